import sys, ctypes as C, numpy as np
sys.path.insert(0, 'tests'); sys.path.insert(0, 'oracle')
import test_march_exact as T
from conftest import native_lib
L = C.CDLL(native_lib("libmarch.so"))
L.march_heart_coop.argtypes = [C.c_double, C.c_int] + [C.POINTER(C.c_double)] * 3 + [C.c_double, C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_uint32)]
sc = T.heart_scene([212.5, 200, 147.5], [-95, -18, 0], [82.5, 82.5, 82.5])
inv = (C.c_double * 12)(*list(sc.shape(0).inverse)[:12])
rng = np.random.default_rng(5)
n = 20000
o = rng.uniform([0, 0, 0], [555, 555, 555], size=(n, 3))
tgt = rng.uniform([110, 140, 50], [320, 260, 250], size=(n, 3))
d = tgt - o; d /= np.linalg.norm(d, axis=1, keepdims=True)
t = C.c_double(); lat = (C.c_uint32 * 2)()
P = []; Q = []
for i in range(n):
    got = L.march_heart_coop(0.01, 4, inv, (C.c_double*3)(*o[i]), (C.c_double*3)(*d[i]), 0.001, float('inf'), C.byref(t), lat)
    P.append(lat[1]); Q.append(lat[0])
P = np.array(P); Q = np.array(Q)
m = P > 0
P, Q = P[m], Q[m]
print('rays marched', len(P))
for q in (50, 90, 99, 99.9, 100):
    print('pct %5.1f plain %6.1f coop %6.1f' % (q, np.percentile(P, q), np.percentile(Q, q)))
big = P >= np.percentile(P, 99)
print('on the top 1%% plain jobs: plain mean %.1f coop mean %.1f' % (P[big].mean(), Q[big].mean()))
