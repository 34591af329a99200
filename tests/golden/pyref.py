"""Independent pure-Python f64 restatement of the reference primitives.

Python floats are IEEE doubles, evaluated left to right with no contraction,
and math.sqrt / math.sin / math.cos / math.tan call the same correctly rounded
or libm routines as the reference, so this restatement is expected to agree
with the C oracle bit for bit.  It is kept in tests/ only and is written from
the reference Rust (cited per function), not from the oracle.
"""
import math


def dot(a, b):  # src/algebra/mod.rs:319-349
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def norm(a):  # :107-110
    l = math.sqrt(dot(a, a))
    return (a[0] / l, a[1] / l, a[2] / l)


def matmul(a, b):  # src/algebra/transform.rs:553-570
    return [[a[i][0] * b[0][j] + a[i][1] * b[1][j] + a[i][2] * b[2][j] + a[i][3] * b[3][j] for j in range(4)]
            for i in range(4)]


def eye():
    return [[1.0 if i == j else 0.0 for j in range(4)] for i in range(4)]


def rad(deg):
    return deg * (math.pi / 180.0)


def roll(deg):  # :364-372
    r = rad(deg)
    m = eye()
    m[1][1], m[1][2], m[2][1], m[2][2] = math.cos(r), -math.sin(r), math.sin(r), math.cos(r)
    return m


def pitch(deg):  # :374-382
    r = rad(deg)
    m = eye()
    m[0][0], m[0][2], m[2][0], m[2][2] = math.cos(r), math.sin(r), -math.sin(r), math.cos(r)
    return m


def yaw(deg):  # :384-392
    r = rad(deg)
    m = eye()
    m[0][0], m[0][1], m[1][0], m[1][1] = math.cos(r), -math.sin(r), math.sin(r), math.cos(r)
    return m


def transform(t, r, s):  # InversableTransform::new, :16-23
    T, S = eye(), eye()
    Ti, Si = eye(), eye()
    for k in range(3):
        T[k][3] = t[k]
        S[k][k] = s[k]
        Ti[k][3] = -t[k]
        Si[k][k] = 1.0 / s[k]
    R = matmul(matmul(roll(r[0]), pitch(r[1])), yaw(r[2]))
    Rinv = matmul(matmul(yaw(-r[2]), pitch(-r[1])), roll(-r[0]))
    return matmul(matmul(T, R), S), matmul(matmul(Si, Rinv), Ti)


def xpoint(m, p):  # :394-409
    return tuple(p[0] * m[i][0] + p[1] * m[i][1] + p[2] * m[i][2] + m[i][3] for i in range(3))


def xvector(m, v):  # :411-417
    return tuple(v[0] * m[i][0] + v[1] * m[i][1] + v[2] * m[i][2] for i in range(3))


def xnormal(m, n):  # :419-425
    return tuple(n[0] * m[0][j] + n[1] * m[1][j] + n[2] * m[2][j] for j in range(3))


def sphere_t(o, d, tmin, tmax):  # src/world/shapes/mod.rs:330-374
    a = dot(d, d)
    hb = dot(d, o)
    c = dot(o, o) - 1.0
    disc = hb * hb - a * c
    if disc < 0.0:
        return None
    if disc == 0.0:
        return -hb * a
    x = (-hb - math.sqrt(disc)) / a
    if x < tmin or x > tmax:
        x = (-hb + math.sqrt(disc)) / a
        if x < tmin or x > tmax:
            return None
    return x


def rect_t(sh, o, d, tmin, tmax):  # :181-204
    t = -o[2] / d[2]
    if t < tmin or t > tmax:
        return None
    px, py = o[0] + d[0] * t, o[1] + d[1] * t
    if px < sh["x0"] or px > sh["x1"] or py < sh["y0"] or py > sh["y1"]:
        return None
    return t


def fmin(a, b):  # f64::min ignores NaN
    if a != a:
        return b
    if b != b:
        return a
    return a if a < b else b


def fmax(a, b):
    if a != a:
        return b
    if b != b:
        return a
    return a if a > b else b


def _div(a, b):
    if b == 0.0:
        if a == 0.0 or a != a:
            return math.nan
        return math.copysign(math.inf, a) * math.copysign(1.0, b)
    return a / b


def cube_t(o, d, tmin, tmax):  # :250-285
    tl = [_div(-1.0 - o[k], d[k]) for k in range(3)]
    tu = [_div(1.0 - o[k], d[k]) for k in range(3)]
    mins = [fmin(tl[k], tu[k]) for k in range(3)]
    maxs = [fmax(tl[k], tu[k]) for k in range(3)]
    lo = fmax(fmax(fmax(mins[0], mins[1]), mins[2]), tmin)
    hi = fmin(fmin(fmin(maxs[0], maxs[1]), maxs[2]), tmax)
    if lo > hi or lo > tmax:
        return None
    return lo


def heart_f(p):  # src/world/shapes/ray_marching.rs:147-155
    x2, y2, z2 = p[0] * p[0], p[1] * p[1], p[2] * p[2]
    z3 = z2 * p[2]
    a = x2 + (9.0 / 4.0) * y2 + z2 - 1.0
    return a * a * a - x2 * z3 - (9.0 / 80.0) * y2 * z3


def heart_grad(p):  # :157-168
    a = p[0] * p[0] + (9.0 / 4.0) * p[1] * p[1] + p[2] * p[2] - 1.0
    a = 3.0 * a * a
    z2 = p[2] * p[2]
    z3 = z2 * p[2]
    return (2.0 * p[0] * (a - z3), (9.0 / 2.0) * p[1] * (a - 0.05 * z3),
            2.0 * p[2] * (a - p[2] * (1.5 * p[0] * p[0] + (27.0 / 40.0) * p[1] * p[1])))


def heart_bound(o, d):  # :135-145 + algebra/equation.rs:5-15
    R = (1.45, 1.45 / 2.05, 1.45)
    oo = tuple(o[k] / R[k] for k in range(3))
    dd = tuple(d[k] / R[k] for k in range(3))
    a, hb, c = dot(dd, dd), dot(dd, oo), dot(oo, oo) - 1.0
    disc = hb * hb - a * c
    if disc < 0.0:
        return None
    if disc == 0.0:
        x1 = x2 = -hb
    else:
        x1, x2 = (-hb - math.sqrt(disc)) / a, (-hb + math.sqrt(disc)) / a
    if x1 < 0.0 and x2 < 0.0:
        return None
    return fmax(x1, 0.0), fmax(x2, 0.0)


def march_t(sh, o, d, tmin, tmax):  # :20-74
    b = heart_bound(o, d)
    if b is None:
        return None
    start, end = b
    step = sh["step"]
    t = start
    p = [o[k] + d[k] * t for k in range(3)]
    r = heart_f(p)
    done = False
    for _ in range(sh.get("depth", 4)):
        while True:
            if t > end or t < start:
                return None
            t += step
            for k in range(3):
                p[k] += d[k] * step
            nxt = heart_f(p)
            if abs(nxt - 0.0) < 1e-15:
                done = True
                break
            if (r < 0.0 and nxt > 0.0) or (r > 0.0 and nxt < 0.0):
                step *= -0.01
                r = nxt
                break
            r = nxt
        if done:
            break
    if t < tmin or t > tmax:
        return None
    return t


def shape_hit(sh, o, d, tmin=0.001, tmax=math.inf):
    """ray_hit_transformed (shapes/mod.rs:112-124): returns (t, point, normal, front) or None."""
    direct, inverse = transform(sh["translate"], sh["rotate"], sh["scale"])
    oo, od = xpoint(inverse, o), xvector(inverse, d)
    kind = sh["type"]
    t = {"Sphere": lambda: sphere_t(oo, od, tmin, tmax), "Rectangle": lambda: rect_t(sh, oo, od, tmin, tmax),
         "Cube": lambda: cube_t(oo, od, tmin, tmax), "Heart": lambda: march_t(sh, oo, od, tmin, tmax)}[kind]()
    if t is None:
        return None
    p = tuple(oo[k] + od[k] * t for k in range(3))
    if kind == "Sphere":
        n = tuple(-x for x in p) if sh.get("inverse_normal") else p
    elif kind == "Rectangle":
        n = (0.0, 0.0, 1.0)
    elif kind == "Cube":
        pa = [abs(x) for x in p]
        mc = fmax(fmax(pa[0], pa[1]), pa[2])
        n = (p[0], 0.0, 0.0) if mc == pa[0] else (0.0, p[1], 0.0) if mc == pa[1] else (0.0, 0.0, p[2])
    else:
        n = heart_grad(p)
    n = norm(n)  # RayHit::new
    wn = xnormal(inverse, n)
    front = dot(wn, d) < 0.0  # set_normal (ray.rs:60-64)
    wn = norm(wn if front else tuple(-x for x in wn))
    return t, xpoint(direct, p), wn, front
