"""Per-pixel timing and counters of the megakernel on a pixel list (diagnostic)."""
import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np
import __graft_entry__ as ge
pt = ge.load_package()
sc = pt.Scene.from_json(open("scenes/cornell_box.json").read(), seed=1)
r = pt.HipRenderer(sc, device=0, depth=8)
w, h = 1920, 1080
px = [1688069 + 12 * i for i in range(64)]
for p in px:
    a = np.array([p], np.uint32)
    t = time.perf_counter()
    cnt = pt.count_work(r, sc.camera(), pt.ImageParams(w, h), 4, a, seed=1)
    dt = time.perf_counter() - t
    t = time.perf_counter()
    r.trace_pixel_samples(sc.camera(), pt.ImageParams(w, h), 4, a, seed=1)
    dt2 = time.perf_counter() - t
    if dt > 0.05 or dt2 > 0.05:
        print(p, "count %.3f s  trace %.3f s" % (dt, dt2), cnt, flush=True)
t = time.perf_counter()
r.trace_pixel_samples(sc.camera(), pt.ImageParams(w, h), 4, np.array(px, np.uint32), seed=1)
print("whole wave trace_pixel_samples %.3f s" % (time.perf_counter() - t), flush=True)
