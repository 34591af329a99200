"""Find pixels whose count_work launch is slow (diagnostic)."""
import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np
import __graft_entry__ as ge
pt = ge.load_package()
text = open("scenes/cornell_box.json").read()
sc = pt.Scene.from_json(text, seed=1)
r = pt.HipRenderer(sc, device=0, depth=8)
w, h = 1920, 1080
px = (np.arange(3, h, 12)[:, None] * w + np.arange(5, w, 12)[None, :]).ravel().astype(np.uint32)
fn = sys.argv[1] if len(sys.argv) > 1 else "count"
chunk = 1024
for i in range(0, len(px), chunk):
    sub = px[i:i + chunk]
    t = time.perf_counter()
    if fn == "count":
        pt.count_work(r, sc.camera(), pt.ImageParams(w, h), 4, sub, seed=1)
    else:
        r.trace_pixel_samples(sc.camera(), pt.ImageParams(w, h), 4, sub, seed=1)
    dt = time.perf_counter() - t
    print("chunk %d: %.3f s" % (i, dt), flush=True)
    if dt > 1.0:
        for j in range(0, len(sub), 64):
            s2 = sub[j:j + 64]
            t = time.perf_counter()
            if fn == "count":
                pt.count_work(r, sc.camera(), pt.ImageParams(w, h), 4, s2, seed=1)
            else:
                r.trace_pixel_samples(sc.camera(), pt.ImageParams(w, h), 4, s2, seed=1)
            d2 = time.perf_counter() - t
            if d2 > 0.5:
                print("   slow wave pixels", [int(v) for v in s2], "%.3f s" % d2, flush=True)
        break
