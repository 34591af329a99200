"""Time pt_count_work (the megakernel STATS build) on the bench's pixel sample."""
import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np
import __graft_entry__ as ge
pt = ge.load_package()
text = open("scenes/cornell_box.json").read()
sc = pt.Scene.from_json(text, seed=1)
r = pt.HipRenderer(sc, device=0, depth=8)
w, h = 1920, 1080
stride = int(sys.argv[1]) if len(sys.argv) > 1 else 12
px = (np.arange(3, h, stride)[:, None] * w + np.arange(5, w, stride)[None, :]).ravel().astype(np.uint32)
t = time.perf_counter()
cnt = pt.count_work(r, sc.camera(), pt.ImageParams(w, h), 4, px, seed=1)
print("count_work %d px: %.3f s" % (len(px), time.perf_counter() - t), {k: cnt[k] for k in ("samples", "march_steps", "march_tries")}, flush=True)
t = time.perf_counter()
out = r.trace_pixel_samples(sc.camera(), pt.ImageParams(w, h), 4, px, seed=1)
print("trace_pixel_samples: %.3f s" % (time.perf_counter() - t), flush=True)
