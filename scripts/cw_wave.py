"""count_work on the slow 64-pixel wave: time and counters (diagnostic)."""
import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np
import __graft_entry__ as ge
pt = ge.load_package()
sc = pt.Scene.from_json(open("scenes/cornell_box.json").read(), seed=1)
r = pt.HipRenderer(sc, device=0, depth=8)
w, h = 1920, 1080
px = np.array([1688069 + 12 * i for i in range(64)], np.uint32)
for sub in (px, px[:32], px[32:], px[:16], px[16:32], px[32:48], px[48:]):
    t = time.perf_counter()
    cnt = pt.count_work(r, sc.camera(), pt.ImageParams(w, h), 4, sub, seed=1)
    print(len(sub), int(sub[0]), "%.3f s" % (time.perf_counter() - t), cnt, flush=True)
