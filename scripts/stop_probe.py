"""Stop-latency probe of a progressive frame (pt_render_stop): full-frame
times of the progressive and the device path, and the time a stop takes at
several points of a C3-size frame.   python scripts/stop_probe.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib

pt = importlib.import_module("rs-pathtracing_amd")
import torch

text = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "scenes", "cornell_box.json")).read()
ps = pt.Scene.from_json(text, seed=1)
r = pt.HipRenderer(ps, depth=8)
cam = ps.camera()
w, h, spp = 3840, 2160, int(os.environ.get("SPP", "256"))
buf = np.zeros((w * h, 3))
stream = torch.cuda.current_stream().cuda_stream
frame = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
for rep in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r.render_device(cam, w, h, spp, 1, 0, 1, frame.data_ptr(), stream)
    torch.cuda.synchronize()
    print("device frame %dx%d %d spp: %.1f ms" % (w, h, spp, (time.perf_counter() - t0) * 1e3), flush=True)
    t0 = time.perf_counter()
    r.start_rendering(cam, pt.ImageParams(w, h), spp, seed=1)
    while not r.render_step(buf, blocking=False):
        time.sleep(0.001)
    print("progressive frame: %.1f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)
for delay in (0.0, 0.1, 0.3, 0.6):
    r.start_rendering(cam, pt.ImageParams(w, h), spp, seed=1)
    time.sleep(delay)
    t0 = time.perf_counter()
    r.stop_rendering()
    print("stop after %.1f s: %.1f ms" % (delay, (time.perf_counter() - t0) * 1e3), flush=True)
