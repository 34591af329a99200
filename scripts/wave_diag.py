"""Phase diagnostics of the wavefront march kernel on one frame (tuning).  Needs a diagnostics build of the
library (the product build compiles the instrumentation out):
    make -C rs-pathtracing_amd LIB=../variants/diag.so BUILD=build_diag EXTRA=-DPT_WAVE_DIAG=1
    PT_AMD_LIB=variants/diag.so python scripts/wave_diag.py [spp]"""
import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import __graft_entry__ as ge
pt = ge.load_package()
import torch
sc = pt.Scene.from_json(open("scenes/cornell_box.json").read(), seed=1)
r = pt.HipRenderer(sc, device=0, depth=8)
cam = sc.camera()
W, H, spp = 1920, 1080, int(sys.argv[1]) if len(sys.argv) > 1 else 8
frame = torch.zeros(W * H * 3, dtype=torch.float64, device="cuda")
r.render_device(cam, W, H, spp, 1, 0, 1, frame.data_ptr(), 0)
torch.cuda.synchronize()
pt.wave_diag(r, True)  # enable + clear
r.render_device(cam, W, H, spp, 1, 0, 1, frame.data_ptr(), 0)
torch.cuda.synchronize()
d = pt.wave_diag(r, False)
trips, cyc, lanes = d[:16], d[16:32], d[32:36]
bsec = d[36:43]
blan = d[48:55]
print("bounce sections (wave cycles of the diag build, each section ended by a full wait; lanes: "
      "scripts/bounce_lanes.py): " + ", ".join(
    "%s %.1f%%%s" % (n, 100 * x / max(1, sum(bsec)), (" (%.1f lanes)" % (l / x)) if any(blan) and x else "")
    for n, x, l in zip(["list", "state", "shade", "end", "trace", "precheck", "store"], bsec, blan)))
names = ["cheap", "select", "adv", "proof"]
tot_trips, tot_cyc = sum(trips), sum(cyc)
print("total trips %d  cycles %.3g" % (tot_trips, tot_cyc))
for m in range(16):
    if trips[m]:
        print("  mix %-26s trips %5.1f%%  cyc/trip %8.0f  cycles %5.1f%%" % (
            "+".join(n for k, n in enumerate(names) if m >> k & 1), 100 * trips[m] / tot_trips,
            cyc[m] / trips[m], 100 * cyc[m] / tot_cyc))
for k, n in enumerate(names):
    present = sum(trips[m] for m in range(16) if m >> k & 1)
    print("  %-7s present in %5.1f%% of trips, avg lanes when present %.1f" % (n, 100 * present / tot_trips, lanes[k] / max(1, present)))
