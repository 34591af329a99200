"""Lane profile of the bounce kernel on one one-stream cornell frame (tuning).

Needs a build with -DPT_LANE_PROF (scripts/variants.sh lprof "-DPT_LANE_PROF"), loaded through PT_AMD_LIB
(pt_lprof.hpp).  Per profiling point: wave passes, mean active lanes per pass, passes per 1000 live path-bounces;
a point inside a loop counts one pass per trip.

    PT_AMD_LIB=variants/lprof.so python scripts/bounce_lanes.py [spp] [scene] [width height]
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.getcwd())
import __graft_entry__ as ge

pt = ge.load_package()
import torch

NAMES = ["live", "shade_hit", "lambert", "reject_try", "metal", "dielectric", "emit", "ended", "trace",
         "ulist_shape", "rect_rows", "ubox_pass", "bvh_node", "bvh_enter", "bvh_leaf", "pre_slab", "pre_job",
         "any_end", "store"]
L = pt.lib()
f = L.pt_lane_prof
f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
n = f(None, 0)
assert n == len(NAMES), (n, len(NAMES))
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
scene = sys.argv[2] if len(sys.argv) > 2 else "cornell_box.json"
W, H = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (1920, 1080)
if scene.startswith("synthetic_"):
    sys.path.insert(0, "scenes")
    import json
    import make_scenes
    text = json.dumps(make_scenes.synthetic(int(scene.split("_")[1])))
else:
    text = open("scenes/" + scene).read()
sc = pt.Scene.from_json(text, seed=1)
r = pt.HipRenderer(sc, device=0, depth=8)
r.set_option("wf_slots", 1)
cam = sc.camera()
frame = torch.zeros(W * H * 3, dtype=torch.float64, device="cuda")
r.render_device(cam, W, H, spp, 1, 0, 1, frame.data_ptr(), 0)
torch.cuda.synchronize()
buf = (C.c_ulonglong * (2 * n))()
f(buf, 1)
r.render_device(cam, W, H, spp, 1, 0, 1, frame.data_ptr(), 0)
torch.cuda.synchronize()
f(buf, 0)
live_lanes = buf[n + 0]
print("bounce kernel lane profile: %s %dx%d %d spp, one chunk stream; %d live path-bounces (%.2f per sample)"
      % (scene, W, H, spp, live_lanes, live_lanes / (W * H * spp)))
print("  %-12s %14s %8s %16s %18s" % ("point", "wave passes", "lanes", "passes/1k paths", "lane-passes/1k"))
for k, name in enumerate(NAMES):
    w, l = buf[k], buf[n + k]
    if w:
        print("  %-12s %14d %8.1f %16.2f %18.1f" % (name, w, l / w, 1000.0 * w / live_lanes, 1000.0 * l / live_lanes))
