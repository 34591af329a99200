"""Wave wall-clock per region of the march kernel on one C2 frame (tuning).

Needs a build with -DPT_MARCH_REGIONS (scripts/variants.sh mreg
"-DPT_MARCH_REGIONS"), loaded through PT_AMD_LIB.  Regions are timed by
each wave's first active lane (s_memtime), so a region's share is the share
of the march kernel's wave time during which some lane of the wave ran it."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.getcwd())
import __graft_entry__ as ge

pt = ge.load_package()
import torch

L = pt.lib()
f = L.pt_march_regions
f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
names = ["iter", "poly+guess", "prefix", "halvings", "advance", "literal", "refill", "total"]
pnames = ["iters", "lin_init", "lit_adds", "advance_loops", "evals", "sir_inside", "lin_fail_zero", "lin_fail_q",
          "lin_fail_tie", "lin_fail_zone"]
buf = (C.c_ulonglong * (2 * len(names) + 2 * len(pnames)))()
sc = pt.Scene.from_json(open("scenes/cornell_box.json").read(), seed=1)
r = pt.HipRenderer(sc, device=0, depth=8)
r.set_option("wf_slots", 1)
cam = sc.camera()
W, H, spp = 1920, 1080, int(sys.argv[1]) if len(sys.argv) > 1 else 64
frame = torch.zeros(W * H * 3, dtype=torch.float64, device="cuda")
r.render_device(cam, W, H, spp, 1, 0, 1, frame.data_ptr(), 0)
torch.cuda.synchronize()
f(buf, 1)
r.render_device(cam, W, H, spp, 1, 0, 1, frame.data_ptr(), 0)
torch.cuda.synchronize()
f(buf, 0)
tot = buf[7]
print("march kernel wave time by region (%% of total wave cycles %.4g), %dx%d %d spp" % (tot, W, H, spp))
R, P = len(names), len(pnames)
for k, n in enumerate(names):
    x, xl = buf[k], buf[R + k]
    print("  %-11s %6.1f%%   lanes active at its start %5.1f of 64" % (n, 100.0 * x / max(1, tot), xl / max(1, x)))
print("profiling points: wave passes, mean lanes per pass (pt_march.hpp PT_MPROF)")
for k, n in enumerate(pnames):
    w, l = buf[2 * R + k], buf[2 * R + P + k]
    if w:
        print("  %-14s %12d passes  %5.1f lanes" % (n, w, l / w))
