import sys, os, json, time
sys.path.insert(0, os.getcwd())
import __graft_entry__ as ge
pt = ge.load_package()
import torch
text = open("scenes/cornell_box.json").read()
sc = pt.Scene.from_json(text, seed=1)
r = pt.HipRenderer(sc, device=0, depth=8)
cam = sc.camera()
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 16
for w, h in [(1920, 1080)]:
    t = time.perf_counter()
    d = pt.profile_phases(r, cam, pt.ImageParams(w, h), spp)
    dt = time.perf_counter() - t
    tot = d["trace"] + d["march"] + d["select"] + d["shade"]
    d["frac"] = {k: round(d[k] / tot, 4) for k in ["trace", "march", "select", "shade", "shade_finish",
                                                     "shade_scatter", "shade_restart"]}
    d["wall_s"] = dt
    d["msps"] = w * h * spp / dt / 1e6
    d["passes_per_sample"] = d["passes"] / (w * h * spp)
    d["march_passes_per_sample"] = d["march_passes"] / (w * h * spp)
    print(json.dumps(d), flush=True)
