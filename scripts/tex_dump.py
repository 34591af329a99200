import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.getcwd() + "/oracle")
import numpy as np
import __graft_entry__ as ge
import oracle as O
pt = ge.load_package()
out = {}
for name, seed, depth in [("textured.json", 1, 8), ("noise.json", 2, 8)]:
    text = open("scenes/" + name).read()
    ps = pt.Scene.from_json(text, seed=seed)
    r = pt.HipRenderer(ps, depth=depth)
    img = r.render(ps.camera(), pt.ImageParams(64, 36), 4, seed=seed)
    out[name] = img
np.savez("gpurun_out/tex_dump.npz", **out)
print("ok")
