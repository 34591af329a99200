import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import torch
import __graft_entry__ as ge
pt = ge.load_package()
if os.environ.get('PT_LIB'):
    from pathlib import Path
    pt.LIB_PATH = Path(os.environ['PT_LIB'])
SYNC = os.environ.get('SYNC') == '1'
text = open("scenes/" + sys.argv[1]).read()
ps = pt.Scene.from_json(text, seed=4)
r = pt.HipRenderer(ps, depth=8)
cam = ps.camera()
w, h = 96, 54
full = r.render(cam, pt.ImageParams(w, h), 2, seed=1)
full2 = r.render(cam, pt.ImageParams(w, h), 2, seed=1)
print("render repeat equal", np.array_equal(full, full2), np.abs(full - full2).max())
stream = torch.cuda.current_stream().cuda_stream
one = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
r.render_device(cam, w, h, 2, 1, 0, 1, one.data_ptr(), stream)
torch.cuda.synchronize()
one = one.view(-1, 3).cpu().numpy()
print("render_device world1 equal", np.array_equal(one, full), np.abs(one - full).max())
for world in (2, 3):
    per = pt.shard_tiles(w, h, 0, world)
    shards = torch.zeros(world * per * 256 * 3, dtype=torch.float64, device="cuda")
    frame = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
    for k in range(world):
        r.render_device(cam, w, h, 2, 1, k, world, shards.data_ptr() + k * per * 256 * 3 * 8, stream)
        if SYNC:
            torch.cuda.synchronize()
    pt.unshard_device(shards.data_ptr(), w, h, world, frame.data_ptr(), stream)
    torch.cuda.synchronize()
    f = frame.view(-1, 3).cpu().numpy()
    bad = np.any(f != full, axis=1)
    print("world", world, "equal", np.array_equal(f, full), "bad px", bad.sum(), "max", np.abs(f - full).max())
    idx = np.nonzero(bad)[0][:10]
    print("   bad pixels", [(int(i % w), int(i // w)) for i in idx], f[idx[:3]], full[idx[:3]])
