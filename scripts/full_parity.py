"""Every pixel of a full-spp frame against the oracle (a one-off check on the GPU box, not a test: the oracle
needs minutes of host time at C2's 530 M samples).  The GPU frame is rendered as bench.py renders its timed
frames (render_device on a side stream, the wavefront engine with two chunk streams); the oracle, in the
reference's BvhNode mode, renders the same pixels in row bands with a progress line per band.  Prints the
number of pixels whose three f64 channels differ in any bit (0 expected) and writes a JSON summary.

    python scripts/full_parity.py [--config c2] [--out gpurun_out/full_parity_c2.json] [--threads 16]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def main():
    import torch

    import __graft_entry__ as ge
    import bench
    import oracle
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--out", default=None)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--bands", type=int, default=24)
    a = ap.parse_args()
    scene_name, w, h, spp = bench.CONFIGS[a.config]
    depth, seed, scene_seed = 8, 1, 1
    text = bench.scene_text(scene_name)
    pt = ge.load_package()
    ps = pt.Scene.from_json(text, seed=scene_seed)
    r = pt.HipRenderer(ps, depth=depth)
    frame = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
    s = torch.cuda.Stream()
    t0 = time.time()
    r.render_device(ps.camera(), w, h, spp, seed, 0, 1, frame.data_ptr(), s.cuda_stream)
    s.synchronize()
    img = frame.view(-1, 3).cpu().numpy()
    print("gpu frame %dx%d %d spp in %.2f s" % (w, h, spp, time.time() - t0), flush=True)
    osc = oracle.Scene(text, seed=scene_seed).use_bvh(True, 7)
    bad = 0
    t1 = time.time()
    rows = np.array_split(np.arange(h), a.bands)
    for k, band in enumerate(rows):
        px = (band[:, None] * w + np.arange(w)[None, :]).reshape(-1).astype(np.uint32)
        ref = osc.render(w, h, spp, depth, seed, pixels=px, threads=a.threads)
        diff = np.any(img[px].view(np.uint64) != ref.view(np.uint64), axis=1)
        bad += int(diff.sum())
        print("band %d/%d rows %d-%d: %d differing pixels (%.0f s)" % (k + 1, len(rows), band[0], band[-1],
                                                                       int(diff.sum()), time.time() - t1), flush=True)
    rec = {"config": a.config, "workload": "%s %dx%d %dspp depth %d" % (scene_name, w, h, spp, depth),
           "pixels": w * h, "differing_pixels": bad, "oracle_seconds": round(time.time() - t1, 1),
           "oracle_threads": a.threads, "source_id": pt.source_id(),
           "gpu_path": "render_device on a side stream (wavefront engine, two chunk streams), as bench.py's steps"}
    print(json.dumps(rec))
    if a.out:
        Path(a.out).write_text(json.dumps(rec, indent=1) + "\n")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
