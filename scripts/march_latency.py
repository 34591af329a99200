"""Latency of single march jobs on the GPU (development probe, not a test).

Runs the skipping Heart march (pt_march_jobs) over captured cornell march jobs (tools/march_prof capture
format), first all of them in one launch, then the 64 jobs with the most march iterations one launch each, then 64
random ones one launch each.  Run it under rocprofv3 --kernel-trace: the march_probe durations, in launch order,
are the per-job latencies of a lone lane.

    python scripts/march_latency.py <jobs.bin> <out.json>
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import __graft_entry__ as ge
    pt = ge.load_package()
    raw = np.fromfile(sys.argv[1], dtype=[("step", "f8"), ("passes", "i4"), ("pad", "i4"), ("o", "f8", 3),
                                          ("d", "f8", 3)])
    J = np.zeros((len(raw), 8))
    J[:, 0] = raw["step"]
    J[:, 1] = raw["passes"]
    J[:, 2:5] = raw["o"]
    J[:, 5:8] = raw["d"]
    scene = pt.Scene.from_json((ROOT / "scenes" / "cornell_box.json").read_text(), seed=1)
    r = pt.HipRenderer(scene, depth=8)
    t, hit, it = pt.march_jobs(r, J)
    t2, hit2, it2 = pt.march_jobs(r, J)
    top = np.argsort(-it.astype(np.int64), kind="stable")[:64]
    rnd = np.random.default_rng(1).choice(len(J), 64, replace=False)
    for i in list(top) + list(rnd):
        pt.march_jobs(r, J[i:i + 1])
    hist = np.bincount(it.astype(np.int64))
    Path(sys.argv[2]).write_text(json.dumps({
        "jobs": int(len(J)), "hits": int(hit.sum()), "iters_hist": hist.tolist(),
        "top": [[int(i), int(it[i])] for i in top], "random": [[int(i), int(it[i])] for i in rnd]}))


if __name__ == "__main__":
    main()
