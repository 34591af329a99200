"""Replay captured march jobs (tools/march_prof capture) on the GPU through
pt_march_jobs and compare with the host build's results (march_prof run ...
<results>).  Diagnostic."""
import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np
import __graft_entry__ as ge

pt = ge.load_package()
jobs_f, res_f = sys.argv[1], sys.argv[2]
raw = np.fromfile(jobs_f, dtype=np.dtype([("step", "f8"), ("passes", "i4"), ("pad", "i4"), ("o", "f8", 3), ("d", "f8", 3)]))
jobs = np.zeros((len(raw), 8))
jobs[:, 0] = raw["step"]
jobs[:, 1] = raw["passes"]
jobs[:, 2:5] = raw["o"]
jobs[:, 5:8] = raw["d"]
ref = np.fromfile(res_f, dtype=np.float64).reshape(-1, 3)
text = open("scenes/cornell_box.json").read()
sc = pt.Scene.from_json(text, seed=1)
r = pt.HipRenderer(sc, device=0, depth=8)
t0 = time.perf_counter()
t, hit, it = pt.march_jobs(r, jobs)
print("gpu %.3f s for %d jobs" % (time.perf_counter() - t0, len(jobs)))
bad = np.nonzero((hit != (ref[:, 1] > 0)) | (hit & (t != ref[:, 0])))[0]
print("mismatches", len(bad), "iters gpu mean %.2f max %d, host mean %.2f max %d" % (it.mean(), it.max(), ref[:, 2].mean(), ref[:, 2].max()))
slow = np.nonzero(it > ref[:, 2] + 0)[0]
print("jobs where gpu iterations differ:", len(slow))
for i in list(bad[:5]) + list(slow[:5]):
    print(i, "job", jobs[i].tolist(), "gpu", t[i], hit[i], it[i], "host", ref[i].tolist())
