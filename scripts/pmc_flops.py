"""Counter-derived f64 FLOPs per sample of the wavefront kernels, from one
rocprofv3 --pmc pass of SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64,
SQ_THREAD_CYCLES_VALU and SQ_ACTIVE_INST_VALU (scripts/gpu.sh sq) over a bench
run of `frames` frames of `samples` camera samples each:

    python scripts/pmc_flops.py <sq dir> <frames> <samples per frame> <out.json> "<workload>"

The SQ_INSTS_VALU_*_F64 counters count wave instructions; the lanes each one
covers are estimated by the kernel's mean active lanes per VALU instruction
(SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU; 64 = no divergence).

* executed: every f64 lane operation the hardware ran, FMA = 2.  The kernels
  are built with -ffp-contract=off, so every FMA comes from a division or
  square-root expansion (v_rcp/v_rsq seed + Newton FMAs) or from the march's
  explicit reciprocal estimates, never from the reference's own arithmetic.
* algorithmic: ADD + MUL lane operations, the reference's additions,
  subtractions and multiplications; each division or square root adds one MUL
  (the quotient/root product of its expansion) and no ADD, so it counts as
  one FLOP, the convention of bench.py's FLOP_WEIGHTS.
* PMC_FMA_PER_TRANS=R (environment): for a build that does some of the
  reference's arithmetic as explicit FMAs (the FMA_SLAB bounce build for large
  BVHs: b * (1/d) - o/d), the FMAs beyond R per TRANS instruction count as
  algorithmic, 2 FLOPs each; R is the expansion FMAs per TRANS measured on the
  same workload with the subtract-multiply build (C5: 377.5 / 59.7 = 6.32).
"""
import os
import collections
import csv
import glob
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def source_id():
    """The build the counters were collected on (bench.py uses the file only for that build)."""
    import __graft_entry__
    return __graft_entry__.load_package().source_id()

d, frames, samples, out, workload = sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), sys.argv[4], sys.argv[5]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"]
        kind = ("bounce" if "wf_bounce" in name else "march" if "wf_march" in name else
                "walk" if "wf_walk" in name else None)
        if kind:
            acc[kind][row["Counter_Name"]] += float(row["Counter_Value"])
res = {"workload": workload, "source_id": source_id(), "frames": frames, "samples_per_frame": samples,
       "source": "rocprofv3 --pmc SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU",
       "kinds": {}}
for kind, c in acc.items():
    lanes = c["SQ_THREAD_CYCLES_VALU"] / max(1.0, c["SQ_ACTIVE_INST_VALU"])
    per = lambda k: c[k] / frames * lanes / samples  # lane operations per sample
    add, mul, fma, trans = (per("SQ_INSTS_VALU_%s_F64" % k) for k in ("ADD", "MUL", "FMA", "TRANS"))
    res["kinds"][kind] = {
        "mean_active_lanes": round(lanes, 2),
        "wave_instrs_per_frame": {k: c["SQ_INSTS_VALU_%s_F64" % k] / frames for k in ("ADD", "MUL", "FMA", "TRANS")},
        "valu_wave_instrs_per_frame": c["SQ_INSTS_VALU"] / frames,
        "per_sample": {"add": round(add, 1), "mul": round(mul, 1), "fma": round(fma, 1), "trans": round(trans, 1)},
        "executed_flops_per_sample": round(add + mul + 2 * fma + trans, 1),
        "algorithmic_flops_per_sample": round(add + mul, 1),
    }
    if os.environ.get("PMC_FMA_PER_TRANS"):
        r = float(os.environ["PMC_FMA_PER_TRANS"])
        alg_fma = max(0.0, fma - r * trans)
        res["kinds"][kind]["algorithmic_flops_per_sample"] = round(add + mul + 2 * alg_fma, 1)
        res["kinds"][kind]["fma_correction"] = {
            "expansion_fma_per_trans": r, "algorithmic_fma_per_sample": round(alg_fma, 1),
            "note": "FMAs beyond the division / square-root expansions' R per TRANS are the reference's own "
                    "multiply-adds (2 FLOPs each)"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
