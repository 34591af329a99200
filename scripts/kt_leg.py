"""rocprofv3 kernel-trace averages over bench.py's one-stream roofline frame
(every launch alone on the device), to compare with the bench line's
roofline.kernels[*].kernel_ms_avg (HIP events):

    python scripts/kt_leg.py <kernel_trace.csv> <frames in the run>

<frames in the run> = warmup + steps + 1 (the roofline frame).  The roofline
frame is the last frame before the count_work probe; a frame's chunks each
start with one first-iteration bounce launch (wf_bounce<true, ..>).
"""
import collections
import csv
import re
import sys

FIRST = re.compile(r"wf_bounce<true")  # a chunk's first-iteration bounce (the FIRST template argument)

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
total_frames = int(sys.argv[2])
end = max(i for i, r in enumerate(rows) if "count_work" in r["Kernel_Name"])
firsts = [i for i in range(end) if FIRST.search(rows[i]["Kernel_Name"])]
chunks = len(firsts) // total_frames
start = firsts[-chunks]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows[start:end]:
    name = r["Kernel_Name"]
    key = ("wf_bounce" if "wf_bounce" in name else "wf_march" if "wf_march" in name else
           "wf_walk" if "wf_walk" in name else "wf_tail" if "wf_tail" in name else
           "compaction" if "cp_" in name else "wf_reduce" if "wf_reduce" in name else name[:40])
    agg[key][0] += 1
    agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
print("one-stream roofline frame: %d chunks" % chunks)
for k, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("%-32s %6d launches  %10.3f ms  %8.4f ms avg" % (k, n, ms, ms / max(1, n)))
