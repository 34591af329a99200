"""One frame's launch sequence from a rocprofv3 kernel_trace CSV: each kernel's duration and the idle gap before it.
   python3 scripts/kt_gaps.py <kernel_trace.csv> [frame index from the end (default 2)]"""
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].startswith(("void pt::", "pt::", "__amd"))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
firsts = [i for i, r in enumerate(rows) if "wf_bounce<true" in r["Kernel_Name"]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
a, b = firsts[-k], firsts[-k + 1]
t0 = int(rows[a]["Start_Timestamp"]); prev_end = None; busy = gaps = 0.0
for r in rows[a - 2:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
    print("%9.1f us  %8.1f us  gap %6.1f  q%s grid %8s  %s" % ((s - t0) / 1e3, (e - s) / 1e3, g, r["Queue_Id"], r["Grid_Size_X"], name))
    busy += (e - s) / 1e3; gaps += max(g, 0.0); prev_end = max(prev_end or 0, e)
print("frame: kernels %.1f us, gaps %.1f us, next frame starts at %.1f us" % (busy, gaps, (int(rows[b]["Start_Timestamp"]) - t0) / 1e3))
