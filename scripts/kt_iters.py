"""Per-iteration launch profile of the wavefront engine from a rocprofv3 kernel trace of one-stream frames
(`bench.py --slots 1`): for each bounce iteration `it` of a chunk, the mean duration of its bounce and march
launches and of the gap from the bounce's start to the march's end, summed over the chunks of the traced frames; wf_tail
launches (before the bounce of their iteration) are summed per iteration, with the longest one.

    python scripts/kt_iters.py <kernel_trace.csv> [first_frame_index]

A chunk starts with a first-iteration bounce (wf_bounce<true, ..>); iteration it of the chunk is its it-th
bounce launch, and the march launch that follows it belongs to the same iteration.  Only frames before the
count_work probe are counted.
"""
import collections
import csv
import re
import sys

FIRST = re.compile(r"wf_bounce<true")  # a chunk's first-iteration bounce (the FIRST template argument)


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    stop = [i for i, r in enumerate(rows) if "count_work" in r["Kernel_Name"]]
    rows = rows[:stop[0]] if stop else rows
    it = -1
    per = collections.defaultdict(lambda: {"bounce": [0, 0.0], "march": [0, 0.0], "cp": [0, 0.0], "tail": [0, 0.0]})
    chunks = 0
    tmax = {}  # longest tail launch per iteration (us)
    for r in rows:
        name = r["Kernel_Name"]
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        if "wf_bounce" in name:
            if FIRST.search(name):
                it = 0
                chunks += 1
            else:
                it += 1
            kind = "bounce"
        elif "wf_march" in name:
            kind = "march"
        elif "cp_" in name:
            kind = "cp"
        elif "wf_tail" in name:  # launched before the bounce of the next iteration
            if it >= 0:
                per[it + 1]["tail"][0] += 1
                per[it + 1]["tail"][1] += dur
                tmax[it + 1] = max(tmax.get(it + 1, 0.0), dur * 1e3)
            continue
        else:
            continue
        if it < 0:
            continue
        per[it][kind][0] += 1
        per[it][kind][1] += dur
    print("%d chunks traced" % chunks)
    print("%4s %10s %10s %10s %10s %10s %10s %10s" % ("it", "bounce ms", "avg us", "march ms", "avg us", "cp ms",
                                                      "tail ms", "max us"))
    tot = collections.Counter()
    for k in sorted(per):
        b, m, c, t = per[k]["bounce"], per[k]["march"], per[k]["cp"], per[k]["tail"]
        tot["b"] += b[1]
        tot["m"] += m[1]
        tot["c"] += c[1]
        tot["t"] += t[1]
        print("%4d %10.3f %10.1f %10.3f %10.1f %10.3f %10.3f %10.1f" % (
            k, b[1], b[1] / max(1, b[0]) * 1e3, m[1], m[1] / max(1, m[0]) * 1e3, c[1], t[1], tmax.get(k, 0.0)))
    print("total: bounce %.3f ms, march %.3f ms, compaction %.3f ms, tail %.3f ms" % (tot["b"], tot["m"], tot["c"],
                                                                                     tot["t"]))


if __name__ == "__main__":
    main()
