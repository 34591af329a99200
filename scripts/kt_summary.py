"""Per-kernel total/avg time from a rocprofv3 kernel_trace CSV."""
import collections, csv, glob, sys
acc = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:34]
        acc[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        n[k] += 1
for k, v in sorted(acc.items(), key=lambda x: -x[1]):
    print("%-36s %5d launches  %10.3f ms total  %9.3f ms avg" % (k, n[k], v, v / n[k]))
