"""Sum rocprofv3 --pmc counter_collection CSVs per kernel family."""
import collections
import csv
import glob
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0].replace("void ", "")[:32]
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
            n[k].add(row.get("Dispatch_Id"))
for k, c in acc.items():
    print("%s  (%d dispatches)" % (k, len(n[k])))
    for name, v in sorted(c.items()):
        print("    %-26s %.4g" % (name, v))
