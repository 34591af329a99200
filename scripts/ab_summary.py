"""Summary of an A/B log (scripts/ab.sh, scripts/optab.sh): value, exactness and
the one-stream kernel times per variant."""
import collections
import json
import sys

vals = collections.defaultdict(list)
cur = None
for line in open(sys.argv[1]):
    if line.startswith("== "):
        cur = line[3:].split(" rep ")[0] + (" ::" + line.split("::", 1)[1].rstrip() if "::" in line else "")
    elif line.startswith("{"):
        r = json.loads(line)
        k = r["roofline"]["kernels"]
        vals[cur].append((r["value"], r.get("exact_pixels_frac"), k.get("wf_march", {}).get("ms_per_frame"),
                          k.get("wf_bounce", {}).get("ms_per_frame"), k.get("wf_walk", {}).get("ms_per_frame")))
for v, xs in vals.items():
    walk = "  iso walk ms %s" % [x[4] for x in xs] if any(x[4] for x in xs) else ""
    print("%-40s value %s  exact %s  iso march ms %s  iso bounce ms %s%s" % (v, [x[0] for x in xs], [x[1] for x in xs],
          [x[2] for x in xs], [x[3] for x in xs], walk))
