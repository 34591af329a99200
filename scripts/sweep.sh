#!/bin/bash
# Option sweep on one box: bash scripts/sweep.sh <tag> <reps> "opts1" "opts2" ...  (bench.py --option lists)
set -e
tag=$1; reps=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$tag
mkdir -p $OUT
cd $R
for rep in $(seq 1 $reps); do
    for o in "$@"; do
        args=""
        for kv in $o; do args="$args --option $kv"; done
        echo "== $o rep $rep" >> $OUT/sweep.log
        timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-pixels 64 --steps 3 $args >> $OUT/sweep.log 2>&1
    done
done
python3 - "$OUT/sweep.log" > $OUT/sweep_summary.txt <<'PY'
import json, sys, collections
res = collections.defaultdict(list); cur = None
for line in open(sys.argv[1]):
    if line.startswith("=="): cur = line[3:].rsplit(" rep ", 1)[0]; continue
    if line.startswith("{"):
        r = json.loads(line); res[cur].append((r["value"], r.get("exact_pixels_frac")))
for k, v in res.items(): print("%-40s %s" % (k, v))
PY
cat $OUT/sweep_summary.txt
