#!/bin/bash
# A/B bench of renderer options or bench arguments on the GPU box:
#   bash scripts/optab.sh <tag> <reps> "<bench args A>" "<bench args B>" ...
# ("-" = no extra arguments).  One bench line per (rep, variant) in gpurun_out/<tag>/ab.log.
set -e
tag=$1; reps=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$tag
mkdir -p $OUT
cd $R
for rep in $(seq 1 $reps); do
    i=0
    for v in "$@"; do
        i=$((i + 1))
        a=$v; [ "$a" = "-" ] && a=""
        echo "== v$i rep $rep :: $a" >> $OUT/ab.log
        timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-pixels 64 --steps 3 $a >> $OUT/ab.log 2>&1
    done
done
python3 scripts/ab_summary.py $OUT/ab.log > $OUT/ab_summary.txt
cat $OUT/ab_summary.txt
