#!/bin/bash
# A/B bench of (library, bench arguments) pairs on the GPU box:
#   bash scripts/abx.sh <tag> <reps> "<lib>|<bench args>" ...
# <lib>: "default" (the in-tree library) or a name under variants/ (variants/<name>.so).  One bench line per
# (rep, entry) in gpurun_out/<tag>/ab.log, summarized by scripts/ab_summary.py.
set -e
tag=$1; reps=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$tag
mkdir -p $OUT
cd $R
for rep in $(seq 1 $reps); do
    for v in "$@"; do
        name=${v%%|*}; args=${v#*|}; [ "$args" = "-" ] && args=""
        if [ "$name" = default ]; then lib=""; else lib=$R/variants/$name.so; fi
        echo "== $name rep $rep :: $args" >> $OUT/ab.log
        PT_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-pixels 64 --steps 3 $args \
            >> $OUT/ab.log 2>&1
    done
done
python3 scripts/ab_summary.py $OUT/ab.log > $OUT/ab_summary.txt
cat $OUT/ab_summary.txt
