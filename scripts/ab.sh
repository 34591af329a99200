#!/bin/bash
# A/B bench of variant libraries on the GPU box:  bash scripts/ab.sh <tag> <reps> name1 name2 ...
# ("default" = the in-tree library).  One bench line per (rep, variant) in gpurun_out/<tag>/ab.log.
set -e
tag=$1; reps=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$tag
mkdir -p $OUT
cd $R
for rep in $(seq 1 $reps); do
    for v in "$@"; do
        if [ "$v" = default ]; then lib=""; else lib=$R/variants/$v.so; fi
        echo "== $v rep $rep" >> $OUT/ab.log
        PT_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-pixels 64 --steps 3 ${BENCH_ARGS} \
            >> $OUT/ab.log 2>&1
    done
done
python3 scripts/ab_summary.py $OUT/ab.log > $OUT/ab_summary.txt
cat $OUT/ab_summary.txt
