#!/bin/bash
# Kernel timeline of the interactive workload (1600x900 depth 50, 1 spp, progressive render_step)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
T=gpurun_out/$1
mkdir -p $T
timeout -k 10 120 python -u scripts/interactive_bench.py --spp 1 --reps 3 --no-parity > $T/inter_plain.log 2>&1
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $R/$T/kt -o it -- python3 $R/scripts/interactive_bench.py --spp 1 --reps 3 --no-parity) > $T/kt.log 2>&1
du -sh $T
