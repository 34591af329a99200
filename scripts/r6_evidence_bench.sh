#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/evidence.sh $1 bench
bash scripts/evidence.sh $1 kt
find gpurun_out/$1 -name "*.csv" -size +2M -delete
KT_FRAMES=4 PROF_TIMEOUT=300 bash scripts/gpu.sh kt $1/kt_c5 --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-kernel-timing
find gpurun_out/$1 -name "*.csv" -size +2M -delete
du -sh gpurun_out/$1
