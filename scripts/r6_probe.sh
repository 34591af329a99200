#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
timeout -k 10 600 python -u scripts/rank_sim.py --worlds 1,8 > gpurun_out/$1/rank_sim_default.txt 2>&1
PT_AMD_LIB=$R/variants/unw17.so timeout -k 10 600 python -u scripts/rank_sim.py --worlds 1,8 > gpurun_out/$1/rank_sim_unw17.txt 2>&1
timeout -k 10 600 python -u scripts/rank_sim.py --worlds 8 > gpurun_out/$1/rank_sim_default2.txt 2>&1
grep '"world"' gpurun_out/$1/rank_sim_*.txt
