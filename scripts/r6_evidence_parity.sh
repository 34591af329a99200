#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
T=gpurun_out/$1
mkdir -p $T
PROF_TIMEOUT=400 bash scripts/gpu.sh kt $1/kt_c5 --config c5 --no-cpu-baseline --no-parity --no-kernel-timing
timeout -k 10 900 python -u scripts/full_parity.py --config c2 --out $T/full_parity_c2.json > $T/full_parity_c2.txt 2>&1
timeout -k 10 1000 python -u scripts/full_parity.py --config c5 --out $T/full_parity_c5.json > $T/full_parity_c5.txt 2>&1
