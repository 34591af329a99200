#!/bin/bash
# Final-build checks, part 2: every pixel of full 256-spp C2 and C5 frames against the oracle.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
T=gpurun_out/$1
mkdir -p $T
timeout -k 10 540 python -u scripts/full_parity.py --config c2 --out $T/full_parity_c2.json > $T/full_parity_c2.txt 2>&1
timeout -k 10 900 python -u scripts/full_parity.py --config c5 --out $T/full_parity_c5.json > $T/full_parity_c5.txt 2>&1
