#!/bin/bash
# C1 launch timelines (depth 8 and 50): kernel traces for the gap analysis (scripts/kt_gaps.py)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/gpu.sh kt $1_d8 --config c1 --steps 20 --warmup 3 --no-cpu-baseline --parity-pixels 64 --no-roofline-leg
bash scripts/gpu.sh kt $1_d50 --config c1 --depth 50 --steps 10 --warmup 2 --no-cpu-baseline --parity-pixels 64 --no-roofline-leg
