#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
timeout -k 10 400 python -u -m pytest tests/test_gpu_bvh_extremes.py -x -v -m gpu -k "regrouped" --timeout 300 \
    --timeout-method thread > gpurun_out/$1/pytest.log 2>&1
bash scripts/abx.sh $1 2 "default|--config c5" "default|--config c5 --option wf_walk_regroup=16" \
    "default|--config c5 --option wf_walk_regroup=24" "default|--config c5 --option wf_walk_regroup=32"
