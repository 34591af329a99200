#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/$1/pytest_gpu.log 2>&1
tail -3 gpurun_out/$1/pytest_gpu.log
bash scripts/abx.sh $1 2 "default|--config c1 --steps 50" "nograph|--config c1 --steps 50" \
    "default|--config c1 --depth 50 --steps 20" "nograph|--config c1 --depth 50 --steps 20" "default|-" "nograph|-"
