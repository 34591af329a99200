#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/$1/pytest_gpu.log 2>&1
tail -2 gpurun_out/$1/pytest_gpu.log
timeout -k 10 300 python -u scripts/interactive_bench.py --out gpurun_out/$1/interactive.jsonl > gpurun_out/$1/interactive.log 2>&1
cut -c1-330 gpurun_out/$1/interactive.jsonl
