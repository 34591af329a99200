#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
timeout -k 10 300 python -u scripts/interactive_bench.py --display-only --out gpurun_out/$1/interactive_display_only.jsonl > gpurun_out/$1/inter.log 2>&1
cut -c1-400 gpurun_out/$1/interactive_display_only.jsonl
