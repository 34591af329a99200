#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
bash scripts/abx.sh $1 1 "default|--depth 50" "default|--depth 50 --option wf_march_slice=128" "default|--depth 50 --option wf_march_slice=512" "default|--depth 50 --option wf_march_slice=0" "default|--depth 50 --option wf_bounce_waves=4" "default|--depth 50 --option wf_bounce_waves=2"
