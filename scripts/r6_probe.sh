#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
bash scripts/abx.sh $1 1 "default|--config c5" "default|--config c5 --option wf_paths=33554432" "default|--config c5 --option wf_paths=67108864" "default|--config c5 --option wf_paths=100663296" "default|--config c5 --option wf_bounce_waves=4" "default|--config c5 --option wf_bounce_waves=5"
