#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
bash scripts/abx.sh $1 2 "default|--depth 50" "default|--depth 50 --option wf_paths=268435456" "default|--depth 50 --option wf_paths=201326592"
