#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
bash scripts/abx.sh $1 1 "default|--option wf_trace=5 --no-parity" "noappend|--option wf_trace=5 --no-parity" "noappend|--option wf_trace=4 --no-parity"
