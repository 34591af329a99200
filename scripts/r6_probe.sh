#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
bash scripts/abx.sh $1 2 "default|--config c5" "wscal|--config c5"
