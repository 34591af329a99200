#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
bash scripts/abx.sh $1 2 "default|-" "memclause|-" "minreg|-" "default|--config c5" "memclause|--config c5" "minreg|--config c5"
