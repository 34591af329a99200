#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/evidence.sh $1 pmc
bash scripts/evidence.sh $1 stall
# the summaries are written; the raw per-dispatch CSVs would exceed what a call may bring back
find gpurun_out/$1 -name "*.csv" -size +512k -delete
du -sh gpurun_out/$1
