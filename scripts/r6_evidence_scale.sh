#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/evidence.sh $1 bench4
bash scripts/evidence.sh $1 ranksim
