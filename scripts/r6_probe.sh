#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
T=gpurun_out/$1
mkdir -p $T
for o in "" "--option wf_slots=3" "--option wf_min_chunks=4" "--option wf_paths=16777216" "--option wf_slots=3 --option wf_min_chunks=6" "--option wf_paths=25165824"; do
    echo "== $o" >> $T/rs.txt
    timeout -k 10 300 python -u scripts/rank_sim.py --worlds 8 $o 2>&1 | grep '"world"' >> $T/rs.txt
done
cat $T/rs.txt | cut -c1-200
