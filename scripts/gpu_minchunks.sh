# 8-rank C2 share: sample chunks per frame (PT_WF_MIN_CHUNKS) on the slowest and a fast rank
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/minchunks
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
R="python -u scripts/rank_sim.py --worlds 8 --ranks 0,3,4 --reps 3"
timeout -k 10 200 $R > $OUT/mc1.log 2>&1
PT_WF_MIN_CHUNKS=8 timeout -k 10 200 $R > $OUT/mc8.log 2>&1
PT_WF_MIN_CHUNKS=16 timeout -k 10 200 $R > $OUT/mc16.log 2>&1
timeout -k 10 200 $R > $OUT/mc1b.log 2>&1
