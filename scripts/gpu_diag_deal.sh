# diagonal multi-rank tile deal: GPU suite (device shard + unshard parity), rank-share simulation, default bench
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/diag_deal
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 400 python -u scripts/rank_sim.py --worlds 1,2,4,8 > $OUT/rank_sim.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_default.log 2>&1
