# HEAD: GPU suite, smoke, rank-share simulation of the 1/2/4/8-GPU C2 partitions (scripts/rank_sim.py)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/final_check2
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
true
