# GPU suite + smoke + default bench at HEAD (the tree the driver runs at round end)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/head_check
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 300 python bench.py > $OUT/bench_default.log 2>&1
