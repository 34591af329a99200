# Round-1 evidence run on one MI355X: GPU tests, smoke, default bench, rocprofv3
# kernel stats of the same bench command, PMC FETCH/WRITE passes (separate runs).
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/r1final_end
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -q -x -m gpu > $OUT/pytest_gpu.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o bench -- python3 $GRAFT_REPO_ROOT/bench.py > $OUT/kt_bench.log 2>&1
B="python3 $GRAFT_REPO_ROOT/bench.py --spp 8 --steps 1 --warmup 0 --no-cpu-baseline --no-parity"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/pmc_fetch -o p --pmc FETCH_SIZE -- $B > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/pmc_write -o p --pmc WRITE_SIZE -- $B > $OUT/pmc_write.log 2>&1
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --parity-pixels 16 > $OUT/c5.log 2>&1
