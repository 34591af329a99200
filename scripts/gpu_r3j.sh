# A/B of a bounce/march change on C2: GPU suite (parity), two bench runs
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3j}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-pixels 96 > $OUT/bench_c2_a.json 2> $OUT/bench_c2_a.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity > $OUT/bench_c2_b.json 2> $OUT/bench_c2_b.err
