# Octant-ordered threaded BVH: full GPU suite, C5 and C2 bench lines
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/r3c
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -v -m gpu -k c5 --timeout 200 --timeout-method thread > $OUT/pytest_c5.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
