# Ground sphere out of the BVH + leaf-size sweep on C5; GPU suite
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/r3d
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -v -m gpu -k c5 --timeout 200 --timeout-method thread > $OUT/pytest_c5.log 2>&1
for L in 2 1 4; do
  PT_BVH_LEAF=$L timeout -k 10 300 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --parity-pixels 16 > $OUT/bench_c5_leaf$L.json 2> $OUT/bench_c5_leaf$L.err
done
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
