# BVH walk loads both successors while testing a node: GPU suite, C5 (100k spheres, megakernel + BVH) and C2 benches with parity
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/prefetch
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --parity-pixels 16 > $OUT/c5.json 2> $OUT/c5.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err
