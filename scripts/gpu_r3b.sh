# BASELINE configs beyond the headline on one MI355X: C3 and C5 bench lines, C4's per-rank share
# (8-rank tiling simulated on one GPU: two ranks at full size), fused-bounce parity again.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/r3b
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "fused" --timeout 200 --timeout-method thread > $OUT/pytest_fused.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err
timeout -k 10 300 python -u bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline --parity-pixels 12 > $OUT/bench_c3.json 2> $OUT/bench_c3.err
timeout -k 10 300 python -u scripts/rank_sim.py --width 3840 --height 2160 --spp 4096 --worlds 8 --ranks 0,3 --reps 1 > $OUT/rank_sim_c4.json 2> $OUT/rank_sim_c4.err
