# Fused bounces (wf_trace): parity, bench A/B against per-bounce launches, 8-rank simulation, full GPU suite
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/r3a
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "fused or engines_agree or chunks" --timeout 200 --timeout-method thread > $OUT/pytest_fused.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_fused.json 2> $OUT/bench_fused.err
PT_WF_FUSED=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity > $OUT/bench_unfused.json 2> $OUT/bench_unfused.err
timeout -k 10 300 python -u scripts/rank_sim.py --worlds 1,8 > $OUT/rank_sim.json 2> $OUT/rank_sim.err
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
