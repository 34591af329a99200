# Wave-dealt march (wf_march_w, global cursor) vs per-block shares: GPU suite, C2 A/B
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/r3h
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "engines_agree or chunks or heart_march or marched_functions or shards" --timeout 200 --timeout-method thread > $OUT/pytest_quick.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_wave.json 2> $OUT/bench_wave.err
PT_WF_MARCH_DEAL=block timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity > $OUT/bench_block.json 2> $OUT/bench_block.err
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
