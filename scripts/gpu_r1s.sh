set -e
mkdir -p gpurun_out/r1s
timeout -k 10 400 python -m pytest tests -q -x -m gpu > gpurun_out/r1s/pytest.log 2>&1
timeout -k 10 120 python scripts/cw_time.py 12 > gpurun_out/r1s/cw.log 2>&1
timeout -k 10 300 python bench.py --spp 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r1s/bench64.log 2>&1
