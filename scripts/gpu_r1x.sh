set -e
mkdir -p gpurun_out/r1x
timeout -k 10 400 python -m pytest tests -q -x -m gpu > gpurun_out/r1x/pytest.log 2>&1
timeout -k 10 300 python bench.py --spp 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r1x/bench64.log 2>&1
bash scripts/gpu_prof.sh r1x/prof
