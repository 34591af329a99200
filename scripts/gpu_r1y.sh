set -e
mkdir -p gpurun_out/r1y
timeout -k 10 400 python -m pytest tests -q -x -m gpu > gpurun_out/r1y/pytest.log 2>&1
timeout -k 10 200 python scripts/march_jobs_check.py scratch/jobs_big.bin scratch/res_big.bin > gpurun_out/r1y/big.log 2>&1
timeout -k 10 300 python bench.py --spp 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r1y/bench64.log 2>&1
bash scripts/gpu_prof.sh r1y/prof
