set -e
mkdir -p gpurun_out/r1p
timeout -k 10 200 python scripts/march_jobs_check.py scratch/jobs_wave.bin scratch/res_wave.bin > gpurun_out/r1p/wave.log 2>&1
timeout -k 10 200 python scripts/march_jobs_check.py scratch/jobs_big.bin scratch/res_big.bin > gpurun_out/r1p/big.log 2>&1
