set -e
mkdir -p gpurun_out/r2b
timeout -k 10 200 python scripts/wave_diag.py 8 > gpurun_out/r2b/diag.log 2>&1
