set -e
mkdir -p gpurun_out/r1q
timeout -k 10 300 python scripts/cw_pixels.py > gpurun_out/r1q/px.log 2>&1
