set -e
mkdir -p gpurun_out/r1o
timeout -k 10 200 python scripts/cw_bisect.py count > gpurun_out/r1o/bisect.log 2>&1
