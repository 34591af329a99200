set -e
mkdir -p gpurun_out/r2h
timeout -k 10 300 python bench.py --spp 32 --steps 2 --warmup 1 > gpurun_out/r2h/bench.log 2>&1
