set -e
mkdir -p gpurun_out/r1r
timeout -k 10 150 python scripts/cw_wave.py > gpurun_out/r1r/default.log 2>&1
PT_MARCH_TRIGGER=1 PT_MARCH_KEEP=65 timeout -k 10 150 python scripts/cw_wave.py > gpurun_out/r1r/old.log 2>&1
