set -e
mkdir -p gpurun_out/r1n
timeout -k 10 120 python scripts/cw_time.py 48 > gpurun_out/r1n/cw_default.log 2>&1
PT_MARCH_TRIGGER=1 PT_MARCH_KEEP=65 timeout -k 10 120 python scripts/cw_time.py 48 > gpurun_out/r1n/cw_old.log 2>&1
PT_MARCH_TRIGGER=1 PT_MARCH_KEEP=1 timeout -k 10 120 python scripts/cw_time.py 48 > gpurun_out/r1n/cw_k1.log 2>&1
