set -e
mkdir -p gpurun_out/r1u
for cfg in "16777216 0" "67108864 0" "16777216 1" "16777216 2" "67108864 1"; do
  set -- $cfg
  echo "paths=$1 blocks_per_cu=$2" >> gpurun_out/r1u/sweep.log
  PT_WF_PATHS=$1 PT_WF_MARCH_BLOCKS_PER_CU=$2 timeout -k 10 200 python bench.py --spp 32 --steps 1 --warmup 1 --no-cpu-baseline --no-parity >> gpurun_out/r1u/sweep.log 2>&1
done
