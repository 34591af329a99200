set -e
mkdir -p gpurun_out/r2d
for L in sb0_w1 sb8_w1 sb16_w1 sb32_w1 sb16_w5 sb0_w1; do
  echo "L=$L" >> gpurun_out/r2d/sweep.log
  PT_AMD_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python bench.py --spp 32 --steps 2 --warmup 1 --no-cpu-baseline >> gpurun_out/r2d/sweep.log 2>&1
done
