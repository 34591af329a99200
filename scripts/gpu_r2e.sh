set -e
mkdir -p gpurun_out/r2e
for L in head pc_w1 pc_w5 head pc_w1; do
  echo "L=$L" >> gpurun_out/r2e/sweep.log
  PT_AMD_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python bench.py --spp 32 --steps 2 --warmup 1 --no-cpu-baseline --no-parity >> gpurun_out/r2e/sweep.log 2>&1
done
