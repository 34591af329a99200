set -e
mkdir -p gpurun_out/r2c
for L in pf0 pf1 pf0_w4 pf0_w5; do
  echo "L=$L" >> gpurun_out/r2c/sweep.log
  PT_AMD_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python bench.py --spp 32 --steps 1 --warmup 1 --no-cpu-baseline >> gpurun_out/r2c/sweep.log 2>&1
done
PT_AMD_LIB=$PWD/scratch/libs/pf0.so timeout -k 10 200 python scripts/wave_diag.py 8 > gpurun_out/r2c/diag_pf0.log 2>&1
