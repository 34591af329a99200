set -e
mkdir -p gpurun_out/r2g
rm -f gpurun_out/r2g/sweep.log
for L in ab_best ab_best_w5 ab_best_w4 ab_best_lit1 ab_nolds ab_best; do
  echo "L=$L" >> gpurun_out/r2g/sweep.log
  PT_AMD_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python bench.py --spp 32 --steps 2 --warmup 1 --no-cpu-baseline --no-parity >> gpurun_out/r2g/sweep.log 2>&1
done
