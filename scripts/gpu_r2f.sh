set -e
mkdir -p gpurun_out/r2f
rm -f gpurun_out/r2f/sweep.log
for L in head ab_base ab_pf1 ab_nolit ab_nomiss ab_nolds head ab_base; do
  echo "L=$L" >> gpurun_out/r2f/sweep.log
  PT_AMD_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python bench.py --spp 32 --steps 2 --warmup 1 --no-cpu-baseline --no-parity >> gpurun_out/r2f/sweep.log 2>&1
done
