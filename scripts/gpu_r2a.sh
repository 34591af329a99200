set -e
mkdir -p gpurun_out/r2a
for L in vote0_adv64 vote1_adv4 vote1_adv1 vote1_adv16; do
  echo "L=$L" >> gpurun_out/r2a/sweep.log
  PT_AMD_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python bench.py --spp 32 --steps 1 --warmup 1 --no-cpu-baseline >> gpurun_out/r2a/sweep.log 2>&1
done
