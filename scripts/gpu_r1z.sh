set -e
mkdir -p gpurun_out/r1z
for K in 1 4 64; do
  echo "K=$K" >> gpurun_out/r1z/sweep.log
  PT_AMD_LIB=$PWD/scratch/libs/adv$K.so timeout -k 10 200 python bench.py --spp 32 --steps 1 --warmup 1 --no-cpu-baseline --no-parity >> gpurun_out/r1z/sweep.log 2>&1
done
