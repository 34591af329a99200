set -e
mkdir -p gpurun_out/r1w
for W in 2 3 4; do
  echo "W=$W" >> gpurun_out/r1w/sweep.log
  PT_WF_BOUNCE_WAVES=$W timeout -k 10 200 python bench.py --spp 32 --steps 1 --warmup 1 --no-cpu-baseline --no-parity >> gpurun_out/r1w/sweep.log 2>&1
done
