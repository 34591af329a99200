set -e
mkdir -p gpurun_out/bounce_waves
[ -n "$NOTEST" ] || timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/bounce_waves/tests.log 2>&1
rm -f gpurun_out/bounce_waves/sweep.log
for W in ${WAVES:-3 4 2}; do
  echo "W=$W" >> gpurun_out/bounce_waves/sweep.log
  PT_WF_BOUNCE_WAVES=$W timeout -k 10 200 python bench.py --spp 32 --steps 2 --warmup 1 --no-cpu-baseline --no-parity >> gpurun_out/bounce_waves/sweep.log 2>&1
done
