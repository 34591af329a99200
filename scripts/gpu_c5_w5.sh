# C5 megakernel 4 vs 5 waves/SIMD, interleaved (3 timed frames each)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/c5w5
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
B="python -u bench.py --config c5 --no-cpu-baseline --no-parity"
for i in 1 2; do
  PT_WAVES=4 timeout -k 10 200 $B > $OUT/w4_$i.json 2> $OUT/w4_$i.err
  PT_WAVES=5 timeout -k 10 200 $B > $OUT/w5_$i.json 2> $OUT/w5_$i.err
done
timeout -k 10 300 python -u bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline --parity-pixels 12 > $OUT/c3.json 2> $OUT/c3.err
