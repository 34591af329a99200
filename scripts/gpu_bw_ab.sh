# A/B: bounce kernel register budget 3 (default) vs 4 waves/SIMD on C2, interleaved, 3 runs each; then the default bench
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/bw_ab
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
B="python -u bench.py --no-cpu-baseline --no-parity"
for i in 1 2 3; do
  timeout -k 10 200 $B > $OUT/bw3_$i.json 2> $OUT/bw3_$i.err
  PT_WF_BOUNCE_WAVES=4 timeout -k 10 200 $B > $OUT/bw4_$i.json 2> $OUT/bw4_$i.err
done
timeout -k 10 300 python bench.py > $OUT/bench_default.log 2>&1
