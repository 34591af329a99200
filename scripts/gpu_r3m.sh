# knob sweep at the 4-wave march default: bounce waves, march slice, slots, chunk paths
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/r3m
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
B="python -u bench.py --no-cpu-baseline --no-parity"
timeout -k 10 300 $B > $OUT/base.json 2> $OUT/base.err
PT_WF_BOUNCE_WAVES=4 timeout -k 10 300 $B > $OUT/bw4.json 2> $OUT/bw4.err
PT_WF_BOUNCE_WAVES=4 PT_WF_MARCH_SLICE=128 timeout -k 10 300 $B > $OUT/bw4_s128.json 2> $OUT/bw4_s128.err
PT_WF_BOUNCE_WAVES=4 PT_WF_MARCH_SLICE=64 timeout -k 10 300 $B > $OUT/bw4_s64.json 2> $OUT/bw4_s64.err
PT_WF_BOUNCE_WAVES=4 PT_WF_SLOTS=3 timeout -k 10 300 $B > $OUT/bw4_slots3.json 2> $OUT/bw4_slots3.err
PT_WF_BOUNCE_WAVES=4 PT_WF_PATHS=33554432 timeout -k 10 300 $B > $OUT/bw4_p25.json 2> $OUT/bw4_p25.err
PT_WF_BOUNCE_WAVES=5 timeout -k 10 300 $B > $OUT/bw5.json 2> $OUT/bw5.err
