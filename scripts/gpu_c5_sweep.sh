# C5 megakernel occupancy and BVH leaf size with the compact nodes (3 timed frames each)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/c5sweep
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
B="python -u bench.py --config c5 --no-cpu-baseline --no-parity"
timeout -k 10 200 $B > $OUT/base.json 2> $OUT/base.err
PT_WAVES=3 timeout -k 10 200 $B > $OUT/w3.json 2> $OUT/w3.err
PT_WAVES=4 timeout -k 10 200 $B > $OUT/w4.json 2> $OUT/w4.err
PT_BVH_LEAF=2 timeout -k 10 200 $B > $OUT/leaf2.json 2> $OUT/leaf2.err
timeout -k 10 200 $B > $OUT/base2.json 2> $OUT/base2.err
