# PMC HBM passes (FETCH_SIZE, WRITE_SIZE; separate runs) on the default bench workload (C2 cornell 1920x1080x256spp,
# depth 8), one timed frame, then bytes per launch per kernel kind -> pmc_traffic_c2.json (bench.py roofline.traffic)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_c2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity"
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/fetch -o p --pmc FETCH_SIZE -- $B > $OUT/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/write -o p --pmc WRITE_SIZE -- $B > $OUT/write.log 2>&1
python3 $GRAFT_REPO_ROOT/scripts/pmc_traffic.py $OUT/fetch $OUT/write $OUT/pmc_traffic_c2.json "cornell_box.json 1920x1080 256spp depth 8" > $OUT/traffic.log
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python bench.py > $OUT/bench_default.log 2>&1 || true
