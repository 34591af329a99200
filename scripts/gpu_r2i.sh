set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/r1final
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --spp 8 --steps 1 --warmup 0 --no-cpu-baseline --no-parity"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/pmc_write -o p --pmc WRITE_SIZE -- $B > $OUT/pmc_write.log 2>&1 || echo "WRITE_SIZE pass rc=$?" >> $OUT/pmc_write.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/pmc_wrreq -o p --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -- $B > $OUT/pmc_wrreq.log 2>&1 || echo "WRREQ pass rc=$?" >> $OUT/pmc_wrreq.log
