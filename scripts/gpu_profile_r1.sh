#!/bin/bash
# Round-1 profiling pass on one MI355X (run through gpurun from the repo root).
# Occupancy A/B of render_tiles, rocprofv3 kernel stats, then PMC counters in
# separate passes (never combined with tracing domains).
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r1
export TMPDIR=/tmp
for W in 2 3 4; do
  PT_WAVES=$W timeout -k 10 300 python bench.py --spp 32 --steps 2 --warmup 1 --no-cpu-baseline --no-parity \
    > gpurun_out/r1/bench_w$W.log 2>&1 || exit 1
done
cd /tmp
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r1/counters.txt 2>&1 || true
B="python3 $GRAFT_REPO_ROOT/bench.py --spp 8 --steps 1 --warmup 0 --no-cpu-baseline --no-parity"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r1/pmc1 -o p \
  --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS \
  -- $B > $GRAFT_REPO_ROOT/gpurun_out/r1/pmc1.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r1/pmc2 -o p \
  --pmc SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
  -- $B > $GRAFT_REPO_ROOT/gpurun_out/r1/pmc2.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r1/pmc3 -o p \
  --pmc FETCH_SIZE -- $B > $GRAFT_REPO_ROOT/gpurun_out/r1/pmc3.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r1/pmc4 -o p \
  --pmc WRITE_SIZE -- $B > $GRAFT_REPO_ROOT/gpurun_out/r1/pmc4.log 2>&1 || exit 5
