#!/bin/bash
# One driver for every GPU-box run (replaces round 1's one-off gpu_r*.sh runners).
# Each GPU step runs under its own timeout; steps are chained so the first
# failure ends the run.  Output goes to gpurun_out/<tag>/.
#
#   bash scripts/gpu.sh tests    <tag> [pytest -k expr]   GPU test suite
#   bash scripts/gpu.sh smoke    <tag>                    __graft_entry__.smoke()
#   bash scripts/gpu.sh bench    <tag> [bench args...]    one bench.py line -> <tag>/bench.log
#   bench A/B of tuning knobs:   bash scripts/gpu.sh bench <tag> --no-cpu-baseline --option wf_slots=1
#   bash scripts/gpu.sh kt       <tag> [bench args...]    rocprofv3 --kernel-trace --stats of bench.py
#   bash scripts/gpu.sh pmc      <tag> [bench args...]    FETCH_SIZE / WRITE_SIZE passes (separate runs)
#                                                         -> <tag>/pmc_traffic.json (scripts/pmc_traffic.py)
#   bash scripts/gpu.sh sq       <tag> [bench args...]    SQ instruction-mix and lane-activity pass
#   bash scripts/gpu.sh stall    <tag> [bench args...]    wave-cycle split: active / waiting on memory / issue-stalled
#   bash scripts/gpu.sh evidence <tag>                    tests, smoke, bench, kt (default and one-stream)
set -e
cmd=$1; tag=$2; shift 2 || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$tag
mkdir -p $OUT
cd $R
# PMC_FILTER (optional): a kernel-name regex; counter passes collect only those kernels' dispatches.  Not needed
# for C3: run its passes at --slots 4 (profiles/r4/c3_profiler_abort.txt: at one stream, ~8,300 dispatches on one
# HSA queue per frame meet a profiler defect at the queue's ring wrap)
FILT=(); if [ -n "$PMC_FILTER" ]; then FILT=(--kernel-include-regex "$PMC_FILTER"); fi
prof() {  # rocprofv3 with the program itself after -- (no launcher hops)
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL ${PROF_TIMEOUT:-400} rocprofv3 "$@")
}
case $cmd in
tests)
    K=(); if [ -n "$1" ]; then K=(-k "$1"); fi
    timeout -k 10 900 python -u -m pytest tests -x -v -m gpu "${K[@]}" --timeout 300 --timeout-method thread \
        > $OUT/pytest_gpu.log 2>&1 ;;
smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 ;;
bench)
    timeout -k 10 600 python -u bench.py "$@" > $OUT/bench.log 2>&1 ;;
kt)
    prof --kernel-trace --stats --output-format csv -d $OUT/kt -o bench -- python3 $R/bench.py "$@" \
        > $OUT/kt.log 2>&1
    python3 scripts/kt_summary.py $OUT/kt > $OUT/kt_summary.txt
    python3 scripts/kt_leg.py $OUT/kt/bench_kernel_trace.csv $(( ${KT_FRAMES:-5} )) > $OUT/kt_one_stream_frame.txt || true ;;
pmc)
    prof --kernel-trace --output-format csv -d $OUT/fetch -o p "${FILT[@]}" --pmc FETCH_SIZE -- python3 $R/bench.py "$@" \
        > $OUT/fetch.log 2>&1
    prof --kernel-trace --output-format csv -d $OUT/write -o p "${FILT[@]}" --pmc WRITE_SIZE -- python3 $R/bench.py "$@" \
        > $OUT/write.log 2>&1
    python3 scripts/pmc_traffic.py $OUT/fetch $OUT/write $OUT/pmc_traffic.json "${WORKLOAD:-cornell_box.json 1920x1080 256spp depth 8}" ${PMC_FRAMES:-1} \
        > $OUT/traffic.log ;;
sq)
    prof --kernel-trace --output-format csv -d $OUT/sq -o p "${FILT[@]}" --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 \
        SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVES \
        -- python3 $R/bench.py "$@" > $OUT/sq.log 2>&1
    python3 scripts/pmc_summary.py $OUT/sq > $OUT/sq_summary.txt
    python3 scripts/pmc_flops.py $OUT/sq ${SQ_FRAMES:-2} ${SQ_SAMPLES:-530841600} $OUT/pmc_flops.json \
        "${WORKLOAD:-cornell_box.json 1920x1080 256spp depth 8}" > /dev/null ;;
stall)
    prof --kernel-trace --output-format csv -d $OUT/stall -o p --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT \
        -- python3 $R/bench.py "$@" > $OUT/stall.log 2>&1
    python3 scripts/pmc_summary.py $OUT/stall > $OUT/stall_summary.txt ;;
cache)  # L2 hit rate and vector-memory request mix per kernel (one pass; list the names with rocprofv3 -L)
    prof --kernel-trace --output-format csv -d $OUT/cache -o p --pmc ${CACHE_PMC:-TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TA_BUSY_avr} \
        -- python3 $R/bench.py "$@" > $OUT/cache.log 2>&1
    python3 scripts/pmc_summary.py $OUT/cache > $OUT/cache_summary.txt ;;
list)
    (cd /tmp && timeout -s KILL 120 rocprofv3 -L) > $OUT/counters.txt 2>&1 || true ;;
evidence)
    bash scripts/gpu.sh tests $tag
    bash scripts/gpu.sh smoke $tag
    bash scripts/gpu.sh bench $tag
    bash scripts/gpu.sh kt $tag/kt_default --no-cpu-baseline --no-parity --no-kernel-timing
    KT_FRAMES=4 bash scripts/gpu.sh kt $tag/kt_one_stream --slots 1 --no-cpu-baseline --no-parity --no-roofline-leg --no-kernel-timing ;;
*)
    echo "usage: scripts/gpu.sh tests|smoke|bench|kt|pmc|sq|evidence <tag> [args]"; exit 2 ;;
esac
