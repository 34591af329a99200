set -e
mkdir -p gpurun_out/r1f
timeout -k 10 200 python scripts/phase_profile.py 16 > gpurun_out/r1f/phase.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r1f/ic --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH -- python3 $GRAFT_REPO_ROOT/bench.py --spp 16 --steps 1 --warmup 0 --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/gpurun_out/r1f/ic.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r1f/wt --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -- python3 $GRAFT_REPO_ROOT/bench.py --spp 16 --steps 1 --warmup 0 --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/gpurun_out/r1f/wt.log 2>&1
