set -e
mkdir -p gpurun_out/r1l
timeout -k 10 400 python -m pytest tests -q -x -m gpu > gpurun_out/r1l/pytest.log 2>&1
timeout -k 10 300 python bench.py --spp 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r1l/bench64.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r1l/kt -o p -- python3 $GRAFT_REPO_ROOT/bench.py --spp 8 --steps 1 --warmup 0 --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/gpurun_out/r1l/kt.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r1l/a -o p --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU -- python3 $GRAFT_REPO_ROOT/bench.py --spp 8 --steps 1 --warmup 0 --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/gpurun_out/r1l/a.log 2>&1
