set -e
mkdir -p gpurun_out/r1j
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r1j/kt -o p -- python3 $GRAFT_REPO_ROOT/bench.py --spp 16 --steps 1 --warmup 0 --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/gpurun_out/r1j/kt.log 2>&1
