# GPU test suite on one MI355X (usage: bash scripts/gpu_tests.sh <tag> [pytest -k expr])
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
K=()
if [ -n "$2" ]; then K=(-k "$2"); fi
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu "${K[@]}" --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
