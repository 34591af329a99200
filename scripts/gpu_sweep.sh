# A/B sweep of tuning knobs on one MI355X: GPU tests first, then short benches.
# usage: bash scripts/gpu_sweep.sh <tag> "<ENV=.. ENV=..>" "<ENV=..>" ...
set -e
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
for cfg in "$@"; do
  echo "== $cfg" >> $OUT/sweep.log
  env $cfg timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $OUT/b.log 2>&1
  python -c "import json,sys; d=json.loads([l for l in open('$OUT/b.log') if l.startswith('{')][-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms_avg'], r['kernel_ms_by_kind'])" >> $OUT/sweep.log
done
cat $OUT/sweep.log
