#!/bin/bash
# Round 6: the GPU suite, the default bench line and a 2-rank gloo rehearsal of the multi-rank path.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
T=gpurun_out/$1
mkdir -p $T
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $T/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > $T/bench.json 2> $T/bench.err
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --config c2 --steps 2 --no-cpu-baseline \
    > $T/bench_gloo2.json 2> $T/bench_gloo2.err
