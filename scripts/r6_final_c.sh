#!/bin/bash
# Final build: GPU suite, smoke, PMC passes
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
T=gpurun_out/$1
mkdir -p $T
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $T/pytest_gpu.txt 2>&1
tail -1 $T/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.txt 2>&1
bash scripts/r6_evidence_pmc.sh $1
