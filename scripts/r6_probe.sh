#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -k "register_budgets" --timeout 300 \
    --timeout-method thread > gpurun_out/$1/pytest.log 2>&1 || true
bash scripts/abx.sh $1 2 "default|--config c5" "default|--config c5 --option wf_slots=3" "default|--config c5 --option wf_slots=4"
