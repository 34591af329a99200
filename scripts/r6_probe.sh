#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$1
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullframe.py tests/test_gpu_parity.py -x -v -m gpu \
    -k "c5 or c1_full or textured_deep" --timeout 300 --timeout-method thread > gpurun_out/$1/pytest.log 2>&1
PT_AMD_LIB=$R/variants/qrec.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullframe.py -x -v -m gpu -k "c5" \
    --timeout 200 --timeout-method thread > gpurun_out/$1/pytest_qrec.log 2>&1
bash scripts/abx.sh $1 2 "default|--config c5 --option bvh_wide=0" "default|--config c5" "qrec|--config c5 --option bvh_wide=0"
