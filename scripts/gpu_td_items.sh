#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 2 4; do
PBX_TD_ITEMS=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_td$v.log 2>&1 || { tail -30 gpurun_out/pytest_td$v.log; exit 1; }
tail -1 gpurun_out/pytest_td$v.log
done
bash scripts/gpu_env_ab.sh PBX_TD_ITEMS "1 2 4"
