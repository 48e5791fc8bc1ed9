#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 4 6; do
PBX_TOWER_PF=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_tower.py tests/test_gpu_dcn.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_pf$v.log 2>&1 || { tail -30 gpurun_out/pytest_pf$v.log; exit 1; }
tail -1 gpurun_out/pytest_pf$v.log
done
bash scripts/gpu_env_ab.sh PBX_TOWER_PF "8 6 4"
