#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PBX_HEAD_BWD_RB=4 PBX_TD_SEG_ITEMS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_knobs.log 2>&1 || { tail -30 gpurun_out/pytest_knobs.log; exit 1; }
tail -1 gpurun_out/pytest_knobs.log
bash scripts/gpu_env_ab.sh PBX_HEAD_BWD_RB "8 4"
bash scripts/gpu_env_ab.sh PBX_TD_SEG_ITEMS "4 2 1"
