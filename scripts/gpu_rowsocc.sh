#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_graph.py tests/test_gpu_feature_types.py tests/test_gpu_fluid.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ro.log 2>&1 || { tail -30 gpurun_out/pytest_ro.log; exit 1; }
tail -1 gpurun_out/pytest_ro.log
bash scripts/gpu_env_ab.sh PBX_SEQPOOL_ROWS_OCC "1 0"
