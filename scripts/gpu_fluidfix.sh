#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fluid.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_fluid.log 2>&1 || { tail -30 gpurun_out/pytest_fluid.log; exit 1; }
tail -1 gpurun_out/pytest_fluid.log
bash scripts/gpu_final2.sh
