#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tower.py tests/test_gpu_tower32.py tests/test_gpu_kernels.py tests/test_gpu_graph.py tests/test_gpu_fluid.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_adam.log 2>&1 || { tail -30 gpurun_out/pytest_adam.log; exit 1; }
tail -1 gpurun_out/pytest_adam.log
bash scripts/gpu_env_ab.sh PBX_ADAM_MAX_BLOCKS "100000 512 256"
bash scripts/gpu_step_trace.sh adam
