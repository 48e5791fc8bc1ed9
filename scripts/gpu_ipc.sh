#!/bin/bash
# GPU box: IPC mesh + multi-process sharded step tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipc.py tests/test_gpu_sharded_ipc.py -v -x --timeout 420 \
  --timeout-method thread > gpurun_out/ipc_tests.log 2>&1
rc=$?
tail -30 gpurun_out/ipc_tests.log
exit $rc
