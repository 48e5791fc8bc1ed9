#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 250 --timeout-method thread tests/test_gpu_fluid.py tests/test_gpu_fluid_multirank.py > $O/r5_fluid_ov_tests.log 2>&1
timeout -k 10 600 python -u scripts/bench_fluid.py --batches 200 > $O/r5_bench_fluid200_ov.txt 2>&1
PBX_ADAM_OVERLAP=0 timeout -k 10 600 python -u scripts/bench_fluid.py --batches 200 > $O/r5_bench_fluid200_noov.txt 2>&1
