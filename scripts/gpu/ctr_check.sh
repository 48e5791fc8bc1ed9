#!/bin/bash
# CTR op GPU tests, then the microbench (graph-replay bwd times)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ctr_ops.py > gpurun_out/ctr_tests.log 2>&1
timeout -k 10 400 python -u scripts/micro/bench_ctr_ops.py --iters 200 > gpurun_out/ctr_micro.jsonl
