#!/bin/bash
# CTR op backwards (k_sfc_dw scaled_fc dW + db; bf16x3 int8fc dx / dW): tests, per-launch times, the op microbench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ctr_ops.py -k "scaled" > gpurun_out/r6_ctr_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r6_ctr_tests.log; exit 3; }
tail -2 gpurun_out/r6_ctr_tests.log
timeout -k 10 300 python -u scripts/micro/scaled_fc_parts.py > gpurun_out/r6_sfc_parts.json 2>&1 || { echo parts failed; tail -10 gpurun_out/r6_sfc_parts.json; exit 4; }
cat gpurun_out/r6_sfc_parts.json | grep "{"
timeout -k 10 600 python -u scripts/micro/bench_ctr_ops.py --iters 30 > gpurun_out/r6_ctr_ops.jsonl 2>&1 || { echo bench failed; tail -10 gpurun_out/r6_ctr_ops.jsonl; exit 5; }
grep "scaled" gpurun_out/r6_ctr_ops.jsonl
