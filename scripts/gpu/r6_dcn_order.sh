#!/bin/bash
# DCN-V2 side-stream enqueue order: cross dW after the head backward (PBX_CROSS_DW_AFTER_HEAD=1) and/or tower dW
# after the head (PBX_DW_AFTER_HEAD=1), so the compute stream runs dX chain -> cross dX chain -> head without forks
set -o pipefail
mkdir -p gpurun_out
PBX_CROSS_DW_AFTER_HEAD=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dcn.py tests/test_gpu_pipeline.py -k "dcn" > gpurun_out/r6_dcn_order_tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" gpurun_out/r6_dcn_order_tests.log | head; exit 3; }
tail -1 gpurun_out/r6_dcn_order_tests.log
for rep in 1 2 3; do
  for cfg in "0 0" "1 0" "0 1" "1 1"; do
    set -- $cfg
    PBX_CROSS_DW_AFTER_HEAD=$1 PBX_DW_AFTER_HEAD=$2 timeout -k 10 300 python -u bench.py --model dcn_v2 --steps 200 --warmup 50 --secondary-dtype none > gpurun_out/r6_dcn_order.json 2>/dev/null || { echo "bench $cfg failed"; exit 4; }
    echo "rep$rep cross_dw_after_head=$1 dw_after_head=$2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_dcn_order.json)"
  done
done
