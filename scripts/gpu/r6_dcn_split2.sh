#!/bin/bash
# DCN-V2 with the tower dW after the head (new default): next-batch dedup placement A/B (PBX_SPLIT_PREFETCH 2 default, 0, 1, 3)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dcn.py tests/test_gpu_pipeline.py > gpurun_out/r6_dcn_split2_tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" gpurun_out/r6_dcn_split2_tests.log | head; exit 3; }
tail -1 gpurun_out/r6_dcn_split2_tests.log
for rep in 1 2 3; do
  for sp in 2 0 1 3; do
    PBX_SPLIT_PREFETCH=$sp timeout -k 10 300 python -u bench.py --model dcn_v2 --steps 200 --warmup 50 --secondary-dtype none > gpurun_out/r6_dcn_split2.json 2>/dev/null || { echo "bench $sp failed"; exit 4; }
    echo "rep$rep split=$sp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_dcn_split2.json)"
  done
done
