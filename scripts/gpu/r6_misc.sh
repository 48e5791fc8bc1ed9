#!/bin/bash
# scaled_fc backward with k_sfc_dw beside the dx launch (PBX_CTR_BWD_SIDE=1) vs one stream; tiered GPU tests after
# the staging change; config 4 again
set -o pipefail
mkdir -p gpurun_out
for side in 0 1; do
  PBX_CTR_BWD_SIDE=$side timeout -k 10 600 python -u scripts/micro/bench_ctr_ops.py --iters 30 > gpurun_out/r6_ctr_side$side.jsonl 2>&1 || { echo "ctr bench failed"; tail -5 gpurun_out/r6_ctr_side$side.jsonl; exit 3; }
  echo "side=$side $(grep '"op": "scaled_fc"' gpurun_out/r6_ctr_side$side.jsonl | grep -o '"bwd_graph_us": [0-9.]*\|"fwd_bwd_graph_us": [0-9.]*' | tr '\n' ' ')"
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tiered.py > gpurun_out/r6_tiered_tests.log 2>&1 || { echo "tiered tests failed"; grep -E "FAILED|Error" gpurun_out/r6_tiered_tests.log | head; exit 4; }
tail -1 gpurun_out/r6_tiered_tests.log
bash scripts/gpu/r6_tier.sh
