#!/bin/bash
# DCN-V2 (config 5): tests, then the cross dW on the side stream vs inline (PBX_CROSS_DW_SIDE), same box, interleaved
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_dcn.py tests/test_gpu_pipeline.py tests/test_gpu_tower.py 2>&1 | tail -3
for rep in 1 2; do
  for sd in 0 1; do
    PBX_CROSS_DW_SIDE=$sd timeout -k 10 300 python -u bench.py --steps 200 --warmup 50 --secondary-dtype none --secondary-dcn off --model dcn_v2 --mlp-dtype bf16 > gpurun_out/r6_dcn.log 2>&1 || { echo "bench failed ($sd)"; tail -5 gpurun_out/r6_dcn.log; exit 3; }
    echo "cross_dw_side=$sd rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_dcn.log)"
  done
done
ANCHOR=k_cross_fwd bash scripts/gpu/step_trace.sh r6_dcn2 --model dcn_v2 --mlp-dtype bf16 | head -45
