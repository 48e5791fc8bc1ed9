#!/bin/bash
# pipelined front on / off for the bf16 configs (DCN-V2 config 5, bf16 DeepFM), same box, interleaved
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_dcn.py tests/test_gpu_pipeline.py 2>&1 | tail -3
for rep in 1 2; do
  for cfg in "--model dcn_v2 --mlp-dtype bf16" "--mlp-dtype bf16"; do
    for p in off on; do
      timeout -k 10 300 python -u bench.py --steps 200 --warmup 50 --secondary-dtype none --secondary-dcn off $cfg --pipeline $p > gpurun_out/r6_pipe.log 2>&1 || { echo "bench failed ($cfg $p)"; tail -5 gpurun_out/r6_pipe.log; exit 3; }
      echo "$cfg pipeline=$p rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_pipe.log)"
    done
  done
done
