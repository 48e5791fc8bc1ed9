#!/bin/bash
# DCN-V2 cross kernels after the select-chain layer pointers / halved top batch / hardware bf16 rounding:
# bf16-path tests, DCN-V2 + bf16 DeepFM + default benches, DCN step trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dcn.py tests/test_gpu_tower.py tests/test_gpu_pipeline.py tests/test_gpu_kernels.py tests/test_gpu_graph.py tests/test_gpu_fluid.py > gpurun_out/r6_dcn2_tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error|assert" gpurun_out/r6_dcn2_tests.log | head -20; tail -3 gpurun_out/r6_dcn2_tests.log; exit 3; }
tail -1 gpurun_out/r6_dcn2_tests.log
for rep in 1 2; do
  timeout -k 10 400 python -u bench.py --model dcn_v2 --steps 200 --warmup 50 --secondary-dtype none > gpurun_out/r6_dcn2_b$rep.json 2> gpurun_out/r6_dcn2_b$rep.err || { echo "dcn bench failed"; tail -20 gpurun_out/r6_dcn2_b$rep.err; exit 4; }
  echo "dcn rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_dcn2_b$rep.json)"
done
timeout -k 10 400 python -u bench.py --mlp-dtype bf16 --steps 200 --warmup 50 --secondary-dtype none --secondary-dcn off > gpurun_out/r6_dcn2_bf16.json 2> gpurun_out/r6_dcn2_bf16.err || { echo "bf16 bench failed"; tail -20 gpurun_out/r6_dcn2_bf16.err; exit 5; }
echo "bf16 deepfm $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_dcn2_bf16.json)"
timeout -k 10 400 python -u bench.py > gpurun_out/r6_dcn2_def.json 2> gpurun_out/r6_dcn2_def.err || { echo "bench failed"; tail -20 gpurun_out/r6_dcn2_def.err; exit 6; }
grep -o '"ms_per_step": [0-9.]*\|"bf16_ms_per_step": [0-9.]*\|"dcn_v2_ms_per_step": [0-9.]*' gpurun_out/r6_dcn2_def.json | tr '\n' ' '; echo
ANCHOR=k_cross_fwd bash scripts/gpu/step_trace.sh r6_dcn2 --model dcn_v2 | head -30
