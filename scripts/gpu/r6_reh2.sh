#!/bin/bash
# fused sharded exchanges (pack inside the key exchange, probe + gather inside the answer exchange) and
# system-coherent inbox accesses without per-block fences: IPC / sharded / n-rank tests, then the 1-rank
# rehearsal A/B against the plain step and the unfused / fenced variants, then the rehearsal kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ipc.py tests/test_gpu_sharded_ipc.py tests/test_gpu_nrank_step.py > gpurun_out/r6_reh2_tests.log 2>&1 || { echo tests failed; grep -E "PASS|FAIL|Error" gpurun_out/r6_reh2_tests.log | tail -30; exit 3; }
grep -cE "PASSED" gpurun_out/r6_reh2_tests.log; tail -1 gpurun_out/r6_reh2_tests.log
export MASTER_ADDR=127.0.0.1
run() {  # tag, env...
  local tag=$1; shift
  env "$@" RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_PORT=$((29700 + RANDOM % 200)) timeout -k 10 300 python -u bench.py --steps 100 --warmup 20 --secondary-dtype none --secondary-dcn off --force-collectives > gpurun_out/r6_reh2_$tag.log 2>&1 || { echo "$tag failed"; tail -15 gpurun_out/r6_reh2_$tag.log; exit 4; }
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_reh2_$tag.log)"
}
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 100 --warmup 20 --secondary-dtype none --secondary-dcn off > gpurun_out/r6_reh2_plain.log 2>&1 || { echo plain failed; exit 5; }
  echo "plain$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_reh2_plain.log)"
  run fused$rep PBX_PACK_EXCHANGE=1
  run unfused$rep PBX_PACK_EXCHANGE=0
  run fenced$rep PBX_IPC_FENCE=1
done
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_PORT=29941
bash scripts/gpu/step_trace.sh r6_reh2 --force-collectives | head -40
