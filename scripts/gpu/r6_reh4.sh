#!/bin/bash
# sharded split prefetch with the next batch's pack + key exchange right after its dedup (on the dW stream, off the
# step's sparse chain): sharded / n-rank tests, rehearsal A/B (early vs after the push), rehearsal kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sharded_ipc.py tests/test_gpu_nrank_step.py tests/test_gpu_fluid_multirank.py tests/test_gpu_pipeline.py > gpurun_out/r6_reh4_tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" gpurun_out/r6_reh4_tests.log | head -20; exit 4; }
tail -1 gpurun_out/r6_reh4_tests.log
export MASTER_ADDR=127.0.0.1
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 100 --warmup 20 --secondary-dtype none --secondary-dcn off > gpurun_out/r6_reh4_plain.log 2>&1 || { echo plain failed; exit 5; }
  echo "plain$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_reh4_plain.log)"
  for ek in 1 0; do
    PBX_EARLY_KEY_EXCHANGE=$ek RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_PORT=$((29850 + rep * 10 + ek)) timeout -k 10 300 python -u bench.py --steps 100 --warmup 20 --secondary-dtype none --secondary-dcn off --force-collectives > gpurun_out/r6_reh4_$ek.log 2>&1 || { echo "reh $ek failed"; tail -10 gpurun_out/r6_reh4_$ek.log; exit 6; }
    echo "rehearsal early_key_exchange=$ek rep$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_reh4_$ek.log)"
  done
done
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_PORT=29961
bash scripts/gpu/step_trace.sh r6_reh4 --force-collectives | head -45
