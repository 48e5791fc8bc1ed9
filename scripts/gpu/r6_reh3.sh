#!/bin/bash
# IPC grids capped at 64 workgroups (was up to 256): exchange micro, IPC / sharded / n-rank tests, rehearsal A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/micro/ipc_exchange_bench.py > gpurun_out/r6_ipc_bench2.jsonl 2>&1 || { echo "ipc bench failed"; tail -20 gpurun_out/r6_ipc_bench2.jsonl; exit 3; }
grep "{" gpurun_out/r6_ipc_bench2.jsonl
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ipc.py tests/test_gpu_sharded_ipc.py tests/test_gpu_nrank_step.py tests/test_gpu_fluid_multirank.py > gpurun_out/r6_reh3_tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" gpurun_out/r6_reh3_tests.log | head -20; exit 4; }
tail -1 gpurun_out/r6_reh3_tests.log
export MASTER_ADDR=127.0.0.1
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 100 --warmup 20 --secondary-dtype none --secondary-dcn off > gpurun_out/r6_reh3_plain.log 2>&1 || { echo plain failed; exit 5; }
  echo "plain$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_reh3_plain.log)"
  for mb in 64 256; do
    PBX_IPC_MAX_BLOCKS=$mb RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_PORT=$((29800 + rep * 10 + mb % 7)) timeout -k 10 300 python -u bench.py --steps 100 --warmup 20 --secondary-dtype none --secondary-dcn off --force-collectives > gpurun_out/r6_reh3_$mb.log 2>&1 || { echo "reh $mb failed"; tail -10 gpurun_out/r6_reh3_$mb.log; exit 6; }
    echo "rehearsal blocks<=$mb rep$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_reh3_$mb.log)"
  done
done
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_PORT=29951
bash scripts/gpu/step_trace.sh r6_reh3 --force-collectives | head -40
