#!/bin/bash
# sharded step rehearsed on one GPU (bench.py --force-collectives: sharded pull/push over the IPC exchange meshes +
# IPC dense all-reduce, now on uncached mesh memory), against the plain 1-rank headline on the same box; then a
# 2-process same-GPU run (two ranks on one GPU over the IPC meshes)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 100 --warmup 20 --secondary-dtype none --secondary-dcn off > gpurun_out/r6_reh_plain.log 2>&1 || { echo plain failed; tail -5 gpurun_out/r6_reh_plain.log; exit 3; }
  echo "plain rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_reh_plain.log)"
  RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=2961$rep timeout -k 10 300 python -u bench.py --steps 100 --warmup 20 --secondary-dtype none --secondary-dcn off --force-collectives > gpurun_out/r6_reh.log 2>&1 || { echo reh failed; tail -15 gpurun_out/r6_reh.log; exit 3; }
  echo "rehearsal rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_reh.log) $(grep -o '"sparse_exchange": "[a-z]*"\|"dense_allreduce": "[a-z_]*"' gpurun_out/r6_reh.log | tr '\n' ' ')"
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --same-gpu --steps 40 --warmup 10 --total-features 2e8 --secondary-dtype none --secondary-dcn off > gpurun_out/r6_2rank.log 2>&1 || { echo "2-rank failed"; tail -20 gpurun_out/r6_2rank.log; exit 4; }
grep -h '"metric"' gpurun_out/r6_2rank.log | head -1 | cut -c1-700
# kernel trace of the rehearsal step (single-rank process group)
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29641
bash scripts/gpu/step_trace.sh r6_reh --force-collectives | head -40
