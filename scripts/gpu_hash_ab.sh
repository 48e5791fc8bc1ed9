#!/bin/bash
# GPU box: hash-dedup item counts on the 1-rank IPC rehearsal step (the sharded path's dedup)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29556
PBX_HASH_RANK_ITEMS=1 PBX_HASH_SEG_ITEMS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_sharded_ipc.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_hash.log 2>&1 || { tail -30 gpurun_out/pytest_hash.log; exit 1; }
tail -1 gpurun_out/pytest_hash.log
for rep in 1 2; do
for cfg in "4 4" "4 1" "2 1" "1 1"; do
  set -- $cfg
  PBX_HASH_RANK_ITEMS=$1 PBX_HASH_SEG_ITEMS=$2 timeout -k 10 300 python -u bench.py --force-collectives --steps 300 --warmup 50 --secondary-dtype none > gpurun_out/hab.json 2> gpurun_out/hab.err || { echo "bench failed"; tail -20 gpurun_out/hab.err; exit 3; }
  echo "rank_items=$1 seg_items=$2 rep=$rep $(grep -h 'wall' gpurun_out/hab.err | grep -o 'wall [0-9.]* ms/step')"
done
done
