#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1
p=29600
for i in 1 2; do
  for m in 0 2 3; do
    p=$((p+1))
    MASTER_PORT=$p PBX_SPLIT_PREFETCH=$m timeout -k 10 300 python -u bench.py --force-collectives --steps 100 --warmup 20 --secondary-dtype none --secondary-dcn off > $O/r5_reh_split${m}_$i.txt 2>&1 || exit 1
  done
done
