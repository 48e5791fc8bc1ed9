#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
for i in 1 2; do
  for m in 0 3 2; do
    PBX_SPLIT_PREFETCH=$m timeout -k 10 240 python -u bench.py --steps 200 --warmup 20 --secondary-dtype none --secondary-dcn off > $O/r5_split_${m}_$i.txt 2>&1
  done
done
