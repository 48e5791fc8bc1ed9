#!/bin/bash
# fp32 tower kernel times under the PBX_TOWER_DEBUG timing flags (0 normal,
# 8 no MP32 stores, 64 no weight loads, 72 both)
set -o pipefail
mkdir -p gpurun_out
for d in 0 8 64 72 0; do
  echo "== PBX_TOWER_DEBUG=$d"
  PBX_TOWER_DEBUG=$d timeout -k 10 120 python -u scripts/bench_tower.py --fp32 --iters 50 2>&1 | grep "\[tower\]" || exit 1
done
