#!/bin/bash
# GPU box: fp32 tower timing experiments (PBX_TOWER_DEBUG bits; numerics irrelevant)
set -o pipefail
mkdir -p gpurun_out
for d in 0 16 24 64 88; do
  echo "== debug $d"
  PBX_TOWER_DEBUG=$d timeout -k 10 120 python -u scripts/bench_tower.py --fp32 --iters 50 2>&1 | grep -E "forward|dX" || exit 2
done
