#!/bin/bash
# steps per captured graph on the headline (K = 4 default vs 8): the graph-launch boundary once per K steps
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
  for k in 4 8; do
    timeout -k 10 300 python -u bench.py --steps 200 --warmup 48 --graph-steps $k --secondary-dtype none --secondary-dcn off > gpurun_out/r6_gs$k.json 2>/dev/null || { echo "K=$k failed"; exit 3; }
    echo "rep$rep K=$k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_gs$k.json)"
  done
done
