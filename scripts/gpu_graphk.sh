#!/bin/bash
# GPU box: same-box interleaved A/B of steps per captured graph
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for k in 1 8 5; do
  timeout -k 10 300 python -u bench.py --steps 400 --warmup 40 --secondary-dtype none --graph-steps $k \
    > gpurun_out/gk_$k.json 2> gpurun_out/gk_$k.err || { echo "bench failed"; tail -30 gpurun_out/gk_$k.err; exit 3; }
  echo "graph-steps=$k rep=$rep $(grep -h 'wall' gpurun_out/gk_$k.err | grep -o '[0-9.]* ms/step' | tr '\n' ' ')"
done
done
for k in 1 5; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --graph-steps $k > gpurun_out/gk_driver$k.json 2> gpurun_out/gk_driver$k.err || { echo "bench failed"; tail -30 gpurun_out/gk_driver$k.err; exit 3; }
echo "driver-style K=$k: $(grep -o '"ms_per_step": [0-9.]*\|"fp32_ms_per_step": [0-9.]*' gpurun_out/gk_driver$k.json | tr '\n' ' ')"
done
