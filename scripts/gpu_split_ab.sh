#!/bin/bash
# GPU box: same-box interleaved A/B of the split pull (PBX_SPLIT_PULL)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
for sp in 1 0; do
  PBX_SPLIT_PULL=$sp timeout -k 10 300 python -u bench.py --steps 400 --warmup 50 --secondary-dtype none --diag-windows 2 \
    > gpurun_out/ab_split$sp.json 2> gpurun_out/ab_split$sp.err || { echo "bench failed"; tail -30 gpurun_out/ab_split$sp.err; exit 3; }
  echo "split=$sp rep=$rep $(grep -h 'wall\|diag window' gpurun_out/ab_split$sp.err | grep -o '[0-9.]* ms/step' | tr '\n' ' ')"
done
done
