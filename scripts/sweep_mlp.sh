#!/bin/bash
# GPU-box sweep of the MLP GEMM knobs on the flagship bench (interleaved rounds).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/sweep.txt
: > $out
for round in 1 2 3; do
  for cfg in "128 1024" "128 512" "64 512" "64 256" "64 1024"; do
    set -- $cfg
    PBX_MLP_TILE=$1 PBX_KSPLIT_DW=$2 timeout -k 10 120 python -u bench.py --steps 300 --warmup 30 > gpurun_out/sw.json 2> gpurun_out/sw.err || exit $?
    echo "tile=$1 ksplit=$2 $(python -c 'import json;d=json.load(open("gpurun_out/sw.json"));print(d["ms_per_step"])')" | tee -a $out
  done
done
