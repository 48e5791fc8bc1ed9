#!/bin/bash
# GPU box: same-box interleaved A/B of an environment knob.
# usage: scripts/gpu_env_ab.sh VAR "valA valB" [extra bench args]
set -o pipefail
var=$1; vals=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
for v in $vals; do
  env $var=$v timeout -k 10 300 python -u bench.py --steps 400 --warmup 50 --secondary-dtype none --diag-windows 1 "$@" \
    > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "bench failed"; tail -30 gpurun_out/ab_$v.err; exit 3; }
  echo "$var=$v rep=$rep $(grep -h 'wall\|diag window' gpurun_out/ab_$v.err | grep -o '[0-9.]* ms/step' | tr '\n' ' ')"
done
done
