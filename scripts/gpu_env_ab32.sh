#!/bin/bash
# GPU box: same-box interleaved A/B of an env knob on the fp32-MLP step (primary dtype fp32)
set -o pipefail
var=$1; vals=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
for v in $vals; do
  env $var=$v timeout -k 10 300 python -u bench.py --steps 300 --warmup 50 --mlp-dtype fp32 --secondary-dtype none "$@" \
    > gpurun_out/ab32_$v.json 2> gpurun_out/ab32_$v.err || { echo "bench failed"; tail -30 gpurun_out/ab32_$v.err; exit 3; }
  echo "$var=$v rep=$rep $(grep -h 'wall' gpurun_out/ab32_$v.err | grep -o 'wall [0-9.]* ms/step')"
done
done
