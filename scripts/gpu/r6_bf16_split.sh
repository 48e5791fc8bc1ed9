#!/bin/bash
# bf16 DeepFM: pipeline off vs on with PBX_SPLIT_PREFETCH 0 / 2; then the default bench (all same-run secondaries)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "off 0" "on 0" "on 2"; do
    set -- $v
    PBX_SPLIT_PREFETCH=$2 timeout -k 10 300 python -u bench.py --steps 200 --warmup 50 --secondary-dtype none --secondary-dcn off --mlp-dtype bf16 --pipeline $1 > gpurun_out/r6_b16.log 2>&1 || { echo "bench failed ($v)"; tail -5 gpurun_out/r6_b16.log; exit 3; }
    echo "bf16 pipeline=$1 split=$2 rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_b16.log)"
  done
done
timeout -k 10 400 python -u bench.py > gpurun_out/r6_bdef.json 2> gpurun_out/r6_bdef.err || { echo "bench failed"; tail -20 gpurun_out/r6_bdef.err; exit 3; }
grep -h "^\[bench\]" gpurun_out/r6_bdef.err | tail -6; cat gpurun_out/r6_bdef.json
