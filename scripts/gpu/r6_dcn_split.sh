#!/bin/bash
# DCN-V2 (config 5): pipelined front with the next batch's dedup placement (PBX_SPLIT_PREFETCH 0 / 3 / 2) vs no pipeline, same box, interleaved
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "off 0" "on 0" "on 3" "on 2"; do
    set -- $v
    PBX_SPLIT_PREFETCH=$2 timeout -k 10 300 python -u bench.py --steps 200 --warmup 50 --secondary-dtype none --secondary-dcn off --model dcn_v2 --mlp-dtype bf16 --pipeline $1 > gpurun_out/r6_dcn.log 2>&1 || { echo "bench failed ($v)"; tail -5 gpurun_out/r6_dcn.log; exit 3; }
    echo "pipeline=$1 split=$2 rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_dcn.log)"
  done
done
