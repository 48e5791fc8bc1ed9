#!/bin/bash
# fp32 headline A/B of the next batch's dedup placement (PBX_SPLIT_PREFETCH
# 0 / 3 / 2, interleaved twice) on one box; plus the chip-wide f32 MFMA rate.
set -o pipefail
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -o /tmp/mfr scripts/micro/mfma_f32_rate.hip 2>/dev/null && timeout -k 10 120 /tmp/mfr > gpurun_out/r6_mfma_rate.log 2>&1
cat gpurun_out/r6_mfma_rate.log
for rep in 1 2; do
  for m in 0 3 2; do
    PBX_SPLIT_PREFETCH=$m timeout -k 10 300 python -u bench.py --steps 200 --warmup 50 --secondary-dtype none --secondary-dcn off > gpurun_out/r6_split_$m.log 2>&1 || { echo "bench failed ($m)"; tail -5 gpurun_out/r6_split_$m.log; exit 3; }
    echo "split=$m rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_split_$m.log)"
  done
done
