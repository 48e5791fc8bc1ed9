#!/bin/bash
# config 4 with the SSD live after the SSD-index / flush changes: the SSD put micro on the box's disk, then
# scripts/gpu/r6_tier.sh (8 passes x 1000 steps, host cap 3e7, headline step)
set -o pipefail
mkdir -p gpurun_out
PBX_SSD_TIMING=1 timeout -k 10 300 python -u scripts/micro/ssd_put_bench.py /tmp/pbx_ssd_put > gpurun_out/r6_ssd_put.log 2>&1 || { echo "ssd put failed"; tail gpurun_out/r6_ssd_put.log; exit 3; }
cat gpurun_out/r6_ssd_put.log
bash scripts/gpu/r6_tier.sh
