#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/micro/scaled_fc_parts.py > gpurun_out/r6_sfc_parts2.json 2>&1 || { echo "parts failed"; tail -10 gpurun_out/r6_sfc_parts2.json; exit 3; }
grep "{" gpurun_out/r6_sfc_parts2.json
