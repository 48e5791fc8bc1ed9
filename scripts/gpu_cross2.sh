#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/diag_t32_adam.py || exit 5
timeout -k 10 300 python -u bench.py --model dcn_v2 --steps 200 --warmup 50 --secondary-dtype none > gpurun_out/dcnf.json 2> gpurun_out/dcnf.err || { echo "dcn bench failed"; tail -30 gpurun_out/dcnf.err; exit 3; }
grep -h 'wall' gpurun_out/dcnf.err
bash scripts/gpu_step_trace.sh dcnf2 --model dcn_v2 | head -8
