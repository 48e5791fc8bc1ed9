#!/bin/bash
# GPU box: driver-style bench (bf16 headline + fp32 secondary in the same run).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b_default.json 2> gpurun_out/b_default.err \
  || { echo "bench failed"; tail -30 gpurun_out/b_default.err; exit 2; }
grep "^{" gpurun_out/b_default.json
grep "ms/step" gpurun_out/b_default.err
