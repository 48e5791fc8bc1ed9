#!/bin/bash
# GPU box: secondary-fp32 timing with the named side streams, and with more HW queues.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --total-features 2e8 > gpurun_out/s1.json 2> gpurun_out/s1.err \
  || { echo "s1 failed"; tail -20 gpurun_out/s1.err; exit 2; }
grep "ms/step" gpurun_out/s1.err
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --total-features 2e8 > gpurun_out/s2.json 2> gpurun_out/s2.err \
  || { echo "s2 failed"; tail -20 gpurun_out/s2.err; exit 3; }
grep "ms/step" gpurun_out/s2.err
