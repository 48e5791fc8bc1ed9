#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dcn.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_dcn.log 2>&1 || { tail -40 gpurun_out/pytest_dcn.log; exit 1; }
tail -1 gpurun_out/pytest_dcn.log
for f in 1 0 1; do
  PBX_CROSS_FUSED=$f timeout -k 10 300 python -u bench.py --model dcn_v2 --steps 200 --warmup 50 --secondary-dtype none > gpurun_out/dcnf$f.json 2> gpurun_out/dcnf$f.err || { echo "dcn bench failed"; tail -30 gpurun_out/dcnf$f.err; exit 3; }
  echo "fused=$f $(grep -h 'wall' gpurun_out/dcnf$f.err)"
done
bash scripts/gpu_step_trace.sh dcnf3 --model dcn_v2 | head -24
