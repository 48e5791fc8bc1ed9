#!/bin/bash
# GPU box: whole GPU suite, driver-style bench, step kernel trace (tag $1)
set -o pipefail
tag=${1:-iter}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$tag.log
if [ $rc -ne 0 ]; then grep -E "Error|error|FAIL" gpurun_out/pytest_$tag.log | head -20; exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 200 --warmup 50 > gpurun_out/b_$tag.json 2> gpurun_out/b_$tag.err || { echo "bench failed"; tail -30 gpurun_out/b_$tag.err; exit 3; }
grep "ms/step" gpurun_out/b_$tag.err; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"fp32_ms_per_step": [0-9.]*' gpurun_out/b_$tag.json
bash scripts/gpu_step_trace.sh $tag
