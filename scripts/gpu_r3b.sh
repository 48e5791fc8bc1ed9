#!/bin/bash
# GPU box: feature types (variable codec), tiered codecs, no-dedup + streaming ckpt
# tests, then the no-dedup bench and its trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_feature_types.py tests/test_gpu_tiered.py tests/test_gpu_nodedup.py \
  tests/test_gpu_ckpt_stream.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r3b.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_r3b.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --dedup off --diag-windows 2 \
  > gpurun_out/b_dd_off.json 2> gpurun_out/b_dd_off.err || { echo "bench failed"; tail -30 gpurun_out/b_dd_off.err; exit 2; }
grep "^{" gpurun_out/b_dd_off.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('dedup off', d['ms_per_step'], d['value'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_nd" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --dedup off --steps 30 --warmup 5 --total-features 2e8 \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof_nd.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_nd.log"; exit 4; }
echo done
