#!/bin/bash
# GPU box: single-shard table dedup -- engine GPU tests, then bench + trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_graph.py tests/test_gpu_feature_types.py \
  tests/test_gpu_nodedup.py tests/test_gpu_tower.py tests/test_gpu_fluid.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_td.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_td.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --diag-windows 2 > gpurun_out/b_td.json 2> gpurun_out/b_td.err \
  || { echo "bench failed"; tail -30 gpurun_out/b_td.err; exit 2; }
grep "^{" gpurun_out/b_td.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bf16', d['ms_per_step'], d['value'], 'fp32', d['config'].get('fp32_ms_per_step'))"
grep "diag window" gpurun_out/b_td.err
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_td" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 5 --total-features 2e8 --secondary-dtype none \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof_td.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_td.log"; exit 4; }
echo done
