#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_td2.log 2>&1 \
  || { tail -5 gpurun_out/pytest_td2.log; exit 1; }
for td in 1 0; do
  PBX_TABLE_DEDUP=$td timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --diag-windows 2 --secondary-dtype none \
    > gpurun_out/b_td$td.json 2> gpurun_out/b_td$td.err || { echo "bench failed"; tail -30 gpurun_out/b_td$td.err; exit 2; }
  echo "table_dedup=$td"; grep "ms/step" gpurun_out/b_td$td.err
done
export PBX_TABLE_DEDUP=1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_td" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 5 --total-features 2e8 --secondary-dtype none \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof_td.log" 2>&1 || { echo "rocprof failed"; exit 4; }
echo done
