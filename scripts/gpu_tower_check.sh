#!/bin/bash
# GPU box: tower numerics tests, per-kernel tower times (rocprof) and the driver-style bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tower.py tests/test_gpu_tower32.py tests/test_gpu_graph.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_tower.log 2>&1 || { tail -30 gpurun_out/pytest_tower.log; exit 1; }
tail -1 gpurun_out/pytest_tower.log
for f in "" "--fp32"; do
  cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$GRAFT_REPO_ROOT/gpurun_out/tchk$f" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/bench_tower.py" --iters 20 $f \
    > "$GRAFT_REPO_ROOT/gpurun_out/tchk$f.log" 2>&1 || { echo "rocprof failed $f"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/tchk$f.log"; exit 2; }
  echo "== tower $f"; cut -d, -f1-4 "$GRAFT_REPO_ROOT/gpurun_out/tchk$f/run_kernel_stats.csv" | grep -i "tower\|t32"
done
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u bench.py --steps 200 --warmup 50 > gpurun_out/bchk.json 2> gpurun_out/bchk.err || { echo "bench failed"; tail -30 gpurun_out/bchk.err; exit 3; }
grep "ms/step" gpurun_out/bchk.err; grep -o '"ms_per_step": [0-9.]*\|"fp32_ms_per_step": [0-9.]*' gpurun_out/bchk.json
