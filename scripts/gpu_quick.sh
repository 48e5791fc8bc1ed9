#!/bin/bash
# GPU box: tower tests, full GPU suite, driver-style bench, rocprof step profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 python -u -m pytest tests/test_gpu_tower.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_tower.log 2>&1 || { echo "tower tests failed rc=$?"; tail -60 gpurun_out/pytest_tower.log; exit 1; }
tail -3 gpurun_out/pytest_tower.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --diag-windows 3 > gpurun_out/bench_drv.json 2> gpurun_out/bench_drv.err \
  || { echo "bench failed"; tail -30 gpurun_out/bench_drv.err; exit 1; }
cat gpurun_out/bench_drv.json; grep "\[bench\]" gpurun_out/bench_drv.err
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 5 --total-features 2e8 \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
echo done
