#!/bin/bash
# One GPU-box pass: GPU tests, 1-GPU bench (graph + diag windows), 1-rank
# forced-collectives rehearsal of the sharded path, rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py --steps 200 --warmup 20 --diag-windows 3 > gpurun_out/bench.json 2> gpurun_out/bench.err \
  || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json; grep "\[bench\]" gpurun_out/bench.err | tail -6
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 1 --steps 100 --warmup 10 --force-collectives \
  > gpurun_out/bench_fc.json 2> gpurun_out/bench_fc.err || { echo "forced-collectives bench failed"; tail -30 gpurun_out/bench_fc.err; exit 1; }
grep metric gpurun_out/bench_fc.json; grep "\[bench\]" gpurun_out/bench_fc.err | tail -3
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 5 --total-features 2e8 \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
echo done
