#!/bin/bash
# GPU box: kernel trace of the 1-rank IPC rehearsal step (bf16) and of the plain 1-GPU step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_1" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 5 --total-features 2e8 \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof_1.log" 2>&1 || { echo "rocprof 1 failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_1.log"; exit 3; }
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_fc" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --force-collectives --steps 30 --warmup 5 --total-features 2e8 \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof_fc.log" 2>&1 || { echo "rocprof fc failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_fc.log"; exit 3; }
ls -R "$GRAFT_REPO_ROOT/gpurun_out" | head -30
echo done
