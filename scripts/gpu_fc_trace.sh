#!/bin/bash
# GPU box: kernel trace of the 1-rank IPC rehearsal step (--force-collectives)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29557
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/st_fc" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --force-collectives --steps 30 --warmup 5 --total-features 2e8 --secondary-dtype none \
  > "$GRAFT_REPO_ROOT/gpurun_out/st_fc.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/st_fc.log"; exit 4; }
cd "$GRAFT_REPO_ROOT" && python3 scripts/step_breakdown.py gpurun_out/st_fc/run_kernel_trace.csv > gpurun_out/st_fc.txt && head -30 gpurun_out/st_fc.txt
