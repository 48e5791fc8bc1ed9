#!/bin/bash
# GPU box: kernel trace of the driver-style bench step (table at 2e8 features to keep the prefill short)
# usage: scripts/gpu_step_trace.sh <tag> [extra bench args]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/st_$tag" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 5 --total-features 2e8 --secondary-dtype none "$@" \
  > "$GRAFT_REPO_ROOT/gpurun_out/st_$tag.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/st_$tag.log"; exit 4; }
cd "$GRAFT_REPO_ROOT" && python3 scripts/step_breakdown.py gpurun_out/st_$tag/run_kernel_trace.csv > gpurun_out/st_$tag.txt && cat gpurun_out/st_$tag.txt
