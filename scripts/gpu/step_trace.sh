#!/bin/bash
# GPU box: kernel (+ memory copy) trace of the driver-style bench step; table at 2e8 features to keep the prefill short.
# usage: scripts/gpu/step_trace.sh <tag> [extra bench args]   -> gpurun_out/st_<tag>.txt (per-kernel table + timeline)
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
anchor=${ANCHOR:-k_t32_fwd}
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/st_$tag" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 5 --total-features ${TRACE_FEATURES:-2e8} --secondary-dtype none --secondary-dcn off "$@" \
  > "$GRAFT_REPO_ROOT/gpurun_out/st_$tag.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/st_$tag.log"; exit 4; }
cd "$GRAFT_REPO_ROOT" && python3 scripts/step_breakdown.py gpurun_out/st_$tag/run_kernel_trace.csv --anchor "$anchor" \
  --copies gpurun_out/st_$tag/run_memory_copy_trace.csv > gpurun_out/st_$tag.txt && cat gpurun_out/st_$tag.txt
