#!/bin/bash
# GPU box: HIP API + kernel trace of a short driver-style bench (20 timed steps), to time the host-side API calls
# around the timed window.  usage: scripts/gpu/api_trace.sh <tag> [bench args]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/api_$tag" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --secondary-dtype none --secondary-dcn off --trace-timed "$@" \
  > "$GRAFT_REPO_ROOT/gpurun_out/api_$tag.log" 2>&1
