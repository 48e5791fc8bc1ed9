#!/bin/bash
# GPU box: kernel trace of the default bench (bf16 headline + fp32 secondary)
# and of a standalone fp32 bench, to compare the fp32 step inside one run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_sec" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --total-features 2e8 \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof_sec.log" 2>&1 || { echo "rocprof sec failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_sec.log"; exit 4; }
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_f32" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --total-features 2e8 --mlp-dtype fp32 \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof_f32.log" 2>&1 || { echo "rocprof f32 failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_f32.log"; exit 5; }
grep "ms/step" "$GRAFT_REPO_ROOT/gpurun_out/prof_sec.log" "$GRAFT_REPO_ROOT/gpurun_out/prof_f32.log"
echo done
