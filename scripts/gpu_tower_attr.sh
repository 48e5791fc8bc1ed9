#!/bin/bash
# GPU box: attribute k_tower_fwd time (PBX_TOWER_DEBUG bits 8 = no m-packed stores, 16 = no output layer)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in 0 8 16 24; do
  cd /tmp && PBX_TOWER_DEBUG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$GRAFT_REPO_ROOT/gpurun_out/tattr$d" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/bench_tower.py" --iters 20 \
    > "$GRAFT_REPO_ROOT/gpurun_out/tattr$d.log" 2>&1 || { echo "rocprof failed d=$d"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/tattr$d.log"; exit 2; }
  echo "== debug=$d"; cut -d, -f1-4 "$GRAFT_REPO_ROOT/gpurun_out/tattr$d/run_kernel_stats.csv" | grep -i tower
done
