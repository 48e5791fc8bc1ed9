#!/bin/bash
# GPU box: 1-rank rehearsal of the multi-GPU step (sparse exchange + dense
# all-reduce on the IPC meshes, captured in the graph), plus a kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555
for dt in bf16 fp32; do
  timeout -k 10 300 python -u bench.py --force-collectives --steps 20 --warmup 5 --mlp-dtype $dt --diag-windows 2 \
    > gpurun_out/fc_$dt.json 2> gpurun_out/fc_$dt.err || { echo "fc $dt failed"; tail -30 gpurun_out/fc_$dt.err; exit 2; }
  cat gpurun_out/fc_$dt.json; grep "\[bench\]\|\[sparse\]" gpurun_out/fc_$dt.err
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_fc" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --force-collectives --steps 30 --warmup 5 --total-features 2e8 \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof_fc.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_fc.log"; exit 3; }
cd "$GRAFT_REPO_ROOT" && timeout -k 10 120 python scripts/tower32_stamps.py > gpurun_out/stamps.log 2>&1; cat gpurun_out/stamps.log | tail -30
echo done
