#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python scripts/micro/graph_overhead.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipc.py tests/test_gpu_sharded_ipc.py -q -x --timeout 420 \
  --timeout-method thread > gpurun_out/ipc_tests.log 2>&1 || { tail -40 gpurun_out/ipc_tests.log; exit 1; }
tail -2 gpurun_out/ipc_tests.log
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_fc" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --force-collectives --steps 30 --warmup 5 --total-features 2e8 \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof_fc.log" 2>&1 || { echo "rocprof fc failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_fc.log"; exit 3; }
grep "\[bench\]" "$GRAFT_REPO_ROOT/gpurun_out/prof_fc.log"
echo done
