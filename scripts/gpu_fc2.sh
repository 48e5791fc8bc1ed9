#!/bin/bash
# GPU box: IPC / sharded tests, then the 1-rank IPC rehearsal bench + its trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipc.py tests/test_gpu_sharded_ipc.py tests/test_gpu_kernels.py tests/test_gpu_graph.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_fc2.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_fc2.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555
timeout -k 10 300 python -u bench.py --force-collectives --steps 20 --warmup 5 > gpurun_out/fc.json 2> gpurun_out/fc.err \
  || { echo "fc failed"; tail -30 gpurun_out/fc.err; exit 3; }
grep "^{" gpurun_out/fc.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fc bf16', d['ms_per_step'], d['value'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_fc" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --force-collectives --steps 30 --warmup 5 --total-features 2e8 \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof_fc.log" 2>&1 || { echo "rocprof fc failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_fc.log"; exit 4; }
echo done
