#!/bin/bash
# GPU box: the whole GPU test suite, driver-style benches (bf16 / fp32), the
# 1-rank IPC rehearsal and its kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 420 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests rc=$rc: stopping"; exit $rc; fi
for dt in bf16 fp32; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --mlp-dtype $dt --diag-windows 2 \
    > gpurun_out/b_$dt.json 2> gpurun_out/b_$dt.err || { echo "bench $dt failed"; tail -30 gpurun_out/b_$dt.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/b_$dt.json')); print('$dt', d['ms_per_step'], d['value'])"
done
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555
timeout -k 10 300 python -u bench.py --force-collectives --steps 20 --warmup 5 > gpurun_out/fc.json 2> gpurun_out/fc.err \
  || { echo "fc failed"; tail -30 gpurun_out/fc.err; exit 3; }
grep "^{" gpurun_out/fc.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fc bf16', d['ms_per_step'], d['value'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_fc" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --force-collectives --steps 30 --warmup 5 --total-features 2e8 \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof_fc.log" 2>&1 || { echo "rocprof fc failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_fc.log"; exit 4; }
echo done
