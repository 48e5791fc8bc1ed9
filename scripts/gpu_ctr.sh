#!/bin/bash
# GPU box: CTR op tests + microbenchmarks + kernel trace of the microbenchmark.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ctr_ops.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_ctr.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_ctr.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u scripts/micro/bench_ctr_ops.py > gpurun_out/ctr_bench.jsonl 2> gpurun_out/ctr_bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/ctr_bench.err; exit 2; }
cat gpurun_out/ctr_bench.jsonl
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_ctr" \
  -o run -- python3 "$GRAFT_REPO_ROOT/scripts/micro/bench_ctr_ops.py" --iters 20 \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof_ctr.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_ctr.log"; exit 4; }
echo done
