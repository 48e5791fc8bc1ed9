#!/bin/bash
# GPU box: fp32 tower tests, fp32 / bf16 driver-style benches, rocprof of the fp32 step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tower32.py tests/test_gpu_tower.py -v --timeout 200 \
  --timeout-method thread > gpurun_out/t32_tests.log 2>&1
rc=$?
tail -25 gpurun_out/t32_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --mlp-dtype fp32 --diag-windows 3 > gpurun_out/t32_bench_fp32.json 2> gpurun_out/t32_bench_fp32.err \
  || { echo "fp32 bench failed"; tail -30 gpurun_out/t32_bench_fp32.err; exit 2; }
cat gpurun_out/t32_bench_fp32.json; grep "\[bench\]" gpurun_out/t32_bench_fp32.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --diag-windows 3 > gpurun_out/t32_bench_bf16.json 2> gpurun_out/t32_bench_bf16.err \
  || { echo "bf16 bench failed"; tail -30 gpurun_out/t32_bench_bf16.err; exit 2; }
cat gpurun_out/t32_bench_bf16.json; grep "\[bench\]" gpurun_out/t32_bench_bf16.err
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof32" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 5 --total-features 2e8 --mlp-dtype fp32 \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof32.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof32.log"; exit 3; }
echo done
