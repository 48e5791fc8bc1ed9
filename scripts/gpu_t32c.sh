#!/bin/bash
# GPU box: fp32 tower tests + microbench + fp32 bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_tower32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t32_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/t32_tests.log; exit 1; }
tail -2 gpurun_out/t32_tests.log
timeout -k 10 120 python -u scripts/bench_tower.py --fp32 --iters 50 > gpurun_out/t32_micro.log 2>&1 || { tail gpurun_out/t32_micro.log; exit 2; }
cat gpurun_out/t32_micro.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --mlp-dtype fp32 --diag-windows 3 > gpurun_out/t32_bench_fp32.json 2> gpurun_out/t32_bench_fp32.err \
  || { echo "fp32 bench failed"; tail -30 gpurun_out/t32_bench_fp32.err; exit 4; }
cat gpurun_out/t32_bench_fp32.json; grep "\[bench\]" gpurun_out/t32_bench_fp32.err
echo done
