#!/bin/bash
# GPU box: driver-style bench (bf16 tower) and the fp32-MLP precision variant.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --diag-windows 2 > gpurun_out/bench_bf16.json 2> gpurun_out/bench_bf16.err \
  || { echo "bf16 bench failed"; tail -30 gpurun_out/bench_bf16.err; exit 1; }
cat gpurun_out/bench_bf16.json; grep "\[bench\]" gpurun_out/bench_bf16.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --diag-windows 2 --mlp-dtype fp32 > gpurun_out/bench_fp32.json 2> gpurun_out/bench_fp32.err \
  || { echo "fp32 bench failed"; tail -30 gpurun_out/bench_fp32.err; exit 1; }
cat gpurun_out/bench_fp32.json; grep "\[bench\]" gpurun_out/bench_fp32.err
