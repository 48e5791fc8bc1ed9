#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/micro/ipc_exchange_bench.py > gpurun_out/r6_ipc_bench.jsonl 2>&1 || { echo failed; tail -20 gpurun_out/r6_ipc_bench.jsonl; exit 3; }
cat gpurun_out/r6_ipc_bench.jsonl | grep "{"
