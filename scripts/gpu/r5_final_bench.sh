#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
timeout -k 10 300 python -u bench.py > $O/r5_bench_default.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/r5_bench_20.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 200 --warmup 50 > $O/r5_bench_200.txt 2>&1
timeout -k 10 400 python -u scripts/bench_fluid.py > $O/r5_bench_fluid.txt 2>&1
