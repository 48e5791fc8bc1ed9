#!/bin/bash
# fp32 tower remainder placement: tests, kernel times, bench, stamps
set -e
mkdir -p gpurun_out
o=gpurun_out/rem_ab_$1.txt
: > $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tower32.py tests/test_gpu_tower.py tests/test_gpu_fluid.py > gpurun_out/rem_tests_$1.log 2>&1
tail -1 gpurun_out/rem_tests_$1.log >> $o
timeout -k 10 200 python -u scripts/bench_tower.py --fp32 2>&1 | grep "\[tower\]" >> $o
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 200 --warmup 50 --secondary-dtype none --secondary-dcn off 2>&1 | grep -o "wall [0-9.]* ms/step" >> $o
done
timeout -k 10 100 python -u scripts/tower32_stamps.py >> $o 2>&1
cat $o
