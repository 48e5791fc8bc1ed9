#!/bin/bash
# fp32 tower: non-temporal MP32 accesses (default) vs plain (PBX_TOWER_DEBUG=256)
set -e
mkdir -p gpurun_out
o=gpurun_out/nt_ab.txt
: > $o
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tower32.py tests/test_gpu_tower.py > gpurun_out/nt_tests.log 2>&1
for rep in 1 2; do
  for d in 0 256; do
    echo "PBX_TOWER_DEBUG=$d" >> $o
    PBX_TOWER_DEBUG=$d timeout -k 10 200 python -u scripts/bench_tower.py --fp32 2>&1 | grep "\[tower\]" >> $o
    PBX_TOWER_DEBUG=$d timeout -k 10 300 python -u bench.py --steps 200 --warmup 50 --secondary-dtype none --secondary-dcn off 2>&1 | grep -o "wall [0-9.]* ms/step" >> $o
  done
done
timeout -k 10 100 python -u scripts/tower32_stamps.py >> $o 2>&1
cat $o
