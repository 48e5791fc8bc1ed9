#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tower.py tests/test_gpu_tower32.py tests/test_gpu_dcn.py tests/test_gpu_graph.py tests/test_gpu_fluid.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_dwh.log 2>&1 || { tail -30 gpurun_out/pytest_dwh.log; exit 1; }
tail -1 gpurun_out/pytest_dwh.log
for rep in 1 2; do
for v in 1 0; do
  PBX_DW_AFTER_HEAD=$v timeout -k 10 300 python -u bench.py --steps 400 --warmup 50 > gpurun_out/dwh_$v.json 2> gpurun_out/dwh_$v.err || { echo "bench failed"; tail -30 gpurun_out/dwh_$v.err; exit 3; }
  echo "PBX_DW_AFTER_HEAD=$v rep=$rep $(grep -h 'wall' gpurun_out/dwh_$v.err | grep -o 'wall [0-9.]* ms/step' | tr '\n' ' ')"
done
done
bash scripts/gpu_step_trace.sh dwh --mlp-dtype fp32 > /dev/null 2>&1; python3 scripts/step_breakdown.py gpurun_out/st_dwh/run_kernel_trace.csv --anchor k_t32_fwd > gpurun_out/st_dwh32.txt; head -14 gpurun_out/st_dwh32.txt
