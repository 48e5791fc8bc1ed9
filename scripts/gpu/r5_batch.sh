#!/bin/bash
# one gpurun call, several measurements: each step under its own time limit,
# the first failure ends the script (no further GPU work after a fault)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_tiered.py > $O/r5_t.log 2>&1
timeout -k 10 300 python -u scripts/tier_bench.py --hbm-cap 4e7 --host-cap 3e7 --ssd /tmp/pbx_ssd_tier_a > $O/r5_tier_retain_bg.txt 2>&1
rm -rf /tmp/pbx_ssd_tier_a
timeout -k 10 500 python -u scripts/tier_bench.py --passes 10 --hbm-cap 4e7 --host-cap 3e7 --ssd /tmp/pbx_ssd_tier_b > $O/r5_tier_retain_bg10.txt 2>&1
rm -rf /tmp/pbx_ssd_tier_b
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --inputs host --trace-timed > $O/r5_h2d_host_$i.txt 2>&1
  HSA_ENABLE_SDMA=0 timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --inputs host --trace-timed > $O/r5_h2d_host_nosdma_$i.txt 2>&1
done
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof_bench -o bench -- python3 bench.py --steps 200 --warmup 20 --secondary-dtype none --secondary-dcn off > $O/r5_prof_bench.txt 2>&1
