#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 250 --timeout-method thread tests/test_gpu_nrank_step.py -k "both" > $O/r5_nr_tests.log 2>&1 || { echo tests failed; exit 1; }
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1
for i in 1 2; do
  MASTER_PORT=2980$i timeout -k 10 300 python -u bench.py --force-collectives --steps 100 --warmup 20 --secondary-dtype none --secondary-dcn off > $O/r5_reh_dn_$i.txt 2>&1 || exit 1
done
