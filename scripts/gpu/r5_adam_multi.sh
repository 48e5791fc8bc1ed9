#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 250 --timeout-method thread tests/test_gpu_nrank_step.py -k "both" tests/test_gpu_fluid.py > $O/r5_am_tests.log 2>&1; echo "tests rc=$?"
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1
for i in 1 2; do
  MASTER_PORT=2952$i timeout -k 10 300 python -u bench.py --force-collectives --steps 100 --warmup 20 --secondary-dtype none --secondary-dcn off > $O/r5_am_reh0_$i.txt 2>&1
  MASTER_PORT=2953$i PBX_ADAM_OVERLAP_MULTI=1 timeout -k 10 300 python -u bench.py --force-collectives --steps 100 --warmup 20 --secondary-dtype none --secondary-dcn off > $O/r5_am_reh1_$i.txt 2>&1
done
unset RANK WORLD_SIZE LOCAL_RANK MASTER_ADDR
timeout -k 10 600 python -u scripts/bench_fluid.py > $O/r5_am_fluid_ov.txt 2>&1
PBX_ADAM_OVERLAP=0 timeout -k 10 600 python -u scripts/bench_fluid.py > $O/r5_am_fluid_noov.txt 2>&1
exit 0
