#!/bin/bash
# rank_attention backward part timings under the PBX_RA_* knobs, after the CTR op tests
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ctr_ops.py > gpurun_out/ra_tests.log 2>&1
o=gpurun_out/ra_parts.jsonl
: > $o
for cfg in "0 0" "0 1" "0 2" "0 4" "0 8" "10 0" "20 0"; do
  set -- $cfg
  PBX_RA_DW_SPLITS=$1 PBX_RA_G_BLOCKS=$2 timeout -k 10 120 python -u scripts/micro/ra_bwd_parts.py | sed "s/}/, \"g_blocks\": $2}/" >> $o
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/ra_prof -o ra -- python3 scripts/micro/ra_bwd_parts.py > gpurun_out/ra_prof.log 2>&1
timeout -k 10 300 python -u scripts/micro/bench_ctr_ops.py --iters 50 > gpurun_out/ctr_micro.jsonl
cat $o
