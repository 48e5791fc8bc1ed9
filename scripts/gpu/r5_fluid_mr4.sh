#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
FLAGS_padbox_pipelined_front=false timeout -k 10 200 python -u scripts/debug_fluid_mr.py --oracle --timeout 120 > $O/r5_mr_cmp_k2.log 2>&1; echo "k2 rc=$?"
FLAGS_padbox_pipelined_front=false FLAGS_padbox_train_steps_per_graph=1 timeout -k 10 200 python -u scripts/debug_fluid_mr.py --oracle --timeout 120 > $O/r5_mr_cmp_k1.log 2>&1; echo "k1 rc=$?"
exit 0
