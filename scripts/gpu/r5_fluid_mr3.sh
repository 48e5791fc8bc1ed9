#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
PBX_IPC_TRACE=1 PBX_TEST_FLUID_GRAPH=0 timeout -k 10 200 python -u scripts/debug_fluid_mr.py --timeout 60 > $O/r5_mr_dbg.log 2>&1; echo "eager rc=$?"
T="timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread"
FLAGS_padbox_pipelined_front=false $T "tests/test_gpu_fluid_multirank.py::test_fluid_two_ranks_match_union_oracle[False]" > $O/r5_mr_nopipe.log 2>&1; echo "nopipe rc=$?"
FLAGS_padbox_train_steps_per_graph=1 $T "tests/test_gpu_fluid_multirank.py::test_fluid_two_ranks_match_union_oracle[False]" > $O/r5_mr_k1pipe.log 2>&1; echo "k1pipe rc=$?"
exit 0
