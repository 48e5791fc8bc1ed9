#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
T="timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread"
$T tests/test_gpu_nrank_step.py -k "2-plain or 2-both" > $O/r5_mr_nrank.log 2>&1; echo "nrank rc=$?"
$T "tests/test_gpu_fluid_multirank.py::test_fluid_two_ranks_match_union_oracle[False]" > $O/r5_mr_default.log 2>&1; echo "default rc=$?"
FLAGS_padbox_fc_precision=bf16 $T "tests/test_gpu_fluid_multirank.py::test_fluid_two_ranks_match_union_oracle[False]" > $O/r5_mr_bf16.log 2>&1; echo "bf16 rc=$?"
FLAGS_padbox_pipelined_front=false FLAGS_padbox_train_steps_per_graph=1 $T "tests/test_gpu_fluid_multirank.py::test_fluid_two_ranks_match_union_oracle[False]" > $O/r5_mr_k1.log 2>&1; echo "k1 rc=$?"
PBX_TEST_FLUID_GRAPH=0 $T "tests/test_gpu_fluid_multirank.py::test_fluid_two_ranks_match_union_oracle[False]" > $O/r5_mr_eager.log 2>&1; echo "eager rc=$?"
exit 0
