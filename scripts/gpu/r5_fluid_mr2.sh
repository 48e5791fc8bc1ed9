#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
T="timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread"
PBX_TEST_FLUID_GRAPH=0 $T "tests/test_gpu_fluid_multirank.py::test_fluid_two_ranks_match_union_oracle[False]" > $O/r5_mr_eager.log 2>&1; echo "eager rc=$?"
