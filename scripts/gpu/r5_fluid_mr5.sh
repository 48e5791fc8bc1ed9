#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
timeout -k 10 200 python -u scripts/debug_fluid_eager_vs_graph.py --k 2 > $O/r5_eg_k2.log 2>&1; echo "eg rc=$?"
timeout -k 10 600 python -u -m pytest -v --timeout 250 --timeout-method thread tests/test_gpu_fluid_multirank.py tests/test_gpu_fluid.py tests/test_gpu_nrank_step.py > $O/r5_mr_tests.log 2>&1; echo "tests rc=$?"
exit 0
