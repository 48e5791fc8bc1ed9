set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_sharded_ipc.py tests/test_gpu_nrank_step.py -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_suite_sharded.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_suite_sharded.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -3 gpurun_out/smoke.log; exit $rc
