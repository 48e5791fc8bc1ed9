set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_tower_x3.py > gpurun_out/x3_tests.log 2>&1
rc=$?; echo "x3 tests rc=$rc"; tail -5 gpurun_out/x3_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/bench_tower.py --x3 > gpurun_out/x3_micro.txt 2>&1 && timeout -k 10 120 python -u scripts/bench_tower.py --fp32 >> gpurun_out/x3_micro.txt 2>&1
rc=$?; cat gpurun_out/x3_micro.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --mlp-dtype fp32x3 --secondary-dtype fp32 --secondary-dcn off --steps 200 --warmup 20 > gpurun_out/x3_bench.txt 2>&1
rc=$?; tail -12 gpurun_out/x3_bench.txt; exit $rc
