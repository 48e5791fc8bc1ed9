# x3 dW split-M A/B: tests, microbench per split count, full bench per split count
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_tower_x3.py > gpurun_out/x3_tests3.log 2>&1
rc=$?; echo "x3 tests rc=$rc"; tail -3 gpurun_out/x3_tests3.log; [ $rc -eq 0 ] || exit $rc
for sp in 1 2 4; do
  PBX_TOWER_X3_DW_SPLITS=$sp timeout -k 10 120 python -u scripts/bench_tower.py --x3 > gpurun_out/x3_micro_s$sp.txt 2>&1 || exit 1
  echo "splits=$sp"; grep -E "dW|forward|chain" gpurun_out/x3_micro_s$sp.txt
done
for sp in 1 2 4 2 1 4; do
  PBX_TOWER_X3_DW_SPLITS=$sp timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --secondary-dtype none --secondary-dcn off > gpurun_out/x3_bench_s$sp.txt 2>&1 || exit 1
  echo "splits=$sp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/x3_bench_s$sp.txt)"
done
