set -o pipefail
mkdir -p gpurun_out
timeout -k 10 100 python -u -m pytest tests/test_gpu_tower.py -q --timeout 90 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 100 python -u scripts/bench_tower.py
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tprof -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_tower.py --iters 20 > $GRAFT_REPO_ROOT/gpurun_out/tprof.log 2>&1
cat $GRAFT_REPO_ROOT/gpurun_out/tprof/run_kernel_stats.csv | cut -d, -f1-8 | head -12
