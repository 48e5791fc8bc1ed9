# 1-GPU rehearsal of the multi-GPU step: every collective of the N-GPU path
# (key / value / gradient all-to-all, dense all-reduce) runs on one rank
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 --diag-windows 2 --force-collectives \
  > gpurun_out/bench_fc.json 2> gpurun_out/bench_fc.err || { echo "forced-collectives bench failed"; tail -30 gpurun_out/bench_fc.err; exit 1; }
cat gpurun_out/bench_fc.json; grep "\[bench\]" gpurun_out/bench_fc.err
# single rank via env:// (no launcher process under the profiler)
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29512
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_fc" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 5 --total-features 2e8 --force-collectives \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof_fc.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_fc.log"; exit 1; }
echo done
