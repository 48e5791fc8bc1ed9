#!/bin/bash
# GPU box: fp32 tower microbench + PMC passes, fp32 bench + rocprof.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_tower32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t32_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/t32_tests.log; exit 1; }
tail -2 gpurun_out/t32_tests.log
timeout -k 10 120 python -u scripts/bench_tower.py --fp32 --iters 50 > gpurun_out/t32_micro.log 2>&1 || { tail gpurun_out/t32_micro.log; exit 2; }
cat gpurun_out/t32_micro.log
timeout -k 10 120 python -u scripts/bench_tower.py --iters 50 > gpurun_out/t16_micro.log 2>&1 || { tail gpurun_out/t16_micro.log; exit 2; }
cat gpurun_out/t16_micro.log
cd /tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/t32pmc
mkdir -p $OUT
i=0
for P in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_tower.py --fp32 --iters 3 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 3; }
done
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --mlp-dtype fp32 --diag-windows 3 > gpurun_out/t32_bench_fp32.json 2> gpurun_out/t32_bench_fp32.err \
  || { echo "fp32 bench failed"; tail -30 gpurun_out/t32_bench_fp32.err; exit 4; }
cat gpurun_out/t32_bench_fp32.json; grep "\[bench\]" gpurun_out/t32_bench_fp32.err
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof32" \
  -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 5 --total-features 2e8 --mlp-dtype fp32 \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof32.log" 2>&1 || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof32.log"; exit 5; }
echo done
