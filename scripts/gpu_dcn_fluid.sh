#!/bin/bash
# GPU box: DCN-V2 (config 5) bench + step kernel trace, fluid train_from_dataset bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --model dcn_v2 --steps 200 --warmup 50 > gpurun_out/dcn.json 2> gpurun_out/dcn.err || { echo "dcn bench failed"; tail -30 gpurun_out/dcn.err; exit 3; }
grep "ms/step" gpurun_out/dcn.err; cat gpurun_out/dcn.json
bash scripts/gpu_step_trace.sh dcn --model dcn_v2 || true
timeout -k 10 400 python -u scripts/bench_fluid.py > gpurun_out/fluid.log 2>&1 || { echo "fluid bench failed"; tail -30 gpurun_out/fluid.log; exit 4; }
tail -5 gpurun_out/fluid.log
