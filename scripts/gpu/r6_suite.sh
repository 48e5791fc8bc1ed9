#!/bin/bash
# GPU box: whole GPU suite, smoke(), driver-style bench (defaults and 20/5), step kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6_pytest.log 2>&1
rc=$?
tail -1 gpurun_out/r6_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r6_pytest.log | head -20; if [ $rc -ne 1 ]; then exit $rc; fi; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke_final.log; exit 2; }
tail -1 gpurun_out/r6_smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6_b.json 2> gpurun_out/r6_b.err || { echo "bench failed"; tail -30 gpurun_out/r6_b.err; exit 3; }
cat gpurun_out/r6_b.json
timeout -k 10 400 python -u bench.py > gpurun_out/r6_b_def.json 2> gpurun_out/r6_b_def.err || { echo "bench failed"; tail -30 gpurun_out/r6_b_def.err; exit 3; }
grep -o '"ms_per_step": [0-9.]*\|"fp32_ms_per_step": [0-9.]*\|"steps": [0-9]*' gpurun_out/r6_b_def.json | tr '\n' ' '; echo
bash scripts/gpu/step_trace.sh r6_final | head -16
timeout -k 10 400 python -u bench.py --model dcn_v2 --steps 200 --warmup 50 --secondary-dtype none > gpurun_out/r6_b_dcn.json 2> gpurun_out/r6_b_dcn.err || { echo "dcn bench failed"; tail -30 gpurun_out/r6_b_dcn.err; exit 3; }
grep -h "wall" gpurun_out/r6_b_dcn.err
ANCHOR=k_cross_fwd bash scripts/gpu/step_trace.sh r6_dcn --model dcn_v2 | head -30
