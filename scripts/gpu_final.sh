#!/bin/bash
# GPU box: the whole GPU suite the way the driver runs it, smoke(), and the driver-style bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_all.log
if [ $rc -ne 0 ]; then echo "gpu tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 2; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/b_nodefault.json 2> gpurun_out/b_nodefault.err || { echo "bench failed"; tail -30 gpurun_out/b_nodefault.err; exit 3; }
grep "^{" gpurun_out/b_nodefault.json
