#!/bin/bash
# GPU box, round 6: a chosen set of GPU tests (each under its own timeout)
# then a bench.  usage: scripts/gpu/r6_run.sh <tag> "<test files>" "<bench args>"
set -o pipefail
tag=$1; tests=$2; bargs=$3
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
if [ -n "$tests" ]; then
  timeout -k 10 1000 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu $tests > gpurun_out/${tag}_tests.log 2>&1
  rc=$?
  tail -3 gpurun_out/${tag}_tests.log
  # test failures (1) or none (0): the GPU is fine, go on; anything else: stop here
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
if [ -n "$bargs" ]; then
  timeout -k 10 400 python -u bench.py $bargs > gpurun_out/${tag}_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.log; exit 3; }
  grep -h "^\[bench\]\|metric" gpurun_out/${tag}_bench.log | tail -12
fi
