#!/bin/bash
# GPU box: graph tests, then same-box interleaved A/B of steps per graph (1 vs auto)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_graph.log 2>&1 || { tail -30 gpurun_out/pytest_graph.log; exit 1; }
tail -1 gpurun_out/pytest_graph.log
for rep in 1 2; do
for k in 1 0 8; do
  timeout -k 10 300 python -u bench.py --steps 400 --warmup 40 --secondary-dtype none --graph-steps $k \
    > gpurun_out/gk_$k.json 2> gpurun_out/gk_$k.err || { echo "bench failed"; tail -30 gpurun_out/gk_$k.err; exit 3; }
  echo "graph-steps=$k rep=$rep $(grep -h 'wall' gpurun_out/gk_$k.err | grep -o '[0-9.]* ms/step' | tr '\n' ' ') $(grep -o '"steps_per_graph": [0-9]*' gpurun_out/gk_$k.json)"
done
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/gk_driver.json 2> gpurun_out/gk_driver.err || { echo "bench failed"; tail -30 gpurun_out/gk_driver.err; exit 3; }
cat gpurun_out/gk_driver.json
