#!/bin/bash
# GPU box: N-rank step rehearsals on one GPU: --force-collectives (1 rank, IPC meshes) and --same-gpu with 2 ranks
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555 timeout -k 10 300 python -u bench.py --force-collectives --steps 200 --warmup 50 --secondary-dtype none > gpurun_out/fc.json 2> gpurun_out/fc.err \
  || { echo "fc bench failed"; tail -30 gpurun_out/fc.err; exit 3; }
grep -h "wall" gpurun_out/fc.err; grep -o '"sparse_exchange": "[a-z]*"\|"dense_allreduce": "[a-z]*"' gpurun_out/fc.json | tr '\n' ' '; echo
timeout -k 10 400 python -u bench.py --gpus 2 --same-gpu --steps 100 --warmup 20 --secondary-dtype none --total-features 2e8 > gpurun_out/sg2.json 2> gpurun_out/sg2.err \
  || { echo "same-gpu bench failed"; tail -30 gpurun_out/sg2.err; exit 4; }
grep -h "wall" gpurun_out/sg2.err | head -2; grep -o '"value": [0-9.]*\|"ranks_seen": [0-9]*\|"sparse_exchange": "[a-z]*"\|"launcher": "[a-z-]*"' gpurun_out/sg2.json | tr '\n' ' '; echo
