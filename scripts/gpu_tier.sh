#!/bin/bash
# GPU box: BASELINE config 4 shape at 1e9 features -- tiered (HBM cap 2e7 rows,
# every written-back row spilled to SSD, reloaded when a later pass needs it)
# vs the all-in-HBM table on the same passes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf /tmp/pbx_ssd
timeout -k 10 500 python -u scripts/tier_bench.py --passes 6 --steps 30 --features 1e9 --hbm-cap 2e7 \
  --ssd /tmp/pbx_ssd --spill-unseen 0 > gpurun_out/tier_1e9.json 2> gpurun_out/tier_1e9.err \
  || { echo "tiered failed"; tail -30 gpurun_out/tier_1e9.err; exit 2; }
cat gpurun_out/tier_1e9.json
rm -rf /tmp/pbx_ssd
timeout -k 10 500 python -u scripts/tier_bench.py --passes 6 --steps 30 --features 1e9 --mode hbm \
  > gpurun_out/tier_hbm_1e9.json 2> gpurun_out/tier_hbm_1e9.err \
  || { echo "hbm failed"; tail -30 gpurun_out/tier_hbm_1e9.err; exit 3; }
cat gpurun_out/tier_hbm_1e9.json
