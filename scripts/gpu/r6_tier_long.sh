#!/bin/bash
# BASELINE config 4 with the SSD tier live: 10 passes of 1000 steps, 1e9 features, HBM table 4e7 rows,
# host tier capped at 3e7 rows (every pass spills to the O_DIRECT SSD log and reloads from it), the headline
# step (K = 4 steps per graph, pipelined front); ratio vs bench.py's ms/step measured on the same box first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 200 --warmup 50 --secondary-dtype none --secondary-dcn off > gpurun_out/r6_tier_head.json 2>/dev/null || exit 3
hm=$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_tier_head.json | awk '{print $2}')
echo "headline ms/step $hm"
rm -rf /tmp/pbx_ssd_r6
timeout -k 10 900 python -u scripts/tier_bench.py --passes 8 --steps ${STEPS:-2500} --hbm-cap ${HBMCAP:-6e7} --host-cap 3e7 --ssd /tmp/pbx_ssd_r6 \
  --headline-ms "$hm" > gpurun_out/r6_tier.json 2> gpurun_out/r6_tier.err
rc=$?
rm -rf /tmp/pbx_ssd_r6
grep "\[tier\]" gpurun_out/r6_tier.err | tail -12
cat gpurun_out/r6_tier.json
exit $rc
