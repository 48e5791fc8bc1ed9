#!/bin/bash
# knob A/B on the current build: fp32 dW LDS ring (PBX_T32_DW_RING 23 default, 24, 25, 16) on the headline bench;
# tower weight prefetch depth (PBX_TOWER_PF 6 default, 4, 8) on DCN-V2
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for r in 23 24 25 16; do
    PBX_T32_DW_RING=$r timeout -k 10 300 python -u bench.py --steps 200 --warmup 50 --secondary-dtype none --secondary-dcn off > gpurun_out/r6_knob_ring$r.json 2>/dev/null || { echo "ring $r failed"; exit 3; }
    echo "rep$rep ring=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_knob_ring$r.json)"
  done
done
for rep in 1 2; do
  for pf in 6 4 8; do
    PBX_TOWER_PF=$pf timeout -k 10 300 python -u bench.py --model dcn_v2 --steps 200 --warmup 50 --secondary-dtype none > gpurun_out/r6_knob_pf$pf.json 2>/dev/null || { echo "pf $pf failed"; exit 4; }
    echo "rep$rep dcn pf=$pf $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6_knob_pf$pf.json)"
  done
done
