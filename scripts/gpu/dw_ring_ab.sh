#!/bin/bash
# full-bench A/B of the fp32 dW ring variants (PBX_T32_DW_RING = DS*10 + NS)
set -e
mkdir -p gpurun_out
o=gpurun_out/dw_ring_ab.txt
: > $o
for rep in 1 2; do
  for r in 23 16 24 25 0; do
    echo -n "PBX_T32_DW_RING=$r " >> $o
    PBX_T32_DW_RING=$r timeout -k 10 300 python -u bench.py --steps 200 --warmup 50 --secondary-dtype none --secondary-dcn off 2>&1 | grep -o "wall [0-9.]* ms/step" >> $o
  done
done
cat $o
