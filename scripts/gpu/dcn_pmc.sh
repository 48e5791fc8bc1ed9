#!/bin/bash
# GPU box: PMC passes over the DCN-V2 bench step (k_cross_bwd / k_cross_fwd and the rest), one run per pass
# usage: scripts/gpu/dcn_pmc.sh <tag>  -> gpurun_out/dpmc_<tag>/p*/ + summary
set -o pipefail
tag=$1; shift
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/dpmc_$tag
mkdir -p $OUT
cd /tmp
i=0
for P in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model dcn_v2 --steps 6 --warmup 3 --total-features 2e8 --secondary-dtype none > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
cd $GRAFT_REPO_ROOT && python3 scripts/pmc_summary.py $OUT/p*/run_counter_collection.csv > $OUT/summary.txt 2>&1; cat $OUT/summary.txt | head -40
