#!/bin/bash
# k_ra_g store cost + occupancy counters
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=gpurun_out/ra_parts2.jsonl
: > $o
for d in 0 2; do
  PBX_RA_DEBUG=$d timeout -k 10 120 python -u scripts/micro/ra_bwd_parts.py >> $o
done
PBX_RA_DEBUG=2 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/ra_prof2 -o ra -- python3 scripts/micro/ra_bwd_parts.py > gpurun_out/ra_prof2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/ra_pmc -o ra -- python3 scripts/micro/ra_bwd_parts.py > gpurun_out/ra_pmc.log 2>&1
cat $o
