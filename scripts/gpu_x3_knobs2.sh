# x3 headline: re-sweep the sparse / head kernel knobs on the new critical path
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python -u bench.py --steps 200 --warmup 20 --secondary-dtype none --secondary-dcn off"
i=0
for e in PBX_NOOP=1 PBX_TD_ITEMS=1 PBX_TD_ITEMS=4 PBX_TD_SEG_ITEMS=2 PBX_HEAD_BWD_RB=4 PBX_TD_FINISH_SIDE=1 PBX_ADAM_MAX_BLOCKS=256 PBX_NOOP=1 PBX_TD_ITEMS=1 PBX_HEAD_BWD_RB=4 PBX_TD_FINISH_SIDE=1; do
  i=$((i+1)); env $e timeout -k 10 300 $B > gpurun_out/kn2_$i.txt 2>&1 || exit 1
  echo "$e $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/kn2_$i.txt)"
done
