# x3 1-rank sharded rehearsal: dW enqueue position / split count A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python -u bench.py --steps 100 --warmup 20 --secondary-dtype none --secondary-dcn off --force-collectives"
i=0
for e in PBX_NOOP=1 PBX_DW_AFTER_HEAD=0 PBX_TOWER_X3_DW_SPLITS=4 PBX_ADAM_OVERLAP_MULTI=0 PBX_NOOP=1 PBX_DW_AFTER_HEAD=0; do
  i=$((i+1))
  env $e RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29640 + i)) timeout -k 10 300 $B > gpurun_out/rehab2_$i.txt 2>&1 || exit 1
  echo "$e $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rehab2_$i.txt)"
done
