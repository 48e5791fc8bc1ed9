# x3 1-rank sharded rehearsal: next-batch dedup placement A/B (PBX_SPLIT_PREFETCH; multi default 3)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python -u bench.py --steps 100 --warmup 20 --secondary-dtype none --secondary-dcn off --force-collectives"
i=0
for m in 3 2 0 1 3 2 0; do
  i=$((i+1))
  PBX_SPLIT_PREFETCH=$m RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29620 + i)) timeout -k 10 300 $B > gpurun_out/rehab_$i.txt 2>&1 || exit 1
  echo "split=$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rehab_$i.txt)"
done
