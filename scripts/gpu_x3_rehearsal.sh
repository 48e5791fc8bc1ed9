# sharded step rehearsal at the x3 headline: plain 1-rank vs --force-collectives (IPC exchanges + IPC dense all-reduce)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python -u bench.py --steps 100 --warmup 20 --secondary-dtype none --secondary-dcn off"
for rep in 1 2; do
  timeout -k 10 300 $B > gpurun_out/reh_plain$rep.txt 2>&1 || exit 1
  RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29600 + rep)) timeout -k 10 300 $B --force-collectives > gpurun_out/reh_coll$rep.txt 2>&1 || exit 1
  echo "rep $rep plain $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/reh_plain$rep.txt) / rehearsal $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/reh_coll$rep.txt)"
done
