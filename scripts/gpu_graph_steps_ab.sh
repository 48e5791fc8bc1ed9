# driver command (--steps 20 --warmup 5, x3 only) with K steps per graph, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python -u bench.py --steps 20 --warmup 5 --secondary-dtype none --secondary-dcn off"
i=0
for k in 4 5 10 20 4 5 10 20; do
  i=$((i+1)); timeout -k 10 300 $B --graph-steps $k > gpurun_out/gs_$i.txt 2>&1 || exit 1
  echo "K=$k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gs_$i.txt)"
done
