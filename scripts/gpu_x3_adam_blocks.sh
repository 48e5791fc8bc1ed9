# x3 headline: fused-Adam grid cap A/B (PBX_ADAM_MAX_BLOCKS; default 512), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python -u bench.py --steps 200 --warmup 20 --secondary-dtype none --secondary-dcn off"
i=0
for v in 512 256 128 64 512 256 128 64; do
  i=$((i+1)); PBX_ADAM_MAX_BLOCKS=$v timeout -k 10 300 $B > gpurun_out/ab_$i.txt 2>&1 || exit 1
  echo "adam_max_blocks=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$i.txt)"
done
