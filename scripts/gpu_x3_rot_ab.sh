# x3 k-step rotation multiplier A/B (PBX_X3_ROT): microbench + full bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 5 7 1 13; do PBX_X3_ROT=$r timeout -k 10 120 python -u scripts/bench_tower.py --x3 > gpurun_out/rot_micro_$r.txt 2>&1 || exit 1; echo "rot=$r $(grep -E 'forward|chain' gpurun_out/rot_micro_$r.txt | tr '\n' ' ')"; done
B="python -u bench.py --steps 200 --warmup 20 --secondary-dtype none --secondary-dcn off"
i=0
for r in 5 7 13 5 7 13; do i=$((i+1)); PBX_X3_ROT=$r timeout -k 10 300 $B > gpurun_out/rot_bench_$i.txt 2>&1 || exit 1; echo "bench rot=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rot_bench_$i.txt)"; done
