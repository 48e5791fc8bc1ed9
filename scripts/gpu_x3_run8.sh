# x3 ring depth A/B with the separate head backward, then the final bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python -u bench.py --steps 200 --warmup 20 --secondary-dtype none --secondary-dcn off"
run() { name=$1; envs=$2; shift 2; env $envs timeout -k 10 300 $B "$@" > gpurun_out/x3f_$name.txt 2>&1 || exit 1; echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/x3f_$name.txt)"; }
run base0 PBX_NOOP=1
run pff3 PBX_X3_PF_F=3
run pff5 PBX_X3_PF_F=5
run pfb2 PBX_X3_PF_B=2
run base1 PBX_NOOP=1
run pff3b PBX_X3_PF_F=3
bash scripts/gpu_final_bench.sh
