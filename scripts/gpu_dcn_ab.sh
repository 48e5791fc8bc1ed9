# DCN-V2 knob A/Bs after the one-launch push (bench.py --model dcn_v2 --steps 200 --warmup 20)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python -u bench.py --model dcn_v2 --steps 200 --warmup 20 --secondary-dtype none --secondary-dcn off"
run() { name=$1; envs=$2; shift 2; env $envs timeout -k 10 300 $B "$@" > gpurun_out/dcn_$name.txt 2>&1 || exit 1; echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dcn_$name.txt)"; }
run base0 PBX_NOOP=1
run split0 PBX_SPLIT_PREFETCH=0
run split3 PBX_SPLIT_PREFETCH=3
run cross_after PBX_CROSS_DW_AFTER_HEAD=1
run pipe_off PBX_NOOP=1 --pipeline off
run gs2 PBX_NOOP=1 --graph-steps 2
run base1 PBX_NOOP=1
run split0b PBX_SPLIT_PREFETCH=0
