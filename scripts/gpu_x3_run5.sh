# x3 headline: sparse-chain / edge knob A/Bs, interleaved (bench.py --steps 200 --warmup 20, x3 only)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python -u bench.py --steps 200 --warmup 20 --secondary-dtype none --secondary-dcn off"
run() { name=$1; envs=$2; shift 2; env $envs timeout -k 10 300 $B "$@" > gpurun_out/x3c_$name.txt 2>&1 || exit 1; echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/x3c_$name.txt)"; }
run base0 PBX_NOOP=1
run head_after_adam PBX_HEAD_AFTER_ADAM=1
run push_finish0 PBX_PUSH_FINISH=0
run fused_scatter PBX_FUSED_SCATTER=1
run td_inrow PBX_TD_INROW=1
run base1 PBX_NOOP=1
run head_after_adam2 PBX_HEAD_AFTER_ADAM=1
run push_finish0_2 PBX_PUSH_FINISH=0
run fused_scatter2 PBX_FUSED_SCATTER=1
run base2 PBX_NOOP=1
