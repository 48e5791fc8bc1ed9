# x3 headline at dW splits=2: kernel trace + step timeline, then knob A/Bs on the full bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_x3b -o bench -- python -u bench.py --steps 40 --warmup 10 --secondary-dtype none --secondary-dcn off > gpurun_out/x3b_prof_bench.txt 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
db=$(find gpurun_out/prof_x3b -name "*results.db" | head -1)
python scripts/prof/step_timeline.py "$db" --marker k_tx3_fwd --steps 30 > gpurun_out/x3b_step_timeline.txt 2>&1; cat gpurun_out/x3b_step_timeline.txt | head -60
B="python -u bench.py --steps 200 --warmup 20 --secondary-dtype none --secondary-dcn off"
run() { name=$1; envs=$2; shift 2; env $envs timeout -k 10 300 $B "$@" > gpurun_out/x3ab_$name.txt 2>&1 || exit 1; echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/x3ab_$name.txt)"; }
run base0 PBX_NOOP=1
run pipe_off PBX_NOOP=1 --pipeline off
run dw_before_head PBX_DW_AFTER_HEAD=0
run adam_ovl_off PBX_ADAM_OVERLAP=0
run gs2 PBX_NOOP=1 --graph-steps 2
run split_pref2 PBX_SPLIT_PREFETCH=2
run base1 PBX_NOOP=1
