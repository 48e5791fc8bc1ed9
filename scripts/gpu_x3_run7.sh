# fused head backward: x3 tests, then ring-depth + fused-head A/B on the full bench, then the final bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_tower_x3.py tests/test_gpu_pipeline.py > gpurun_out/x3_tests7.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/x3_tests7.log; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --steps 200 --warmup 20 --secondary-dtype none --secondary-dcn off"
run() { name=$1; envs=$2; shift 2; env $envs timeout -k 10 300 $B "$@" > gpurun_out/x3e_$name.txt 2>&1 || exit 1; echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/x3e_$name.txt)"; }
run base0 PBX_NOOP=1
run head_unfused PBX_X3_FUSED_HEAD=0
run pff5 PBX_X3_PF_F=5
run pff3 PBX_X3_PF_F=3
run pfb2 PBX_X3_PF_B=2
run base1 PBX_NOOP=1
run head_unfused2 PBX_X3_FUSED_HEAD=0
bash scripts/gpu_final_bench.sh
