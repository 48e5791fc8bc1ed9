# x3 ring-depth A/B (microbench + full bench), then the driver's command and a default run
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for f in 3 4 5; do PBX_X3_PF_F=$f timeout -k 10 120 python -u scripts/bench_tower.py --x3 > gpurun_out/x3pf_f$f.txt 2>&1 || exit 1; echo "PF_F=$f $(grep forward gpurun_out/x3pf_f$f.txt)"; done
for b in 2 3; do PBX_X3_PF_B=$b timeout -k 10 120 python -u scripts/bench_tower.py --x3 > gpurun_out/x3pf_b$b.txt 2>&1 || exit 1; echo "PF_B=$b $(grep chain gpurun_out/x3pf_b$b.txt)"; done
B="python -u bench.py --steps 200 --warmup 20 --secondary-dtype none --secondary-dcn off"
run() { name=$1; envs=$2; shift 2; env $envs timeout -k 10 300 $B "$@" > gpurun_out/x3d_$name.txt 2>&1 || exit 1; echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/x3d_$name.txt)"; }
run base0 PBX_NOOP=1
run pff5 PBX_X3_PF_F=5
run pff3 PBX_X3_PF_F=3
run pfb2 PBX_X3_PF_B=2
run base1 PBX_NOOP=1
bash scripts/gpu_final_bench.sh
