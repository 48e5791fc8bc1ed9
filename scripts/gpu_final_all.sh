# final validation: GPU suite + smoke, the driver's bench command, a kernel trace of the headline step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_suite2.sh || exit 1
bash scripts/gpu_final_bench.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o bench -- python -u bench.py --steps 40 --warmup 10 --secondary-dtype none --secondary-dcn off > gpurun_out/final_prof_bench.txt 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
db=$(find gpurun_out/prof_final -name "*results.db" | head -1)
python scripts/prof/step_timeline.py "$db" --marker k_tx3_fwd --steps 30 --timeline --which 2 > gpurun_out/final_step_timeline.txt 2>&1; head -20 gpurun_out/final_step_timeline.txt
