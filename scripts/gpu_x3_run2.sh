# round 6: the x3 headline -- driver-style bench, kernel trace + timeline, 2-rank same-GPU rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/x3_driver_style.txt 2>&1
rc=$?; tail -3 gpurun_out/x3_driver_style.txt | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_x3 -o bench -- python -u bench.py --steps 40 --warmup 10 --secondary-dtype none --secondary-dcn off > gpurun_out/x3_prof_bench.txt 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
db=$(find gpurun_out/prof_x3 -name "*results.db" | head -1); echo "db=$db"
python scripts/prof/step_timeline.py "$db" --marker k_tx3_fwd --steps 30 > gpurun_out/x3_step_timeline.txt 2>&1; tail -45 gpurun_out/x3_step_timeline.txt
timeout -k 10 400 python -u bench.py --gpus 2 --same-gpu --steps 20 --warmup 5 --total-features 200000000 > gpurun_out/x3_rehearsal2.txt 2>&1
rc=$?; tail -4 gpurun_out/x3_rehearsal2.txt | cut -c1-400; exit $rc
