# kernel trace of the x3 1-rank sharded rehearsal step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_reh -o bench -- python -u bench.py --steps 40 --warmup 10 --secondary-dtype none --secondary-dcn off --force-collectives > gpurun_out/reh_prof.txt 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
db=$(find gpurun_out/prof_reh -name "*results.db" | head -1)
python scripts/prof/step_timeline.py "$db" --marker k_tx3_fwd --steps 30 --timeline --which 2 > gpurun_out/reh_step_timeline.txt 2>&1; cat gpurun_out/reh_step_timeline.txt
