# PMC pass (MFMA busy / wave states) on the x3 and exact-fp32 tower microbenchmarks
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 200 rocprofv3 --pmc $C -d gpurun_out/pmc_x3 -o pmc -- python -u scripts/bench_tower.py --x3 --iters 5 > gpurun_out/pmc_x3.txt 2>&1
rc=$?; echo "x3 pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 200 rocprofv3 --pmc $C -d gpurun_out/pmc_t32 -o pmc -- python -u scripts/bench_tower.py --fp32 --iters 5 > gpurun_out/pmc_t32.txt 2>&1
rc=$?; echo "fp32 pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
for d in pmc_x3 pmc_t32; do f=$(find gpurun_out/$d -name "*counter_collection.csv" | head -1); echo "== $d $f"; python scripts/prof/pmc_mfma.py "$f" --simds 1024 | head -14; done
