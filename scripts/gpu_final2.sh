# final: GPU suite + smoke, the driver's bench command twice and a default run
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_suite2.sh || exit 1
bash scripts/gpu_final_bench.sh
