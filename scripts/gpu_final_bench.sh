# the driver's command (default run) twice + a 200-step default run
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/final_driver1.txt 2>&1 || exit 1
tail -1 gpurun_out/final_driver1.txt | cut -c1-300
timeout -k 10 300 python -u bench.py > gpurun_out/final_default.txt 2>&1 || exit 1
grep "\[bench\]" gpurun_out/final_default.txt | tail -6; tail -1 gpurun_out/final_default.txt | cut -c1-300
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/final_driver2.txt 2>&1 || exit 1
tail -1 gpurun_out/final_driver2.txt | cut -c1-300
