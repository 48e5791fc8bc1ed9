# kernel trace of DCN measured twice in one process (first vs second measurement)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/secprof -o run -- python3 -u bench.py --model dcn_v2 --secondary-dcn on --steps 100 --warmup 20 > gpurun_out/secprof.log 2>&1 && grep "ms/step" gpurun_out/secprof.log &&
python3 scripts/micro/split_trace.py gpurun_out/secprof > gpurun_out/secprof_split.txt && cat gpurun_out/secprof_split.txt && rm -f $(find gpurun_out/secprof -name "*kernel_trace.csv")
