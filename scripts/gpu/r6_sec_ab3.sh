# second in-process measurement: with / without returning the cached blocks to HIP in between
set -o pipefail
mkdir -p gpurun_out
PBX_BENCH_KEEP_CACHE=1 timeout -k 10 200 python -u bench.py --model dcn_v2 --secondary-dcn on > gpurun_out/sec3_keep.json 2>gpurun_out/sec3_keep.err && grep "ms/step" gpurun_out/sec3_keep.err &&
timeout -k 10 200 python -u bench.py --model dcn_v2 --secondary-dcn on > gpurun_out/sec3_empty.json 2>gpurun_out/sec3_empty.err && grep "ms/step" gpurun_out/sec3_empty.err
