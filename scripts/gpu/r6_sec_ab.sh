# secondary-measurement A/B: DCN-V2 standalone vs as the same-run secondary
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --model dcn_v2 > gpurun_out/sec_dcn_alone.json 2>gpurun_out/sec_dcn_alone.err && cat gpurun_out/sec_dcn_alone.json &&
timeout -k 10 200 python -u bench.py --secondary-dtype none > gpurun_out/sec_fp32_dcn.json 2>gpurun_out/sec_fp32_dcn.err && cat gpurun_out/sec_fp32_dcn.json &&
timeout -k 10 200 python -u bench.py --mlp-dtype bf16 --secondary-dtype none --secondary-dcn off > gpurun_out/sec_bf16_alone.json 2>gpurun_out/sec_bf16_alone.err && cat gpurun_out/sec_bf16_alone.json &&
timeout -k 10 200 python -u bench.py --model dcn_v2 > gpurun_out/sec_dcn_alone2.json 2>gpurun_out/sec_dcn_alone2.err && cat gpurun_out/sec_dcn_alone2.json
