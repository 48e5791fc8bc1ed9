# does any second measurement in one process run slower? (DCN twice; fp32 after bf16)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --model dcn_v2 --secondary-dcn on > gpurun_out/sec2_dcn_dcn.json 2>gpurun_out/sec2_dcn_dcn.err && grep "ms/step" gpurun_out/sec2_dcn_dcn.err &&
timeout -k 10 200 python -u bench.py --mlp-dtype bf16 --secondary-dtype fp32 --secondary-dcn off > gpurun_out/sec2_bf16_fp32.json 2>gpurun_out/sec2_bf16_fp32.err && grep "ms/step" gpurun_out/sec2_bf16_fp32.err
