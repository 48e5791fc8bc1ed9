# does the step time drift as one measurement keeps training? (diag windows after the timed K steps)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --model dcn_v2 --diag-windows 8 > gpurun_out/drift_dcn.json 2>gpurun_out/drift_dcn.err && grep "ms/step" gpurun_out/drift_dcn.err &&
timeout -k 10 300 python -u bench.py --secondary-dtype none --secondary-dcn off --diag-windows 8 > gpurun_out/drift_fp32.json 2>gpurun_out/drift_fp32.err && grep "ms/step" gpurun_out/drift_fp32.err
