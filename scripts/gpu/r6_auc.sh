# AUC histogram merge: exactness tests, then the step-time drift over 8 extra windows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tower.py tests/test_gpu_tower32.py tests/test_gpu_dcn.py -m gpu > gpurun_out/auc_tests.log 2>&1 && tail -2 gpurun_out/auc_tests.log &&
timeout -k 10 300 python -u bench.py --secondary-dtype none --secondary-dcn off --diag-windows 8 > gpurun_out/auc_fp32.json 2>gpurun_out/auc_fp32.err && grep "ms/step" gpurun_out/auc_fp32.err &&
timeout -k 10 300 python -u bench.py --model dcn_v2 --diag-windows 8 > gpurun_out/auc_dcn.json 2>gpurun_out/auc_dcn.err && grep "ms/step" gpurun_out/auc_dcn.err &&
timeout -k 10 300 python -u bench.py > gpurun_out/auc_default.json 2>gpurun_out/auc_default.err && grep "ms/step" gpurun_out/auc_default.err
