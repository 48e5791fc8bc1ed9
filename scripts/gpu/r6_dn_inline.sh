set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tower.py tests/test_gpu_tower32.py tests/test_gpu_dcn.py tests/test_gpu_pipeline.py -m gpu > gpurun_out/dnin_tests.log 2>&1 && tail -3 gpurun_out/dnin_tests.log &&
timeout -k 10 200 python -u bench.py > gpurun_out/dnin_bench1.json 2>gpurun_out/dnin_bench1.err && cat gpurun_out/dnin_bench1.json &&
PBX_DN_INLINE_UPDATE=0 timeout -k 10 200 python -u bench.py > gpurun_out/dnin_bench0.json 2>gpurun_out/dnin_bench0.err && cat gpurun_out/dnin_bench0.json &&
timeout -k 10 200 python -u bench.py > gpurun_out/dnin_bench1b.json 2>gpurun_out/dnin_bench1b.err && cat gpurun_out/dnin_bench1b.json
