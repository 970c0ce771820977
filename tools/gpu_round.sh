set -o pipefail
mkdir -p gpurun_out/r01c
timeout -k 10 300 python -u -m pytest tests/test_gpu_sense.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r01c/sense_tests.log 2>&1 || { echo SENSE_TESTS_FAILED; tail -30 gpurun_out/r01c/sense_tests.log; exit 1; }
tail -2 gpurun_out/r01c/sense_tests.log
timeout -k 10 120 python tools/sense_bench.py > gpurun_out/r01c/sense_fast.log 2>&1 && cat gpurun_out/r01c/sense_fast.log
DLCS_SENSE_GENERIC=1 timeout -k 10 120 python tools/sense_bench.py > gpurun_out/r01c/sense_generic.log 2>&1 && cat gpurun_out/r01c/sense_generic.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r01c/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAILED; tail -30 gpurun_out/r01c/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r01c/gpu_tests.log
timeout -k 10 600 python bench.py > gpurun_out/r01c/bench.log 2>&1 && tail -1 gpurun_out/r01c/bench.log
