set -o pipefail
mkdir -p gpurun_out/r06j
for dt in fp32 bf16; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches --dtype $dt > gpurun_out/r06j/bench_$dt.log 2>&1 || { tail -20 gpurun_out/r06j/bench_$dt.log; exit 1; }
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r06j/bench_$dt.log | head -2
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_bench_launch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06j/tests.log 2>&1; tail -3 gpurun_out/r06j/tests.log
