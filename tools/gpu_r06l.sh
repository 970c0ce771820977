set -o pipefail
mkdir -p gpurun_out/r06l
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "wgrad or relu_out or bf16_v6 or thin" tests/test_gpu_swin.py -k "bf16 or wgrad or relu_out or v6 or thin" -x -q --timeout 180 --timeout-method thread > gpurun_out/r06l/tests.log 2>&1 || { tail -30 gpurun_out/r06l/tests.log; exit 1; }
tail -2 gpurun_out/r06l/tests.log
for dt in bf16 fp32; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches --dtype $dt > gpurun_out/r06l/bench_$dt.log 2>&1 || { tail -20 gpurun_out/r06l/bench_$dt.log; exit 1; }
  echo "$dt $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06l/bench_$dt.log | head -1)"
done
