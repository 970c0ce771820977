#!/bin/bash
# c160 bf16 wgrad without the spilling bias path: kernel tests, then the bf16 step
set -o pipefail
mkdir -p gpurun_out/r06y
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad" > gpurun_out/r06y/tests.log 2>&1 || { tail -30 gpurun_out/r06y/tests.log; exit 1; }
tail -2 gpurun_out/r06y/tests.log
for rep in 1 2; do
  f=gpurun_out/r06y/b_bf16_$rep.log
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches --dtype bf16 > $f 2>&1 || { tail -20 $f; exit 1; }
  python tools/bline.py $f
done
