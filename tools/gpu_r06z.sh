#!/bin/bash
# bf16 thin-input conv without the scratch round trip: tests, microbench, bf16 step
set -o pipefail
mkdir -p gpurun_out/r06z
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_modules.py -k "thin" > gpurun_out/r06z/tests.log 2>&1 || { tail -30 gpurun_out/r06z/tests.log; exit 1; }
tail -2 gpurun_out/r06z/tests.log
timeout -k 10 120 python tools/conv_bench.py thin 30 2>&1 | grep -v amdgpu.ids
f=gpurun_out/r06z/b_bf16.log
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches --dtype bf16 > $f 2>&1 || { tail -20 $f; exit 1; }
python tools/bline.py $f
