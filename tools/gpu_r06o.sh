#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dit.py tests/test_gpu_latte.py > gpurun_out/r06o_test.log 2>&1 || { tail -30 gpurun_out/r06o_test.log; exit 1; }
tail -3 gpurun_out/r06o_test.log
./tools/profile_c5.sh r06c5b
