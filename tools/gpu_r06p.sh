#!/bin/bash
# bf16 conv v7: kernel tests, then same-box A/B of the bf16 step (v7 vs v6)
set -o pipefail
mkdir -p gpurun_out/r06p
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "bf16_v6" > gpurun_out/r06p/tests.log 2>&1 || { tail -30 gpurun_out/r06p/tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r06p/tests.log | tail -8
for rep in 1 2; do for v in 0 1; do
  f=gpurun_out/r06p/b_v6${v}_$rep.log
  DLCS_DIAG=1 DLCS_CONV_V6=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches --dtype bf16 > $f 2>&1 || { tail -20 $f; exit 1; }
  python tools/bline.py $f
done; done
