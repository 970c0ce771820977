#!/bin/bash
# fused Adam with the version bump vs foreach Adam (same box), after the weight-cache fix
set -o pipefail
mkdir -p gpurun_out/r06aa
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_swin.py -k "weight_cache" > gpurun_out/r06aa/tests.log 2>&1 || { tail -30 gpurun_out/r06aa/tests.log; exit 1; }
tail -1 gpurun_out/r06aa/tests.log
for rep in 1 2; do for fe in 0 1; do for dt in fp32 bf16; do
  f=gpurun_out/r06aa/b_fe${fe}_${dt}_$rep.log
  DLCS_DIAG=1 DLCS_ADAM_FOREACH=$fe timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches --dtype $dt > $f 2>&1 || { tail -20 $f; exit 1; }
  echo "foreach=$fe $(python tools/bline.py $f)"
done; done; done
