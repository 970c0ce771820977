#!/bin/bash
# grouped fp32 dW: fma fold + permlane swaps (new) vs HEAD (abold), same box; then the dW tests
set -o pipefail
export DLCS_DIAG=1
for rep in 1 2; do
  DLCS_HIP_LIB=dl-swin-gan_amd/dl_cs/libdlcs_hip_abold.so timeout -k 10 120 python tools/dw_bench.py 30 2>&1 | grep -v amdgpu.ids | sed 's/^/old /'
  timeout -k 10 120 python tools/dw_bench.py 30 2>&1 | grep -v amdgpu.ids | sed 's/^/new /'
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "dw_grouped or gemm_dw" 2>&1 | tail -3
