#!/bin/bash
# K = 160 GEMM epilogue with 8-channel items (new) vs HEAD (abold), same box; tests
set -o pipefail
for rep in 1 2; do
  DLCS_HIP_LIB=dl-swin-gan_amd/dl_cs/libdlcs_hip_abold.so timeout -k 10 180 python tools/conv_bench.py f16x3 20 fp32 2>&1 | grep -E "k160" | sed 's/^/old /'
  timeout -k 10 180 python tools/conv_bench.py f16x3 20 fp32 2>&1 | grep -E "k160" | sed 's/^/new /'
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "k160 or producer_planes or embed or unembed" 2>&1 | tail -2
