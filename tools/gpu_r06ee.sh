#!/bin/bash
# DPP 8-lane max / sum (h3r row scale, attention staging) vs HEAD (abold); tests
set -o pipefail
for rep in 1 2; do
  DLCS_HIP_LIB=dl-swin-gan_amd/dl_cs/libdlcs_hip_abold.so timeout -k 10 120 python tools/h3r_bench.py 2>&1 | grep -v amdgpu.ids | sed 's/^/old /'
  timeout -k 10 120 python tools/h3r_bench.py 2>&1 | grep -v amdgpu.ids | sed 's/^/new /'
  DLCS_HIP_LIB=dl-swin-gan_amd/dl_cs/libdlcs_hip_abold.so timeout -k 10 120 python tools/attn_bench.py 20 fp32 2>&1 | grep -v amdgpu.ids | sed 's/^/old /'
  timeout -k 10 120 python tools/attn_bench.py 20 fp32 2>&1 | grep -v amdgpu.ids | sed 's/^/new /'
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "h3r or attention" 2>&1 | tail -2
