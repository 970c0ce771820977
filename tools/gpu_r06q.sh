#!/bin/bash
# bf16 conv v7 DIAG timing experiments (DLCS_V7_EXP bits) vs v6, tools/conv_bench.py
set -o pipefail
mkdir -p gpurun_out/r06q
export DLCS_DIAG=1 DLCS_HIP_LIB=dl-swin-gan_amd/dl_cs/libdlcs_hip_diag.so
DLCS_CONV_V6=1 timeout -k 10 120 python tools/conv_bench.py fwd 20 2>&1 | grep -v amdgpu.ids | sed 's/^/v6 /'
DLCS_CONV_V6=1 timeout -k 10 120 python tools/conv_bench.py dgrad 20 2>&1 | grep -v amdgpu.ids | sed 's/^/v6 /'
for e in 0 16 1 2 3 8 4 12 15; do
  DLCS_V7_EXP=$e timeout -k 10 120 python tools/conv_bench.py fwd 20 2>&1 | grep -v amdgpu.ids | sed "s/^/v7 exp=$e /"
done
DLCS_V7_EXP=16 timeout -k 10 120 python tools/conv_bench.py dgrad 20 2>&1 | grep -v amdgpu.ids | sed "s/^/v7 exp=16 /"
DLCS_V7_EXP=0 timeout -k 10 120 python tools/conv_bench.py dgrad 20 2>&1 | grep -v amdgpu.ids | sed "s/^/v7 exp=0 /"
