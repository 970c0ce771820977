#!/bin/bash
# scheduling fences in the bf16 160-channel conv: v6 / v7 with and without (bit 128), same box
set -o pipefail
export DLCS_DIAG=1 DLCS_HIP_LIB=dl-swin-gan_amd/dl_cs/libdlcs_hip_diag.so
for rep in 1 2; do
for e in 0 128; do
  DLCS_V6_EXP=$e timeout -k 10 120 python tools/conv_bench.py fwd 30 2>&1 | grep -v amdgpu.ids | sed "s/^/v6 exp=$e /"
  DLCS_V6_EXP=$e timeout -k 10 120 python tools/conv_bench.py dgrad 30 2>&1 | grep -v amdgpu.ids | sed "s/^/v6 exp=$e /"
  DLCS_CONV_V7=1 DLCS_V7_EXP=$e timeout -k 10 120 python tools/conv_bench.py fwd 30 2>&1 | grep -v amdgpu.ids | sed "s/^/v7 exp=$e /"
done; done
