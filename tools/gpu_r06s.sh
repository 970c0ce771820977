#!/bin/bash
set -o pipefail
export DLCS_DIAG=1 DLCS_HIP_LIB=dl-swin-gan_amd/dl_cs/libdlcs_hip_diag.so
for e in 0 64 4 32 96 36 72 8; do
  DLCS_V7_EXP=$e timeout -k 10 120 python tools/conv_bench.py fwd 20 2>&1 | grep -v amdgpu.ids | sed "s/^/v7 exp=$e /"
done
