#!/bin/bash
# h3r timing experiments (results invalid): 1 no per-chunk vmcnt wait, 2 no MFMA,
# 4 no per-chunk barrier, 8 no B DMA in the loop
set -o pipefail
for e in "" 1 2 4 8; do
  L=dl-swin-gan_amd/dl_cs/libdlcs_hip${e:+_exp$e}.so
  echo "== exp '$e'"
  DLCS_HIP_LIB=$L timeout -k 10 120 python tools/h3r_bench.py 2>&1 | grep "h3r" | sed 's/f32 .* h3r/h3r/' || exit 1
done
