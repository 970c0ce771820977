#!/bin/bash
# same-box A/B, bf16 160-channel conv: v7 vs v6, microbench x3 alternating, then the bf16 step x2
set -o pipefail
export DLCS_DIAG=1
for rep in 1 2 3; do for v in 1 0; do
  DLCS_CONV_V6=$v timeout -k 10 120 python tools/conv_bench.py fwd 30 2>&1 | grep -v amdgpu.ids | sed "s/^/v6=$v /"
  DLCS_CONV_V6=$v timeout -k 10 120 python tools/conv_bench.py dgrad 30 2>&1 | grep -v amdgpu.ids | sed "s/^/v6=$v /"
done; done
mkdir -p gpurun_out/r06u
for rep in 1 2; do for v in 1 0; do
  f=gpurun_out/r06u/b_v6${v}_$rep.log
  DLCS_CONV_V6=$v timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches --dtype bf16 > $f 2>&1 || { tail -20 $f; exit 1; }
  python tools/bline.py $f
done; done
