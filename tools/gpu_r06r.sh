#!/bin/bash
# SQ counters of the bf16 160-channel forward: v6 vs v7 (tools/conv_bench.py)
set -o pipefail
export DLCS_DIAG=1
DLCS_CONV_V6=1 bash tools/pmc_sq.sh r06r_v6 python3 $(pwd)/tools/conv_bench.py fwd 3 > gpurun_out/r06r_v6.txt 2>&1 || { cat gpurun_out/r06r_v6.txt | tail; exit 1; }
DLCS_CONV_V6=0 bash tools/pmc_sq.sh r06r_v7 python3 $(pwd)/tools/conv_bench.py fwd 3 > gpurun_out/r06r_v7.txt 2>&1 || { cat gpurun_out/r06r_v7.txt | tail; exit 1; }
grep -A12 "conv3d_k3_v6_kernel<32\|conv3d_k3_v6_kernel<2,\|v6_kernel<" gpurun_out/r06r_v6.txt | head -30
grep -A12 "v7_kernel<" gpurun_out/r06r_v7.txt | head -30
