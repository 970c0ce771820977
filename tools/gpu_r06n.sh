#!/bin/bash
# round 6: fp16-split MHSA backward -- parity tests, then config-5 A/B timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dit.py -k "mhsa" > gpurun_out/r06n_test.log 2>&1 || { tail -30 gpurun_out/r06n_test.log; exit 1; }
tail -5 gpurun_out/r06n_test.log
timeout -k 10 120 python -u tools/mhsa_bench.py > gpurun_out/r06n_h3.log 2>&1 && cat gpurun_out/r06n_h3.log &&
DLCS_DIAG=1 DLCS_MHSA_H3_BWD=0 DLCS_HIP_LIB=dl-swin-gan_amd/dl_cs/libdlcs_hip_diag.so timeout -k 10 120 python -u tools/mhsa_bench.py > gpurun_out/r06n_f32.log 2>&1 && cat gpurun_out/r06n_f32.log
