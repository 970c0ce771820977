set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "bf16_v6 or relu_out_residual or fwd_dgrad_wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/r06d/tests.log 2>&1 || { tail -30 gpurun_out/r06d/tests.log; exit 1; }
tail -2 gpurun_out/r06d/tests.log
echo "v6:"; timeout -k 10 120 python tools/conv_bench.py fwd 20 && timeout -k 10 120 python tools/conv_bench.py dgrad 20
echo "v5 (DIAG):"; DLCS_DIAG=1 DLCS_CONV_V5=1 DLCS_HIP_LIB=dl-swin-gan_amd/dl_cs/libdlcs_hip_diag.so timeout -k 10 120 python tools/conv_bench.py fwd 20 && DLCS_DIAG=1 DLCS_CONV_V5=1 DLCS_HIP_LIB=dl-swin-gan_amd/dl_cs/libdlcs_hip_diag.so timeout -k 10 120 python tools/conv_bench.py dgrad 20
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
DLCS_DIAG=1 DLCS_HIP_LIB=dl-swin-gan_amd/dl_cs/libdlcs_hip_diag.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06d/prof -o run -- python3 tools/attn_exp.py fp32 base > gpurun_out/r06d/attn.log 2>&1
tail -4 gpurun_out/r06d/attn.log
f=$(find gpurun_out/r06d/prof -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -d, -f1-8
