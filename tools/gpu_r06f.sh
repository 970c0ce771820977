set -o pipefail
mkdir -p gpurun_out/r06f
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "thin_planes or thin_f16x3" -x -q --timeout 120 --timeout-method thread > gpurun_out/r06f/tests.log 2>&1 || { tail -30 gpurun_out/r06f/tests.log; exit 1; }
tail -2 gpurun_out/r06f/tests.log
echo "p3:"; timeout -k 10 120 python tools/thin_bench.py 20 2>&1 | grep -E "thin_out_p|wgrad_.*_p|thin_in"
echo "p2 (DIAG):"; DLCS_DIAG=1 DLCS_THIN_OUT_P2=1 DLCS_HIP_LIB=dl-swin-gan_amd/dl_cs/libdlcs_hip_diag.so timeout -k 10 120 python tools/thin_bench.py 20 2>&1 | grep -E "thin_out_p"
tools/trace_r06.sh r06f
