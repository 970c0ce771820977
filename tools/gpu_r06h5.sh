#!/bin/bash
# h3r epilogue with every global read before the first store: tests, h3r / DiT micro-benches, fp32 step A/B
set -o pipefail
OUT=gpurun_out/r06h5
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_modules.py tests/test_gpu_swin.py tests/test_gpu_dit.py tests/test_gpu_latte.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for lib in abold new abold new; do
  L=dl-swin-gan_amd/dl_cs/libdlcs_hip.so; [ $lib = abold ] && L=dl-swin-gan_amd/dl_cs/libdlcs_hip_abold.so
  echo "== $lib"
  DLCS_HIP_LIB=$L timeout -k 10 120 python tools/h3r_bench.py 2>&1 | grep "h3r" | sed 's/f32 .* h3r/h3r/' || exit 1
done
for rep in 1 2; do for lib in abold new; do
  L=dl-swin-gan_amd/dl_cs/libdlcs_hip.so; [ $lib = abold ] && L=dl-swin-gan_amd/dl_cs/libdlcs_hip_abold.so
  f=$OUT/b_fp32_${lib}_$rep.log
  DLCS_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches > $f 2>&1 || { tail -20 $f; exit 1; }
  echo -n "$lib $rep "; python tools/bline.py $f
done; done
