# thin convs with unconditional halo loads; unembed input gradient on the x6 NT GEMM
mkdir -p gpurun_out/r03aa
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "thin" tests/test_gpu_swin.py tests/test_gpu_fullsize.py -k "thin or swinnet or pgd or window or block or mlp or direct or hqs or bf16" > gpurun_out/r03aa/t.log 2>&1; tail -3 gpurun_out/r03aa/t.log
timeout -k 10 200 python tools/thin_bench.py 20 > gpurun_out/r03aa/thin.log 2>&1; grep -v amdgpu.ids gpurun_out/r03aa/thin.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-configs > gpurun_out/r03aa/bench.json 2> gpurun_out/r03aa/bench.err; grep "^{" gpurun_out/r03aa/bench.json | cut -c1-260
