# h3 attention staging rework: parity tests, then kernel times (full and staging-only)
mkdir -p gpurun_out/r03y
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "window_attention_f32 or h3_floor" -s > gpurun_out/r03y/t1.log 2>&1; tail -3 gpurun_out/r03y/t1.log; grep "tail=True" gpurun_out/r03y/t1.log | head -12
for n in 0 99; do DLCS_ATTN_H3_NLOOP=$n bash tools/ktrace.sh r03y_s$n python3 $PWD/tools/attn_bench.py 10 fp32 2>&1 | grep h3_kernel; done
