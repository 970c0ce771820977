# x6 embed GEMM (unconditional loads) + h3 attention: tests, benches, kernel trace
mkdir -p gpurun_out/r03x
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "nt_x6 or window_attention_f32 or h3_floor" -s > gpurun_out/r03x/t1.log 2>&1; tail -3 gpurun_out/r03x/t1.log; grep "tail=True" gpurun_out/r03x/t1.log | head -12
timeout -k 10 120 python tools/embed_bench.py > gpurun_out/r03x/eb.log 2>&1 && grep -v amdgpu.ids gpurun_out/r03x/eb.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03x/prof_attn -o run -- python3 $GRAFT_REPO_ROOT/tools/attn_bench.py 20 fp32 > $GRAFT_REPO_ROOT/gpurun_out/r03x/ab.log 2>&1; cd $GRAFT_REPO_ROOT; grep -v amdgpu.ids gpurun_out/r03x/ab.log | tail -3
find gpurun_out/r03x/prof_attn -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-8 {} | head -8'
