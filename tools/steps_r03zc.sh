# model-level GPU tests and a bench line on the final attention kernels
mkdir -p gpurun_out/r03zc
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_swin.py tests/test_gpu_fullsize.py tests/test_gpu_modules.py > gpurun_out/r03zc/t.log 2>&1; tail -2 gpurun_out/r03zc/t.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r03zc/bench.json 2> gpurun_out/r03zc/bench.err; grep "^{" gpurun_out/r03zc/bench.json | cut -c1-250
