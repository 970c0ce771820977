set -o pipefail
mkdir -p gpurun_out/r06g
tools/pmc_r06.sh r06g 2>&1 | grep -v "^W2026\|amdgpu.ids" | tail -8
for dt in fp32 bf16; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches --dtype $dt > gpurun_out/r06g/bench_$dt.log 2>&1 || { tail -20 gpurun_out/r06g/bench_$dt.log; exit 1; }
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r06g/bench_$dt.log | head -2
done
