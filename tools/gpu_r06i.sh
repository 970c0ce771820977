set -o pipefail
mkdir -p gpurun_out/r06i
timeout -k 10 400 python -m cProfile -o gpurun_out/r06i/prof_bf16.out bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches --dtype bf16 > gpurun_out/r06i/bench_bf16.log 2>&1 || { tail -20 gpurun_out/r06i/bench_bf16.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r06i/bench_bf16.log | head -2
python - <<'PY'
import pstats
p = pstats.Stats("gpurun_out/r06i/prof_bf16.out")
p.sort_stats("tottime").print_stats(35)
PY
tools/trace_r06.sh r06i bf16
