set -o pipefail
mkdir -p gpurun_out/r06k
for rep in 1 2; do for o in foreach fused flat; do for dt in fp32 bf16; do
  BENCH_OPT=$o timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches --dtype $dt > gpurun_out/r06k/bench_${o}_${dt}_$rep.log 2>&1 || { tail -20 gpurun_out/r06k/bench_${o}_${dt}_$rep.log; exit 1; }
  echo "$o $dt $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06k/bench_${o}_${dt}_$rep.log | head -1)"
done; done; done
