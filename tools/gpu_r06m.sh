set -o pipefail
mkdir -p gpurun_out/r06m
for rep in 1 2; do for v in new oldstream oldbias; do for dt in bf16 fp32; do
  env=""; [ $v = oldstream ] && env="AB_OLD_STREAM=1"; [ $v = oldbias ] && env="AB_OLD_BIAS=1"
  env $env timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches --dtype $dt > gpurun_out/r06m/b_${v}_${dt}_$rep.log 2>&1 || { tail -20 gpurun_out/r06m/b_${v}_${dt}_$rep.log; exit 1; }
  echo "$v $dt $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r06m/b_${v}_${dt}_$rep.log | head -1)"
done; done; done
