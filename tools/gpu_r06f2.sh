#!/bin/bash
# final: bf16 trace + bf16 conv-trio PMC traffic, then the full default bench line
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r06fin
mkdir -p $OUT
( cd /tmp && export TMPDIR=/tmp && \
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_bf16" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches --dtype bf16 > "$OUT/bench_traced_bf16.log" 2>&1 && \
  python3 "$R/tools/kstats.py" "$(find "$OUT/trace_bf16" -name '*kernel_stats.csv' | head -1)" 5 60 > "$OUT/summary_bf16.txt" && \
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_bf16_FETCH_SIZE" -o run -- python3 "$R/tools/conv_bench.py" all 3 > "$OUT/pmc_f.log" 2>&1 && \
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_bf16_WRITE_SIZE" -o run -- python3 "$R/tools/conv_bench.py" all 3 > "$OUT/pmc_w.log" 2>&1 ) || { echo PROFILE_FAILED; tail -5 $OUT/*.log; exit 1; }
head -6 $OUT/summary_bf16.txt
cc() { find "$OUT/$1" -name '*counter_collection.csv' | head -1; }
for k in "conv3d_k3_v6_kernel<1,:fwd" "conv3d_k3_v6_kernel<4,:dgrad" "conv3d_wgrad_c160_kernel:wgrad"; do
  python3 tools/pmc_traffic.py "$(cc pmc_bf16_FETCH_SIZE)" "$(cc pmc_bf16_WRITE_SIZE)" "${k%%:*}" > $OUT/traffic_bf16_conv_${k##*:}.json
done
cat $OUT/traffic_*.json
timeout -k 10 1100 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
grep "^{" $OUT/bench.json | tail -1 | cut -c1-600
