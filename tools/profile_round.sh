#!/bin/bash
# Round profile on the GPU box (run via gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats of a short bench.py run  -> per-kernel time
#   2. PMC passes, one counter per run (FETCH_SIZE, WRITE_SIZE do not fit one pass
#      on gfx950): the roofline conv (tools/conv_bench.py fwd) and the SENSE
#      forward (tools/sense_bench.py)                             -> HBM bytes per launch
# Outputs under gpurun_out/$TAG; summaries are copied into profiles/ by hand.
set -euo pipefail
TAG=${1:-r01}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/bench_traced.log" 2>&1
python3 "$R/tools/kstats.py" "$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)" 5 40 > "$OUT/summary.txt"
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_conv_$c" -o run -- \
        python3 "$R/tools/conv_bench.py" fwd 3 > "$OUT/pmc_conv_$c.log" 2>&1
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_sense_$c" -o run -- \
        python3 "$R/tools/sense_bench.py" 3 > "$OUT/pmc_sense_$c.log" 2>&1
done
cc() { find "$OUT/$1" -name '*counter_collection.csv' | head -1; }
python3 "$R/tools/pmc_traffic.py" "$(cc pmc_conv_FETCH_SIZE)" "$(cc pmc_conv_WRITE_SIZE)" conv3d_k3_v5_kernel > "$OUT/traffic_conv3d_k3_v5.json"
python3 "$R/tools/pmc_traffic.py" "$(cc pmc_sense_FETCH_SIZE)" "$(cc pmc_sense_WRITE_SIZE)" "sense_rows_fast_kernel<160, 1," > "$OUT/traffic_sense_rows_fwd.json"
python3 "$R/tools/pmc_traffic.py" "$(cc pmc_sense_FETCH_SIZE)" "$(cc pmc_sense_WRITE_SIZE)" "sense_cols_fast_kernel<192, false>" > "$OUT/traffic_sense_cols_fwd.json"
echo "profile done: $OUT"
cat "$OUT/summary.txt" | head -30
cat "$OUT"/traffic_*.json
