#!/bin/bash
# rocprofv3 --kernel-trace --stats of a short bench.py run (any bench flags after TAG)
#   bash tools/trace_bench.sh TAG --dtype fp32
set -euo pipefail
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 2 --no-cpu-baseline "$@" > "$OUT/bench_traced.log" 2>&1
python3 "$R/tools/kstats.py" "$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)" 5 45 > "$OUT/summary.txt"
tail -1 "$OUT/bench_traced.log"
cat "$OUT/summary.txt"
