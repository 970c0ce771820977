#!/bin/bash
# kernel traces of the last tree (the trace half of tools/profile_r06.sh)
set -euo pipefail
TAG=${1:-r06fin_prof}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for dt in fp32 bf16; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$dt" -o run -- \
        python3 "$R/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches --dtype $dt > "$OUT/bench_traced_$dt.log" 2>&1
    python3 "$R/tools/kstats.py" "$(find "$OUT/trace_$dt" -name '*kernel_stats.csv' | head -1)" 5 60 > "$OUT/summary_$dt.txt"
    echo "== $dt"; head -8 "$OUT/summary_$dt.txt"
done
rm -rf "$OUT"/trace_*/*/*kernel_trace.csv 2>/dev/null || true
