#!/bin/bash
# Round-6 step traces (run via gpurun from the repo root): rocprofv3 --kernel-trace
# --stats of a short headline-only bench.py run per dtype; the per-dispatch CSV is
# kept for per-launch-shape analysis (tools/kshapes.py).   tools/trace_r06.sh TAG [dtypes]
set -euo pipefail
TAG=${1:-r06}
DTS=${2:-"fp32 bf16"}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for dt in $DTS; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$dt" -o run -- \
        python3 "$R/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches --dtype $dt > "$OUT/bench_traced_$dt.log" 2>&1
    python3 "$R/tools/kstats.py" "$(find "$OUT/trace_$dt" -name '*kernel_stats.csv' | head -1)" 5 60 > "$OUT/summary_$dt.txt"
    echo "== $dt"; head -14 "$OUT/summary_$dt.txt"; tail -1 "$OUT/bench_traced_$dt.log" | cut -c1-300
done
