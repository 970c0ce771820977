#!/bin/bash
# rocprofv3 --kernel-trace --stats of any command; prints the per-kernel summary
#   bash tools/ktrace.sh TAG python3 $PWD/tools/attn_bench.py 5 fp32
set -euo pipefail
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "$@" > "$OUT/run.log" 2>&1
python3 "$R/tools/kstats.py" "$(find "$OUT/trace" -name "*kernel_stats.csv" | head -1)" ${KSTEPS:-1} ${KTOP:-25}
