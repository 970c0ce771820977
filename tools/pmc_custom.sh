#!/bin/bash
# One rocprofv3 --pmc pass with the given counters (respect the per-block limits):
#   bash tools/pmc_custom.sh TAG "SQ_A SQ_B GRBM_GUI_ACTIVE" python3 $PWD/tools/attn_bench.py 5 fp32
set -euo pipefail
TAG=$1; shift
CTRS=$1; shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/pmc" -o run -- "$@" > "$OUT/pmc.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$(find "$OUT/pmc" -name '*counter_collection.csv' | head -1)"
