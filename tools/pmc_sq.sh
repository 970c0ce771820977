#!/bin/bash
# SQ stall / utilisation counters for one micro-benchmark (run via gpurun from the repo root):
#   bash tools/pmc_sq.sh TAG python3 tools/conv_bench.py fwd 3
set -euo pipefail
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT/sq" -o run -- "$@" > "$OUT/sq.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$(find "$OUT/sq" -name '*counter_collection.csv' | head -1)"
