#!/bin/bash
# HBM bytes per launch of the SENSE kernels (tools/sense_bench.py, BASELINE slice):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc runs, summarised per kernel
# with tools/pmc_traffic.py.  Outputs under gpurun_out/$TAG.
set -euo pipefail
TAG=${1:-sense}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_sense_$c" -o run -- \
        python3 "$R/tools/sense_bench.py" 3 > "$OUT/pmc_sense_$c.log" 2>&1
done
cc() { find "$OUT/$1" -name '*counter_collection.csv' | head -1; }
for k in "sense_rows_fast_kernel<160, 1, false" "sense_cols_fast_kernel<192, false, true>" "sense_rows_fast_kernel<160, 2, true, 4, 2, 2>" "sense_rows_fast_kernel<160, 2, true, 4, 2, 1>"; do
    python3 "$R/tools/pmc_traffic.py" "$(cc pmc_sense_FETCH_SIZE)" "$(cc pmc_sense_WRITE_SIZE)" "$k" || true
done > "$OUT/traffic_sense.jsonl"
cat "$OUT/traffic_sense.jsonl"
