#!/bin/bash
# Round profile on the GPU box (run via gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats of a short bench.py run  -> per-kernel time
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE; they do not fit one pass on gfx950)
#      over tools/conv_bench.py fwd                               -> HBM bytes of the roofline kernel
# Outputs under gpurun_out/$TAG; summaries are copied into profiles/ by hand.
set -euo pipefail
TAG=${1:-r01}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/bench_traced.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 "$R/tools/conv_bench.py" fwd 3 > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 "$R/tools/conv_bench.py" fwd 3 > "$OUT/pmc_write.log" 2>&1
echo "profile done: $OUT"
