#!/bin/bash
# Round-5 profile on the GPU box (run via gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats of a short fp32 bench.py run (headline step only)
#      [and of the bf16 step with WITH_BF16=1]
#   2. one SQ PMC pass over the f16x3 160 -> 160 conv trio (tools/conv_bench.py)
#   3. FETCH_SIZE / WRITE_SIZE passes (separate runs) over the conv trio
# Outputs under gpurun_out/$TAG; summaries are copied into profiles/ by hand.
set -euo pipefail
TAG=${1:-r05}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
DTS="fp32"
[ "${WITH_BF16:-0}" = "1" ] && DTS="fp32 bf16"
for dt in $DTS; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$dt" -o run -- \
        python3 "$R/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches --dtype $dt > "$OUT/bench_traced_$dt.log" 2>&1
    python3 "$R/tools/kstats.py" "$(find "$OUT/trace_$dt" -name '*kernel_stats.csv' | head -1)" 5 60 > "$OUT/summary_$dt.txt"
    echo "== $dt"; head -14 "$OUT/summary_$dt.txt"
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT/sq_h3" -o run -- python3 "$R/tools/conv_bench.py" f16x3 3 fp32 > "$OUT/sq_h3.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$(find "$OUT/sq_h3" -name '*counter_collection.csv' | head -1)" f16x3 > "$OUT/sq_h3.txt"
grep -A10 "conv3d_k3_f16x3_kernel<1, 0, false>\|conv3d_k3_f16x3_kernel<4, 3, false>\|conv3d_wgrad_f16x3_kernel" "$OUT/sq_h3.txt" | head -40
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_h3_$c" -o run -- \
        python3 "$R/tools/conv_bench.py" f16x3 3 fp32 > "$OUT/pmc_h3_$c.log" 2>&1
done
cc() { find "$OUT/$1" -name '*counter_collection.csv' | head -1; }
tr() { python3 "$R/tools/pmc_traffic.py" "$(cc pmc_$1_FETCH_SIZE)" "$(cc pmc_$1_WRITE_SIZE)" "$2" > "$OUT/$3.json" || true; }
tr h3 "conv3d_k3_f16x3_kernel<1," traffic_f16x3_conv_fwd
tr h3 "conv3d_k3_f16x3_kernel<4," traffic_f16x3_conv_dgrad
tr h3 "conv3d_wgrad_f16x3_kernel" traffic_f16x3_conv_wgrad
cat "$OUT"/traffic_*.json
echo "profile done: $OUT"
