#!/bin/bash
# Round-2 profile on the GPU box (run via gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats of short fp32 and bf16 bench.py runs -> per-kernel time per step
#   2. one SQ PMC pass over the fp32-on-bf16-MFMA (x6) conv kernels  -> MFMA busy, LDS conflicts, waits
#   3. FETCH_SIZE / WRITE_SIZE passes (separate runs) over the x6 conv kernels -> HBM bytes per launch
# Outputs under gpurun_out/$TAG; summaries are copied into profiles/ by hand.
set -euo pipefail
TAG=${1:-r02}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for dt in fp32 bf16; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$dt" -o run -- \
        python3 "$R/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --no-secondary --no-configs --no-all-branches --dtype $dt > "$OUT/bench_traced_$dt.log" 2>&1
    python3 "$R/tools/kstats.py" "$(find "$OUT/trace_$dt" -name '*kernel_stats.csv' | head -1)" 5 45 > "$OUT/summary_$dt.txt"
    echo "== $dt"; head -30 "$OUT/summary_$dt.txt"
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT/sq_h3" -o run -- python3 "$R/tools/conv_bench.py" f16x3 3 fp32 > "$OUT/sq_h3.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$(find "$OUT/sq_h3" -name '*counter_collection.csv' | head -1)" f16x3 | tee "$OUT/sq_h3.txt"
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_h3_$c" -o run -- \
        python3 "$R/tools/conv_bench.py" f16x3 3 fp32 > "$OUT/pmc_h3_$c.log" 2>&1
done
cc() { find "$OUT/$1" -name '*counter_collection.csv' | head -1; }
python3 "$R/tools/pmc_traffic.py" "$(cc pmc_h3_FETCH_SIZE)" "$(cc pmc_h3_WRITE_SIZE)" "conv3d_k3_f16x3_kernel<1," > "$OUT/traffic_f16x3_conv_fwd.json" || true
python3 "$R/tools/pmc_traffic.py" "$(cc pmc_h3_FETCH_SIZE)" "$(cc pmc_h3_WRITE_SIZE)" "conv3d_wgrad_f16x3_kernel" > "$OUT/traffic_f16x3_conv_wgrad.json" || true
cat "$OUT"/traffic_f16x3_*.json
echo "profile done: $OUT"
