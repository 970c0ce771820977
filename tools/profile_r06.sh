#!/bin/bash
# Round-6 profile on the GPU box (run via gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats of a short fp32 and bf16 bench.py run (headline step only)
#   2. one SQ pass over the f16x3 160 -> 160 conv trio and one over the bf16 trio (tools/conv_bench.py)
#   3. FETCH_SIZE / WRITE_SIZE passes (separate runs) over both trios -> per-launch HBM bytes
# Outputs under gpurun_out/$TAG; summaries are copied into profiles/ by hand.
set -euo pipefail
TAG=${1:-r06}
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
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d "$OUT/sq_h3" -o run -- python3 "$R/tools/conv_bench.py" f16x3 3 fp32 > "$OUT/sq_h3.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$(find "$OUT/sq_h3" -name '*counter_collection.csv' | head -1)" > "$OUT/sq_h3.txt"
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d "$OUT/sq_bf16" -o run -- python3 "$R/tools/conv_bench.py" all 3 > "$OUT/sq_bf16.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$(find "$OUT/sq_bf16" -name '*counter_collection.csv' | head -1)" > "$OUT/sq_bf16.txt"
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_h3_$c" -o run -- \
        python3 "$R/tools/conv_bench.py" f16x3 3 fp32 > "$OUT/pmc_h3_$c.log" 2>&1
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_bf16_$c" -o run -- \
        python3 "$R/tools/conv_bench.py" all 3 > "$OUT/pmc_bf16_$c.log" 2>&1
done
cc() { find "$OUT/$1" -name '*counter_collection.csv' | head -1; }
tr() { python3 "$R/tools/pmc_traffic.py" "$(cc pmc_$1_FETCH_SIZE)" "$(cc pmc_$1_WRITE_SIZE)" "$2" > "$OUT/$3.json" || true; }
tr h3 "conv3d_k3_f16x3_kernel<1," traffic_f16x3_conv_fwd
tr h3 "conv3d_k3_f16x3_kernel<4," traffic_f16x3_conv_dgrad
tr h3 "conv3d_wgrad_f16x3_kernel" traffic_f16x3_conv_wgrad
tr bf16 "conv3d_k3_v6_kernel<1," traffic_bf16_conv_fwd
tr bf16 "conv3d_k3_v6_kernel<4," traffic_bf16_conv_dgrad
tr bf16 "conv3d_wgrad_c160_kernel" traffic_bf16_conv_wgrad
cat "$OUT"/traffic_*.json
echo "profile done: $OUT"
