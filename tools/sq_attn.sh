#!/bin/bash
# SQ counter pass (one rocprofv3 --pmc run, counters within the per-block limits) over the
# fp32 window attention (fp16-split kernels) and the x6 patch-embed GEMM; summaries per kernel
set -euo pipefail
TAG=${1:-r03x_sq}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CNT="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d "$OUT/attn" -o run -- python3 "$R/tools/attn_bench.py" 3 fp32 > "$OUT/attn.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d "$OUT/emb" -o run -- python3 "$R/tools/embed_bench.py" > "$OUT/emb.log" 2>&1
ca=$(find "$OUT/attn" -name '*counter_collection.csv' | head -1)
ce=$(find "$OUT/emb" -name '*counter_collection.csv' | head -1)
for k in attn_fwd_h3 attn_bwd_kv_h3 attn_bwd_q_h3; do echo "== $k"; python3 "$R/tools/pmc_summary.py" "$ca" $k; done
echo "== gemm_nt_x6"; python3 "$R/tools/pmc_summary.py" "$ce" gemm_nt_x6
