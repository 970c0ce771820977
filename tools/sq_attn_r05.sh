#!/bin/bash
# Round-5 SQ pass over the fp32 window attention (fp16-split kernels, tools/attn_bench.py):
# matrix-core, VALU and LDS issue utilisation per kernel (tools/sq_derived.py), one
# rocprofv3 --pmc run within the per-block counter limits (8 SQ + 1 GRBM).
set -euo pipefail
TAG=${1:-r05_sq_attn}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CNT="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d "$OUT/attn" -o run -- python3 "$R/tools/attn_bench.py" 3 fp32 > "$OUT/attn.log" 2>&1
ca=$(find "$OUT/attn" -name '*counter_collection.csv' | head -1)
python3 "$R/tools/sq_derived.py" "$ca" attn_fwd_h3 attn_bwd_kv_h3 attn_bwd_q_h3 | tee "$OUT/sq_attn.txt"
