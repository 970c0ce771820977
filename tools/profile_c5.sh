#!/bin/bash
# Config-5 (DiT / Latte DDPM_X training step) kernel traces: rocprofv3 --kernel-trace --stats
# of tools/config_prof.py {dit|latte} (2 warmup + 2 timed steps + the inference evals).
set -euo pipefail
TAG=${1:-r06c5}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for ph in dit latte; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$ph" -o run -- \
        python3 "$R/tools/config_prof.py" $ph 2 > "$OUT/phase_$ph.json" 2> "$OUT/phase_$ph.err"
    python3 "$R/tools/kstats.py" "$(find "$OUT/trace_$ph" -name '*kernel_stats.csv' | head -1)" 1 40 > "$OUT/summary_$ph.txt"
    echo "== $ph"; head -16 "$OUT/summary_$ph.txt"
    python3 -c "import json,sys; d=json.load(open('$OUT/phase_$ph.json')); v=list(d.values())[0]; print({k: v[k] for k in ('value','ms_per_step')})"
done
