#!/bin/bash
# per-kernel times of the SENSE micro-benchmark under rocprofv3 (GPU box);
# extra env settings for an A/B leg are passed as "NAME=VALUE" arguments
set -o pipefail
R=$(pwd); TAG=${TAG:-sp}
cd /tmp && export TMPDIR=/tmp
for leg in "base" "$@"; do
    d=$R/gpurun_out/$TAG/$leg; mkdir -p "$d"
    if [ "$leg" = base ]; then envs=(); else envs=("$leg"); fi
    env "${envs[@]}" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- \
        python3 "$R/tools/sense_bench.py" 20 > "$d.log" 2>&1 || { echo "leg $leg failed"; tail -5 "$d.log"; exit 1; }
    echo "== $leg"; grep -E "forward|adjoint|normal" "$d.log"
    python3 "$R/tools/kstats.py" "$(find "$d" -name '*kernel_stats.csv' | head -1)" 20 5
done
