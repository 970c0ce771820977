#!/bin/bash
# PMC HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the non-conv HBM kernels:
# thin ends (tools/thin_bench.py) and the K = 160 patch GEMMs (tools/k160_bench.py).
set -uo pipefail
TAG=${1:-r06g}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for b in thin_bench k160_bench; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${b}_$c" -o run -- python3 "$R/tools/$b.py" 3 > "$OUT/pmc_${b}_$c.log" 2>&1 || { echo "pmc $b $c failed"; tail -5 "$OUT/pmc_${b}_$c.log"; exit 1; }
  done
done
cc() { find "$OUT/$1" -name '*counter_collection.csv' | head -1; }
for k in conv3d_thin_out_p3 conv3d_wgrad_thin_p conv3d_thin_in_f16x3_kernel.Li0 conv3d_thin_in_f16x3_kernel.Li4 split2_f16; do
  python3 "$R/tools/pmc_traffic.py" "$(cc pmc_thin_bench_FETCH_SIZE)" "$(cc pmc_thin_bench_WRITE_SIZE)" "$k" || true
done
python3 "$R/tools/pmc_traffic.py" "$(cc pmc_k160_bench_FETCH_SIZE)" "$(cc pmc_k160_bench_WRITE_SIZE)" "gemm_k160" || true
