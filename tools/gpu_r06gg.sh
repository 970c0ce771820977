#!/bin/bash
# final-tree bench line
set -o pipefail
OUT=gpurun_out/r06gg
mkdir -p $OUT
timeout -k 10 1000 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
grep "^{" $OUT/bench.json | tail -1 | cut -c1-200
