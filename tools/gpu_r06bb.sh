#!/bin/bash
# final bench line (after the fused-Adam version fix), then the config-5 traces
set -o pipefail
OUT=gpurun_out/r06bb
mkdir -p $OUT
timeout -k 10 1000 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
grep "^{" $OUT/bench.json | tail -1 | cut -c1-300
./tools/profile_c5.sh r06c5c
