#!/bin/bash
# final-tree pass: every -m gpu test, smoke(), the default bench line
set -o pipefail
OUT=gpurun_out/r06fin
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/gpu_tests.log | tail -20
tail -2 $OUT/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
grep "^{" $OUT/bench.json | tail -1 | cut -c1-300
echo "final pass done (tests rc=$rc)"
