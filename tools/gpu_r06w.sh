#!/bin/bash
# end-of-round GPU pass, part 1: every -m gpu test, then smoke()
set -o pipefail
OUT=gpurun_out/${1:-r06w}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/gpu_tests.log | tail -20
tail -2 $OUT/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
exit $rc
