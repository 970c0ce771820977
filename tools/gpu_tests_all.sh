#!/bin/bash
# GPU test pass without -x (to see every failure at once).
#   tools/gpu_tests_all.sh TAG [test files ...]   (default: all of tests/)
set -o pipefail
TAG=${1:-r02a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
TARGETS="${@:2}"
[ -z "$TARGETS" ] && TARGETS=tests
timeout -k 10 900 python -u -m pytest $TARGETS -v -s -m gpu --timeout 180 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $OUT/gpu_tests.log | grep -v PASSED | tail -40
grep -E "vs f64|floor|err vs" $OUT/gpu_tests.log | tail -60
tail -3 $OUT/gpu_tests.log
exit $rc
