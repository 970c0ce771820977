#!/bin/bash
# Full GPU test pass without -x (to see every failure at once).
set -o pipefail
TAG=${1:-r02a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread ${@:2} > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $OUT/gpu_tests.log | grep -v PASSED | tail -40
tail -3 $OUT/gpu_tests.log
exit $rc
