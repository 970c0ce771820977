#!/bin/bash
# Round-6 GPU pass: named test files (or all of tests/), then optionally smoke.
#   tools/gpu_r06.sh TAG [test files ...]
set -o pipefail
TAG=${1:-r06a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
TARGETS="${@:2}"
[ -z "$TARGETS" ] && TARGETS=tests
timeout -k 10 1000 python -u -m pytest $TARGETS -v -s -m gpu -x --timeout 180 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $OUT/gpu_tests.log | grep -v PASSED | tail -20
grep -E "bf16 vs fp32|fresh network|NRMSE" $OUT/gpu_tests.log | tail -20
tail -3 $OUT/gpu_tests.log
exit $rc
