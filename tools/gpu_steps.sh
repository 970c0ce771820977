#!/bin/bash
# Run GPU steps from a file of "name|command" lines, each under its own time limit,
# stopping at the first step that crashed / timed out (rc not in {0, 1}; rc 1 = test failures).
#   tools/gpu_steps.sh TAG STEPFILE
TAG=$1; STEPS=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
while IFS='|' read -r name cmd; do
    [ -z "$name" ] && continue
    echo "=== $name"
    timeout -k 10 ${STEP_TIMEOUT:-420} bash -c "$cmd" > $OUT/$name.log 2>&1
    rc=$?
    echo "rc=$rc"
    grep -E "vs f64|floor|NRMSE|FAILED|passed|failed|Error" $OUT/$name.log | tail -25
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done < $STEPS
