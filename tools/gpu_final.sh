#!/bin/bash
# End-of-round GPU pass (run via gpurun from the repo root): every -m gpu test,
# smoke(), the default bench line, then tools/profile_r02.sh $TAG.
set -o pipefail
TAG=${1:-r02z}
OUT=gpurun_out/$TAG
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
bash tools/profile_r02.sh $TAG > $OUT/profile.log 2>&1 || { echo PROFILE_FAILED; tail -20 $OUT/profile.log; exit 1; }
echo "final pass done (tests rc=$rc)"
