#!/bin/bash
# Full GPU pass of the current tree (run via gpurun from the repo root):
#   GPU parity tests, smoke(), default bench line, then tools/profile_round.sh $TAG.
set -o pipefail
TAG=${1:-r01e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -30 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
bash tools/profile_round.sh $TAG
