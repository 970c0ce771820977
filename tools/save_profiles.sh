#!/bin/bash
# Copy the judged summaries of a gpu_final.sh / profile_r02.sh pass into profiles/ (run here, not on the box).
set -e
TAG=$1
O=gpurun_out/$TAG
grep '^{' $O/bench.json | tail -1 > profiles/${TAG}_bench.json
tail -3 $O/gpu_tests.log > profiles/${TAG}_gpu_tests_tail.txt
tail -1 $O/smoke.log > profiles/${TAG}_smoke.txt
cp $O/summary_fp32.txt profiles/${TAG}_summary_fp32.txt
cp $O/summary_bf16.txt profiles/${TAG}_summary_bf16.txt
cp $O/sq_h3.txt profiles/${TAG}_sq_f16x3.txt
for f in $O/traffic_f16x3_*.json; do cp $f profiles/${TAG}_$(basename $f); done
cp "$(find $O/trace_fp32 -name '*kernel_stats.csv' | head -1)" profiles/${TAG}_kernel_stats_fp32.csv
cp "$(find $O/trace_bf16 -name '*kernel_stats.csv' | head -1)" profiles/${TAG}_kernel_stats_bf16.csv
grep '^{' $O/bench_traced_fp32.log | tail -1 > profiles/${TAG}_bench_traced_fp32.json
