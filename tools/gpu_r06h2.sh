#!/bin/bash
# h3r token-Linear latency floor: time vs M
set -o pipefail
timeout -k 10 120 python tools/h3r_bench.py 2>&1 | grep -v amdgpu.ids && timeout -k 10 120 python tools/h3r_bench.py sweep 2>&1 | grep -v amdgpu.ids
