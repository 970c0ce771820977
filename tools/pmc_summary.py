"""Per-kernel mean of every counter in a rocprofv3 --pmc counter_collection.csv.

    python tools/pmc_summary.py run_counter_collection.csv [kernel_regex]
"""
import collections
import csv
import re
import sys

rx = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"]
    if rx and not rx.search(name):
        continue
    acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in acc.items():
    n = max(len(v) for v in cs.values())
    print(f"{name[:110]}  (dispatches {n})")
    m = {k: sum(v) / len(v) for k, v in cs.items()}
    for k in sorted(m):
        print(f"    {k:28s} {m[k]:16.1f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CYCLES" in m and m["SQ_BUSY_CYCLES"] > 0:
        print(f"    MFMA busy / SQ busy (per-SIMD normalised by the guide's recipe): see MI355X_MICROARCH.md")
