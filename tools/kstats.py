"""Summarise a rocprofv3 --stats kernel CSV: top kernels by total time."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total GPU time {tot / 1e6:.1f} ms  ({tot / 1e6 / steps:.1f} ms per step over {steps:g} steps)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.2f} ms/step {float(r['Percentage']):5.1f}% "
          f"calls/step={int(r['Calls']) / steps:7.1f} avg={float(r['AverageNs']) / 1e3:9.1f}us  {r['Name'][:100]}")
