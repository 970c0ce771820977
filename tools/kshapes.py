"""Per-launch-shape durations from a rocprofv3 kernel_trace.csv: for kernels whose
name matches a substring, group dispatches by grid size and report count / mean /
median us; also the gaps between consecutive dispatches (launch overhead).
  python tools/kshapes.py run_kernel_trace.csv [substring ...]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    pats = sys.argv[2:] or [""]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    agg = collections.defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"]
        if not any(p in n for p in pats):
            continue
        key = (n[:70], int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), int(r["Grid_Size_Y"]),
               int(r["Grid_Size_Z"]))
        agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        v2 = sorted(v)
        print(f"{sum(v) / 1e3:8.2f} ms {len(v):5d} x mean {sum(v) / len(v):8.1f} med {v2[len(v) // 2]:8.1f} us  "
              f"wg {k[1]} x {k[2]} x {k[3]}  {k[0]}")
    gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])]
    gaps = [g for g in gaps if 0 <= g < 1000]
    if gaps:
        gaps.sort()
        print(f"inter-dispatch gaps: n {len(gaps)} median {gaps[len(gaps) // 2]:.1f} us, sum {sum(gaps) / 1e3:.1f} ms")


if __name__ == "__main__":
    main()
