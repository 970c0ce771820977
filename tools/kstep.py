"""Per-step kernel statistics from a rocprofv3 kernel_trace.csv of bench.py: the
training steps are the segments that end with the optimizer's multi_tensor_apply
cluster; the last N segments (the timed steps) are summarised per step -- busy time,
wall span, idle gaps, launches, and the top kernels.
  python tools/kstep.py run_kernel_trace.csv [N=3] [top=25]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    nlast = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    opt = [i for i, r in enumerate(rows) if "multi_tensor_apply" in r["Kernel_Name"] or "fused_adam" in r["Kernel_Name"].lower()]
    ends = [i for j, i in enumerate(opt) if j + 1 == len(opt) or opt[j + 1] > i + 1]   # last launch of each cluster
    seg = [(a + 1, b + 1) for a, b in zip(ends[:-1], ends[1:])][-nlast:]
    tot = collections.Counter()
    cnt = collections.Counter()
    busy = span = 0.0
    nl = 0
    for a, b in seg:
        for r in rows[a:b]:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            tot[r["Kernel_Name"][:100]] += d
            cnt[r["Kernel_Name"][:100]] += 1
            busy += d
        span += (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
        nl += b - a
    n = len(seg)
    print(f"{n} steps: busy {busy / n / 1e3:.2f} ms/step, span {span / n / 1e3:.2f} ms/step, "
          f"idle {(span - busy) / n / 1e3:.2f} ms/step, {nl / n:.0f} launches/step")
    for k, v in tot.most_common(top):
        print(f"{v / n / 1e3:8.3f} ms/step {cnt[k] / n:7.1f}/step {v / cnt[k]:9.1f} us  {k}")


if __name__ == "__main__":
    main()
