"""Print ms/step and the conv kernels' per-launch time / roofline fraction of bench.py logs (the JSON line)."""
import json
import sys

for path in sys.argv[1:]:
    d = json.loads([ln for ln in open(path) if ln.startswith("{")][-1])
    rc = d.get("roofline_conv") or {}
    conv = " ".join(f"{k} {v.get('avg_us', 0):.0f}us/{v.get('frac', 0):.3f}" for k, v in rc.items())
    print(f"{path}: {d['ms_per_step']:.1f} ms/step {d['value']:.3f} {d['unit']} | {conv}")
