"""Derived SQ utilisations per kernel from a rocprofv3 --pmc counter_collection.csv
(rocprofiler-sdk's derived_counters.xml formulas, gfx950: GRBM_GUI_ACTIVE is summed
over the 8 XCDs in the CSV, so its per-XCD value -- the 'max' reduce of the formulas
-- is the sum / 8; 256 CUs, 1024 SIMDs):
    MfmaUtil  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM / 8 x 1024)
    VALUBusy  = SQ_ACTIVE_INST_VALU / 256 / (GRBM / 8)      (SQ_ACTIVE_INST_* in quad-cycles per wave)
    LDSBusy   = SQ_ACTIVE_INST_LDS  / 256 / (GRBM / 8)
plus instructions per dispatch (SQ_INSTS_*).
    python tools/sq_derived.py run_counter_collection.csv [kernel_regex ...]
"""
import collections
import csv
import re
import sys

rxs = [re.compile(a) for a in sys.argv[2:]]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"]
    if rxs and not any(x.search(name) for x in rxs):
        continue
    acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in acc.items():
    m = {k: sum(v) / len(v) for k, v in cs.items()}
    n = max(len(v) for v in cs.values())
    g = m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    print(f"{name[:100]}  (dispatches {n}, {g / 2.1e3:.1f} us at 2.1 GHz)")
    if g > 0:
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            print(f"    MfmaUtil  {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (g * 1024):.3f}")
        if "SQ_ACTIVE_INST_VALU" in m:
            print(f"    VALUBusy  {m['SQ_ACTIVE_INST_VALU'] / 256 / g:.3f}")
        if "SQ_ACTIVE_INST_LDS" in m:
            print(f"    LDSBusy   {m['SQ_ACTIVE_INST_LDS'] / 256 / g:.3f}")
    for k in sorted(m):
        if k.startswith("SQ_INSTS"):
            print(f"    {k:24s} {m[k]:16.0f}")
    if "SQ_INSTS_VALU" in m and "SQ_INSTS_MFMA" in m and m["SQ_INSTS_MFMA"] > 0:
        print(f"    VALU / MFMA instructions {m['SQ_INSTS_VALU'] / m['SQ_INSTS_MFMA']:.1f}")
