"""HBM bytes per dispatch of one kernel from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE in KiB per dispatch).  gfx950 correction
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of wide
coalesced streaming reads -> doubled; WRITE_SIZE is exact for 16-B stores.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv KERNEL_REGEX [skip_first]
"""
import csv
import json
import re
import sys


def per_dispatch(path, rx, counter):
    vals = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and re.search(rx, r["Kernel_Name"]):
            vals.append(float(r["Counter_Value"]))
    return vals


fetch_csv, write_csv, rx = sys.argv[1:4]
skip = int(sys.argv[4]) if len(sys.argv) > 4 else 1
f = per_dispatch(fetch_csv, rx, "FETCH_SIZE")[skip:]
w = per_dispatch(write_csv, rx, "WRITE_SIZE")[skip:]
fetch_b = 2.0 * 1024 * sum(f) / len(f)
write_b = 1024 * sum(w) / len(w)
print(json.dumps({"kernel_regex": rx, "dispatches": [len(f), len(w)],
                  "fetch_bytes_corrected": fetch_b, "write_bytes": write_b,
                  "hbm_bytes_per_launch": fetch_b + write_b}))
