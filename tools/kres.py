"""Per-kernel VGPR / spill / LDS summary of a hipcc --save-temps device .s file.

usage: python tools/kres.py file-hip-amdgcn-amd-amdhsa-gfx950.s [name-filter]"""
import re
import subprocess
import sys

text = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
meta = text[text.find("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    f = dict(re.findall(r"^\s*\.(\w+):\s+(\S+)", blk, re.M))
    name = f.get("name", "?")
    if flt not in name:
        continue
    try:
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    except OSError:
        dem = name
    print(f"vgpr {f.get('vgpr_count'):>4} agpr {f.get('agpr_count'):>3} spill {f.get('vgpr_spill_count'):>3} "
          f"lds {f.get('group_segment_fixed_size'):>6} scratch {f.get('private_segment_fixed_size'):>4}  {dem[:110]}")
