#!/usr/bin/env python3
"""Compact per-kernel resource usage (VGPR / AGPR / scratch / occupancy) of one HIP source,
from hipcc -Rpass-analysis=kernel-resource-usage. usage: python tools/kres.py FILE [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", "include",
                    "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"],
                   capture_output=True, text=True)
cur = None
rows = {}
for line in r.stderr.splitlines():
    m = re.search(r"remark: +(.+?): (\S+) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for name, d in rows.items():
    if flt in name:
        print(f"{name[:90]:90s} V{d.get('VGPRs')} A{d.get('AGPRs')} S{d.get('SGPRs')} "
              f"scratch{d.get('ScratchSize [bytes/lane]')} occ{d.get('Occupancy [waves/SIMD]')} "
              f"lds{d.get('LDS Size [bytes/block]')}")
if r.returncode:
    print(r.stderr[-3000:])
