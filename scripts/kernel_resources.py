#!/usr/bin/env python3
"""Per-kernel VGPRs / scratch / occupancy of a HIP source (hipcc -Rpass-analysis).

Usage: scripts/kernel_resources.py srbd-nmpc-solver_amd/csrc/ipm_box.hip [filter]
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(
    ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-c", src,
     "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"],
    capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
        continue
    for key in ("VGPRs", "AGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]"):
        m = re.search(key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0].split("\\")[0]] = int(m.group(1))
for r in rows:
    if flt in r["name"]:
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('AGPRs', 0):>3} agpr {r.get('ScratchSize', '?'):>4} B scratch "
              f"occ {r.get('Occupancy', '?')}  lds {r.get('LDS', '?'):>6}  {r['name'][:110]}")
