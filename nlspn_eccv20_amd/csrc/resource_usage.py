#!/usr/bin/env python3
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks as a table."""
import re
import subprocess
import sys

cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
       "-ffp-contract=off", "-Rpass-analysis=kernel-resource-usage", "-o", "/tmp/nlspn_ru.so", "nlspn_capi.hip"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|TotalSGPRs): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split()[0]] = int(m.group(2))
filt = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if filt in r["name"]:
        dem = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        dem = dem.replace("nlspn::", "").replace("(StepArgs)", "").replace("void ", "")
        print(f"{dem[:90]:90s} vgpr={r.get('VGPRs')} sgpr={r.get('TotalSGPRs')} scratch={r.get('ScratchSize')} "
              f"occ={r.get('Occupancy')} lds={r.get('LDS')}")
