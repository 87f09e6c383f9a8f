#!/usr/bin/env python3
"""Kernel resource usage (VGPR, SGPR, LDS, occupancy) of one HIP source, from
hipcc -Rpass-analysis=kernel-resource-usage. usage: tools/kres.py <src.hip> [regex]"""
import re, subprocess, sys
from pathlib import Path
R = Path(__file__).resolve().parents[1]
src, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else ".")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{R/'include'}",
       f"-I{R/'swift_subtask_dev_amd/csrc'}", "-DSWH_BUILD", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r"remark: +([A-Za-z ]+?)(?: \[[^\]]*\])?: (\S+)", line)
    if cur and m:
        rows[cur][m.group(1).strip()] = m.group(2)
dm = subprocess.run(["c++filt"], input="\n".join(rows), capture_output=True, text=True).stdout.split("\n")
for (name, d), dn in zip(rows.items(), dm):
    if re.search(pat, dn):
        short = re.sub(r"\(.*", "", dn)
        print(f"{short:45s} vgpr {d.get('VGPRs','?'):>4} agpr {d.get('AGPRs','?'):>3} sgpr {d.get('TotalSGPRs','?'):>4} "
              f"lds {d.get('LDS Size','?'):>6} scratch {d.get('ScratchSize','?'):>4} occ {d.get('Occupancy','?')}")
