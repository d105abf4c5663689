#!/usr/bin/env python3
"""Register / occupancy table of the kernels in one HIP source (hipcc -Rpass-analysis).
usage: scripts/kernel_regs.py cuda_iblb_11_amd/csrc/lbm_sweep.hip [name-filter]"""
import re, subprocess, sys
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-c", src,
                    "-o", "/tmp/_regs.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
cur, rows = None, []
for ln in r.stderr.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|Occupancy \[waves/SIMD\]|ScratchSize \[bytes/lane\]|SGPRs Spill): (\S+)", ln)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    else:
        cur[k.split()[0]] = v
for d in rows:
    if flt in d["name"]:
        print(f"{d.get('VGPRs','?'):>4} {d.get('AGPRs','?'):>4} occ {d.get('Occupancy','?'):>2} scratch {d.get('ScratchSize','?'):>3} sspill {d.get('SGPRs','?'):>3}  {d['name'][:110]}")
