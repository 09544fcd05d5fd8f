#!/usr/bin/env python3
"""Per-kernel VGPR / spill / scratch table of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage).

    python scripts/kernel_resources.py gnot-replication_amd/csrc/chain2.hip [extra hipcc flags]
"""
import os
import re
import subprocess
import sys

src = os.path.abspath(sys.argv[1])
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-fno-slp-vectorize", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
       "-I" + os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(src))), "include"), "-c", src,
       "-o", "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
err = subprocess.run(cmd, capture_output=True, text=True, cwd=os.path.dirname(src)).stderr
rows, cur = [], None
for line in err.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs Spill|SGPRs Spill): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt"], input=v, capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    else:
        cur[k] = v
for r in rows:
    print(f"{r.get('VGPRs','?'):>4} vgpr {r.get('AGPRs','?'):>3} agpr spill {r.get('VGPRs Spill','?'):>3} "
          f"scratch {r.get('ScratchSize [bytes/lane]','?'):>4} occ {r.get('Occupancy [waves/SIMD]','?')}  {r['name'][:110]}")
