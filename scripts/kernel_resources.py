#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy of a HIP TU for gfx950 (the
compiler's kernel-resource-usage remarks), e.g.
  python3 scripts/kernel_resources.py chaos-ray-tracing-course-2025_amd/csrc/crt_render.hip [name-filter]
Run from the package dir of the tree to inspect (headers resolve relative to it)."""
import re
import subprocess
import sys

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fPIC",
       "--offload-arch=gfx950", "-munsafe-fp-atomics", "-fno-slp-vectorize", "--cuda-device-only", "-c", src,
       "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[3:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/lane\])?: (\S+) \[", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for name, r in rows.items():
    if filt and filt not in name:
        continue
    dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    dm = re.sub(r"\(.*\)$", "", dm)
    print(f"{dm:70s} vgpr {r.get('VGPRs','?'):>4} sgpr {r.get('TotalSGPRs','?'):>4} scratch {r.get('ScratchSize','?'):>5} "
          f"occ {r.get('Occupancy [waves/SIMD]', r.get('Occupancy','?')):>2} sgpr_spill {r.get('SGPRs Spill','?'):>3} "
          f"vgpr_spill {r.get('VGPRs Spill','?'):>3} lds {r.get('LDS Size','?')}")
