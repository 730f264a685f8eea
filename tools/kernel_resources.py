#!/usr/bin/env python3
"""Per-kernel VGPR / spill / scratch / occupancy table of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage).

    python tools/kernel_resources.py csrc/kernels/conv_chain.hip [name-filter]
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics",
       "-mllvm", "-amdgpu-mfma-vgpr-form=1", "-Icsrc/kernels", "-c", src, "-o", "/tmp/_kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+([\w \[\]/]+?):\s+(.*?)\s+\[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k in ("Function Name", "Name"):
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if flt in r["name"]:
        # scratch also counts private arrays the compiler did not promote to registers (not reported as spills)
        print(f"{r.get('VGPRs','?'):>4} vgpr {r.get('AGPRs','?'):>3} agpr spill {r.get('VGPRs Spill','?'):>3} "
              f"scratch {r.get('ScratchSize [bytes/lane]','?'):>4} "
              f"occ {r.get('Occupancy [waves/SIMD]','?'):>2}  {r['name'][:150]}")
