"""Per-kernel register / spill / occupancy table of a HIP source for gfx950
(hipcc -Rpass-analysis=kernel-resource-usage). Usage: python scripts/kres.py FILE.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-c",
       "--offload-device-only", "-Rpass-analysis=kernel-resource-usage", src, "-o", "/tmp/kres.o"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark:\s+Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for name, r in rows.items():
    if flt in name:
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('VGPRs Spill', '?'):>3} vspill {r.get('SGPRs Spill', '?'):>4} sspill "
              f"occ {r.get('Occupancy [waves/SIMD]', '?')}  lds {r.get('LDS Size [bytes/block]', '?'):>6}  {name}")
