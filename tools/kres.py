#!/usr/bin/env python3
"""Per-kernel register / spill / occupancy table of one HIP source (gfx950),
from hipcc's -Rpass-analysis=kernel-resource-usage remarks.

usage: python tools/kres.py <file.hip> [filter-substring]
"""
import re
import subprocess
import sys
from pathlib import Path

src = Path(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
csrc = Path(__file__).resolve().parent.parent / "idunno" / "csrc"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{csrc}", "--cuda-device-only",
       "-c", str(src), "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for ln in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", ln)
    if not m:
        continue
    body = m.group(1)
    if body.startswith("Function Name:"):
        cur = {"name": body.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in body:
        k, v = body.split(":", 1)
        cur[k.strip()] = v.strip()
try:
    names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                           text=True).stdout.splitlines()
except OSError:
    names = [r["name"] for r in rows]
print(f"{'kernel':90s} {'vgpr':>5s} {'agpr':>5s} {'spill':>5s} {'sgpr':>5s} {'occ':>4s}")
for r, n in zip(rows, names):
    if flt and flt not in n:
        continue
    n = re.sub(r"\(idunno::\w+\)$", "", n.replace("void idunno::", ""))
    print(f"{n[:90]:90s} {r.get('VGPRs', '?'):>5s} {r.get('AGPRs', '?'):>5s} {r.get('VGPRs Spill', '?'):>5s} "
          f"{r.get('SGPRs', '?'):>5s} {r.get('Occupancy [waves/SIMD]', '?'):>4s}")
