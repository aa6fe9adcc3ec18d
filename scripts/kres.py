#!/usr/bin/env python3
"""Register / LDS / occupancy table of the kernels of one source file (compiler remarks).
   python scripts/kres.py antidote_amd/csrc/am_lanes.hip [name-regex] [extra hipcc flags...]"""
import re
import subprocess
import sys

src, pat, extra = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "."), sys.argv[3:]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
       "-I/opt/rocm/include", *extra, "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
dem = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, d in zip(rows, dem):
    d = re.sub(r"\(anonymous namespace\)::", "", d).split("(")[0]
    if not re.search(pat, d):
        continue
    g = lambda k: r.get(k, "?")
    print(f"{d[:64]:64s} vgpr {g('VGPRs'):>4} agpr {g('AGPRs'):>3} vspill {g('VGPRs Spill'):>4} "
          f"sspill {g('SGPRs Spill'):>4} occ {g('Occupancy [waves/SIMD]'):>2} lds {g('LDS Size [bytes/block]')}")
