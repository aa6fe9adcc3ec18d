#!/usr/bin/env python3
"""Memory-op / wait skeleton of one kernel's gfx950 assembly (vmcnt waits between loads show
where a wave stalls).  python scripts/kasm.py SRC.hip MANGLED-SUBSTRING [extra hipcc flags...]"""
import re
import subprocess
import sys

src, key, extra = sys.argv[1], sys.argv[2], sys.argv[3:]
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
                "-I/opt/rocm/include", *extra, "-S", "--offload-device-only", src, "-o", "/tmp/kasm.s"], check=True,
               capture_output=True)
s = open("/tmp/kasm.s").read()
name = [m for m in re.findall(r"^(_Z\S+):", s, re.M) if key in m][0]
body = s[s.index(name + ":"):]
body = body[:body.index(".Lfunc_end")]
n = 0
for l in body.split("\n"):
    t = l.strip()
    if not t or t.startswith((";", ".")) and not t.startswith(".LBB"):
        continue
    n += 1
    op = t.split()[0]
    if op.startswith(("global_", "buffer_", "s_waitcnt vmcnt", "ds_bpermute")) or (op == "s_waitcnt" and "vmcnt" in t) \
            or t.startswith(".LBB"):
        print(f"{n:5d} {t[:100]}")
