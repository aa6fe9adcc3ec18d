#!/usr/bin/env python3
"""Per-kernel averages of the counters in gpurun_out/pmcsq_* (scripts/pmc_sq.sh).
   python scripts/pmc_sq_summary.py gpurun_out/pmcsq_c4_old [kernel-regex]"""
import csv
import glob
import re
import sys
from collections import defaultdict

d, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "k_lane|k_grp|k_rows|k_big|k_bc|k_sets|k_stream")
files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
acc = defaultdict(lambda: defaultdict(list))
for f in files:
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        if not re.search(pat, k):
            continue
        k = re.sub(r"\(anonymous namespace\)::", "", k).split("(")[0]
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    n = len(next(iter(cs.values())))
    for c, vs in sorted(cs.items()):
        print(f"   {c:24s} {sum(vs) / len(vs):16.4g}   (n={len(vs)})")
    w = cs.get("SQ_WAVE_CYCLES")
    if w:
        W = sum(w)
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in cs:
                print(f"   {c + ' / WAVE_CYCLES':38s} {sum(cs[c]) / W:.3f}")
