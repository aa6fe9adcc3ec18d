"""Average PMC counter values per kernel over the rocprofv3 --pmc output dirs given."""
import collections
import csv
import glob
import os
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    if not any(s in k for s in ("grp", "stream", "rows", "sets", "big", "lane", "plan")):
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.4g}  (n={len(v)})")
