#!/usr/bin/env python3
"""Print the top kernels of rocprofv3 --stats summaries: kstats.py DIR [DIR...]"""
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        print("==", f)
        for r in list(csv.DictReader(open(f)))[:8]:
            print(f"  {r['Name'][:72]:72s} {r['Calls']:>4s} {float(r['AverageNs'])/1e6:9.3f} ms {float(r['Percentage']):6.2f}%")
