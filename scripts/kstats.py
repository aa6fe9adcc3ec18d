"""Print the read kernels of rocprofv3 kernel-stats CSVs side by side: kstats.py DIR... [--match k_grp]"""
import csv
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--match=")), "")
for d in args:
    rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
    print("==", d)
    for x in rows:
        if match in x["Name"] and int(x["Calls"]) >= 10:
            print(f"  {x['Name'][:60]:60s} {x['Calls']:>5s} {float(x['AverageNs']) / 1e3:9.1f} us")
