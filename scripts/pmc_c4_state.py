#!/usr/bin/env python3
"""Per-state averages of k_lane_q's counters and durations from scripts/pmc_c4_state.sh.
The dispatches before the first C3 kernel are the "plain" state, those after it "c3first".
   python scripts/pmc_c4_state.py gpurun_out/c4state_*"""
import csv
import glob
import re
import sys
from collections import defaultdict


def rows(d, name):
    out = []
    for f in glob.glob(f"{d}/**/*{name}.csv", recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def main():
    for d in sys.argv[1:]:
        kt = rows(d, "kernel_trace")
        cc = rows(d, "counter_collection")
        split = min((int(r["Dispatch_Id"]) for r in kt if re.search(r"k_grp_incl|k_grp_wave", r["Kernel_Name"])),
                    default=1 << 62)
        dur = {int(r["Dispatch_Id"]): (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
               for r in kt if "k_lane_q" in r["Kernel_Name"]}
        acc = defaultdict(lambda: defaultdict(list))
        for r in cc:
            i = int(r["Dispatch_Id"])
            if i not in dur:
                continue
            acc["plain" if i < split else "c3first"][r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(d)
        for st in ("plain", "c3first"):
            ids = [i for i in dur if (i < split) == (st == "plain")]
            if not ids:
                continue
            ms = sorted(dur[i] for i in ids)
            print(f"  {st}: {len(ids)} dispatches, ms median {ms[len(ms) // 2]:.3f} min {ms[0]:.3f} max {ms[-1]:.3f}")
            for c, vs in sorted(acc[st].items()):
                print(f"     {c:40s} {sum(vs) / len(vs):16.6g}")


if __name__ == "__main__":
    main()
