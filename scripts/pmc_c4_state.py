#!/usr/bin/env python3
"""Per-state averages of k_lane_q's counters and durations from scripts/pmc_c4_state.sh.
The dispatches before the first C3 kernel are the "plain" state, those after it "c3first".
   python scripts/pmc_c4_state.py gpurun_out/c4state_*"""
import csv
import glob
import re
import sys
from collections import defaultdict

KERNEL = r"k_lane_q<3,"  # C4's lane kernel (C3's own planner runs k_lane_q<8, ...>)


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
               for r in kt if re.search(KERNEL, r["Kernel_Name"])}
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
            avg = {c: sum(vs) / len(vs) for c, vs in acc[st].items()}
            for c, v in sorted(avg.items()):
                print(f"     {c:40s} {v:16.6g}")
            if "TCP_TCC_READ_REQ_sum" in avg:
                print(f"     -> mean L2 read latency (cycles)         {avg['TCP_TCC_READ_REQ_LATENCY_sum'] / avg['TCP_TCC_READ_REQ_sum']:16.1f}")
            if "TCP_UTCL1_REQUEST_sum" in avg:
                print(f"     -> UTCL1 miss rate                       {avg['TCP_UTCL1_TRANSLATION_MISS_sum'] / avg['TCP_UTCL1_REQUEST_sum']:16.4f}")
            if "SQ_WAVE_CYCLES" in avg:
                for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                    print(f"     -> {c + ' / WAVE_CYCLES':38s} {avg[c] / avg['SQ_WAVE_CYCLES']:16.3f}")


if __name__ == "__main__":
    main()
