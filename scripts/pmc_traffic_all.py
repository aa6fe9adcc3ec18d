"""HBM traffic per materialize launch summed over EVERY materialize kernel (the lane, row,
stream, group, LDS-sort and big-read tiers and the planner) from rocprofv3 --pmc FETCH_SIZE
and WRITE_SIZE passes (separate runs) of `bench.py --config CFG`; one launch = one k_lane
(or k_grp_wave) dispatch.  Writes profiles/pmc_traffic.json[CFG].
Usage: pmc_traffic_all.py FETCH_DIR WRITE_DIR CFG WORKLOAD LAUNCH_KERNEL [OUT [ZONE_INDEX]]
(ZONE_INDEX: the store's zone index level name, bench.py INDEX_NAMES; default "none")"""
import csv
import glob
import json
import sys

MAT = ("k_lane", "k_plan", "k_rows", "k_bc_rows", "k_stream", "k_grp_wave", "k_grp_wg", "k_grp_row", "k_grp_incl",
       "k_grp_recs", "k_sets", "k_big_", "k_bc_wave")


def totals(d, counter, launch):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    tot, n = {}, 0
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if r["Counter_Name"] != counter or not any(m in k for m in MAT):
            continue
        tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"]) * 1024
        n += launch in k
    return tot, n


def main():
    fdir, wdir, cfg, workload, launch = sys.argv[1:6]
    out = sys.argv[6] if len(sys.argv) > 6 else "profiles/pmc_traffic.json"
    zone_index = sys.argv[7] if len(sys.argv) > 7 else "none"
    f, nf = totals(fdir, "FETCH_SIZE", launch)
    w, nw = totals(wdir, "WRITE_SIZE", launch)
    fetch_raw = sum(f.values()) / nf
    write = sum(w.values()) / nw
    d = {"workload": workload, "zone_index": zone_index, "kernel": "all materialize kernels (" + ", ".join(MAT) + ")", "launches": [nf, nw],
         "fetch_raw_bytes_per_launch": fetch_raw, "fetch_bytes_per_launch": 2 * fetch_raw,
         "write_bytes_per_launch": write, "bytes_per_launch": 2 * fetch_raw + write,
         "per_kernel_fetch_raw": {k[:80]: v / nf for k, v in sorted(f.items(), key=lambda x: -x[1])},
         "per_kernel_write": {k[:80]: v / nw for k, v in sorted(w.items(), key=lambda x: -x[1])},
         "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes, KiB -> bytes, summed over "
                   "the launch's kernels; FETCH_SIZE x2 (MI355X_MICROARCH.md: 128-B requests tallied at 64 B). "
                   "Upper bound: reads served by 64-B requests (the lane tier's 32-B per-lane pieces, gathers) "
                   "are counted exactly by FETCH_SIZE, so x2 over-states them; fetch_raw is the lower bound."}
    try:
        allc = json.load(open(out))
    except Exception:
        allc = {}
    # the sources the passes ran (bench.py reports traffic only for a record of its own sources)
    sys.path.insert(0, ".")
    from bench import src_sha16
    d["src_sha16"] = src_sha16()
    allc[cfg] = d
    json.dump(allc, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in d.items() if not k.startswith("per_kernel")}))


if __name__ == "__main__":
    main()
