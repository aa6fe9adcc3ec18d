"""HBM traffic per cached-mode read call (bench.py --base cached: am_snapcache_read = k_sc_claim +
k_sc_select + the materialize tiers + k_sc_store + k_sc_release) from rocprofv3 --pmc FETCH_SIZE
and WRITE_SIZE passes (separate runs).  bench.py alternates an untimed populate call (the q = 0.5
reads that fill the cache) with the timed q = 0.75 call, so the dispatches are split into calls
at every k_sc_claim and only the odd (timed) calls are averaged.  Writes
profiles/pmc_traffic.json[CFG].
Usage: pmc_traffic_cached.py FETCH_DIR WRITE_DIR CFG WORKLOAD [OUT [ZONE_INDEX]]  (default "none")"""
import csv
import glob
import json
import sys

MAT = ("k_lane", "k_plan", "k_rows", "k_bc_rows", "k_stream", "k_grp_wave", "k_grp_wg", "k_grp_row", "k_sets", "k_big_",
       "k_bc_wave",
       "k_sc_")


def calls(d, counter):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"]
        per.setdefault(int(r["Dispatch_Id"]), [k, 0.0])[1] += float(r["Counter_Value"]) * 1024
    out, cur = [], None
    for did in sorted(per):
        k, v = per[did]
        if "k_sc_claim" in k:
            cur = {}
            out.append(cur)
        if cur is not None and any(m in k for m in MAT):
            cur[k[:80]] = cur.get(k[:80], 0.0) + v
    return out


def main():
    fdir, wdir, cfg, workload = sys.argv[1:5]
    out = sys.argv[5] if len(sys.argv) > 5 else "profiles/pmc_traffic.json"
    zone_index = sys.argv[6] if len(sys.argv) > 6 else "none"
    fc, wc = calls(fdir, "FETCH_SIZE"), calls(wdir, "WRITE_SIZE")
    ft, wt = fc[1::2], wc[1::2]  # the timed calls
    fetch_raw = sum(sum(c.values()) for c in ft) / len(ft)
    write = sum(sum(c.values()) for c in wt) / len(wt)
    d = {"workload": workload, "zone_index": zone_index, "kernel": "am_snapcache_read: k_sc_* + every materialize tier", "calls": [len(ft), len(wt)],
         "fetch_raw_bytes_per_launch": fetch_raw, "fetch_bytes_per_launch": 2 * fetch_raw,
         "write_bytes_per_launch": write, "bytes_per_launch": 2 * fetch_raw + write,
         "per_kernel_fetch_raw": {k: sum(c.get(k, 0.0) for c in ft) / len(ft) for k in sorted({k for c in ft for k in c})},
         "per_kernel_write": {k: sum(c.get(k, 0.0) for c in wt) / len(wt) for k in sorted({k for c in wt for k in c})},
         "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of bench.py --base cached, "
                   "KiB -> bytes; dispatches split into read calls at k_sc_claim, the timed (odd) calls averaged; "
                   "FETCH_SIZE x2 (MI355X_MICROARCH.md: 128-B requests tallied at 64 B; upper bound, fetch_raw the "
                   "lower bound)"}
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
