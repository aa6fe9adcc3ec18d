"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch of the
materialize kernel (profiles/pmc_traffic.json, read by bench.py for roofline.traffic).

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KiB) counts exactly
half the bytes of a wide coalesced streaming read -> x2; WRITE_SIZE (KiB) is exact for
16-B-per-lane streaming stores (our result stores are 1-8 B per lane: uncalibrated)."""
import csv
import json
import sys


def per_kernel(path, counter, match):
    """counter value per dispatch of every kernel whose name contains `match`, by name"""
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and match in r["Kernel_Name"]:
            vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return vals


def avg_sum(vals):
    """one materialize launch = one dispatch of each matched kernel: sum of per-kernel means"""
    return sum(sum(v) / len(v) for v in vals.values())


def main():
    fetch_csv, write_csv, config, workload, out = sys.argv[1:6]
    match = sys.argv[6] if len(sys.argv) > 6 else "k_grp_wave"
    f = per_kernel(fetch_csv, "FETCH_SIZE", match)
    w = per_kernel(write_csv, "WRITE_SIZE", match)
    if not f or not w:
        raise SystemExit(f"no {match} dispatches found")
    fetch = avg_sum(f) * 1024 * 2
    write = avg_sum(w) * 1024
    d = {"workload": workload, "kernel": match, "dispatches": [sum(len(v) for v in f.values()),
                                                               sum(len(v) for v in w.values())],
         "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
         "bytes_per_launch": fetch + write,
         "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; FETCH_SIZE x2 "
                   "(gfx950 half-count on wide streaming reads), KiB -> bytes"}
    try:
        allc = json.load(open(out))
        if "workload" in allc:  # the r01 single-config layout
            allc = {}
    except Exception:
        allc = {}
    allc[config] = d
    json.dump(allc, open(out, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
