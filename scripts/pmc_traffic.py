"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch of the
materialize kernel (profiles/pmc_traffic.json, read by bench.py for roofline.traffic).

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KiB) counts exactly
half the bytes of a wide coalesced streaming read -> x2; WRITE_SIZE (KiB) is exact for
16-B-per-lane streaming stores (our result stores are 1-8 B per lane: uncalibrated)."""
import csv
import json
import sys


def per_kernel(path, counter, match):
    vals = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and match in r["Kernel_Name"]:
            vals.append(float(r["Counter_Value"]))
    return vals


def main():
    fetch_csv, write_csv, workload, out = sys.argv[1:5]
    match = sys.argv[5] if len(sys.argv) > 5 else "k_stream"
    f = per_kernel(fetch_csv, "FETCH_SIZE", match)
    w = per_kernel(write_csv, "WRITE_SIZE", match)
    if not f or not w:
        raise SystemExit(f"no {match} dispatches found")
    fetch = sum(f) / len(f) * 1024 * 2
    write = sum(w) / len(w) * 1024
    d = {"workload": workload, "kernel": match, "dispatches": [len(f), len(w)],
         "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
         "bytes_per_launch": fetch + write,
         "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; FETCH_SIZE x2 "
                   "(gfx950 half-count on wide streaming reads), KiB -> bytes"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
