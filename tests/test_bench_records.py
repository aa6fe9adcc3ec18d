"""bench.py's committed PMC record (profiles/pmc_traffic.json) is keyed on the exact workload
string the bench prints, so a renamed config would silently turn `roofline.traffic` into
null.  Every recorded config must still match bench.CONFIGS, and the default config must
have a record."""
import json
import os

import bench


def test_pmc_traffic_records_match_bench_workloads():
    with open(os.path.join(os.path.dirname(bench.__file__), "profiles", "pmc_traffic.json")) as f:
        rec = json.load(f)
    assert "c3" in rec and "c3_cached" in rec
    for key, e in rec.items():
        cfg = key[:-len("_cached")] if key.endswith("_cached") else key  # bench.py --base cached
        assert cfg in bench.CONFIGS, key
        w = f"{cfg}: {bench.CONFIGS[cfg]['desc']}"
        assert bench.load_traffic(key, w, e["zone_index"]) == e.get("calibrated_bytes_per_launch", e["bytes_per_launch"]), key
        assert e["bytes_per_launch"] > 0
