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
    assert "c3" in rec
    for cfg, e in rec.items():
        assert cfg in bench.CONFIGS, cfg
        w = f"{cfg}: {bench.CONFIGS[cfg]['desc']}"
        assert bench.load_traffic(cfg, w) == e.get("calibrated_bytes_per_launch", e["bytes_per_launch"]), cfg
        assert e["bytes_per_launch"] > 0
