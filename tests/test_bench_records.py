"""bench.py's committed PMC record (profiles/pmc_traffic.json) is keyed on the exact workload
string the bench prints and on the hash of the library sources it was measured on
(src_sha16): a renamed config, or a record taken on older kernels, turns `roofline.traffic`
into null instead of reporting another build's bytes.  Every recorded config must still match
bench.CONFIGS, and the default config must have a record."""
import json
import os

import bench


def _records():
    with open(os.path.join(os.path.dirname(bench.__file__), "profiles", "pmc_traffic.json")) as f:
        return json.load(f)


def test_pmc_traffic_records_match_bench_workloads():
    rec = _records()
    assert "c3" in rec and "c3_cached" in rec
    for key, e in rec.items():
        cfg = key[:-len("_cached")] if key.endswith("_cached") else key  # bench.py --base cached
        assert cfg in bench.CONFIGS, key
        assert e["workload"] == f"{cfg}: {bench.CONFIGS[cfg]['desc']}", key
        assert e["bytes_per_launch"] > 0


def test_pmc_traffic_reported_only_for_its_sources(tmp_path, monkeypatch):
    rec = _records()
    e = rec["c3"]
    w = e["workload"]
    want = e.get("calibrated_bytes_per_launch", e["bytes_per_launch"])
    got = bench.load_traffic("c3", w, e["zone_index"])
    assert got == (want if e.get("src_sha16") == bench.src_sha16() else None)
    # a record stamped with the current sources is reported, another stamp is not
    for stamp, expect in ((bench.src_sha16(), want), ("0" * 16, None), (None, None)):
        d = dict(rec)
        d["c3"] = dict(e, src_sha16=stamp)
        prof = tmp_path / "profiles"
        prof.mkdir(exist_ok=True)
        (prof / "pmc_traffic.json").write_text(json.dumps(d))
        monkeypatch.setattr(bench, "HERE", str(tmp_path))
        csrc = os.path.join(os.path.dirname(bench.__file__), "antidote_amd", "csrc")
        inc = os.path.join(os.path.dirname(bench.__file__), "include")
        for link, src in ((tmp_path / "antidote_amd" / "csrc", csrc), (tmp_path / "include", inc)):
            if not link.exists():
                link.parent.mkdir(exist_ok=True)
                link.symlink_to(src)
        assert bench.load_traffic("c3", w, e["zone_index"]) == expect, stamp
        monkeypatch.undo()
