#!/usr/bin/env python3
"""Markdown rows for BASELINE.md / DESIGN.md from bench.py JSON lines:
   python scripts/baseline_table.py profiles/r04/final/bench_c3.json ...  (one JSON line per file)"""
import json
import sys

print("| config | workload per GPU | ms / step (median HIP-event step) | G ops/s | layout bytes / launch | frac (layout) | "
      "logical bytes / launch | frac (logical) | PMC traffic / layout | CPU 1 thread | CPU threads |")
print("|---|---|---|---|---|---|---|---|---|---|---|")
for f in sys.argv[1:]:
    line = [l for l in open(f) if l.startswith("{")][-1]
    d = json.loads(line)
    rf, cb = d["roofline"], d.get("cpu_baseline") or {}
    lg = rf.get("logical", {})
    step = d.get("step_ms_hip_events", {}).get("median")
    tr = rf.get("traffic")
    tr_ratio = f"{tr / rf['alg_bytes_per_launch']:.2f}" if tr else "—"
    st = cb.get("single_thread") or {}
    print(f"| {d['config']['workload'].split(':')[0]} | {d['config']['workload'].split(': ', 1)[1][:60]} | "
          f"{d['ms_per_step']:.2f} ({step:.2f}) | {d['value'] / 1e9:.1f} | {rf['alg_bytes_per_launch'] / 1e9:.2f} GB | "
          f"{rf['frac']:.3f} | {lg.get('bytes_per_launch', 0) / 1e9:.2f} GB | {lg.get('frac_of_peak', 0):.3f} | "
          f"{tr_ratio} | {st.get('value', 0) / 1e6:.1f} M {cb.get('unit', '')} | "
          f"{cb.get('value', 0) / 1e6:.1f} M ({cb.get('cores', '—')} thr) |")
