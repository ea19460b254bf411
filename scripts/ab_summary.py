#!/usr/bin/env python3
"""Summarise scripts/ab_bench.sh output: per run, C91 / S91 value, ms/step and k_ms4 ms."""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except (ValueError, IndexError):
        print(os.path.basename(f), "no JSON line")
        continue
    row = [os.path.basename(f)]
    if "roofline" in j and j.get("config", {}).get("workload", "").startswith("C"):
        row.append(f"C91 {j['value'] / 1e3:.1f} G {j['ms_per_step']:.3f} ms k_ms4 {j['roofline'].get('kernel_ms')}")
    c = j.get("c31")
    if c:
        row.append(f"C31 {c['value'] / 1e3:.1f} G {c['ms_per_step']:.3f} ms k_ms4 {c['roofline'].get('kernel_ms')}")
    s = j.get("strains")
    if s:
        row.append(f"S91 {s['value'] / 1e3:.1f} G {s['ms_per_step']:.3f} ms k_ms4 {s['roofline'].get('kernel_ms')}")
    print("  ".join(row))
