#!/usr/bin/env python3
"""summary of scripts/ab_run.sh results: step and dominant-kernel ms per build and run"""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(os.path.basename(f), "unreadable", e)
        continue
    out = [os.path.basename(f)]
    if "ms_per_step" in j:
        w = j.get("config", {}).get("workload", "?")[:1]
        out.append(f"{w} step {j['ms_per_step']:.3f} k {j['roofline'].get('kernel_ms')}")
    if "decode" in j:
        out.append(f"D step {j['decode']['ms_per_step']:.3f} k {j['decode']['roofline'].get('kernel_ms')}")
    s = j.get("strains")
    if s:
        out.append(f"S step {s['ms_per_step']:.3f} k {s['roofline'].get('kernel_ms')}")
    print(" | ".join(out))
