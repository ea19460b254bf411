#!/usr/bin/env python3
"""One-line digest of bench.py JSON lines (A/B comparisons): encode / decode / strains values,
kernel times and roofline fractions."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        if not line.startswith("{"):
            continue
        j = json.loads(line)
        out = [path.split("/")[-1]]

        def add(tag, blk):
            if not blk or blk.get("value") is None:
                return
            r = blk.get("roofline") or {}
            out.append(f"{tag} {blk['value'] / 1e3:.1f} Gb/s k={r.get('kernel_ms')}ms frac={r.get('frac')}")
        add("enc", j)
        add("dec", j.get("decode"))
        s = j.get("strains") or {}
        add("S-enc", s)
        add("S-dec", s.get("decode"))
        par = [j.get("parity", {}).get("encode_bit_exact_all_ranks"),
               (j.get("decode") or {}).get("parity", {}).get("round_trip_exact_all_ranks"),
               s.get("parity", {}).get("encode_bit_exact_all_ranks")]
        out.append(f"parity {par}")
        print(" | ".join(out))
