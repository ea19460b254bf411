#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output of scripts/profile_encode.sh into a markdown table and
profiles/pmc_traffic.json (HBM bytes per launch, gfx950 FETCH_SIZE correction applied).

FETCH_SIZE / WRITE_SIZE are in KiB.  MI355X_MICROARCH.md "HBM": on gfx950 FETCH_SIZE
reports exactly half the bytes of wide coalesced streaming reads, so the read side is
doubled; WRITE_SIZE is taken as reported.  Other access widths are uncalibrated: the
number is the guide's prescribed correction, reported as such."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(path_glob):
    out = []
    for p in glob.glob(path_glob, recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def short(name):
    for k in ("k_encode", "k_ms4", "k_parse4", "k_pack", "k_emit4", "k_dec_rec", "k_emit", "k_scan_apply",
              "k_scan_reduce", "k_dec_tiles", "k_dec_reduce", "k_dec_apply", "k_dec_expand", "k_walk_double", "k_walk_init", "k_tile_rows", "k_tab_level",
              "k_tab_bits"):
        if k in name:
            return k
    return name[:40]


def main(prof_dir, out_md, out_json):
    lines = []
    stats = rows(os.path.join(prof_dir, "kt", "**", "*kernel_stats.csv"))
    lines.append("| kernel | calls | total ms | avg us | min us | max us | % |")
    lines.append("|---|---|---|---|---|---|---|")
    avg_ns = {}
    for r in sorted(stats, key=lambda r: -float(r["TotalDurationNs"])):
        nm = short(r["Name"])
        avg_ns[nm] = float(r["AverageNs"])
        lines.append(f"| {nm} | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.2f} | {float(r['AverageNs'])/1e3:.1f} | "
                     f"{float(r['MinNs'])/1e3:.1f} | {float(r['MaxNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |")
    per = defaultdict(lambda: defaultdict(list))
    for name in ("pmc_fetch", "pmc_write", "pmc_tcc", "pmc_sq", "pmc_grbm"):
        for r in rows(os.path.join(prof_dir, name, "**", "*counter_collection.csv")):
            per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    lines.append("")
    lines.append("| kernel | counter | mean per launch |")
    lines.append("|---|---|---|")
    traffic = {}
    for k, cs in per.items():
        for c, vals in sorted(cs.items()):
            lines.append(f"| {k} | {c} | {sum(vals)/len(vals):.4g} |")
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024
            w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
            traffic[k] = {"fetch_bytes_reported": f, "write_bytes": w,
                          "hbm_bytes_per_launch": 2 * f + w,
                          "note": "2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE half-count correction)"}
            if "TCC_EA0_RDREQ_sum" in cs:
                traffic[k]["ea_rdreq_per_launch"] = sum(cs["TCC_EA0_RDREQ_sum"]) / len(cs["TCC_EA0_RDREQ_sum"])
            if "TCC_HIT_sum" in cs:
                h, m = sum(cs["TCC_HIT_sum"]), sum(cs["TCC_MISS_sum"])
                traffic[k]["l2_hit_rate"] = h / (h + m) if h + m else None
            if "GRBM_GUI_ACTIVE" in cs and k in avg_ns:
                g = sum(cs["GRBM_GUI_ACTIVE"]) / len(cs["GRBM_GUI_ACTIVE"])
                traffic[k]["effective_clock_ghz"] = g / 8 / avg_ns[k]
            if k in avg_ns:
                traffic[k]["avg_duration_ns"] = avg_ns[k]
    lines.append("")
    lines.append("```json")
    lines.append(json.dumps(traffic, indent=1))
    lines.append("```")
    open(out_md, "w").write("\n".join(lines) + "\n")
    if out_json:
        json.dump(traffic, open(out_json, "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
