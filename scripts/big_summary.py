#!/usr/bin/env python3
"""scripts/big_point.sh output -> one JSON record: the large-collection encode point (3.0 Gbp,
~177 M nodes, k = 31) with k_ms4's requests per read and roofline fraction, beside S91's from a
bench line.

usage: big_summary.py OUT_DIR RESULT_JSON [--bench BENCH_JSON]
"""
import argparse
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import per_dispatch, short  # noqa: E402

HBM = 8000.0


def mean(xs):
    return sum(xs) / len(xs) if xs else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir")
    ap.add_argument("result")
    ap.add_argument("--bench", help="a bench.py JSON line: S91's numbers go beside this point")
    a = ap.parse_args()
    pt = json.loads(open(os.path.join(a.out_dir, "point.json")).read().strip().splitlines()[-1])
    pt.setdefault("reps", 3)
    n = pt["reads"]
    rd = per_dispatch(a.out_dir, "pmc_rd")
    wr = per_dispatch(a.out_dir, "pmc_wr")
    kt = []
    for p in glob.glob(os.path.join(a.out_dir, "kt", "**", "*kernel_trace.csv"), recursive=True):
        kt += list(csv.DictReader(open(p)))
    dur = {}
    for r in kt:
        dur.setdefault(short(r["Kernel_Name"]), []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    kern = {}
    for k in ("k_ms4", "k_parse4", "k_pack", "k_emit4"):
        # the last dispatch of each pass is the timed call (the first call learns the pools and
        # may run twice); the kernel trace's last --reps dispatches are the timed ones
        c = pt.get("calls_per_rep", 1)
        r_, w_ = rd.get(k, [])[-c:], wr.get(k, [])[-c:]
        dur[k] = dur.get(k, [])[-pt.get("reps", 3) * c:]
        if not r_:
            continue
        # per call (mean over the rep's calls) x calls = per rep; n reads per rep
        rb = c * mean([32 * x.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * x.get("TCC_EA0_RDREQ_64B_sum", 0) +
                   128 * x.get("TCC_EA0_RDREQ_128B_sum", 0) for x in r_])
        rq = c * mean([x.get("TCC_EA0_RDREQ_sum", 0) for x in r_])
        wq = c * mean([x.get("TCC_EA0_WRREQ_sum", 0) for x in w_]) if w_ else None
        wb = c * mean([32 * (x.get("TCC_EA0_WRREQ_sum", 0) - x.get("TCC_EA0_WRREQ_64B_sum", 0)) +
                   64 * x.get("TCC_EA0_WRREQ_64B_sum", 0) for x in w_]) if w_ else 0
        ms = c * mean(dur.get(k, [])) / 1e6 if dur.get(k) else None
        e = {"avg_ms_trace": round(ms, 4) if ms else None, "read_requests_per_read": round(rq / n, 3),
             "write_requests_per_read": round(wq / n, 3) if wq is not None else None,
             "bytes_per_read": round((rb + wb) / n, 1)}
        if ms:
            e["achieved_gbs"] = round((rb + wb) / (ms / 1e3) / 1e9, 1)
            e["frac_of_8tbs"] = round(e["achieved_gbs"] / HBM, 4)
        kern[k] = e
    res = {"workload": f"L31: {n} x {pt['read_len']}bp reads (1% subst) drawn from a {pt['bases'] / 1e9:.2f} Gbp "
                       f"collection (the 5 Mbp genome + {pt['strains']} strains at {pt['snp_ppm'] / 1e4:g}% "
                       f"substitutions), SBWT k={pt['k']} (+revcomp)",
           "point": pt, "kernels": kern,
           "encode_gbases_per_s_kernel": pt.get("encode_gbases_per_s_kernel"),
           "note": "encode = one device call of all reads (kernel-only: ntc_last_timing, every kernel of the call); "
                   "counters: rocprofv3 PMC passes of the same command (scripts/big_point.sh), bytes past L2 at each "
                   "request's size"}
    if a.bench:
        b = json.loads(open(a.bench).read().strip().splitlines()[-1])
        s = b.get("strains") or {}
        rl = s.get("roofline") or {}
        res["s91_beside"] = {"value_mbases_s": s.get("value"), "ms_per_step": s.get("ms_per_step"),
                             "k_ms4_ms": rl.get("kernel_ms"), "frac": rl.get("frac"),
                             "read_requests_per_read": (rl.get("line_rate") or {}).get("read_requests_per_read"),
                             "index_nodes": (s.get("config") or {}).get("index_nodes")}
    with open(a.result, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
