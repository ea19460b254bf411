#!/usr/bin/env python3
"""rocprofv3 output of scripts/profile_bench.sh -> profiles/pmc_traffic.json + a markdown summary.

Per workload and kernel, the mean per launch of:
  read_bytes   = 32 * TCC_EA0_RDREQ_32B + 64 * TCC_EA0_RDREQ_64B + 128 * TCC_EA0_RDREQ_128B
                 (every L2->fabric read request at its own size; on gfx950 random 4..16 B loads
                 and streaming loads alike go out as 128 B requests -- the FETCH_SIZE half-count
                 the guide describes is those 128 B requests tallied at 64 B through TCC_BUBBLE = 0)
  write_bytes  = 32 * (TCC_EA0_WRREQ - TCC_EA0_WRREQ_64B) + 64 * TCC_EA0_WRREQ_64B (= WRITE_SIZE)
  dram_read_bytes = 32 * TCC_EA0_RDREQ_DRAM_32B
  fetch_size_bytes = the rocprofv3 FETCH_SIZE expression for gfx950 from the same counters
Kernel durations come from the kernel-trace pass of the default bench command, split into
its workloads by dispatch order (bench.py with --inflight I contexts):
  C91 encode calls: I (every context's outputs) + W + K (timed, I in flight) + N isolated
      (one at a time, I > 1 only: the roofline's denominator) + I (outputs refreshed)
  D91 decode calls: W + K (timed) + N isolated (I > 1 only)
  C31 encode calls (when the trace has them): as C91, after D91
  S91: 1 + W + K encode calls, SD91: W + K decode calls (one context)
avg_ns is the isolated launches' mean (the timed ones where I = 1); avg_ns_inflight the
timed launches' mean.

usage: pmc_traffic.py PROF_DIR OUT_JSON OUT_MD [--steps K --warmup W --reads R --read-len L]
"""
import argparse
import csv
import glob
import json
import os
import sys
import time
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

KERNELS = ("k_ms4", "k_parse4", "k_pack", "k_emit4", "k_dec_rec", "k_dec_tiles", "k_scan_apply", "k_scan_reduce",
           "k_tab_level", "k_walk_double", "k_walk_init", "k_walk_ext", "k_path")


def short(name):
    for k in KERNELS:
        if k in name:
            return k
    return name.split("(")[0][:40]


def rows(pattern):
    out = []
    for p in sorted(glob.glob(pattern, recursive=True)):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def per_dispatch(prof_dir, pass_name):
    """kernel -> list (dispatch order) of {counter: value}"""
    d = defaultdict(dict)
    names = {}
    for r in rows(os.path.join(prof_dir, pass_name, "**", "*counter_collection.csv")):
        did = int(r["Dispatch_Id"])
        d[did][r["Counter_Name"]] = d[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[did] = short(r["Kernel_Name"])
    out = defaultdict(list)
    for did in sorted(d):
        out[names[did]].append(d[did])
    return out


def mean(xs):
    return sum(xs) / len(xs) if xs else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("out_json")
    ap.add_argument("out_md")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--inflight", type=int, default=2, help="bench.py --inflight of the kernel-trace pass")
    ap.add_argument("--iso", type=int, default=3, help="isolated calls bench.py times after the timed region")
    ap.add_argument("--no-c31", dest="with_c31", action="store_false",
                    help="the kernel-trace pass ran without the C31 block (bench.py --configs without c31)")
    a = ap.parse_args()
    import ntcomp_amd as nt

    # ---- kernel durations per workload from the kernel trace of the default command ----
    kt = rows(os.path.join(a.prof_dir, "kt", "**", "*kernel_trace.csv"))
    if not kt:  # an incomplete profile must not replace the committed counters
        sys.exit(f"no kernel trace under {a.prof_dir}/kt: nothing written")
    kt.sort(key=lambda r: int(r["Start_Timestamp"]))
    seq = defaultdict(list)
    for r in kt:
        seq[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    I, WK = a.inflight, a.warmup + a.steps
    N = a.iso if I > 1 else 0
    c_total = I + WK + N + I
    dur = {"C91": {}, "D91": {}, "C31": {}, "S91": {}, "SD91": {}}
    inflight = {"C91": {}, "D91": {}, "C31": {}}
    n_c = 2 if a.with_c31 else 1  # C blocks before S91
    for kname in ("k_ms4", "k_parse4", "k_pack", "k_emit4"):
        xs = seq.get(kname, [])
        timed = xs[I:I + WK]
        dur["C91"][kname] = mean(xs[I + WK:I + WK + N]) if N else mean(timed)
        inflight["C91"][kname] = mean(timed)
        if a.with_c31:
            c = c_total
            dur["C31"][kname] = mean(xs[c + I + WK:c + I + WK + N]) if N else mean(xs[c + I:c + I + WK])
            inflight["C31"][kname] = mean(xs[c + I:c + I + WK])
        s0 = n_c * c_total + 1
        dur["S91"][kname] = mean(xs[s0:s0 + WK]) if len(xs) >= s0 + WK else None
    for kname in ("k_dec_rec", "k_dec_tiles"):
        xs = seq.get(kname, [])
        dur["D91"][kname] = mean(xs[WK:WK + N]) if N else mean(xs[:WK])
        inflight["D91"][kname] = mean(xs[:WK])
        dur["SD91"][kname] = mean(xs[WK + N:WK + N + WK]) if len(xs) >= WK + N + WK else None

    units = {"C91": (a.reads, "read"), "S91": (a.reads, "read"), "C31": (a.reads, "read"),
             "D91": (a.reads * a.read_len, "base"), "SD91": (a.reads * a.read_len, "base")}
    src = {"C91": ("encode", ("k_ms4", "k_parse4", "k_pack", "k_emit4")),
           "D91": ("decode", ("k_dec_rec", "k_dec_tiles")),
           "C31": ("c31", ("k_ms4", "k_parse4", "k_pack", "k_emit4")),
           "S91": ("strains", ("k_ms4", "k_parse4", "k_pack", "k_emit4")),
           "SD91": ("strains", ("k_dec_rec", "k_dec_tiles"))}
    out = {"device_source_hash": nt.device_source_hash(), "collected": time.strftime("%Y-%m-%d %H:%M"),
           "source": f"scripts/profile_bench.sh -> {os.path.relpath(a.prof_dir, REPO)}", "workloads": {}}
    md = ["# rocprofv3 summary (bench.py, one MI355X)", "",
          f"device source hash `{out['device_source_hash']}`; kernel-trace pass = `bench.py --steps {a.steps} "
          f"--warmup {a.warmup}` (all configs, --inflight {a.inflight}); counter passes = `bench.py --configs <w> --no-cpu --steps 3 "
          f"--warmup 0`, one pass per counter group.", "",
          "| workload | kernel | avg ms (trace) | read B/launch | write B/launch | B/unit | RDREQ/unit | 32/64/128 B req | "
          "DRAM rd B | L2 hit | GB/s | frac of 8 TB/s |", "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for wl, (wname, kernels) in src.items():
        rd = per_dispatch(a.prof_dir, f"pmc_rd_{wname}")
        wr = per_dispatch(a.prof_dir, f"pmc_wr_{wname}")
        mi = per_dispatch(a.prof_dir, f"pmc_misc_{wname}")
        u, un = units[wl]
        kd = {}
        for kname in kernels:
            R, W, M = rd.get(kname, []), wr.get(kname, []), mi.get(kname, [])
            if not R or not W:
                continue

            def m(lst, c):
                return mean([x[c] for x in lst if c in x])
            n32, n64, n128, nreq = (m(R, "TCC_EA0_RDREQ_32B_sum"), m(R, "TCC_EA0_RDREQ_64B_sum"),
                                    m(R, "TCC_EA0_RDREQ_128B_sum"), m(R, "TCC_EA0_RDREQ_sum"))
            wreq, w64 = m(W, "TCC_EA0_WRREQ_sum"), m(W, "TCC_EA0_WRREQ_64B_sum")
            dram32, bub = m(W, "TCC_EA0_RDREQ_DRAM_32B_sum"), m(W, "TCC_BUBBLE_sum")
            e = {"read_bytes": 32 * n32 + 64 * n64 + 128 * n128,
                 "write_bytes": 32 * (wreq - w64) + 64 * w64,
                 "rdreq": nreq, "rdreq_32b": n32, "rdreq_64b": n64, "rdreq_128b": n128,
                 "wrreq": wreq, "wrreq_64b": w64, "bubble": bub,
                 "dram_read_bytes": 32 * dram32 if dram32 is not None else None,
                 "fetch_size_bytes": (bub * 128 + (nreq - bub - n32) * 64 + n32 * 32) if bub is not None else None}
            if M:
                h, mm = m(M, "TCC_HIT_sum"), m(M, "TCC_MISS_sum")
                e["l2_hit_rate"] = h / (h + mm) if h is not None and mm and h + mm else None
                for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
                          "GRBM_GUI_ACTIVE"):
                    e[c] = m(M, c)
            ns = dur[wl].get(kname)
            if inflight.get(wl, {}).get(kname):
                e["avg_ns_inflight"] = inflight[wl][kname]
            if ns:
                e["avg_ns"] = ns
                if e.get("GRBM_GUI_ACTIVE"):
                    e["effective_clock_ghz"] = e["GRBM_GUI_ACTIVE"] / 8 / ns
            kd[kname] = e
            tb = e["read_bytes"] + e["write_bytes"]
            gbs = tb / ns if ns else None
            md.append(f"| {wl} | {kname} | {ns / 1e6 if ns else float('nan'):.4f} | {e['read_bytes']:.4g} | "
                      f"{e['write_bytes']:.4g} | {tb / u:.2f} | {nreq / u:.3f} | {n32:.3g}/{n64:.3g}/{n128:.3g} | "
                      f"{e['dram_read_bytes'] or 0:.4g} | {e.get('l2_hit_rate') or 0:.3f} | "
                      f"{gbs or 0:.0f} | {(gbs or 0) / 8000:.3f} |")
        out["workloads"][wl] = {"units_per_launch": u, "unit": un, "kernels": kd}
    stats = rows(os.path.join(a.prof_dir, "kt", "**", "*kernel_stats.csv"))
    md += ["", "rocprofv3 `--stats` (kernel_stats.csv of the kernel-trace pass, all workloads together):", "",
           "| kernel | calls | total ms | avg us | min us | max us | % |", "|---|---|---|---|---|---|---|"]
    for r in sorted(stats, key=lambda r: -float(r["TotalDurationNs"]))[:24]:
        md.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                  f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['MinNs']) / 1e3:.1f} | {float(r['MaxNs']) / 1e3:.1f} | "
                  f"{float(r['Percentage']):.1f} |")
    md += ["", "Per-workload trace averages (dispatch order split; C91/D91: isolated launches, the roofline's "
           "denominator):", "", "```json", json.dumps(dur, indent=1), "```", "",
           "C91/D91 timed launches with calls in flight (each shares the GPU with the other context's kernels):",
           "", "```json", json.dumps(inflight, indent=1), "```"]
    if not all(out["workloads"].get(w, {}).get("kernels") for w in ("C91", "D91")):
        sys.exit("counter passes missing for C91/D91: nothing written")
    json.dump(out, open(a.out_json, "w"), indent=1)
    open(a.out_md, "w").write("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main()
