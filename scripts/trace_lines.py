#!/usr/bin/env python3
"""Per-read cache-line footprint of the encode lanes (k_ms4 / k_parse4 logic), on the CPU.

Runs the kernels' lane functions through the TEST-ONLY emulator built with -DNTC_TRACE
(tests/emu libntc_emu_trace.so) and prints, per phase and per structure, the loads and the
distinct 128-byte lines each read touches.  Distinct lines per read approximate the L2
misses of a structure far larger than L2 (suffix table, bitmaps, colex_at, ...).

usage: python scripts/trace_lines.py [--genome-bp 5000000] [--k 91] [--reads 20000] [--err-ppm 10000]
"""
import argparse
import ctypes
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

KINDS = ["rank", "lcs", "uniq", "tabU", "tabLo", "bits", "filt", "colex", "pos_of_node", "pstream", "Q", "E",
         "puniq", "E-store"]


def minimizer_order(reads, n, L, w=20):
    """read order grouped by each read's minimizer (smallest hashed w-mer, strand as read)"""
    codes = ((reads.reshape(n, L).astype(np.uint64) >> np.uint64(1)) ^ (reads.reshape(n, L).astype(np.uint64) >> np.uint64(2))) & np.uint64(3)
    v = np.zeros((n, L - w + 1), dtype=np.uint64)
    for i in range(w):
        v = (v << np.uint64(2)) | codes[:, i:i + L - w + 1]
    h = (v * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(20)
    return np.argsort(h.min(axis=1), kind="stable")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genome-bp", type=int, default=5_000_000)
    ap.add_argument("--k", type=int, default=91)
    ap.add_argument("--reads", type=int, default=20_000)
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--err-ppm", type=int, default=10_000)
    ap.add_argument("--tab-u", type=int, default=0)
    ap.add_argument("--strains", type=int, default=0, help="index a collection: the genome + N strains")
    ap.add_argument("--snp-ppm", type=int, default=10_000)
    ap.add_argument("--group", type=int, default=1, help="count distinct lines per this many consecutive reads")
    ap.add_argument("--order", choices=["input", "minimizer"], default="input",
                    help="process reads as generated, or grouped by their minimizer (locality experiment)")
    ap.add_argument("--json", help="merge this workload's lines per read into this JSON file "
                                   "(profiles/algorithmic_lines.json, read by bench.py)")
    ap.add_argument("--label", help="workload key in --json (C91, C31, S91)")
    ap.add_argument("--waves", action="store_true",
                    help="also run one 64-lane wave in lock step (emu_wave_modes): iterations and steps per read")
    args = ap.parse_args()
    so = os.path.join(REPO, "tests", "emu", "libntc_emu_trace.so")
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "tests", "emu"), "libntc_emu_trace.so"])
    import emu_lib
    import ntcomp_amd as nt

    emu_lib.EMU_SO = so
    L = emu_lib.emu_lib()
    L.emu_trace_report.argtypes = [ctypes.c_void_p]
    L.emu_trace_overlap.argtypes = [ctypes.c_void_p]
    genome = nt.synth_genome(1, args.genome_bp)
    texts = [genome]
    if args.strains:
        st = nt.synth_strains(genome, 3, args.strains, args.snp_ppm)
        texts += [st[i] for i in range(args.strains)]
    ix = nt.Index.build([t.tobytes() for t in texts], args.k, threads=8)
    reads = nt.synth_reads(np.concatenate(texts), 2, 0, args.reads, args.read_len, args.err_ppm)
    if args.order == "minimizer":
        reads = reads.reshape(args.reads, args.read_len)[minimizer_order(reads, args.reads, args.read_len)].ravel()
    os.environ["NTC_TRACE_GROUP"] = str(args.group)
    offs = np.arange(0, args.reads * args.read_len + 1, args.read_len, dtype=np.uint64)
    recs, _ = emu_lib.emu_encode(ix.n, args.k, ix.rows, ix.C, ix.lcs, reads, offs, tab_u=args.tab_u)
    K = len(KINDS)
    out = np.zeros(1 + 4 * K, dtype=np.uint64)
    ov = np.zeros(K, dtype=np.uint64)
    L.emu_trace_report(out.ctypes.data)
    L.emu_trace_overlap(ov.ctypes.data)
    stp = np.zeros(K, dtype=np.uint64)
    L.emu_trace_steps.argtypes = [ctypes.c_void_p]
    L.emu_trace_steps(stp.ctypes.data)
    st = np.zeros(16, dtype=np.uint64)
    L.emu_stats.argtypes = [ctypes.c_void_p]
    L.emu_stats(st.ctypes.data)
    n = int(out[0])
    req = out[1:1 + 2 * K].reshape(2, K) / n
    lines = out[1 + 2 * K:].reshape(2, K) / n
    print(f"reads {n}, records/read {len(recs) / n:.2f}, k={args.k}, err_ppm={args.err_ppm}, "
          f"order {args.order}, lines counted per {args.group} reads")
    for ph, name in enumerate(["ms", "parse"]):
        print(f"-- {name}: loads/read {req[ph].sum():.2f}, lines/read {lines[ph].sum():.2f}"
              + (f", lines distinct per step (no L2 reuse across steps) {stp.sum() / n:.2f}" if ph == 0 else ""))
        for i in np.argsort(-lines[ph]):
            if req[ph][i] > 0:
                extra = f"  (also touched by ms: {ov[i] / n:5.2f})" if ph == 1 else f"  per step {stp[i] / n:6.2f}"
                print(f"   {KINDS[i]:12s} loads {req[ph][i]:7.2f}  lines {lines[ph][i]:6.2f}{extra}")
    if args.json:
        import hashlib
        import json
        core = os.path.join(REPO, "ntcomp_amd", "csrc", "encode_core.h")
        try:
            with open(args.json) as f:
                j = json.load(f)
        except (OSError, ValueError):
            j = {}
        j["note"] = ("distinct 128-byte lines each read touches in the encode lanes (tests/emu emulator of "
                     "encode_core.h, NTC_TRACE), per kernel phase: the algorithmic traffic of this design, "
                     "scripts/trace_lines.py --json")
        j.setdefault("workloads", {})[args.label] = {
            "encode_core_sha256": hashlib.sha256(open(core, "rb").read()).hexdigest()[:16],
            "reads": n, "k": args.k, "genome_bp": args.genome_bp, "strains": args.strains,
            "err_ppm": args.err_ppm, "records_per_read": round(len(recs) / n, 4),
            "k_ms4_lines_per_read": round(float(lines[0].sum()), 4),
            "k_ms4_step_lines_per_read": round(float(stp.sum()) / n, 4),
            "k_parse4_lines_per_read": round(float(lines[1].sum()), 4),
            "k_ms4_by_structure": {KINDS[i]: round(float(lines[0][i]), 4) for i in range(K) if lines[0][i] > 0},
            "k_parse4_by_structure": {KINDS[i]: round(float(lines[1][i]), 4) for i in range(K) if lines[1][i] > 0}}
        with open(args.json, "w") as f:
            json.dump(j, f, indent=1, sort_keys=True)
    if st.any():  # NTC_STAT counters of the MS lanes (encode_core.h), per read
        print("-- unit counters per read: " + ", ".join(f"[{i}] {st[i] / n:.2f}" for i in range(16) if st[i]))
    if args.waves:
        w = emu_lib.emu_wave_modes(ix.n, args.k, ix.rows, ix.C, ix.lcs, reads, offs)
        modes = ["Scan", "Ext", "P1", "Bs", "Brk", "First", "Enter", "BrkLong", "ExtFail", "run"]
        nr = args.reads
        print(f"-- wave (64 lanes, lock step): iterations per 64 reads {64 * w[0] / nr:.2f}, "
              f"lane steps per read {w[2] / nr:.2f}, distinct modes per iteration {w[1] / max(w[0], 1):.2f}")
        print("   steps per read: " + ", ".join(f"{m} {w[3 + i] / nr:.2f}" for i, m in enumerate(modes) if w[3 + i]))


if __name__ == "__main__":
    main()
