#!/usr/bin/env python3
"""A strain collection past 2^32 k-mer occurrences, built on the GPU and used to encode.

The 5 Mbp synthetic genome plus S strains at R substitutions per million (default 600 x
0.1 %: 3.0 Gbp, 6.0 G k-mer occurrences with reverse complements at k = 31, about 0.2 G
nodes) -- the scale of ntcomp's intended use, a genome collection (README.md:2).  The GPU
build (ntc_build_index_device_ex, build.hip) runs in memory-bounded passes (-m/--mem-gb,
src/cli.rs:56-61: --budget-gb, default 85 % of the free HBM); no pass sorts 2^32 keys.
Then the index is uploaded, reads drawn from the whole collection are encoded on the GPU,
a sample is checked bit for bit against the C oracle (the checker), and every read is
decoded back.  Prints one JSON line (stats, timings, parity).

  python scripts/big_build.py [--strains 600] [--snp-ppm 1000] [--budget-gb 0] [--reads 10000000] [--reps 3]

The encode is timed with the library's HIP events (ntc_last_timing: every kernel of the call,
k_ms4 alone), one call of --reads reads per repetition, inputs in host memory (the call's H2D
is outside the kernels' span); rocprofv3 PMC passes over the same command
(scripts/big_point.sh) give k_ms4's requests per read.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402

import ntcomp_amd as nt  # noqa: E402


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--strains", type=int, default=600)
    ap.add_argument("--glen", type=int, default=5_000_000)
    ap.add_argument("--snp-ppm", type=int, default=1000)
    ap.add_argument("--k", type=int, default=31)
    ap.add_argument("--budget-gb", type=float, default=0)
    ap.add_argument("--host-budget-gb", type=float, default=0)
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch-reads", type=int, default=5_000_000,
                    help="reads per device call (10 M in one call ran out of its overflow pools after two re-runs)")
    ap.add_argument("--no-check", action="store_true", help="skip the oracle sample and the decode (PMC passes)")
    ap.add_argument("--sample", type=int, default=3000)
    ap.add_argument("--skip-encode", action="store_true")
    a = ap.parse_args()
    out = {"strains": a.strains, "glen": a.glen, "snp_ppm": a.snp_ppm, "k": a.k}
    t = time.time()
    genome = nt.synth_genome(1, a.glen)
    coll = np.empty((a.strains + 1) * a.glen, dtype=np.uint8)
    coll[:a.glen] = genome
    step = 50
    for s0 in range(0, a.strains, step):  # strains in slices (seed, s, i) -> same bases
        n = min(step, a.strains - s0)
        st = nt.synth_strains(genome, 1000 + s0, n, a.snp_ppm)
        coll[(1 + s0) * a.glen:(1 + s0 + n) * a.glen] = st.reshape(-1)
    offs = np.arange(0, (a.strains + 2) * a.glen, a.glen, dtype=np.uint64)
    out["bases"] = int(offs[-1])
    out["synth_s"] = round(time.time() - t, 2)
    log(f"collection: {out['bases'] / 1e9:.2f} Gbp in {out['synth_s']} s")
    ctx = nt.GpuContext(0)
    stats = {}
    t = time.time()
    ix = nt.Index.build_gpu(ctx, (coll, offs), a.k, device_budget=int(a.budget_gb * (1 << 30)),
                            host_budget=int(a.host_budget_gb * (1 << 30)), stats=stats)
    out["build_s"] = round(time.time() - t, 2)
    out["build"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in stats.items()}
    out["occurrences_over_2_32"] = stats["occurrences"] >= (1 << 32)
    log(f"build: {out['build_s']} s, {json.dumps(out['build'])}")
    if not a.skip_encode:
        t = time.time()
        ctx.upload(ix)
        out["upload_s"] = round(time.time() - t, 2)
        n, L = a.reads, 150
        reads = nt.synth_reads(coll, 2, 0, n, L, 10_000)
        roffs = np.arange(0, n * L + 1, L, dtype=np.uint64)
        out["reads"] = n
        out["read_len"] = L
        out["err_ppm"] = 10_000
        out["reps"] = max(1, a.reps)
        # device calls of --batch-reads reads (inputs resident in HBM, as bench.py's batches), all
        # timed with the library's HIP events and summed per repetition; a first pass learns the
        # overflow pools
        nb = a.batch_reads or n
        spans = [(s0, min(n, s0 + nb)) for s0 in range(0, n, nb)]
        bufs = []
        for s0, s1 in spans:
            m = s1 - s0
            cap = m * L // 4 + 64
            o = np.arange(0, m * L + 1, L, dtype=np.uint64)
            d = {"b": ctx.alloc(m * L), "o": ctx.alloc(o.nbytes), "r": ctx.alloc(cap * 8), "ro": ctx.alloc(o.nbytes),
                 "n": m, "cap": cap}
            ctx.h2d(d["b"], reads[s0 * L:s1 * L])
            ctx.h2d(d["o"], o)
            bufs.append(d)
        tot, main = [], []
        for rep in range(max(1, a.reps) + 1):
            t = time.time()
            tt = mm = 0.0
            for d in bufs:
                ctx.encode_device(d["b"], d["o"], d["n"], L, d["r"], d["cap"], d["ro"])
                d["nrec"] = ctx.encode_status()
                tm = ctx.timing()
                tt += tm["total_ms"]
                mm += tm["main_ms"]
            out["encode_s"] = round(time.time() - t, 3)
            if rep:
                tot.append(tt)
                main.append(mm)
        rl, ro_l, base = [], [np.zeros(1, np.uint64)], 0
        for d in bufs:
            ro = ctx.d2h(np.zeros(d["n"] + 1, dtype=np.uint64), d["ro"])
            rl.append(ctx.d2h(np.zeros(d["nrec"], dtype=np.uint64), d["r"]))
            ro_l.append(ro[1:] + base)
            base += d["nrec"]
            for key in ("b", "o", "r", "ro"):
                ctx.free(d[key])
        recs, rro = np.concatenate(rl), np.concatenate(ro_l)
        out["batch_reads"] = nb
        out["calls_per_rep"] = len(bufs)
        out["spill_reruns"] = ctx.get_option("spill_reruns")
        out["records"] = int(len(recs))
        out["records_per_read"] = round(len(recs) / n, 3)
        out["encode_kernel_ms"] = round(sum(tot) / len(tot), 3)
        out["encode_kernel_ms_all"] = [round(x, 3) for x in tot]
        out["k_ms4_ms"] = round(sum(main) / len(main), 3)
        out["encode_gbases_per_s_kernel"] = round(n * L / out["encode_kernel_ms"] / 1e6, 2)
        out["suffix_table_u"] = ctx.get_option("tab_u")
        out["n_paths"] = ctx.get_option("n_paths")
        out["joint_runs"] = bool(ctx.get_option("joint"))
        if a.no_check:
            ctx.close()
            print(json.dumps(out), flush=True)
            return
        from oracle_lib import OracleIndex
        m = a.sample
        t = time.time()
        exp, eoff = OracleIndex(ix.n, a.k, ix.rows, ix.C, ix.lcs).encode(reads[:m * L], roffs[:m + 1])
        out["oracle_sample_s"] = round(time.time() - t, 2)
        out["parity_sample_reads"] = m
        out["parity_bit_exact"] = bool(np.array_equal(recs[:int(eoff[m])], exp) and
                                       np.array_equal(rro[:m + 1], eoff))
        dec, do = ctx.decode(recs)
        out["round_trip_exact"] = bool(np.array_equal(dec, reads) and np.array_equal(do, roffs))
    ctx.close()
    print(json.dumps(out), flush=True)
    ok = out.get("parity_bit_exact", True) and out.get("round_trip_exact", True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
