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

  python scripts/big_build.py [--strains 600] [--snp-ppm 1000] [--budget-gb 0] [--reads 2000000]
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
    ap.add_argument("--reads", type=int, default=2_000_000)
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
        t = time.time()
        recs, rro = ctx.encode(reads, roffs)
        out["encode_s"] = round(time.time() - t, 3)
        out["records"] = int(len(recs))
        tm = ctx.timing()
        out["encode_kernel_ms"] = round(tm["total_ms"], 3)
        out["encode_gbases_per_s_kernel"] = round(n * L / tm["total_ms"] / 1e6, 2)
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
