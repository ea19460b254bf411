"""Encode workspace sized by need (capi.cpp encode4_impl): per read 4 dense + S secondary
entry slots and 8 record slots, the rest in overflow pools reserved by the reads that need
them (MsLaneT::reserve, parse_read's RecPool).  A call that runs out of a pool is re-run with
the pools grown when its status is read; its records must equal the oracle's like any other
call (lib.rs:163-230, encode.rs:129-166).  Sizes are checked against the round-2 verdict's
bound: <= 15 GB of workspace per 10 M reads of C91."""
import numpy as np
import pytest

import ntcomp_amd as nt
from oracle_lib import OracleIndex

pytestmark = pytest.mark.gpu


def _collection(glen, strains, seed=1):
    genome = nt.synth_genome(seed, glen)
    st = nt.synth_strains(genome, 3, strains, 10_000)
    return [genome] + [st[i] for i in range(strains)]


def test_pools_rerun_on_a_strain_collection():
    """Joint-run index (most reads spill past 4 entries): with 4 secondary slots and empty
    pools the call re-runs, on the host and the device API, with records identical to the
    default sizing and to the oracle."""
    texts = _collection(1_000_000, 3)
    ix = nt.Index.build([t.tobytes() for t in texts], 91)
    coll = np.concatenate(texts)
    n, L = 60_000, 150
    reads = nt.synth_reads(coll, 5, 0, n, L, 10_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    ref = nt.GpuContext(0)
    ref.upload(ix)
    assert ref.get_option("joint") == 1 and ref.get_option("ent_slots") == 16
    exp, eoff = ref.encode(reads, offs)
    orc = OracleIndex(ix.n, 91, ix.rows, ix.C, ix.lcs)
    m = 3000
    oexp, _ = orc.encode(reads[:m * L], offs[:m + 1])
    assert np.array_equal(exp[:int(eoff[m])], oexp)
    ctx = nt.GpuContext(0)
    ctx.set_option("ent_slots", 4)
    ctx.set_option("pool_per_read", 0)
    ctx.upload(ix)
    got, goff = ctx.encode(reads, offs)
    assert ctx.get_option("spill_reruns") >= 1
    assert np.array_equal(goff, eoff) and np.array_equal(got, exp)
    # device API: the re-run happens inside encode_status
    ctx.set_option("pool_per_read", 0)
    before = ctx.get_option("spill_reruns")
    db, do = ctx.alloc(reads.nbytes), ctx.alloc(offs.nbytes)
    dr, dro = ctx.alloc(len(exp) * 8 + 64), ctx.alloc(offs.nbytes)
    try:
        ctx.h2d(db, reads)
        ctx.h2d(do, offs)
        ctx.encode_device(db, do, n, L, dr, len(exp) + 8, dro)
        assert ctx.encode_status() == len(exp)
        assert ctx.get_option("spill_reruns") == before + 1
        assert np.array_equal(ctx.d2h(np.zeros(len(exp), dtype=np.uint64), dr), exp)
    finally:
        for p in (db, do, dr, dro):
            ctx.free(p)
    # a second call of the same size needs no re-run: the pools remember the per-read need
    got2, _ = ctx.encode(reads, offs)
    assert np.array_equal(got2, exp) and ctx.get_option("spill_reruns") == before + 1
    for c in (ref, ctx):
        c.close()


def test_record_pool_rerun_on_long_reads():
    """Reads of 5-20 kb at k = 31 with 2 % errors: hundreds of records per read, all past the
    8 dense slots go to the record pool; empty pools force a re-run."""
    genome = nt.synth_genome(17, 300_000)
    ix = nt.Index.build([genome.tobytes()], 31)
    rng = np.random.default_rng(4)
    g = genome.tobytes()
    reads = []
    for _ in range(60):
        L = int(rng.integers(5_000, 20_000))
        st = int(rng.integers(0, len(g) - L))
        s = bytearray(g[st:st + L])
        for _ in range(L // 50):
            s[int(rng.integers(0, L))] = b"ACGT"[int(rng.integers(0, 4))]
        reads.append(bytes(s))
    offs = np.zeros(len(reads) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(r) for r in reads])
    bases = np.frombuffer(b"".join(reads), dtype=np.uint8)
    exp, eoff = OracleIndex(ix.n, 31, ix.rows, ix.C, ix.lcs).encode(bases, offs)
    assert max(np.diff(eoff)) > 100
    ctx = nt.GpuContext(0)
    ctx.set_option("pool_per_read", 0)
    ctx.upload(ix)
    got, goff = ctx.encode(bases, offs)
    assert ctx.get_option("spill_reruns") >= 1
    assert np.array_equal(goff, eoff) and np.array_equal(got, exp)
    out, o2 = ctx.decode(got)
    assert np.array_equal(out, bases)
    # the pools a later batch of short reads gets follow its own bases, not the long reads'
    # per-read need (rates are learned per base from the latest call)
    n, L = 20_000, 150
    short = nt.synth_reads(genome, 6, 0, n, L, 10_000)
    soffs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    sexp, _ = OracleIndex(ix.n, 31, ix.rows, ix.C, ix.lcs).encode(short[:2000 * L], soffs[:2001])
    sgot, _ = ctx.encode(short, soffs)
    assert np.array_equal(sgot[:len(sexp)], sexp)
    assert ctx.get_option("pool_entries") <= n * L + 4 * n + 4096
    assert ctx.get_option("pool_records") <= n * L + 4 * n + 4096
    ctx.close()


def test_c91_workspace_per_read():
    """C91-shaped batch (150 bp, 1 % errors, k = 91): the context's whole device workspace
    after one call stays far under the 1.5 kB per read (15 GB per 10 M reads) bound."""
    genome = nt.synth_genome(1, 5_000_000)
    ix = nt.Index.build([genome.tobytes()], 91)
    ctx = nt.GpuContext(0)
    ctx.upload(ix)
    n, L = 2_000_000, 150
    reads = nt.synth_reads(genome, 2, 0, n, L, 10_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    db, do = ctx.alloc(reads.nbytes), ctx.alloc(offs.nbytes)
    cap = n * 8
    dr, dro = ctx.alloc(cap * 8), ctx.alloc(offs.nbytes)
    try:
        ctx.h2d(db, reads)
        ctx.h2d(do, offs)
        ctx.encode_device(db, do, n, L, dr, cap, dro)
        nrec = ctx.encode_status()
        assert ctx.get_option("spill_reruns") == 0
        ws = ctx.get_option("workspace_bytes")
        assert ws / n < 600, ws / n
        recs = ctx.d2h(np.zeros(nrec, dtype=np.uint64), dr)
        orc = OracleIndex(ix.n, 91, ix.rows, ix.C, ix.lcs)
        m = 2000
        exp, eoff = orc.encode(reads[:m * L], offs[:m + 1])
        assert np.array_equal(recs[:int(eoff[m])], exp)
    finally:
        for p in (db, do, dr, dro):
            ctx.free(p)
    ctx.close()
