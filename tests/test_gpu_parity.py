"""GPU parity: the HIP kernels (through the C ABI of libntcomp_gpu.so) against the golden
vectors and the faithful CPU oracle on the same seeded inputs; bit-exact records and
decoded bases; error behaviour; size-independent properties at full scale."""
import numpy as np
import pytest

import ntcomp_amd as nt
from oracle_lib import OracleIndex, golden_names, load_golden, pack_reads

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = nt.GpuContext(0)
    yield c
    c.close()


@pytest.mark.parametrize("name", golden_names())
def test_gpu_golden_records_ms_decode(ctx, name):
    g = load_golden(name)
    ctx.upload_arrays(g["n"], g["k"], g["rows_u64"], g["C"], g["lcs_u8"])
    bases, offs = pack_reads(g["reads"])
    recs, roff = ctx.encode(bases, offs)
    assert recs.tolist() == [w for r in g["records"] for w in r]
    assert np.diff(roff).tolist() == [len(r) for r in g["records"]]
    d, s = ctx.matching_statistics(bases, offs)
    exp = np.array([x for r in g["ms"] for x in r], dtype=np.uint64).reshape(-1, 2)
    assert np.array_equal(d.astype(np.uint64), exp[:, 0])
    assert np.array_equal(s.astype(np.uint64), exp[:, 1])
    out, o2 = ctx.decode(recs)
    assert [out[o2[i]:o2[i + 1]].tobytes().decode() for i in range(len(o2) - 1)] == g["reads"]


@pytest.mark.parametrize("variant", [4, 1])
@pytest.mark.parametrize("k,err_ppm,glen", [(31, 10_000, 400_000), (91, 10_000, 400_000), (91, 0, 400_000),
                                             (15, 30_000, 200_000), (255, 5_000, 100_000), (11, 10_000, 100_000)])
def test_gpu_matches_oracle_random(ctx, k, err_ppm, glen, variant):
    genome = nt.synth_genome(1000 + k, glen)
    ix = nt.Index.build([genome.tobytes()], k)
    ctx.upload(ix)
    ctx.set_option("encode_variant", variant)
    L = 150 if k < 200 else 400
    n = 4000
    reads = nt.synth_reads(genome, 77, 0, n, L, err_ppm)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    orc = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs)
    exp, eoff = orc.encode(reads, offs)
    got, goff = ctx.encode(reads, offs)
    assert np.array_equal(goff, eoff)
    assert np.array_equal(got, exp)
    out, o2 = ctx.decode(got)
    assert np.array_equal(out, reads)
    assert np.array_equal(o2, offs)
    ctx.set_option("encode_variant", 4)


def test_gpu_v2_repetitive_genome_and_ms(ctx):
    rng = np.random.default_rng(5)
    unit = nt.synth_genome(21, 400).tobytes()
    parts = []
    for _ in range(200):
        u = bytearray(unit)
        for _ in range(3):
            u[int(rng.integers(0, len(u)))] = b"ACGT"[int(rng.integers(0, 4))]
        parts.append(bytes(u) + nt.synth_genome(int(rng.integers(1, 1 << 30)), 97).tobytes())
    genome = np.frombuffer(b"".join(parts), dtype=np.uint8)
    for k, variant, joint in ((31, 4, 1), (91, 4, 1), (91, 4, 0), (91, 1, -1)):
        ix = nt.Index.build([genome.tobytes()], k)
        ctx.set_option("joint", joint)  # repeats: multi-node intervals, joint path runs on and off
        ctx.upload(ix)
        ctx.set_option("encode_variant", variant)
        assert ctx.get_option("n_paths") > 0
        reads = nt.synth_reads(genome, 8, 0, 5000, 150, 10_000)
        offs = np.arange(0, 5000 * 150 + 1, 150, dtype=np.uint64)
        orc = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs)
        exp, eoff = orc.encode(reads, offs)
        got, goff = ctx.encode(reads, offs)
        assert np.array_equal(goff, eoff) and np.array_equal(got, exp)
        d, s = ctx.matching_statistics(reads[:300 * 150], offs[:301])
        for r in range(0, 300, 7):
            od, olo = orc.ms(reads[r * 150:(r + 1) * 150].tobytes())
            assert np.array_equal(d[r * 150:(r + 1) * 150], od)
            assert np.array_equal(s[r * 150:(r + 1) * 150].astype(np.uint64), olo)
    ctx.set_option("encode_variant", 4)
    ctx.set_option("joint", -1)


def test_gpu_ragged_and_edge_lengths(ctx):
    genome = nt.synth_genome(5, 200_000)
    k = 31
    ix = nt.Index.build([genome.tobytes()], k)
    ctx.upload(ix)
    rng = np.random.default_rng(3)
    g = genome.tobytes()
    reads = []
    for L in [1, 2, 11, 12, 30, 31, 32, 33, 34, 63, 64, 65, 150, 151, 1000, 5000]:
        st = int(rng.integers(0, len(g) - L))
        reads.append(g[st:st + L])
    reads += [bytes(rng.choice(list(b"ACGT"), size=int(rng.integers(1, 400))).tolist()) for _ in range(300)]
    bases, offs = pack_reads(reads)
    orc = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs)
    exp, eoff = orc.encode(bases, offs)
    got, goff = ctx.encode(bases, offs)
    assert np.array_equal(goff, eoff) and np.array_equal(got, exp)
    out, o2 = ctx.decode(got)
    assert np.array_equal(out, bases) and np.array_equal(o2, offs)


def test_gpu_device_api_matches_host_api(ctx):
    genome = nt.synth_genome(9, 300_000)
    ix = nt.Index.build([genome.tobytes()], 91)
    ctx.upload(ix)
    n, L = 20_000, 150
    reads = nt.synth_reads(genome, 4, 0, n, L, 10_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    exp, eoff = ctx.encode(reads, offs)
    db, do = ctx.alloc(reads.nbytes), ctx.alloc(offs.nbytes)
    dr, dro = ctx.alloc(n * L * 8), ctx.alloc(offs.nbytes)
    try:
        ctx.h2d(db, reads)
        ctx.h2d(do, offs)
        for max_len in (150, 0):
            ctx.encode_device(db, do, n, max_len, dr, n * L, dro)
            nrec = ctx.encode_status()
            assert nrec == len(exp)
            got = ctx.d2h(np.zeros(nrec, dtype=np.uint64), dr)
            gro = ctx.d2h(np.zeros(n + 1, dtype=np.uint64), dro)
            assert np.array_equal(got, exp) and np.array_equal(gro, eoff)
        dout, doffs = ctx.alloc(n * L), ctx.alloc((n + 1) * 8)
        ctx.decode_device(dr, len(exp), dout, n * L, doffs, n + 1)
        assert ctx.decode_status() == (n, n * L)
        out = ctx.d2h(np.zeros(n * L, dtype=np.uint8), dout)
        assert np.array_equal(out, reads)
        t = ctx.timing()
        assert t["main_ms"] > 0
        ctx.free(dout)
        ctx.free(doffs)
    finally:
        for p in (db, do, dr, dro):
            ctx.free(p)


def test_gpu_error_behaviour(ctx):
    genome = nt.synth_genome(11, 50_000)
    ix = nt.Index.build([genome.tobytes()], 31)
    ctx.upload(ix)
    good = genome[100:250].tobytes()
    for bad_read, code in ((b"", 3), (good[:50] + b"N" + good[51:], 2), (good[:10] + b"a" + good[11:], 2)):
        bases, offs = pack_reads([good, good, bad_read, good])
        with pytest.raises(nt.NtcError) as e:
            ctx.encode(bases, offs)
        assert e.value.code == code
        assert e.value.bad_read == 2
    # decode: records that do not start with a read's first record
    recs, _ = ctx.encode(*pack_reads([good, good]))
    with pytest.raises(nt.NtcError) as e:
        ctx.decode(recs[1:])
    assert e.value.code == 8


def test_gpu_index_without_a_base():
    # an index whose genome lacks 'T' entirely: any read with T must be rejected, not hang
    ix = nt.Index.build(["ACGACGGACCAGACGAGGCAACGAGCACCGA" * 3], 7, add_revcomp=False)
    ctx = nt.GpuContext(0)
    ctx.upload(ix)
    with pytest.raises(nt.NtcError) as e:
        ctx.encode(*pack_reads(["CGGACCAGACGAGGCAACGA", "ACGT"]))  # not "ACGACGGAC": a reference panic
    assert e.value.code == 2 and e.value.bad_read == 1
    ctx.close()


@pytest.mark.parametrize("k", [91, 31])
def test_gpu_full_scale_roundtrip(k):
    """BASELINE configs C91 and C31: the 5 Mbp index at k with 1M reads: decode(encode(x))
    == x for every read, and a 20k-read sample bit-exact against the oracle."""
    genome = nt.synth_genome(1, 5_000_000)
    ix = nt.Index.build([genome.tobytes()], k)
    ctx = nt.GpuContext(0)
    ctx.upload(ix)
    n, L = 1_000_000, 150
    reads = nt.synth_reads(genome, 2, 0, n, L, 10_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    recs, roff = ctx.encode(reads, offs)
    out, o2 = ctx.decode(recs)
    assert np.array_equal(out, reads)
    orc = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs)
    m = 20_000
    exp, eoff = orc.encode(reads[: m * L], offs[: m + 1])
    assert np.array_equal(recs[: int(roff[m])], exp)
    ctx.close()


@pytest.mark.parametrize("ext2,joint", [(0, -1), (1, -1), (0, 0)])
def test_gpu_strain_collection(ext2, joint):
    """An index of a genome + 3 strains at 1 % substitutions (fragmented path cover, many
    branching nodes): 300k reads from the collection round-trip exactly, 10k bit-exact vs
    the oracle (bench.py's S91 config at reduced size); also with the two-character rank
    chunks (ctx option ext2), and without joint path runs (ctx option joint; auto turns
    them on for this cover).  (d, S) of every position of a read sample equals the
    oracle's matching statistics."""
    genome = nt.synth_genome(1, 2_000_000)
    strains = nt.synth_strains(genome, 3, 3, 10_000)
    texts = [genome] + [strains[i] for i in range(3)]
    ix = nt.Index.build([t.tobytes() for t in texts], 91)
    ctx = nt.GpuContext(0)
    ctx.set_option("ext2", ext2)
    ctx.set_option("joint", joint)
    ctx.upload(ix)
    assert ctx.get_option("ext2") == ext2
    assert ctx.get_option("joint") == (1 if joint < 0 else joint)
    assert ctx.get_option("n_paths") > 1000
    coll = np.concatenate(texts)
    n, L = 300_000, 150
    reads = nt.synth_reads(coll, 2, 0, n, L, 10_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    recs, roff = ctx.encode(reads, offs)
    out, o2 = ctx.decode(recs)
    assert np.array_equal(out, reads) and np.array_equal(o2, offs)
    orc = OracleIndex(ix.n, 91, ix.rows, ix.C, ix.lcs)
    m = 10_000
    exp, eoff = orc.encode(reads[: m * L], offs[: m + 1])
    assert np.array_equal(recs[: int(roff[m])], exp)
    d, s = ctx.matching_statistics(reads[:500 * L], offs[:501])
    for r in range(0, 500, 5):
        od, olo = orc.ms(reads[r * L:(r + 1) * L].tobytes())
        assert np.array_equal(d[r * L:(r + 1) * L], od), r
        assert np.array_equal(s[r * L:(r + 1) * L].astype(np.uint64), olo), r
    ctx.close()


@pytest.mark.parametrize("k,glen", [(5, 300), (7, 20_000), (9, 2_000), (9, 20_000)])
def test_gpu_small_k_reference_panic_status(ctx, k, glen):
    """k <= 10: a short record with k < len <= 11 panics in the reference (encode.rs:151-152);
    the GPU reports NTC_ERR_REFERENCE_PANIC at the oracle's first panicking read, and the other
    reads encode bit-exact."""
    g = nt.synth_genome(50 + k, glen)
    ix = nt.Index.build([g.tobytes()], k)
    ctx.upload(ix)
    L, n = 150, 200
    reads = nt.synth_reads(g, 3, 0, n, L, 10_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    orc = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs)
    one = np.array([0, L], dtype=np.uint64)
    panics = [r for r in range(n) if orc.try_encode(reads[r * L:(r + 1) * L], one)[0] == -5]
    assert panics
    with pytest.raises(nt.NtcError) as e:
        ctx.encode(reads, offs)
    assert e.value.code == 11 and e.value.bad_read == panics[0]
    keep = [r for r in range(n) if r not in set(panics)]
    if keep:
        kr = np.concatenate([reads[r * L:(r + 1) * L] for r in keep])
        ko = np.arange(0, len(keep) * L + 1, L, dtype=np.uint64)
        got, goff = ctx.encode(kr, ko)
        exp, eoff = orc.encode(kr, ko)
        assert np.array_equal(got, exp) and np.array_equal(goff, eoff)


def test_gpu_decode_bad_colex_over_many_tiles(ctx):
    """Malformed records (colex rank >= n) spread over many 256-record tiles: the decode
    reports NTC_ERR_FORMAT, writes nothing out of bounds and leaves the context usable."""
    genome = nt.synth_genome(21, 400_000)
    ix = nt.Index.build([genome.tobytes()], 31)
    ctx.upload(ix)
    n, L = 60_000, 150
    reads = nt.synth_reads(genome, 5, 0, n, L, 10_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    recs, _ = ctx.encode(reads, offs)
    assert len(recs) > 50 * 256
    flags = (recs >> np.uint64(56)) & np.uint64(2)
    longs = np.nonzero(flags == 0)[0]
    bad = recs.copy()
    pick = longs[:: max(1, len(longs) // 200)]
    bad[pick] = (bad[pick] & ~np.uint64(0xFFFFFFFF)) | np.uint64(0xFFFFFFF0)
    for _ in range(3):
        with pytest.raises(nt.NtcError) as e:
            ctx.decode(bad)
        assert e.value.code == 8
    out, o2 = ctx.decode(recs)
    assert np.array_equal(out, reads) and np.array_equal(o2, offs)


@pytest.mark.parametrize("lead", [0, 3, 16, 37])
def test_gpu_device_api_unaligned_ragged(ctx, lead):
    """Batch starting `lead` bytes into the caller's buffer (offs[0] = lead), ragged reads and
    an over-estimated max_read_len: records equal the host API's, nothing read past the end."""
    genome = nt.synth_genome(12, 200_000)
    ix = nt.Index.build([genome.tobytes()], 31)
    ctx.upload(ix)
    rng = np.random.default_rng(lead)
    g = genome.tobytes()
    reads = []
    for _ in range(3000):
        L = int(rng.integers(1, 300))
        st = int(rng.integers(0, len(g) - L))
        reads.append(g[st:st + L])
    bases, offs = pack_reads(reads)
    exp, eoff = ctx.encode(bases, offs)
    buf = np.concatenate([np.frombuffer(b"N" * lead, dtype=np.uint8), bases])
    offs_l = offs + np.uint64(lead)
    n = len(reads)
    db, do = ctx.alloc(buf.nbytes), ctx.alloc(offs_l.nbytes)
    dr, dro = ctx.alloc(len(bases) * 8 + 64), ctx.alloc(offs_l.nbytes)
    try:
        ctx.h2d(db, buf)
        ctx.h2d(do, offs_l)
        for max_len in (400, 0):
            ctx.encode_device(db, do, n, max_len, dr, len(bases) + 8, dro)
            nrec = ctx.encode_status()
            got = ctx.d2h(np.zeros(nrec, dtype=np.uint64), dr)
            gro = ctx.d2h(np.zeros(n + 1, dtype=np.uint64), dro)
            assert np.array_equal(got, exp) and np.array_equal(gro, eoff)
    finally:
        for p in (db, do, dr, dro):
            ctx.free(p)


def _repeat_genome(seed, units, unit_len, mut, spacer):
    rng = np.random.default_rng(seed)
    unit = nt.synth_genome(seed, unit_len).tobytes()
    parts = []
    for _ in range(units):
        u = bytearray(unit)
        for _ in range(mut):
            u[int(rng.integers(0, len(u)))] = b"ACGT"[int(rng.integers(0, 4))]
        parts.append(bytes(u) + nt.synth_genome(int(rng.integers(1, 1 << 30)), spacer).tobytes())
    return np.frombuffer(b"".join(parts), dtype=np.uint8)


@pytest.mark.parametrize("k,err_ppm,genome_kind,L", [
    (31, 10_000, "random", 150), (91, 20_000, "random", 150), (63, 5_000, "repeats", 150),
    (91, 10_000, "repeats", 250), (127, 10_000, "random", 300), (21, 50_000, "random", 100)])
def test_gpu_parity_sweep(ctx, k, err_ppm, genome_kind, L):
    """Larger sweep: 60k reads per config, bit-exact records and exact round trips, on
    random genomes and on genomes of near-identical repeats (long LCS runs, branching
    paths, contraction probes above U - 1 and binary searches)."""
    genome = nt.synth_genome(70 + k, 2_000_000) if genome_kind == "random" else _repeat_genome(k, 600, 700, 4, 150)
    ix = nt.Index.build([genome.tobytes()], k, threads=8)
    ctx.upload(ix)
    n = 60_000
    reads = nt.synth_reads(genome, 31, 0, n, L, err_ppm, threads=8)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    exp, eoff = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs).encode(reads, offs)
    got, goff = ctx.encode(reads, offs)
    assert np.array_equal(goff, eoff) and np.array_equal(got, exp)
    out, o2 = ctx.decode(got)
    assert np.array_equal(out, reads) and np.array_equal(o2, offs)


def test_gpu_reads_with_n_report_the_first_bad_read(ctx):
    genome = nt.synth_genome(15, 100_000)
    ctx.upload(nt.Index.build([genome.tobytes()], 31))
    reads = bytearray(nt.synth_reads(genome, 3, 0, 5000, 150, 10_000).tobytes())
    for r in (3210, 4000, 77):
        reads[r * 150 + 40] = ord("N")
    bases = np.frombuffer(bytes(reads), dtype=np.uint8)
    offs = np.arange(0, 5000 * 150 + 1, 150, dtype=np.uint64)
    with pytest.raises(nt.NtcError) as e:
        ctx.encode(bases, offs)
    assert e.value.code == 2 and e.value.bad_read == 77


def test_gpu_long_reads(ctx):
    """Nanopore-length reads (10-30 kb) at k = 31: many runs and errors per read."""
    genome = nt.synth_genome(16, 400_000)
    ix = nt.Index.build([genome.tobytes()], 31)
    ctx.upload(ix)
    rng = np.random.default_rng(8)
    g = genome.tobytes()
    reads = []
    for _ in range(40):
        L = int(rng.integers(10_000, 30_000))
        st = int(rng.integers(0, len(g) - L))
        s = bytearray(g[st:st + L])
        for _ in range(L // 100):
            s[int(rng.integers(0, L))] = b"ACGT"[int(rng.integers(0, 4))]
        reads.append(bytes(s))
    bases, offs = pack_reads(reads)
    exp, eoff = OracleIndex(ix.n, 31, ix.rows, ix.C, ix.lcs).encode(bases, offs)
    got, goff = ctx.encode(bases, offs)
    assert np.array_equal(goff, eoff) and np.array_equal(got, exp)
    out, o2 = ctx.decode(got)
    assert np.array_equal(out, bases) and np.array_equal(o2, offs)


@pytest.mark.parametrize("k", [255, 91, 31])
def test_gpu_reference_fasta_data_shape(ctx, k):
    """The reference's own test (tests/fasta_data.rs:28-101) in its shape, on the GPU: 7
    random contigs shorter than 2,000 bases, an index of them at k = 255 with reverse
    complements, each contig encoded against it, blocks of 3 records written after a file
    header (write_block_to, the last block num_records % 3) and decoded back block by block
    (`while let Ok(records) = decode_block`).  Seeded numpy contigs, not the `random` crate's
    (absent here).  A contig of more than k bases parses into long records plus a head that
    is short only when it has <= 11 bases (one shorter than k has no k-mer in the index and
    parses into short records), and a block with no short record makes write_block_to err
    (minimal_binary_encode of the empty stream 4, encode.rs:80), which the test's `let _ =`
    drops: at k = 255 with this seed blocks 1 and 2 are written and block 3 (contig 7) is
    dropped, so the decode returns the first 6 contigs in order.  SURVEY 8(c)'s k = 91 / 31
    variants the same way: the decode returns exactly the written blocks' contigs; records
    bit-exact against the oracle's throughout."""
    rng = np.random.default_rng(5)
    alpha = np.frombuffer(b"ACGT", dtype=np.uint8)
    contigs = [alpha[rng.integers(0, 4, int(rng.integers(1, 2000)))].tobytes() for _ in range(7)]
    ix = nt.Index.build(contigs, k)
    ctx.upload(ix)
    orc = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs)
    buf, written = nt.file_header(), []
    for i in range(0, 7, 3):
        grp = contigs[i:i + 3]
        bases, offs = pack_reads(grp)
        recs, roff = ctx.encode(bases, offs)
        exp, eoff = orc.encode(bases, offs)
        assert np.array_equal(roff, eoff) and np.array_equal(recs, exp)
        try:
            buf += nt.write_block(recs, len(grp))
            written += grp
        except nt.NtcError as e:
            assert e.code == 3  # write_block_to's Err (no short record in the block)
    assert written == contigs[:6] if k == 255 else written
    pos, got = 32, []
    while True:
        try:
            recs, used, nrec = nt.read_block(buf[pos:])
        except nt.NtcError:
            break
        pos += used
        out, o2 = ctx.decode(recs)
        got += [out[o2[j]:o2[j + 1]].tobytes() for j in range(len(o2) - 1)]
    assert pos == len(buf) and got == written


def test_gpu_record_length_limit(ctx):
    """The 24-bit match length (lib.rs:226: dictionary_max < 16777216, NTC_ERR_LENGTH for the
    reference's assert): one exact read of a unique 16.8 Mbp sequence at k = 31 parses into a
    record of 31m + 1 bases (the jump loop steps back k at a time, lib.rs:193-203) and a
    short head.  At 2^24 + 16 bases the long record is 2^24 - 15 (bit-exact vs the oracle,
    decoded back); at 2^24 + 17 it would be 2^24 + 16: the call fails with NTC_ERR_LENGTH."""
    genome = nt.synth_genome(21, (1 << 24) + 1000)
    ix = nt.Index.build([genome.tobytes()], 31, threads=8)
    ctx.upload(ix)
    g = genome.tobytes()
    bases, offs = pack_reads([g[5:5 + (1 << 24) + 16]])
    got, goff = ctx.encode(bases, offs)
    exp, eoff = OracleIndex(ix.n, 31, ix.rows, ix.C, ix.lcs).encode(bases, offs)
    assert np.array_equal(goff, eoff) and np.array_equal(got, exp)
    assert len(got) == 2 and (int(got[0]) >> 32) & 0xFFFFFF == (1 << 24) - 15 and (int(got[1]) >> 32) & 0xFFFFFF == 31
    out, o2 = ctx.decode(got)
    assert np.array_equal(out, bases) and np.array_equal(o2, offs)
    bases, offs = pack_reads([g[100:300], g[5:5 + (1 << 24) + 17]])
    with pytest.raises(nt.NtcError) as e:
        ctx.encode(bases, offs)
    assert e.value.code == 4 and e.value.bad_read == 1


@pytest.mark.parametrize("link", [1, 0])
def test_gpu_path_cover_equals_host_cover(ctx, monkeypatch, link):
    """ntc_index_upload builds the path cover on the device (list ranking, cycle cuts, and
    with path_link the unitigs linked across branches: k_link_want / k_link_apply); it must
    be the host build_paths cover byte for byte (the one the emulation tests run), on single
    genomes, repeats, cycles and strain collections (where the linking changes the cover)."""
    from emu_lib import emu_path_cover
    monkeypatch.setenv("NTC_PATH_LINK", str(link))
    g = nt.synth_genome(44, 60_000).tobytes()
    gg = nt.synth_genome(45, 40_000)
    st = nt.synth_strains(gg, 5, 40, 2000)
    coll = [gg.tobytes()] + [st[i].tobytes() for i in range(40)]
    cases = [([g], 31), ([g], 91), ([g[:20_000]], 7), ([b"ACGGTCATTC" * 20, b"TTGACCAGGATC" * 15, g[:3000]], 31),
             ([(g[:500] * 30), g[:7000]], 15), ([b"ACGTTGCA" * 100], 2), ([g[:30_000]], 255), (coll, 31),
             (coll, 91), (coll[:6], 23)]
    ctx.set_option("path_link", link)
    try:
        for seqs, k in cases:
            ix = nt.Index.build(seqs, k)
            ctx.upload(ix)
            h, tlen, npaths = emu_path_cover(ix.n, k, ix.rows, ix.C, ix.lcs)
            assert ctx.get_option("path_text_len") == tlen, k
            assert ctx.get_option("n_paths") == npaths, k
            assert ctx.get_option("path_hash") & ((1 << 64) - 1) == h, k
    finally:
        ctx.set_option("path_link", 1)


def test_gpu_host_api_splits_large_batches_into_passes(ctx):
    """Host-buffer calls run in device passes of at most max_pass_bases (bounded workspace
    for any batch size): records, offsets, decoded bases and the failing read's index are
    the same as in one pass."""
    genome = nt.synth_genome(17, 200_000)
    ix = nt.Index.build([genome.tobytes()], 31)
    ctx.upload(ix)
    rng = np.random.default_rng(4)
    lens = rng.integers(1, 400, 3000)
    g = genome.tobytes()
    reads = [g[s:s + L] for s, L in zip(rng.integers(0, len(g) - 400, 3000), lens)]
    bases, offs = pack_reads(reads)
    exp, eoff = OracleIndex(ix.n, 31, ix.rows, ix.C, ix.lcs).encode(bases, offs)
    default = ctx.get_option("max_pass_bases")
    try:
        for mp in (1, 5_000, 77_777, default):
            ctx.set_option("max_pass_bases", mp)
            got, goff = ctx.encode(bases, offs)
            assert np.array_equal(goff, eoff) and np.array_equal(got, exp), mp
            out, o2 = ctx.decode(got)
            assert np.array_equal(out, bases) and np.array_equal(o2, offs), mp
        bad = bytearray(bases.tobytes())
        bad[int(offs[2500]) + 3] = ord("N")
        for mp in (5_000, default):
            ctx.set_option("max_pass_bases", mp)
            with pytest.raises(nt.NtcError) as e:
                ctx.encode(np.frombuffer(bytes(bad), dtype=np.uint8), offs)
            assert e.value.code == 2 and e.value.bad_read == 2500, mp
    finally:
        ctx.set_option("max_pass_bases", default)


@pytest.mark.parametrize("pair_bytes", [1, 0])
@pytest.mark.parametrize("k,tab_u", [(91, 0), (31, 12), (21, 5)])
@pytest.mark.parametrize("win", [-1, 0])
def test_gpu_scan_exact_test_paths(ctx, k, tab_u, pair_bytes, win):
    """SCAN on window words (win = -1, the default) or, with win = 0, through the filter and
    the pair bytes or the level-U bitmap (pair_bytes = 0): identical records, bit-exact vs the
    oracle, for filtered (U >= 12) and unfiltered table depths."""
    genome = nt.synth_genome(500 + k, 1_000_000)
    ix = nt.Index.build([genome.tobytes()], k, threads=8)
    ctx.set_option("pair_bytes", pair_bytes)
    ctx.set_option("tab_u", tab_u)
    ctx.set_option("win", win)
    try:
        ctx.upload(ix)
        assert ctx.get_option("pair_bytes") == pair_bytes
        assert ctx.get_option("win") == (0 if win == 0 else int(ctx.get_option("tab_u") >= 4))
        n, L = 20_000, 150
        reads = nt.synth_reads(genome, 9, 0, n, L, 15_000, threads=8)
        offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
        exp, eoff = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs).encode(reads, offs)
        got, goff = ctx.encode(reads, offs)
        assert np.array_equal(goff, eoff) and np.array_equal(got, exp)
    finally:
        ctx.set_option("pair_bytes", 1)
        ctx.set_option("tab_u", 0)
        ctx.set_option("win", -1)


def test_gpu_decode_direct_path_for_long_records(ctx):
    """Error-free 30-50 kb reads: one or two records each, so a block of 256 records spans
    far more than kDecStageWords output words and k_dec_rec writes ASCII directly (its
    fallback path), next to blocks that stage through LDS (the short-read batch after it)."""
    genome = nt.synth_genome(17, 300_000)
    ix = nt.Index.build([genome.tobytes()], 31)
    ctx.upload(ix)
    rng = np.random.default_rng(9)
    g = genome.tobytes()
    reads = []
    for _ in range(120):
        L = int(rng.integers(30_000, 50_000))
        st = int(rng.integers(0, len(g) - L))
        reads.append(g[st:st + L])
    reads += [g[i * 7:i * 7 + 150] for i in range(600)]  # then short reads: staged blocks
    bases, offs = pack_reads(reads)
    exp, eoff = OracleIndex(ix.n, 31, ix.rows, ix.C, ix.lcs).encode(bases, offs)
    got, goff = ctx.encode(bases, offs)
    assert np.array_equal(goff, eoff) and np.array_equal(got, exp)
    longm = ((got >> np.uint64(56)) & np.uint64(2)) == 0
    lens = (got[longm] >> np.uint64(32)) & np.uint64(0xFFFFFF)
    assert int(lens.max()) > 32 * 1024  # records longer than a whole staging buffer
    out, o2 = ctx.decode(got)
    assert np.array_equal(out, bases) and np.array_equal(o2, offs)


def test_gpu_random_cases_equal_oracle(ctx):
    """The property test's random cases (tests/test_property.py: random k 11..127, genome,
    repeats, read lengths 1..400, error rates, reverse complements) through the GPU: records
    bit-exact vs the oracle, decode(encode(x)) == x, failures at the oracle's first read."""
    from test_property import _case
    rng = np.random.default_rng(2024)
    for i in range(60):
        k = int(rng.integers(11, 128))
        ix, bases, offs = _case(int(rng.integers(0, 2**32)), k, int(rng.integers(300, 6000)),
                                int(rng.integers(1, 60)), int(rng.integers(1, 400)),
                                float(rng.choice([0.0, 0.005, 0.02, 0.08])), bool(rng.integers(0, 2)))
        ctx.upload(ix)
        orc = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs)
        rc, bad = orc.try_encode(bases, offs)
        if rc < 0:
            with pytest.raises(nt.NtcError) as e:
                ctx.encode(bases, offs)
            assert e.value.bad_read == bad, (i, k)
            continue
        exp, eoff = orc.encode(bases, offs)
        got, goff = ctx.encode(bases, offs)
        assert np.array_equal(goff, eoff) and np.array_equal(got, exp), (i, k)
        out, o2 = ctx.decode(got)
        assert np.array_equal(out, bases) and np.array_equal(o2, offs), (i, k)


def test_gpu_random_collections_equal_oracle():
    """Random strain collections through the GPU (round 6's linked path cover, joint runs and
    fork hops on many small structures): a genome of 2-40 kbp plus 1-11 strains at 0.1-5 %
    substitutions, k from 11 to 255, the cover linked or not (ctx option path_link), reads
    of 20-400 bases drawn across the collection with 0-2 % errors; records bit-exact vs the
    oracle and decode(encode(x)) == x."""
    rng = np.random.default_rng(606)
    ctx = nt.GpuContext(0)
    for i in range(24):
        k = int(rng.choice([11, 15, 23, 31, 47, 63, 91, 127, 191, 255]))
        genome = nt.synth_genome(int(rng.integers(1, 1 << 30)), int(rng.integers(2_000, 40_000)))
        ns = int(rng.integers(1, 12))
        strains = nt.synth_strains(genome, int(rng.integers(1, 1 << 30)), ns,
                                   int(rng.choice([1_000, 5_000, 20_000, 50_000])))
        texts = [genome] + [strains[j] for j in range(ns)]
        ix = nt.Index.build([t.tobytes() for t in texts], k)
        ctx.set_option("path_link", i % 2)
        ctx.upload(ix)
        n, L = int(rng.integers(50, 800)), int(rng.integers(20, 400))
        reads = nt.synth_reads(np.concatenate(texts), int(rng.integers(1, 1 << 30)), 0, n, L,
                               int(rng.choice([0, 5_000, 20_000])))
        offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
        orc = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs)
        exp, eoff = orc.encode(reads, offs)
        got, goff = ctx.encode(reads, offs)
        assert np.array_equal(goff, eoff) and np.array_equal(got, exp), (i, k, ns)
        out, o2 = ctx.decode(got)
        assert np.array_equal(out, reads) and np.array_equal(o2, offs), (i, k, ns)
    ctx.close()


def test_gpu_suffix_table_depth_15():
    """The deepest suffix table (U = 15, 8.6 GB top level; the default for indexes of more than
    ~17 M nodes) gives the same records as the oracle on the C91 index."""
    genome = nt.synth_genome(1, 5_000_000)
    ix = nt.Index.build([genome.tobytes()], 91)
    ctx = nt.GpuContext(0)
    ctx.set_option("tab_u", 15)
    ctx.upload(ix)
    assert ctx.get_option("tab_u") == 15
    n, L = 200_000, 150
    reads = nt.synth_reads(genome, 9, 0, n, L, 10_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    recs, roff = ctx.encode(reads, offs)
    out, o2 = ctx.decode(recs)
    assert np.array_equal(out, reads)
    m = 20_000
    exp, eoff = OracleIndex(ix.n, 91, ix.rows, ix.C, ix.lcs).encode(reads[: m * L], offs[: m + 1])
    assert np.array_equal(recs[: int(roff[m])], exp)
    ctx.close()
