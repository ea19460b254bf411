"""The product index producer (ntc_build_index, stand-in for kbo::build) against the
brute-force SBWT of tests/golden/make_golden.py: node count, C array, subset-matrix rows
and LCS must be identical."""
import numpy as np
import pytest

import ntcomp_amd as nt
from oracle_lib import golden_names, load_golden


@pytest.mark.parametrize("name", golden_names())
def test_builder_matches_golden(name):
    g = load_golden(name)
    ix = nt.Index.build(g["seqs"], g["k"], add_revcomp=True, threads=4)
    assert ix.n == g["n"]
    assert ix.k == g["k"]
    assert ix.C == g["C"]
    for c in range(4):
        assert np.array_equal(ix.row(c), g["rows_u64"][c]), "ACGT"[c]
    assert np.array_equal(ix.lcs, g["lcs_u8"])


def test_builder_thread_count_invariant():
    genome = nt.synth_genome(7, 300_000)
    a = nt.Index.build([genome.tobytes()], 31, threads=1)
    b = nt.Index.build([genome.tobytes()], 31, threads=8)
    assert a.n == b.n and a.C == b.C
    for c in range(4):
        assert np.array_equal(a.row(c), b.row(c))
    assert np.array_equal(a.lcs, b.lcs)


def test_builder_splits_on_non_acgt():
    # k-mers containing N are skipped (kbo/sbwt split sequences at non-ACGT bytes)
    ix1 = nt.Index.build(["ACGTACGTTGCA" + "N" + "GGCATTACGA"], 5)
    ix2 = nt.Index.build(["ACGTACGTTGCA", "GGCATTACGA"], 5)
    assert ix1.n == ix2.n
    for c in range(4):
        assert np.array_equal(ix1.row(c), ix2.row(c))


def test_index_files_roundtrip(tmp_path):
    g = load_golden("small_k15")
    ix = nt.Index.build(g["seqs"], g["k"])
    ix.save(tmp_path / "idx")
    assert (tmp_path / "idx.sbwt").exists() and (tmp_path / "idx.lcs").exists()
    jx = nt.Index.load(tmp_path / "idx")
    assert jx.n == ix.n and jx.k == ix.k and jx.C == ix.C
    for c in range(4):
        assert np.array_equal(jx.row(c), ix.row(c))
    assert np.array_equal(jx.lcs, ix.lcs)
    (tmp_path / "idx.lcs").unlink()
    with pytest.raises(nt.NtcError):
        nt.Index.load(tmp_path / "idx")


@pytest.mark.parametrize("k", [15, 31, 91])
def test_index_sbwt_rs_layout_round_trip(tmp_path, k):
    """own layout -> sbwt-rs layout (restated sbwt 0.3.11 / kbo 0.5.1 serialisation,
    main.rs:138; [ext, recalled], parity unpinned) -> own layout: rows, C, k and LCS survive
    bit for bit, and Index.load detects each layout."""
    g = nt.synth_genome(5 + k, 30_000)
    ix = nt.Index.build([g.tobytes()], k)
    ix.save(tmp_path / "a", layout="sbwt-rs")
    assert (tmp_path / "a.sbwt").read_bytes()[:20] == (12).to_bytes(8, "little") + b"plain-matrix"
    b = nt.Index.load(tmp_path / "a")
    b.save(tmp_path / "b")
    assert (tmp_path / "b.sbwt").read_bytes()[:8] == b"NTCSBWT1"
    c = nt.Index.load(tmp_path / "b")
    for x in (b, c):
        assert (x.n, x.k, x.C) == (ix.n, ix.k, ix.C)
        assert all(np.array_equal(p, q) for p, q in zip(x.rows, ix.rows))
        assert np.array_equal(x.lcs, ix.lcs)


def _words_from(blob, off):
    return np.frombuffer(blob[off:off + (len(blob) - off) // 8 * 8], dtype="<u8")


def _read_rows(blob):
    L = int.from_bytes(blob[:8], "little")
    w = _words_from(blob, 8 + L)
    pos, rows = 0, []
    for _ in range(4):
        ones, bits, nw = int(w[pos]), int(w[pos + 1]), int(w[pos + 2])
        words = w[pos + 3:pos + 3 + nw]
        pos += 3 + nw
        opts = []
        for _ in range(3):
            sz = int(w[pos])
            opts.append(None if sz == 0 else w[pos + 1:pos + 1 + sz].copy())
            pos += 1 + sz
        rows.append((ones, bits, words.copy(), opts))
    return rows, w, pos


def _unpack(words, n, width):
    v = np.zeros(n, dtype=np.uint64)
    for i in range(n):
        b = i * width
        x = int(words[b >> 6]) >> (b & 63)
        if (b & 63) + width > 64:
            x |= int(words[(b >> 6) + 1]) << (64 - (b & 63))
        v[i] = x & ((1 << width) - 1)
    return v


@pytest.mark.parametrize("k,sparse", [(15, False), (31, False), (31, True)])
def test_sbwt_rs_rows_carry_rank_and_select(tmp_path, k, sparse):
    """The reference builds with build_select = true (main.rs:118-119) and its decode calls
    access_kmer, which needs select (lib.rs:258, 286, 291): each subset-matrix row is written
    with Some(rank support), Some(select support), None(select_zero) [simple-sds, ext,
    recalled, unpinned].  Checked by an independent reader: the rank samples equal the ones
    before each 512-bit superblock and the 9-bit in-superblock counts, select answers every
    one's position from its superblock sample + block sample, and the file loads back."""
    g = nt.synth_genome(77 + k, 300_000)
    if sparse:  # T in ~0.3 % of positions: row T's superblocks of 4096 ones span > 2^16 bits ("long")
        rng = np.random.default_rng(k)
        g = np.frombuffer(b"ACG", np.uint8)[rng.integers(0, 3, 600_000)]
        g[rng.integers(0, len(g), 2000)] = ord("T")
    ix = nt.Index.build([g.tobytes()], k, add_revcomp=not sparse)
    ix.save(tmp_path / "a", layout="sbwt-rs")
    rows, _, _ = _read_rows((tmp_path / "a.sbwt").read_bytes())
    n_long = 0
    for c, (ones, bits, words, (rank, sel, selz)) in enumerate(rows):
        assert bits == ix.n and np.array_equal(words, ix.rows[c][:len(words)])
        assert rank is not None and sel is not None and selz is None, c
        row = np.unpackbits(words.view(np.uint8), bitorder="little")[:bits].astype(np.int64)
        assert ones == int(row.sum())
        # rank: Vec<(u64, u64)> of ceil(words / 8) superblocks
        nsb = int(rank[0])
        assert nsb == (len(words) + 7) // 8 and len(rank) == 1 + 2 * nsb
        wc = np.array([bin(int(x)).count("1") for x in words], dtype=np.int64)
        for s in range(nsb):
            assert int(rank[1 + 2 * s]) == int(wc[:8 * s].sum())
            for j in range(1, 8):
                if 8 * s + j < len(words):
                    assert (int(rank[2 + 2 * s]) >> (9 * (j - 1))) & 511 == int(wc[8 * s:8 * s + j].sum())
        # select: samples, long IntVector, short IntVector
        ns = int(sel[0])
        samples = sel[1:1 + 2 * ns].reshape(-1, 2)
        p = 1 + 2 * ns
        ln, lw, _, lnw = (int(x) for x in sel[p:p + 4])
        lvals = _unpack(sel[p + 4:p + 4 + lnw], ln, lw)
        p += 4 + lnw
        sn, sw, _, snw = (int(x) for x in sel[p:p + 4])
        assert sw == 16 and p + 4 + snw == len(sel)
        svals = _unpack(sel[p + 4:p + 4 + snw], sn, sw)
        pos1 = np.flatnonzero(row)
        assert ns == (len(pos1) + 4095) // 4096
        for i in range(0, len(pos1), 997):  # select(i) for a sample of ones
            first, off = (int(x) for x in samples[i // 4096])
            a = i // 4096 * 4096
            assert first == pos1[a]
            b = min(len(pos1), a + 4096)
            if pos1[b - 1] - pos1[a] + 1 > 1 << 16:
                assert lvals[off + i - a] == pos1[i]
                n_long += 1
            else:  # the block's first one, then a scan of the row
                bs = first + int(svals[off + (i - a) // 64])
                assert bs == pos1[a + (i - a) // 64 * 64]
    assert (n_long > 0) == sparse
    b = nt.Index.load(tmp_path / "a")
    assert all(np.array_equal(x, y) for x, y in zip(b.rows, ix.rows)) and np.array_equal(b.lcs, ix.lcs)


def test_sbwt_rs_reader_skips_options_of_any_size(tmp_path):
    """The reader skips each row's Options by their size: a hand-built file with all three
    Some (select_zero too, arbitrary payloads) and one with all three None load the same."""
    import struct
    g = nt.synth_genome(3, 20_000)
    ix = nt.Index.build([g.tobytes()], 21)
    ix.save(tmp_path / "a", layout="sbwt-rs")
    blob = (tmp_path / "a.sbwt").read_bytes()
    L = int.from_bytes(blob[:8], "little")
    head, body = blob[:8 + L], blob[8 + L:]
    rows, w, end = _read_rows(blob)
    for variant in ("all_some", "all_none"):
        out = bytearray(head)
        for ones, bits, words, opts in rows:
            out += struct.pack("<QQQ", ones, bits, len(words)) + words.tobytes()
            for j, o in enumerate(opts):
                if variant == "all_none":
                    out += struct.pack("<Q", 0)
                else:
                    pay = o if o is not None else np.arange(5 + j, dtype="<u8")
                    out += struct.pack("<Q", len(pay)) + pay.astype("<u8").tobytes()
        out += body[end * 8:]
        (tmp_path / f"{variant}.sbwt").write_bytes(bytes(out))
        (tmp_path / f"{variant}.lcs").write_bytes((tmp_path / "a.lcs").read_bytes())
        b = nt.Index.load(tmp_path / variant)
        assert (b.n, b.k) == (ix.n, ix.k)
        assert all(np.array_equal(x, y) for x, y in zip(b.rows, ix.rows)) and np.array_equal(b.lcs, ix.lcs)


@pytest.mark.parametrize("k,p", [(7, 1), (7, 3), (15, 4), (31, 5)])
def test_prefix_table_equals_search_by_definition(k, p):
    """-p/--prefix-precalc (src/cli.rs:46): every p-mer's colex interval (sbwt's
    PrefixLookupTable [ext, recalled]) equals the brute-force SBWT's search of that p-mer
    (tests/golden/make_golden.py NaiveSBWT: the nodes whose suffix is the pattern), [0, 0)
    when absent; index = the p-mer's 2-bit codes, first character most significant."""
    import itertools
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import NaiveSBWT
    rng = np.random.default_rng(k * 10 + p)
    seqs = ["".join(rng.choice(list("ACGT"), int(n))) for n in (300, 41, 120)]
    sb = NaiveSBWT(seqs, k)
    ix = nt.Index.build([s.encode() for s in seqs], k)
    assert ix.n == sb.n
    ix.set_prefix_precalc(p)
    got_p, ranges = ix.prefix_table()
    assert got_p == p and ranges.shape == (4 ** p, 2)
    for idx, t in enumerate(itertools.product("ACGT", repeat=p)):
        r = sb.search("".join(t))
        assert tuple(int(x) for x in ranges[idx]) == (r if r else (0, 0)), "".join(t)


def test_prefix_table_in_sbwt_rs_files(tmp_path):
    ix = nt.Index.build([nt.synth_genome(3, 20_000).tobytes()], 31)
    ix.set_prefix_precalc(6)
    _, exp = ix.prefix_table()
    ix.save(tmp_path / "rs", layout="sbwt-rs")
    jx = nt.Index.load(tmp_path / "rs")
    p, got = jx.prefix_table()
    assert p == 6 and np.array_equal(got, exp)
    # no table: the single range [0, n), read back as none
    ix.set_prefix_precalc(0)
    ix.save(tmp_path / "rs0", layout="sbwt-rs")
    assert nt.Index.load(tmp_path / "rs0").prefix_table() == (0, None)
    with pytest.raises(nt.NtcError):
        ix.set_prefix_precalc(13)
