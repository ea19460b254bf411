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
