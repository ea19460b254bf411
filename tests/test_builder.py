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
