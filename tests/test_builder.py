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
