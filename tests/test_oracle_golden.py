"""Pins the CPU oracle (oracle/ntcomp_oracle.c, the faithful restatement) to the golden
vectors of the independent brute-force restatement (tests/golden/make_golden.py)."""
import numpy as np
import pytest

from oracle_lib import OracleIndex, golden_names, load_golden, pack_reads


@pytest.mark.parametrize("name", golden_names())
def test_oracle_ms_matches_golden(name):
    g = load_golden(name)
    ix = OracleIndex(g["n"], g["k"], g["rows_u64"], g["C"], g["lcs_u8"])
    for read, ms in zip(g["reads"], g["ms"]):
        d, lo = ix.ms(read.encode())
        exp = np.array(ms, dtype=np.uint64).reshape(-1, 2)
        assert np.array_equal(d.astype(np.uint64), exp[:, 0]), read
        # start is defined (and consumed) only where d > 0
        m = exp[:, 0] > 0
        assert np.array_equal(lo[m], exp[m, 1]), read


@pytest.mark.parametrize("name", golden_names())
def test_oracle_records_match_golden(name):
    g = load_golden(name)
    ix = OracleIndex(g["n"], g["k"], g["rows_u64"], g["C"], g["lcs_u8"])
    bases, offs = pack_reads(g["reads"])
    recs, roff = ix.encode(bases, offs)
    exp = [w for r in g["records"] for w in r]
    assert recs.tolist() == exp
    assert np.diff(roff).tolist() == [len(r) for r in g["records"]]


@pytest.mark.parametrize("name", golden_names())
def test_oracle_decode_roundtrip(name):
    g = load_golden(name)
    ix = OracleIndex(g["n"], g["k"], g["rows_u64"], g["C"], g["lcs_u8"])
    recs = np.array([w for r in g["records"] for w in r], dtype=np.uint64)
    out, offs = ix.decode(recs)
    got = [out[offs[i]:offs[i + 1]].tobytes().decode() for i in range(len(offs) - 1)]
    assert got == g["reads"]


def test_oracle_without_prefix_table_is_identical():
    g = load_golden("ecoli_like_k31")
    a = OracleIndex(g["n"], g["k"], g["rows_u64"], g["C"], g["lcs_u8"], precalc=8)
    b = OracleIndex(g["n"], g["k"], g["rows_u64"], g["C"], g["lcs_u8"], precalc=0)
    bases, offs = pack_reads(g["reads"])
    assert np.array_equal(a.encode(bases, offs)[0], b.encode(bases, offs)[0])
