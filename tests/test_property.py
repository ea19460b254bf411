"""Property-based parity (hypothesis): the kernels' lane logic (test-only emulator of
ntcomp_amd/csrc/encode_core.h) against the faithful CPU oracle on random small indexes and
reads -- random k (11..127), genome lengths, read lengths (1..400), error rates, reverse
complements, repeats -- plus decode(encode(x)) == x (tests/fasta_data.rs:93's property).
CPU only; the same lane functions run on the GPU in tests/test_gpu_parity.py."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import ntcomp_amd as nt
from emu_lib import emu_decode, emu_encode
from oracle_lib import OracleIndex

ALPHA = np.frombuffer(b"ACGT", dtype=np.uint8)


def _case(seed, k, glen, n_reads, max_len, err, repeat):
    rng = np.random.default_rng(seed)
    g = ALPHA[rng.integers(0, 4, glen)]
    if repeat:  # a repeated block makes multi-node intervals and long LCS values
        blk = g[: max(k + 5, glen // 8)].copy()
        g = np.concatenate([g, blk, g[glen // 3: glen // 2], blk])
    ix = nt.Index.build([g.tobytes()], k)
    reads, offs = [], [0]
    for _ in range(n_reads):
        L = int(rng.integers(1, max_len + 1))
        s = int(rng.integers(0, max(1, len(g) - L)))
        r = g[s:s + L].copy()
        if rng.random() < 0.5:
            r = (3 - ((r >> 1 ^ r >> 2) & 3)).astype(np.uint8)
            r = ALPHA[r][::-1].copy()
        flip = rng.random(len(r)) < err
        r[flip] = ALPHA[(((r[flip] >> 1 ^ r[flip] >> 2) & 3) + rng.integers(1, 4, int(flip.sum()))) & 3]
        reads.append(r)
        offs.append(offs[-1] + len(r))
    return ix, np.concatenate(reads), np.array(offs, dtype=np.uint64)


import os

N_EXAMPLES = int(os.environ.get("NTC_PROPERTY_EXAMPLES", "200"))  # raise for a longer bug hunt


@settings(max_examples=N_EXAMPLES, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(seed=st.integers(0, 2**32 - 1), k=st.integers(11, 127), glen=st.integers(300, 6000),
       n_reads=st.integers(1, 60), max_len=st.integers(1, 400), err=st.sampled_from([0.0, 0.005, 0.02, 0.08]),
       repeat=st.booleans())
def test_emulated_kernel_equals_oracle_on_random_cases(seed, k, glen, n_reads, max_len, err, repeat):
    ix, bases, offs = _case(seed, k, glen, n_reads, max_len, err, repeat)
    orc = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs)
    rc, bad = orc.try_encode(bases, offs)
    if rc < 0:  # the oracle fails on a read (e.g. a base absent from a tiny index): the emulator too
        with pytest.raises(RuntimeError):
            emu_encode(ix.n, k, ix.rows, ix.C, ix.lcs, bases, offs)
        return
    exp, eoff = orc.encode(bases, offs)
    got, goff = emu_encode(ix.n, k, ix.rows, ix.C, ix.lcs, bases, offs)
    assert np.array_equal(goff, eoff)
    assert np.array_equal(got, exp)
    out, oo = emu_decode(ix.n, k, ix.rows, ix.C, ix.lcs, got)
    assert np.array_equal(out, bases) and np.array_equal(oo, offs)


@settings(max_examples=max(50, N_EXAMPLES // 2), deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(seed=st.integers(0, 2**32 - 1), k=st.integers(11, 127), glen=st.integers(300, 6000),
       n_reads=st.integers(1, 60), max_len=st.integers(1, 400), err=st.sampled_from([0.005, 0.02, 0.08]),
       repeat=st.booleans())
def test_emulated_kernel_without_scan_filter_equals_oracle(seed, k, glen, n_reads, max_len, err, repeat):
    """SCAN with the pre-filter off (the upload's auto mode for dense indexes such as S91):
    every position is a candidate and the pair words alone decide (two positions per word)."""
    ix, bases, offs = _case(seed, k, glen, n_reads, max_len, err, repeat)
    orc = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs)
    rc, bad = orc.try_encode(bases, offs)
    if rc < 0:
        return
    exp, eoff = orc.encode(bases, offs)
    os.environ["NTC_EMU_FILTER"] = "0"
    try:
        got, goff = emu_encode(ix.n, k, ix.rows, ix.C, ix.lcs, bases, offs)
    finally:
        del os.environ["NTC_EMU_FILTER"]
    assert np.array_equal(goff, eoff) and np.array_equal(got, exp)
