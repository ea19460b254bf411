"""The C ABI library loads on a CPU-only machine and exports every symbol that
include/*.h declare (no GPU compute here)."""
import ctypes
import os
import re

import numpy as np

import ntcomp_amd as nt
from oracle_lib import REPO


def declared_symbols():
    names = set()
    for h in ("ntcomp_gpu.h", "ntcomp_host.h", "ntcomp_codec.h", "ntcomp_pipeline.h"):
        src = open(os.path.join(REPO, "include", h)).read()
        names |= set(re.findall(r"\b(ntc_[a-z0-9_]+)\s*\(", src))
    return names


def test_every_declared_symbol_is_exported():
    L = nt.lib()
    decl = declared_symbols()
    assert decl == set(nt.EXPORTED)
    for s in decl:
        assert hasattr(L, s), s


def test_abi_version():
    assert nt.lib().ntc_abi_version() == 1


def test_ctx_create_fails_loudly_without_gpu():
    import torch  # noqa: F401  (only to know whether a GPU exists here)
    if torch.cuda.is_available():
        return
    h = ctypes.c_void_p()
    rc = nt.lib().ntc_ctx_create(0, ctypes.byref(h))
    assert rc != 0 and not h.value
    try:
        nt.GpuContext(0)
        raise AssertionError("GpuContext must raise without a GPU")
    except nt.NtcError:
        pass


def test_synth_is_deterministic_and_shardable():
    g = nt.synth_genome(1, 10_000)
    assert set(np.unique(g).tolist()) <= set(b"ACGT")
    a = nt.synth_reads(g, 2, 0, 100, 150, 10_000, threads=3)
    b = nt.synth_reads(g, 2, 40, 60, 150, 10_000, threads=1)
    assert np.array_equal(a.reshape(100, 150)[40:], b.reshape(60, 150))


def test_index_prepare_needs_no_gpu():
    """ntc_index_prepare (the host half of an upload) runs without a GPU and rejects a null
    view; ntc_index_upload_prepared fails loudly without a context."""
    g = nt.synth_genome(3, 50_000)
    ix = nt.Index.build([g.tobytes()], 31)
    p = nt.IndexPrep(ix)
    assert p.h
    p.close()
    out = ctypes.c_void_p()
    assert nt.lib().ntc_index_prepare(None, ctypes.byref(out)) == 1
    assert nt.lib().ntc_index_upload_prepared(None, None) == 1
