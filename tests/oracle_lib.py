"""ctypes loader for the CPU oracle (oracle/liboracle_ntcomp.so) and the golden fixtures.

Test infrastructure: the oracle is the CHECKER, never the thing under test.
"""
import ctypes
import gzip
import json
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
ORACLE_SO = os.path.join(REPO, "oracle", "liboracle_ntcomp.so")

_lib = None


def oracle_lib():
    global _lib
    if _lib is None:
        src = os.path.join(REPO, "oracle", "ntcomp_oracle.c")
        if (not os.path.exists(ORACLE_SO)) or os.path.getmtime(ORACLE_SO) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])
        lib = ctypes.CDLL(ORACLE_SO)
        P = ctypes.c_void_p
        u64 = ctypes.c_uint64
        lib.orc_index_new.restype = P
        lib.orc_index_new.argtypes = [u64, ctypes.c_uint32, P, P, P, P, P, P, ctypes.c_uint32]
        lib.orc_index_free.argtypes = [P]
        lib.orc_matching_statistics.restype = ctypes.c_int
        lib.orc_matching_statistics.argtypes = [P, P, u64, P, P]
        lib.orc_encode_batch.restype = ctypes.c_int64
        lib.orc_encode_batch.argtypes = [P, P, P, u64, P, u64, P, P]
        lib.orc_decode.restype = ctypes.c_int64
        lib.orc_decode.argtypes = [P, P, u64, P, u64, P, u64, P]
        lib.orc_access_kmer.argtypes = [P, u64, P]
        _lib = lib
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleIndex:
    """Wraps orc_index built from raw SBWT arrays (rows: 4 x uint64 words, C, lcs)."""

    def __init__(self, n, k, rows, C, lcs, precalc=8):
        self.lib = oracle_lib()
        self.n, self.k = int(n), int(k)
        self._rows = [np.ascontiguousarray(r, dtype=np.uint64) for r in rows]
        self._C = np.ascontiguousarray(C, dtype=np.uint64)
        self._lcs = np.ascontiguousarray(lcs, dtype=np.uint8)
        self.h = self.lib.orc_index_new(self.n, self.k, *[_ptr(r) for r in self._rows],
                                        _ptr(self._C), _ptr(self._lcs), precalc)

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.orc_index_free(self.h)
            self.h = None

    def ms(self, read: bytes):
        q = np.frombuffer(read, dtype=np.uint8)
        d = np.zeros(len(q), dtype=np.uint32)
        lo = np.zeros(len(q), dtype=np.uint64)
        rc = self.lib.orc_matching_statistics(self.h, _ptr(q), len(q), _ptr(d), _ptr(lo))
        assert rc == 0, rc
        return d, lo

    def encode(self, bases: np.ndarray, offsets: np.ndarray):
        bases = np.ascontiguousarray(bases, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        nreads = len(offsets) - 1
        cap = int(offsets[-1]) + 1
        recs = np.zeros(cap, dtype=np.uint64)
        roff = np.zeros(nreads + 1, dtype=np.uint64)
        bad = ctypes.c_int64(-1)
        rc = self.lib.orc_encode_batch(self.h, _ptr(bases), _ptr(offsets), nreads, _ptr(recs), cap,
                                       _ptr(roff), ctypes.byref(bad))
        if rc < 0:
            raise RuntimeError(f"oracle encode failed rc={rc} at read {bad.value}")
        return recs[:rc], roff

    def try_encode(self, bases: np.ndarray, offsets: np.ndarray):
        """-> (rc, bad_read): rc < 0 is the oracle's error (ORC_ERR_PANIC = -5 where the
        reference panics), bad_read the first failing read."""
        bases = np.ascontiguousarray(bases, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        cap = int(offsets[-1]) + 1
        recs = np.zeros(cap, dtype=np.uint64)
        roff = np.zeros(len(offsets), dtype=np.uint64)
        bad = ctypes.c_int64(-1)
        rc = self.lib.orc_encode_batch(self.h, _ptr(bases), _ptr(offsets), len(offsets) - 1, _ptr(recs), cap,
                                       _ptr(roff), ctypes.byref(bad))
        return int(rc), int(bad.value)

    def decode(self, recs: np.ndarray):
        recs = np.ascontiguousarray(recs, dtype=np.uint64)
        flags = (recs >> np.uint64(56)).astype(np.uint8)
        total = int(np.where(flags & 2, flags >> 2, (recs >> np.uint64(32)) & np.uint64(0xFFFFFF)).sum())
        nreads = int((flags & 1).sum())
        out = np.zeros(total + 1, dtype=np.uint8)
        offs = np.zeros(nreads + 2, dtype=np.uint64)
        nr = ctypes.c_uint64(0)
        rc = self.lib.orc_decode(self.h, _ptr(recs), len(recs), _ptr(out), len(out), _ptr(offs),
                                 len(offs), ctypes.byref(nr))
        if rc < 0:
            raise RuntimeError(f"oracle decode failed rc={rc}")
        return out[:rc], offs[:nr.value + 1]


def load_golden(name):
    with gzip.open(os.path.join(GOLDEN, name + ".json.gz"), "rt") as f:
        g = json.load(f)
    words = (g["n"] + 63) // 64
    g["rows_u64"] = [np.frombuffer(bytes.fromhex(g["rows"][c]), dtype="<u8")[:words].copy()
                     for c in "ACGT"]
    g["lcs_u8"] = np.frombuffer(bytes.fromhex(g["lcs"]), dtype=np.uint8).copy()
    return g


def golden_names():
    return sorted(f[:-8] for f in os.listdir(GOLDEN) if f.endswith(".json.gz"))


def pack_reads(reads):
    """list[str|bytes] -> (uint8 bases, uint64 offsets[n+1])"""
    bs = [r.encode() if isinstance(r, str) else r for r in reads]
    offs = np.zeros(len(bs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(b) for b in bs])
    return np.frombuffer(b"".join(bs) or b"\0", dtype=np.uint8)[: int(offs[-1])].copy(), offs
