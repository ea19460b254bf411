"""ctypes loader for the TEST-ONLY host emulation of the kernels' lane logic
(tests/emu/emu.cpp -> encode_core.h).  Used by -m "not gpu" tests only."""
import ctypes
import os
import subprocess

import numpy as np

from oracle_lib import REPO

EMU_SO = os.path.join(REPO, "tests", "emu", "libntc_emu.so")
_lib = None


def emu_lib():
    global _lib
    if _lib is None:
        deps = [os.path.join(REPO, "tests", "emu", "emu.cpp"),
                os.path.join(REPO, "ntcomp_amd", "csrc", "derived.h"),
                os.path.join(REPO, "ntcomp_amd", "csrc", "encode_core.h"),
                os.path.join(REPO, "ntcomp_amd", "csrc", "derived.cpp")]
        stale = lambda: (not os.path.exists(EMU_SO)) or any(os.path.getmtime(EMU_SO) < os.path.getmtime(d)
                                                             for d in deps)
        if stale():
            import fcntl  # one build at a time across pytest-xdist workers (re-checked under the lock)
            with open(os.path.join(REPO, "tests", "emu", ".build.lock"), "w") as lock:
                fcntl.flock(lock, fcntl.LOCK_EX)
                if stale():
                    subprocess.check_call(["make", "-s", "-B", "-C", os.path.join(REPO, "tests", "emu")])
                fcntl.flock(lock, fcntl.LOCK_UN)
        L = ctypes.CDLL(EMU_SO)
        P, u64 = ctypes.c_void_p, ctypes.c_uint64
        L.emu_encode.restype = ctypes.c_int
        L.emu_encode.argtypes = [P, P, P, u64, P, u64, P, P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.emu_path_cover.restype = ctypes.c_int
        L.emu_path_cover.argtypes = [P, P]
        L.emu_decode.restype = ctypes.c_int
        L.emu_decode.argtypes = [P, P, u64, P, u64, P, u64, P]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def make_view(n, k, rows, C, lcs):
    from ntcomp_amd import IndexView
    keep = [np.ascontiguousarray(r, dtype=np.uint64) for r in rows] + [np.ascontiguousarray(lcs, dtype=np.uint8)]
    v = IndexView()
    v.n_nodes, v.k = int(n), int(k)
    for c in range(4):
        v.rows[c] = keep[c].ctypes.data
        v.C[c] = int(C[c])
    v.lcs = keep[4].ctypes.data
    return v, keep


def emu_encode(n, k, rows, C, lcs, bases, offs, want_ms=False, variant=4, use_paths=True, tab_u=0):
    v, keep = make_view(n, k, rows, C, lcs)
    bases = np.ascontiguousarray(bases, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    total = int(offs[-1] - offs[0])
    recs = np.zeros(total + 1, dtype=np.uint64)
    roff = np.zeros(len(offs), dtype=np.uint64)
    bad = ctypes.c_int64(-1)
    d = np.zeros(total + 1, dtype=np.uint32)
    s = np.zeros(total + 1, dtype=np.uint32)
    rc = emu_lib().emu_encode(ctypes.byref(v), _p(bases), _p(offs), len(offs) - 1, _p(recs), len(recs), _p(roff),
                              ctypes.byref(bad), _p(d) if want_ms else None, _p(s) if want_ms else None,
                              variant, int(use_paths), int(tab_u))
    if rc:
        raise RuntimeError(f"emu_encode rc={rc} bad={bad.value}")
    out = (recs[: int(roff[-1])], roff)
    return out + ((d[:total], s[:total]) if want_ms else ())


def emu_decode(n, k, rows, C, lcs, recs):
    v, keep = make_view(n, k, rows, C, lcs)
    recs = np.ascontiguousarray(recs, dtype=np.uint64)
    flags = (recs >> np.uint64(56)).astype(np.uint8)
    total = int(np.where(flags & 2, flags >> 2, (recs >> np.uint64(32)) & np.uint64(0xFFFFFF)).sum())
    out = np.zeros(total + 1, dtype=np.uint8)
    offs = np.zeros(int((flags & 1).sum()) + 2, dtype=np.uint64)
    nr = ctypes.c_uint64()
    rc = emu_lib().emu_decode(ctypes.byref(v), _p(recs), len(recs), _p(out), len(out), _p(offs), len(offs),
                              ctypes.byref(nr))
    if rc:
        raise RuntimeError(f"emu_decode rc={rc}")
    return out[:total], offs[: nr.value + 1]


def emu_path_cover(n, k, rows, C, lcs):
    """(hash, text length, paths) of the host-built path cover (derived.cpp build_paths)."""
    v, keep = make_view(n, k, rows, C, lcs)
    out = np.zeros(3, dtype=np.uint64)
    rc = emu_lib().emu_path_cover(ctypes.byref(v), _p(out))
    if rc:
        raise RuntimeError(f"emu_path_cover rc={rc}")
    return int(out[0]), int(out[1]), int(out[2])


def emu_default_tab_u(k, lcs):
    """derived.cpp default_tab_u: the suffix-table depth the upload picks for this LCS array."""
    lib = emu_lib()
    lib.emu_default_tab_u.restype = ctypes.c_uint32
    lib.emu_default_tab_u.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]
    lcs = np.ascontiguousarray(lcs, dtype=np.uint8)
    return int(lib.emu_default_tab_u(len(lcs), k, lcs.ctypes.data))


def emu_wave_modes(n, k, rows, C, lcs, bases, offs):
    """k_ms4 wave divergence statistics (tests/emu/emu.cpp emu_wave_modes)"""
    v, keep = make_view(n, k, rows, C, lcs)
    bases = np.ascontiguousarray(bases, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    out = np.zeros(23, dtype=np.uint64)
    rc = emu_lib().emu_wave_modes(ctypes.byref(v), _p(bases), _p(offs), len(offs) - 1, _p(out))
    if rc:
        raise RuntimeError(f"emu_wave_modes rc={rc}")
    return out
