"""A compiled consumer of the C ABI (tests/abi_c/abi_check.c): it includes only
include/*.h and links libntcomp_gpu.so, so the struct layouts, integer widths and
const-ness that INTEGRATION.md's Rust binding relies on are checked by a compiler
(_Static_assert against the #[repr(C)] layout) and by the linker (every symbol it calls
must resolve).  The GPU half drives upload -> encode -> write_block -> read_block ->
decode (and the GPU packer) from C against the committed golden records."""
import os
import subprocess

import numpy as np
import pytest

from oracle_lib import load_golden, pack_reads

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "abi_c", "abi_check.c")
LIBDIR = os.path.join(REPO, "ntcomp_amd")


def build(tmp_path):
    exe = str(tmp_path / "abi_check")
    cmd = ["gcc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror", "-O1", "-I", os.path.join(REPO, "include"),
           SRC, "-o", exe, "-L", LIBDIR, "-lntcomp_gpu", "-Wl,-rpath," + LIBDIR]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_c99_consumer_compiles_links_and_reports_layout(tmp_path):
    exe = build(tmp_path)
    r = subprocess.run([exe, "--layout"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert '"ntc_index_view": 88' in r.stdout and '"ntc_block_meta": 152' in r.stdout


def test_c_consumer_rejects_a_wrong_layout(tmp_path):
    """The static asserts bite: a header whose ntc_index_view differs fails to compile."""
    bad = tmp_path / "inc"
    bad.mkdir()
    for h in os.listdir(os.path.join(REPO, "include")):
        txt = open(os.path.join(REPO, "include", h)).read()
        if h == "ntcomp_gpu.h":
            txt = txt.replace("    uint32_t reserved;\n    const uint64_t *rows[4];", "    uint64_t reserved;\n    const uint64_t *rows[4];")
            assert "uint64_t reserved;" in txt
        (bad / h).write_text(txt)
    r = subprocess.run(["gcc", "-std=c99", "-fsyntax-only", "-I", str(bad), SRC], capture_output=True, text=True)
    assert r.returncode != 0 and "abi_check.c" in r.stderr  # the layout asserts, not the header, fail


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["k91_err", "ecoli_like_k31"])
def test_c_consumer_round_trip_on_gpu(tmp_path, name):
    exe = build(tmp_path)
    g = load_golden(name)
    d = tmp_path / "data"
    d.mkdir()
    np.concatenate(g["rows_u64"]).astype("<u8").tofile(d / "rows.bin")
    g["lcs_u8"].tofile(d / "lcs.bin")
    bases, offs = pack_reads(g["reads"])
    bases.tofile(d / "bases.bin")
    offs.astype("<u8").tofile(d / "offs.bin")
    recs = np.array([w for r in g["records"] for w in r], dtype="<u8")
    recs.tofile(d / "recs.bin")
    (d / "meta.txt").write_text(" ".join(str(x) for x in [g["n"], g["k"], *g["C"], len(g["reads"]), len(recs)]))
    r = subprocess.run([exe, str(d)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi_check: OK" in r.stdout
