"""The ntcomp CLI (`python -m ntcomp_amd build|encode|decode`, src/cli.rs:27-93): FASTX
ingest + normalize on CPU; end-to-end encode/decode on the GPU, with encoded.dat checked
byte for byte against the container built from the CPU oracle's records."""
import gzip
import os
import subprocess
import sys

import numpy as np
import pytest

import ntcomp_amd as nt
from oracle_lib import OracleIndex

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cli(*args, stdout=None):
    return subprocess.run([sys.executable, "-m", "ntcomp_amd", *args], cwd=REPO, stdout=stdout,
                          stderr=subprocess.PIPE, check=True)


def test_fastx_normalize_fasta_fastq_gzip(tmp_path):
    fa = tmp_path / "x.fa"
    fa.write_text(">a desc\nacgtNNxu\nAC\n>b\n\n>c\nRYgg\r\n.~-\n")
    got = [(b.tobytes(), o.tolist()) for b, o in nt.FastxReader(str(fa))]
    assert got == [(b"ACGTNNNTACRYGG---", [0, 10, 10, 17])]
    fq = tmp_path / "x.fq.gz"
    with gzip.open(fq, "wt") as f:
        f.write("@r1\nACGT\n+\nIIII\n\n@r2 x\nttaa\n+r2\nIIII\n")
    got = [(b.tobytes(), o.tolist()) for b, o in nt.FastxReader(str(fq))]
    assert got == [(b"ACGTTTAA", [0, 4, 8])]
    bad = tmp_path / "bad.txt"
    bad.write_text("hello\n")
    with pytest.raises(nt.NtcError):
        nt.FastxReader(str(bad))


def test_fastx_batches_split_on_read_count(tmp_path):
    fq = tmp_path / "r.fq"
    with open(fq, "w") as f:
        for i in range(1000):
            f.write(f"@r{i}\n{'ACGT'[i % 4] * (1 + i % 7)}\n+\n{'I' * (1 + i % 7)}\n")
    rd = nt.FastxReader(str(fq))
    sizes = []
    while True:
        x = rd.batch(max_reads=300)
        if x is None:
            break
        sizes.append(len(x[1]) - 1)
    assert sizes == [300, 300, 300, 100]


def _norm_table():
    """needletail normalize(iupac=true) restated as a byte map, 0 = dropped (fastx.cpp header)."""
    t = np.full(256, ord("N"), dtype=np.uint8)
    for c in b"ACGTN-BDHVRYSWKM":
        t[c] = c
    for c in b"acgbdhvryswkm":
        t[c] = c - 32
    for c in b"tuU":
        t[c] = ord("T")
    t[ord("n")] = ord("N")
    for c in b".~":
        t[c] = ord("-")
    for c in b" \t\r\n":
        t[c] = 0
    return t


_NORM = _norm_table()


def _normalize(seq):
    v = _NORM[np.frombuffer(seq, dtype=np.uint8)]
    return v[v != 0].tobytes()


@pytest.mark.parametrize("fmt", ["fasta", "fastq"])
@pytest.mark.parametrize("gz", [False, True, "bz2", "xz", "zst", "bgzf", "gzmulti", "gzlib"])
def test_fastx_random_records_across_chunks(tmp_path, monkeypatch, fmt, gz):
    """Records of up to 3 Mbp with mixed case, IUPAC, junk bytes and CRLF endings, spread
    over several 8 MiB input chunks: every record's bases equal the restated normalize."""
    rng = np.random.default_rng(7 if fmt == "fasta" else 8)
    alphabet = np.frombuffer(b"ACGTACGTACGTACGTacgtnNuU.~-RYkmX*\t ", dtype=np.uint8)
    lens = [3_000_000, 0, 17, 150] + rng.integers(1, 40_000, 600).tolist()
    expect, parts = [], []
    for i, L in enumerate(lens):
        pure = rng.random() < 0.5
        seq = (np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, L)] if pure
               else alphabet[rng.integers(0, len(alphabet), L)]).tobytes()
        expect.append(_normalize(seq))
        eol = b"\r\n" if i % 5 == 0 else b"\n"
        if fmt == "fasta":
            w = int(rng.integers(50, 200)) if i % 3 else max(L, 1)
            lines = [seq[a:a + w] for a in range(0, L, w)] or [b""]
            parts.append(b">r%d some description%s%s%s" % (i, eol, eol.join(lines), eol))
        else:
            seq = seq.replace(b"\t", b"A").replace(b" ", b"C")  # one line per FASTQ sequence
            expect[-1] = _normalize(seq)
            parts.append(b"@r%d%s%s%s+%s%s%s" % (i, eol, seq, eol, eol, b"I" * L, eol))
    data = b"".join(parts)
    path = tmp_path / ("x." + fmt + {False: "", True: ".gz", "bz2": ".bz2", "xz": ".xz", "zst": ".zst", "bgzf": ".gz",
                                         "gzmulti": ".gz", "gzlib": ".gz"}[gz])
    if gz is True or gz == "gzlib":  # libdeflate whole-member path; gzlib: zlib's streaming path
        with gzip.open(path, "wb", compresslevel=1) as f:
            f.write(data)
        if gz == "gzlib":
            monkeypatch.setenv("NTC_FASTX_ZLIB", "1")
    elif gz == "bgzf":  # BGZF (bgzip): members of <= 64 KB with the BC extra field
        path.write_bytes(b"".join(_bgzf_member(data[i:i + 65280]) for i in range(0, len(data), 65280)))
    elif gz == "gzmulti":  # concatenated members, the first larger than the last (output size grows)
        h = len(data) * 9 // 10
        path.write_bytes(gzip.compress(data[:h], 1) + gzip.compress(data[h:], 1))
    elif gz == "bz2":  # two concatenated streams (pbzip2-style), decoded back to back
        import bz2
        h = len(data) // 2
        path.write_bytes(bz2.compress(data[:h], 1) + bz2.compress(data[h:], 1))
    elif gz == "xz":
        import lzma
        path.write_bytes(lzma.compress(data, preset=0))
    elif gz == "zst":  # two concatenated frames, decoded back to back
        h = len(data) // 2
        path.write_bytes(_zstd_compress(data[:h]) + _zstd_compress(data[h:]))
    else:
        path.write_bytes(data)
    got = []
    for b, o in nt.FastxReader(str(path)):
        got += [b[int(o[r]):int(o[r + 1])].tobytes() for r in range(len(o) - 1)]
    assert len(got) == len(expect)
    assert got == expect


@pytest.mark.parametrize("threads", [1, 3, 16])
def test_fastx_mapped_parallel_equals_streaming(tmp_path, monkeypatch, threads):
    """Plain FASTQ is memory-mapped and each batch parsed in parallel pieces cut at record
    starts (fastx.cpp parse_fq_range); batches, records and bases must equal the streaming
    parser's (NTC_FASTX_STREAM=1), including quality lines that begin with '@' or '+',
    CRLF endings, blank lines between records and a last line without a newline."""
    rng = np.random.default_rng(11)
    parts = []
    for i in range(60_000):
        L = int(rng.integers(0, 400)) if i % 97 else 0
        seq = np.frombuffer(b"ACGTacgtN", np.uint8)[rng.integers(0, 9, L)].tobytes()
        qual = np.frombuffer(b"@+I#5", np.uint8)[rng.integers(0, 5, L)].tobytes()
        eol = b"\r\n" if i % 7 == 0 else b"\n"
        parts.append(b"@r%d x%s%s%s+%s%s%s" % (i, eol, seq, eol, eol, qual, eol) + (b"\n" if i % 13 == 0 else b""))
    data = b"".join(parts).rstrip(b"\n")
    path = tmp_path / "p.fq"
    path.write_bytes(data)

    def batches(stream):
        if stream:
            monkeypatch.setenv("NTC_FASTX_STREAM", "1")
        else:
            monkeypatch.delenv("NTC_FASTX_STREAM", raising=False)
        rd = nt.FastxReader(str(path))
        if not stream:
            assert nt.lib().ntc_fastx_set_threads(rd.h, threads) == 0
        out = []
        while True:
            x = rd.batch(max_reads=7777, max_bases=1 << 21)
            if x is None:
                break
            out.append((x[0].tobytes(), x[1].tolist()))
        rd.close()
        return out

    a, b = batches(False), batches(True)
    assert len(a) == len(b) and a == b
    assert sum(len(o) - 1 for _, o in a) == 60_000


def test_fastx_fastq_quality_length_must_match(tmp_path):
    """needletail rejects a record whose quality and sequence lengths differ (the reference
    then panics in read_from_fastx_parser, main.rs:46): NTC_ERR_FORMAT, mapped or streamed."""
    for name, data in (("plain.fq", b"@a\nACGT\n+\nIII\n"), ("z.fq.gz", gzip.compress(b"@a\nACGT\n+\nIIIII\n"))):
        p = tmp_path / name
        p.write_bytes(data)
        rd = nt.FastxReader(str(p))
        with pytest.raises(nt.NtcError) as e:
            rd.batch()
        assert e.value.code == 8


def _bgzf_member(chunk):
    import struct
    import zlib
    c = zlib.compressobj(1, zlib.DEFLATED, -15)
    body = c.compress(chunk) + c.flush()
    bsize = 18 + len(body) + 8
    hdr = b"\x1f\x8b\x08\x04" + b"\0" * 4 + b"\x00\xff" + struct.pack("<H", 6) + b"BC" + struct.pack("<HH", 2, bsize - 1)
    return hdr + body + struct.pack("<II", zlib.crc32(chunk), len(chunk))


def _zstd_compress(data, level=1):
    """one zstd frame through the image's libzstd.so.1 (test helper; no zstd module or CLI here)"""
    import ctypes
    z = ctypes.CDLL("libzstd.so.1")
    z.ZSTD_compressBound.restype = ctypes.c_size_t
    z.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
    z.ZSTD_compress.restype = ctypes.c_size_t
    z.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
    z.ZSTD_isError.argtypes = [ctypes.c_size_t]
    cap = z.ZSTD_compressBound(len(data))
    buf = ctypes.create_string_buffer(cap)
    n = z.ZSTD_compress(buf, cap, data, len(data), level)
    assert not z.ZSTD_isError(n)
    return buf.raw[:n]


def test_fastx_truncated_and_corrupt_compression(tmp_path):
    """needletail/niffler-style detection by magic bytes: a truncated bzip2 or zstd stream and
    a corrupt zstd frame are I/O errors, never garbage."""
    import bz2
    data = b"".join(b"@r%d\nACGTACGTAC\n+\nIIIIIIIIII\n" % i for i in range(20000))
    (tmp_path / "t.fq.bz2").write_bytes(bz2.compress(data)[:-200])
    with pytest.raises(nt.NtcError) as e:
        for _ in nt.FastxReader(str(tmp_path / "t.fq.bz2")):
            pass
    assert e.value.code == 9
    (tmp_path / "t.fq.zst").write_bytes(_zstd_compress(data)[:-50])
    (tmp_path / "z.fq.zst").write_bytes(bytes([0x28, 0xB5, 0x2F, 0xFD]) + b"\0" * 64)
    (tmp_path / "t.fq.gz").write_bytes(gzip.compress(data)[:-100])
    (tmp_path / "c.fq.gz").write_bytes(gzip.compress(data)[:-8] + b"\0" * 8)  # bad CRC / ISIZE
    for name in ("t.fq.zst", "z.fq.zst", "t.fq.gz", "c.fq.gz"):
        with pytest.raises(nt.NtcError) as e:
            for _ in nt.FastxReader(str(tmp_path / name)):
                pass
        assert e.value.code == 9


def test_fastx_gzip_padding_and_mixed_members(tmp_path):
    """zlib's gzread ignores bytes after the last member (e.g. zero padding) and reads any
    mix of members; the libdeflate readers must agree: padding ends the input, and a
    non-BGZF member after BGZF ones hands the rest to zlib (delivered bytes skipped)."""
    recs = [b"@r%d\n%s\n+\n%s\n" % (i, b"ACGT" * (1 + i % 9), b"I" * (4 * (1 + i % 9))) for i in range(30000)]
    data = b"".join(recs)
    exp = [r.split(b"\n")[1] for r in recs]
    half = len(data) // 2
    cases = {
        "pad.fq.gz": gzip.compress(data, 1) + b"\0" * 4096,
        "multipad.fq.gz": gzip.compress(data[:half], 1) + gzip.compress(data[half:], 1) + b"\0" * 16,
        "mixed.fq.gz": b"".join(_bgzf_member(data[i:i + 65280]) for i in range(0, half, 65280)) +
        gzip.compress(data[((half + 65279) // 65280) * 65280:], 1),
    }
    for name, blob in cases.items():
        (tmp_path / name).write_bytes(blob)
        got = []
        for b, o in nt.FastxReader(str(tmp_path / name)):
            got += [b[int(o[r]):int(o[r + 1])].tobytes() for r in range(len(o) - 1)]
        assert got == exp, name


def test_fasta_format():
    b = np.frombuffer(b"ACGTTT", dtype=np.uint8)
    assert nt.fasta_format(b, np.array([0, 4, 4, 6], dtype=np.uint64), 9) == b">seq.9\nACGT\n>seq.10\n\n>seq.11\nTT\n"


def test_cli_build_writes_a_loadable_index(tmp_path):
    g = nt.synth_genome(3, 20_000).tobytes().decode()
    fa = tmp_path / "g.fa"
    fa.write_text(">g\n" + "\n".join(g[i:i + 60] for i in range(0, len(g), 60)) + "\n")
    _cli("build", "-o", str(tmp_path / "idx"), "-k", "31", str(fa))
    ix = nt.Index.load(str(tmp_path / "idx"))
    ref = nt.Index.build([g.encode()], 31)
    assert ix.n == ref.n and np.array_equal(ix.lcs, ref.lcs)
    assert all(np.array_equal(a, b) for a, b in zip(ix.rows, ref.rows))


@pytest.mark.gpu
def test_cli_encode_decode_end_to_end(tmp_path):
    genome = nt.synth_genome(4, 300_000)
    fa = tmp_path / "g.fa"
    fa.write_text(">g\n" + genome.tobytes().decode() + "\n")
    _cli("build", "-o", str(tmp_path / "idx"), "-k", "31", "-t", "4", str(fa))
    n, L = 140_000, 100  # three blocks of 65,536 reads (the last one partial)
    reads = nt.synth_reads(genome, 9, 0, n, L, 10_000)
    fq = tmp_path / "r.fq.gz"
    with gzip.open(fq, "wb", compresslevel=1) as f:
        for i in range(n):
            s = reads[i * L:(i + 1) * L].tobytes()
            f.write(b"@r%d\n" % i + s + b"\n+\n" + b"I" * L + b"\n")
    enc = tmp_path / "enc.dat"
    with open(enc, "wb") as f:
        _cli("encode", "-i", str(tmp_path / "idx"), "--blocks-per-batch", "1", "--deflate", "zlib", str(fq), stdout=f)
    # container from the oracle's records, block by block (main.rs:162-177)
    ix = nt.Index.load(str(tmp_path / "idx"))
    orc = OracleIndex(ix.n, 31, ix.rows, ix.C, ix.lcs)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    exp = nt.file_header()
    for b0 in range(0, n, 65536):
        b1 = min(n, b0 + 65536)
        recs, _ = orc.encode(reads[b0 * L:b1 * L], offs[: b1 - b0 + 1])
        exp += nt.write_block(recs, b1 - b0)
    assert enc.read_bytes() == exp
    dec = tmp_path / "dec.fa"
    with open(dec, "wb") as f:
        _cli("decode", "-i", str(tmp_path / "idx"), str(enc), stdout=f)
    lines = dec.read_bytes().split(b"\n")
    assert lines[-1] == b"" and len(lines) == 2 * n + 1
    assert lines[0] == b">seq.1" and lines[2 * (n - 1)] == b">seq.%d" % n
    assert b"".join(lines[1::2]) == reads.tobytes()


NATIVE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ntcomp_amd", "ntcomp")


def test_native_cli_build_equals_python_cli(tmp_path):
    """`ntcomp build` as a native binary (ntcomp_main.cpp, no interpreter) writes the same
    index files as the Python CLI, with -l lists, several files and the sbwt-rs layout + -p;
    without a GPU `--builder auto` uses the host builder."""
    g = nt.synth_genome(5, 30_000).tobytes().decode()
    (tmp_path / "a.fa").write_text(">a\n" + g[:17_000] + "\n")
    (tmp_path / "b.fq").write_text("@b\n" + g[17_000:] + "\n+\n" + "I" * (30_000 - 17_000) + "\n")
    (tmp_path / "list.txt").write_text(f"x\t{tmp_path / 'b.fq'}\n")
    for fmt in ("own", "sbwt-rs"):
        subprocess.run([NATIVE, "build", "-o", str(tmp_path / "n"), "-k", "31", "--builder", "host",
                        "--index-format", fmt, "-p", "5", "-l", str(tmp_path / "list.txt"), str(tmp_path / "a.fa")],
                       check=True, stderr=subprocess.PIPE)
        _cli("build", "-o", str(tmp_path / "p"), "-k", "31", "--builder", "host", "--index-format", fmt, "-p", "5",
             "-l", str(tmp_path / "list.txt"), str(tmp_path / "a.fa"))
        for ext in (".sbwt", ".lcs"):
            assert (tmp_path / ("n" + ext)).read_bytes() == (tmp_path / ("p" + ext)).read_bytes(), (fmt, ext)
    assert nt.Index.load(str(tmp_path / "n")).prefix_table()[0] == 5
    r = subprocess.run([NATIVE], stderr=subprocess.PIPE)
    assert r.returncode == 2 and b"usage" in r.stderr


def test_cli_build_writes_sbwt_rs_layout_by_default(tmp_path):
    """The reference always writes sbwt-rs files (kbo::index::serialize_sbwt, main.rs:138) with
    the -p 8 prefix table (cli.rs:46): both CLIs do so by default, `--index-format own` is the
    opt-in, and Index.load reads either."""
    g = nt.synth_genome(7, 20_000).tobytes().decode()
    (tmp_path / "a.fa").write_text(">a\n" + g + "\n")
    subprocess.run([NATIVE, "build", "-o", str(tmp_path / "n"), "--builder", "host", str(tmp_path / "a.fa")],
                   check=True, stderr=subprocess.PIPE)
    _cli("build", "-o", str(tmp_path / "p"), "--builder", "host", str(tmp_path / "a.fa"))
    _cli("build", "-o", str(tmp_path / "own"), "--builder", "host", "--index-format", "own", str(tmp_path / "a.fa"))
    for ext in (".sbwt", ".lcs"):
        assert (tmp_path / ("n" + ext)).read_bytes() == (tmp_path / ("p" + ext)).read_bytes(), ext
    assert (tmp_path / "n.sbwt").read_bytes()[:8] != b"NTCSBWT1"
    assert (tmp_path / "own.sbwt").read_bytes()[:8] == b"NTCSBWT1"
    # build_select = true (main.rs:118-119): every row carries rank and select, not select_zero
    from test_builder import _read_rows
    for _, _, _, (rank, sel, selz) in _read_rows((tmp_path / "n.sbwt").read_bytes())[0]:
        assert rank is not None and len(rank) > 0 and sel is not None and len(sel) > 0 and selz is None
    a, b = nt.Index.load(str(tmp_path / "n")), nt.Index.load(str(tmp_path / "own"))
    assert a.prefix_table()[0] == 8 and a.k == b.k == 31 and a.n == b.n
    assert all(np.array_equal(x, y) for x, y in zip(a.rows, b.rows)) and np.array_equal(a.lcs, b.lcs)


def test_native_cli_rejects_unknown_options(tmp_path):
    """clap rejects arguments it does not know (src/cli.rs); so does the native CLI, instead of
    taking `--gpu 2` as a switch and '2' as the input file."""
    for args in (["encode", "-i", "x", "--gpu", "2", "r.fq"], ["build", "-o", "x", "--mem", "3", "a.fa"],
                 ["decode", "-i", "x", "--stat", "e.dat"], ["encode", "-i", "x", "--gpux=2", "r.fq"]):
        r = subprocess.run([NATIVE, *args], stderr=subprocess.PIPE, cwd=tmp_path)
        assert r.returncode != 0 and b"unexpected argument" in r.stderr, (args, r.stderr)


def test_native_cli_accepts_clap_forms(tmp_path):
    """Forms clap accepts (src/cli.rs): an attached short value (`-k31`, `-t2`, `-p5`),
    `-h`/`--help` (usage on stdout, exit 0) and `-V`/`--version` (Cargo.toml's version)."""
    g = nt.synth_genome(11, 12_000).tobytes().decode()
    (tmp_path / "a.fa").write_text(">a\n" + g + "\n")
    subprocess.run([NATIVE, "build", "-o", str(tmp_path / "x"), "-k31", "-t2", "-p5", "--builder", "host",
                    str(tmp_path / "a.fa")], check=True, stderr=subprocess.PIPE)
    subprocess.run([NATIVE, "build", "-o", str(tmp_path / "y"), "-k", "31", "-t", "2", "-p", "5", "--builder", "host",
                    str(tmp_path / "a.fa")], check=True, stderr=subprocess.PIPE)
    for ext in (".sbwt", ".lcs"):
        assert (tmp_path / ("x" + ext)).read_bytes() == (tmp_path / ("y" + ext)).read_bytes(), ext
    assert nt.Index.load(str(tmp_path / "x")).k == 31
    for args in (["-h"], ["--help"], ["build", "-h"], ["encode", "--help"]):
        r = subprocess.run([NATIVE, *args], capture_output=True)
        assert r.returncode == 0 and b"usage" in r.stdout, args
    for args in (["-V"], ["--version"], ["decode", "-V"]):
        r = subprocess.run([NATIVE, *args], capture_output=True)
        assert r.returncode == 0 and r.stdout.strip() == b"ntcomp 0.1.0", args
    r = subprocess.run([sys.executable, "-m", "ntcomp_amd", "--version"], cwd=REPO, capture_output=True)
    assert r.returncode == 0 and b"ntcomp 0.1.0" in r.stdout


@pytest.mark.gpu
def test_native_cli_encode_decode_equal_python_cli(tmp_path):
    """`ntcomp encode|decode` (native) and `python -m ntcomp_amd encode|decode` write the same
    bytes: the same native pipelines behind both (ntc_encode_file / ntc_decode_file)."""
    genome = nt.synth_genome(6, 300_000)
    (tmp_path / "g.fa").write_text(">g\n" + genome.tobytes().decode() + "\n")
    subprocess.run([NATIVE, "build", "-o", str(tmp_path / "idx"), "-k", "31", str(tmp_path / "g.fa")], check=True,
                   stderr=subprocess.PIPE)
    # default flags: the sbwt-rs layout with the -p 8 prefix table, read back by encode/decode
    assert (tmp_path / "idx.sbwt").read_bytes()[:8] != b"NTCSBWT1"
    assert nt.Index.load(str(tmp_path / "idx")).prefix_table()[0] == 8
    n, L = 150_000, 100
    reads = nt.synth_reads(genome, 9, 0, n, L, 10_000)
    fq = tmp_path / "r.fq"
    fq.write_bytes(b"".join(b"@r\n" + reads[i * L:(i + 1) * L].tobytes() + b"\n+\n" + b"I" * L + b"\n"
                            for i in range(n)))
    with open(tmp_path / "n.dat", "wb") as f:
        subprocess.run([NATIVE, "encode", "-i", str(tmp_path / "idx"), "--deflate", "zlib", "--devices", "0,0",
                        str(fq)], stdout=f, stderr=subprocess.PIPE, check=True)
    with open(tmp_path / "p.dat", "wb") as f:
        _cli("encode", "-i", str(tmp_path / "idx"), "--deflate", "zlib", str(fq), stdout=f)
    assert (tmp_path / "n.dat").read_bytes() == (tmp_path / "p.dat").read_bytes()
    with open(tmp_path / "n.fa", "wb") as f:
        subprocess.run([NATIVE, "decode", "-i", str(tmp_path / "idx"), str(tmp_path / "n.dat")], stdout=f,
                       stderr=subprocess.PIPE, check=True)
    lines = (tmp_path / "n.fa").read_bytes().split(b"\n")
    assert b"".join(lines[1::2]) == reads.tobytes() and lines[0] == b">seq.1"


@pytest.mark.gpu
def test_native_cli_build_budgets(tmp_path):
    """-m bounds a GPU build pass's device memory; without --temp-dir nothing spills to disk
    however small -m is (the reference builds on disk only with --temp-dir, cli.rs:58-60);
    with it, partitions past -m GB of host memory go there.  The same index either way."""
    genome = nt.synth_genome(3, 400_000)
    (tmp_path / "g.fa").write_text(">g\n" + genome.tobytes().decode() + "\n")
    outs = {}
    for name, extra in (("mem", ["-m", "0.005"]), ("tmp", ["-m", "0.001", "--temp-dir", str(tmp_path)]),
                        ("def", [])):
        r = subprocess.run([NATIVE, "build", "-o", str(tmp_path / name), "--builder", "gpu", "--verbose", *extra,
                            str(tmp_path / "g.fa")], check=True, stderr=subprocess.PIPE)
        err = r.stderr.decode()
        line = [x for x in err.splitlines() if x.startswith("build:")][0]
        outs[name] = (line, (tmp_path / f"{name}.sbwt").read_bytes(), (tmp_path / f"{name}.lcs").read_bytes())
    assert outs["mem"][1:] == outs["def"][1:] == outs["tmp"][1:]
    assert "spilled 0 B" in outs["mem"][0] and "spilled 0 B" in outs["def"][0], outs
    assert " 1 + 1 passes" not in outs["mem"][0], outs["mem"][0]  # -m 5 MB: several passes
    assert "spilled 0 B" not in outs["tmp"][0], outs["tmp"][0]
