"""Host C++ under the sanitizers: tests/san builds the library's host
code -- FASTX ingest (fastx.cpp), the block codec (block_codec.cpp), index files
(index_io.cpp), the threaded host builder (sbwt_build.cpp) and the native file pipelines'
host threads (pipeline.cpp: reader ring, deflate / inflate pool, ordered writer; the GPU
stage stubbed on the CPU by the oracle, tests/san/gpu_stub.cpp) -- once with
-fsanitize=address,undefined and once with -fsanitize=thread, and drives it over valid,
truncated and corrupt inputs: gzip / BGZF / bz2 / xz / zstd FASTX, damaged encoded.dat
blocks (decode_block's Err ends the reference's loop, src/main.rs:202), damaged index
files.  Every run must be free of sanitizer reports and give the production library's
answer."""
import bz2
import gzip
import lzma
import os
import struct
import subprocess

import numpy as np
import pytest

import ntcomp_amd as nt
from oracle_lib import OracleIndex

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(REPO, "tests", "san")
ENV = dict(os.environ,
           ASAN_OPTIONS="halt_on_error=1:detect_leaks=1:abort_on_error=0:exitcode=66",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
           TSAN_OPTIONS="halt_on_error=1:exitcode=66:second_deadlock_stack=1",
           NTC_THREADS="4")
MASK = (1 << 64) - 1


@pytest.fixture(scope="module")
def san():
    # one build at a time (pytest-xdist workers share tests/san: a relink under a binary
    # another worker is running fails with a permission error)
    import fcntl
    with open(os.path.join(SAN, ".build.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        subprocess.check_call(["make", "-s", "-j2", "-C", SAN])
        fcntl.flock(lock, fcntl.LOCK_UN)
    return {"asan": os.path.join(SAN, "san_asan"), "tsan": os.path.join(SAN, "san_tsan")}


def run(binary, *args):
    r = subprocess.run([binary, *map(str, args)], env=ENV, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=600)
    err = r.stderr.decode(errors="replace")
    assert r.returncode == 0 and "Sanitizer" not in err and "runtime error" not in err, err[-4000:]
    return dict(x.split("=", 1) for x in r.stdout.decode().split())


def fnv(h, data):
    for b in data:
        h = ((h ^ b) * 0x100000001B3) & MASK
    return h


def fastx_digest(path, max_reads=1 << 20):
    """(rc, reads, bases, hash) through the production reader, as san_driver prints them."""
    h, reads, bases = 0xCBF29CE484222325, 0, 0
    try:
        rd = nt.FastxReader(path)
        while True:
            x = rd.batch(max_reads)
            if x is None:
                break
            b, o = x
            for r in range(len(o) - 1):
                L = int(o[r + 1] - o[r])
                h = fnv(h, L.to_bytes(8, "little"))
                h = fnv(h, b[int(o[r]):int(o[r + 1])].tobytes())
            reads += len(o) - 1
            bases += int(o[-1] - o[0])
        rd.close()
        rc = 0
    except nt.NtcError as e:
        rc = e.code
    return rc, reads, bases, h


def _reads(n, L, seed):
    rng = np.random.default_rng(seed)
    return [bytes(rng.choice(list(b"ACGTacgtN"), int(rng.integers(1, L)))) for _ in range(n)]


def test_fastx_under_sanitizers(san, tmp_path):
    from test_cli import _bgzf_member, _zstd_compress
    seqs = _reads(2000, 160, 1)
    fq = b"".join(b"@r%d x\n%s\n+\n%s\n" % (i, s, b"I" * len(s)) for i, s in enumerate(seqs))
    fa = b"".join(b">r%d\n%s\n" % (i, b"\n".join(s[j:j + 50] for j in range(0, len(s), 50))) for i, s in enumerate(seqs))
    files = {"p.fq": fq, "p.fa": fa, "g.fq.gz": gzip.compress(fq), "x.fq.xz": lzma.compress(fq),
             "b.fq.bz2": bz2.compress(fq), "z.fa.zst": _zstd_compress(fa),
             "bg.fq.gz": b"".join(_bgzf_member(fq[i:i + 9000]) for i in range(0, len(fq), 9000)),
             "gpad.fq.gz": gzip.compress(fq) + b"\0" * 100,
             # damaged inputs: I/O errors, never garbage or a crash
             "t.fq.gz": gzip.compress(fq)[:-100], "c.fq.gz": gzip.compress(fq)[:-8] + b"\0" * 8,
             "t.fq.bz2": bz2.compress(fq)[:-200], "t.fq.xz": lzma.compress(fq)[:-40],
             "t.fa.zst": _zstd_compress(fa)[:-50], "tbg.fq.gz": files_bgzf_trunc(fq),
             "bad.fq": fq[:-3], "q.fq": b"@r\nACGT\n+\nII\n"}
    for name, data in files.items():
        (tmp_path / name).write_bytes(data)
        exp = fastx_digest(str(tmp_path / name), 300)
        for kind in ("asan", "tsan"):
            for threads, into in ((1, 0), (4, 1)):
                got = run(san[kind], "fastx", tmp_path / name, threads, 300, 1 << 16, into)
                if exp[0]:  # an error: same code, nothing after it matters
                    assert int(got["rc"]) == exp[0], (name, kind, got)
                else:
                    assert (int(got["rc"]), int(got["reads"]), int(got["bases"]), int(got["hash"], 16)) == exp, \
                        (name, kind, threads)


def files_bgzf_trunc(fq):
    from test_cli import _bgzf_member
    return b"".join(_bgzf_member(fq[i:i + 9000]) for i in range(0, len(fq), 9000))[:-30]


@pytest.fixture(scope="module")
def encoded(tmp_path_factory):
    """A 15-mer index of a 40 kbp genome and 3 blocks + a partial one of 50-base reads, as
    encoded.dat built from the oracle's records with the host codec (main.rs:162-177)."""
    d = tmp_path_factory.mktemp("san")
    genome = nt.synth_genome(8, 40_000)
    ix = nt.Index.build([genome.tobytes()], 15)
    ix.save(str(d / "idx"))
    n, L = 3 * 65536 + 77, 50
    reads = nt.synth_reads(genome, 4, 0, n, L, 20_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    recs, roff = OracleIndex(ix.n, 15, ix.rows, ix.C, ix.lcs).encode(reads, offs)
    data = nt.file_header()
    for b0 in range(0, n, 65536):
        b1 = min(n, b0 + 65536)
        data += nt.write_block(recs[int(roff[b0]):int(roff[b1])], b1 - b0)
    (d / "e.dat").write_bytes(data)
    body = reads.reshape(n, L)
    fq = b"".join(b"@r\n" + body[i].tobytes() + b"\n+\n" + b"I" * L + b"\n" for i in range(n))
    (d / "r.fq").write_bytes(fq)
    fasta = b"".join(b">seq.%d\n" % (i + 1) + body[i].tobytes() + b"\n" for i in range(n))
    return d, ix, data, fasta


def blocks_digest(data):
    h, pos, blocks, total, rc = 0xCBF29CE484222325, 32 if len(data) >= 32 else len(data), 0, 0, 0
    while pos < len(data):
        try:
            r, used, num = nt.read_block(data[pos:])
        except nt.NtcError as e:
            rc = e.code
            break
        h = fnv(fnv(h, r.tobytes()), int(num).to_bytes(8, "little"))
        blocks += 1
        total += len(r)
        pos += used
    return rc, blocks, total, h


def test_block_codec_damaged_blocks_under_sanitizers(san, encoded, tmp_path):
    d, ix, data, _ = encoded
    rng = np.random.default_rng(9)
    cases = {"whole": data, "header_only": data[:32], "short": data[:20], "trunc": data[:-11]}
    for i in range(12):  # flipped bytes anywhere: stream headers, gzip headers, deflate data
        b = bytearray(data)
        for p in rng.integers(32, len(b), 3):
            b[int(p)] ^= int(rng.integers(1, 256))
        cases[f"flip{i}"] = bytes(b)
    for i in range(4):  # a stream header's sizes overwritten
        b = bytearray(data)
        p = 32 + 16 * i
        b[p:p + 8] = bytes(rng.integers(0, 256, 8, dtype=np.uint8))
        cases[f"hdr{i}"] = bytes(b)
    for name, blob in cases.items():
        (tmp_path / name).write_bytes(blob)
        exp = blocks_digest(blob)
        got = run(san["asan"], "blocks", tmp_path / name)
        assert (int(got["rc"]), int(got["blocks"]), int(got["recs"]), int(got["hash"], 16)) == exp, name


def test_index_files_under_sanitizers(san, encoded, tmp_path):
    d, ix, _, _ = encoded
    exp = run(san["asan"], "index", d / "idx")
    assert int(exp["rc"]) == 0 and int(exp["n"]) == ix.n
    # own -> sbwt-rs (with a 6-character prefix table) -> loaded again: same index
    got = run(san["asan"], "index", d / "idx", tmp_path / "rs", 1, 6)
    assert got == exp
    assert run(san["asan"], "index", tmp_path / "rs") == exp
    jx = nt.Index.load(str(tmp_path / "rs"))
    assert jx.prefix_table()[0] == 6 and jx.n == ix.n
    # truncated / foreign files fail cleanly
    for ext in (".sbwt", ".lcs"):
        for cut in (7, 60, 1000):
            blob = (tmp_path / ("rs" + ext)).read_bytes()
            for other in (".sbwt", ".lcs"):
                (tmp_path / ("x" + other)).write_bytes((tmp_path / ("rs" + other)).read_bytes())
            (tmp_path / ("x" + ext)).write_bytes(blob[:cut])
            assert int(run(san["asan"], "index", tmp_path / "x")["rc"]) == 1, (ext, cut)
            own = (d / ("idx" + ext)).read_bytes()
            for other in (".sbwt", ".lcs"):
                (tmp_path / ("y" + other)).write_bytes((d / ("idx" + other)).read_bytes())
            (tmp_path / ("y" + ext)).write_bytes(own[:cut])
            assert int(run(san["asan"], "index", tmp_path / "y")["rc"]) == 1, (ext, cut)


def test_host_builder_under_sanitizers(san, tmp_path):
    g = nt.synth_genome(11, 300_000)
    st = nt.synth_strains(g, 2, 2, 10_000)
    text = [g.tobytes(), st[0].tobytes(), st[1].tobytes(), b"ACGTNNACGTAC" * 50]
    (tmp_path / "g.fa").write_bytes(b"".join(b">s%d\n%s\n" % (i, t) for i, t in enumerate(text)))
    ref = nt.Index.build(text, 31, threads=4)
    for kind in ("asan", "tsan"):
        got = run(san[kind], "build", tmp_path / "g.fa", 31, 4)
        assert int(got["n"]) == ref.n, kind


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_pipelines_under_sanitizers(san, encoded, tmp_path, kind):
    """ntc_encode_file / ntc_decode_file with two (stub) contexts, 4 pool threads, one block
    per batch and 1 Mi-base ring buffers: encoded.dat byte-identical to the blockwise host
    codec (zlib), the FASTA to the reads; a damaged block ends the decode after the blocks
    before it; libdeflate's blocks inflate to the same streams."""
    d, ix, data, fasta = encoded
    got = run(san[kind], "encode", d / "idx", d / "r.fq", tmp_path / "e.dat", 4, 1, 2, 0)
    assert int(got["rc"]) == 0 and int(got["blocks"]) == 4, got
    assert (tmp_path / "e.dat").read_bytes() == data
    got = run(san[kind], "decode", d / "idx", tmp_path / "e.dat", tmp_path / "o.fa", 4, 1, 2)
    assert int(got["rc"]) == 0, got
    assert (tmp_path / "o.fa").read_bytes() == fasta
    # batches of 3 blocks after a first batch of one (the writer starts on the first block)
    for fb in ("1", "2", "3"):
        ENV["NTC_FIRST_BATCH_BLOCKS"] = fb
        try:
            got = run(san[kind], "decode", d / "idx", tmp_path / "e.dat", tmp_path / "o3.fa", 4, 3, 2)
        finally:
            del ENV["NTC_FIRST_BATCH_BLOCKS"]
        assert int(got["rc"]) == 0 and int(got["blocks"]) == 4, (fb, got)
        assert (tmp_path / "o3.fa").read_bytes() == fasta, fb
    if nt.libdeflate_available():
        got = run(san[kind], "encode", d / "idx", d / "r.fq", tmp_path / "l.dat", 3, 2, 1, 1)
        assert int(got["rc"]) == 0
        assert blocks_digest((tmp_path / "l.dat").read_bytes()) == blocks_digest(data)
    bad = bytearray(data)
    pos = 32
    for _ in range(2):  # third block: corrupt its first stream's deflate data
        pos += nt.read_block(data[pos:])[1]
    bad[pos + 32 + 12:pos + 32 + 40] = b"\xff" * 28
    (tmp_path / "bad.dat").write_bytes(bytes(bad))
    got = run(san[kind], "decode", d / "idx", tmp_path / "bad.dat", tmp_path / "b.fa", 4, 1, 2)
    assert int(got["rc"]) == 0 and int(got["blocks"]) == 2 and int(got["dropped"]) == 2, got
    assert (tmp_path / "b.fa").read_bytes() == fasta[:fasta.index(b">seq.%d\n" % (2 * 65536 + 1))]
    # third block: a stream header's encoded_size (or num_u64) damaged, its gzip data intact --
    # a damaged block that ends the output, not a 32 GiB pinned allocation
    for field, stream in ((12, 1), (12, 3), (8, 2)):
        bad = bytearray(data)
        p = pos
        for _ in range(stream):
            p += 32 + int.from_bytes(data[p:p + 4], "little")
        bad[p + field:p + field + 4] = b"\xff\xff\xff\xff"
        (tmp_path / "bad2.dat").write_bytes(bytes(bad))
        got = run(san[kind], "decode", d / "idx", tmp_path / "bad2.dat", tmp_path / "b2.fa", 4, 1, 2)
        assert int(got["rc"]) == 0 and int(got["blocks"]) == 2 and int(got["dropped"]) == 2, (field, stream, got)
        assert (tmp_path / "b2.fa").read_bytes() == fasta[:fasta.index(b">seq.%d\n" % (2 * 65536 + 1))]
    # a read with a base absent from the index: the pipeline reports it, nothing hangs
    fq = (d / "r.fq").read_bytes().replace(b"\n+\n", b"\n+\n", 1)
    lines = fq.split(b"\n")
    lines[4 * 70001 + 1] = b"N" + lines[4 * 70001 + 1][1:]
    (tmp_path / "n.fq").write_bytes(b"\n".join(lines))
    got = run(san[kind], "encode", d / "idx", tmp_path / "n.fq", tmp_path / "n.dat", 4, 1, 2, 0)
    assert int(got["rc"]) == 2 and int(got["bad"]) == 70001, got


def test_pipeline_text_reader_edge_cases_under_sanitizers(san, encoded, tmp_path):
    """The encode reader's GPU-parse path (pipeline.cpp fill_text: copy + newline scan, cuts
    after the last whole block, hand-over to the host parser) against the host parser
    (host_parse = 1) on FASTQ shapes the host parser accepts or rejects: CRLF, lower case,
    no final newline, blank lines mid-file / at either end, a truncated last record.  Same
    rc, counts and encoded.dat bytes either way (the stub's GPU parse restates fastq.hip)."""
    d, ix, _, _ = encoded
    genome = nt.synth_genome(8, 40_000)
    n, L = 65536 + 300, 40
    body = nt.synth_reads(genome, 5, 0, n, L, 20_000).reshape(n, L)
    recs = [b"@r%d\n" % i + body[i].tobytes() + b"\n+\n" + b"I" * L + b"\n" for i in range(n)]
    plain = b"".join(recs)
    lower = b"".join(r.replace(body[i].tobytes(), body[i].tobytes().lower()) if i % 7 == 0 else r
                     for i, r in enumerate(recs))
    mid_blank = b"".join(recs[:65600]) + b"\n\r\n" + b"".join(recs[65600:])
    cases = {
        "plain": (plain, True),
        "crlf": (plain.replace(b"\n", b"\r\n"), True),
        "lower": (lower, True),
        "no_final_newline": (plain[:-1], True),
        "mid_blank": (mid_blank, True),
        "trailing_blank": (plain + b"\n\n\n", True),
        "leading_blank": (b"\n" + plain, False),
        "truncated": (plain[:plain.rindex(b"\n+\n")], True),
    }
    # read lengths changing mid-file (the batch-size estimate and the carried text disagree)
    long_body = nt.synth_reads(genome, 6, 0, 300, 400, 20_000).reshape(300, 400)
    ragged = b"".join(recs[:65536 + 100]) + b"".join(
        b"@l%d\n" % i + long_body[i].tobytes() + b"\n+\n" + b"I" * 400 + b"\n" for i in range(300))
    cases["ragged"] = (ragged, True)
    # the same through a decoder (the streamed text path): gzip and BGZF
    from test_cli import _bgzf_member
    for name in ("plain", "crlf", "mid_blank", "truncated", "no_final_newline", "ragged"):
        blob, tf = cases[name]
        cases[name + ".gz"] = (gzip.compress(blob, 1), tf)
        cases[name + ".bgzf"] = (b"".join(_bgzf_member(blob[i:i + 60000]) for i in range(0, len(blob), 60000)), tf)
    # BGZF members the direct (parallel, libdeflate) path rejects: the reader drops to its
    # buffered path and zlib, as the host-parse path does -- same rc and bytes
    import struct
    members = [_bgzf_member(plain[i:i + 60000]) for i in range(0, len(plain), 60000)]
    bad_crc = bytearray(members[40])
    bad_crc[-8] ^= 0xFF
    cases["bad_crc.bgzf"] = (b"".join(members[:40]) + bytes(bad_crc) + b"".join(members[41:]), None)
    slack = bytearray(members[40]) + b"\0" * 8  # BSIZE covers 8 bytes past the gzip trailer
    struct.pack_into("<H", slack, 16, len(slack) - 1)
    cases["slack.bgzf"] = (b"".join(members[:40]) + bytes(slack) + b"".join(members[41:]), None)
    for name, (blob, text_first) in cases.items():
        (tmp_path / f"{name}.fq").write_bytes(blob)
        got = {}
        for hp in (0, 1):
            got[hp] = run(san["asan"], "encode", d / "idx", tmp_path / f"{name}.fq", tmp_path / f"{name}{hp}.dat",
                          4, 1, 2, 0, hp)
        assert int(got[1]["text"]) == 0
        assert text_first is None or (int(got[0]["text"]) > 0) == text_first, (name, got[0])
        if name.endswith(".bgzf"):  # BGZF inflated in parallel straight into the batch: under TSan too
            t = run(san["tsan"], "encode", d / "idx", tmp_path / f"{name}.fq", tmp_path / f"{name}t.dat", 4, 1, 2, 0, 0)
            assert t == got[0], (name, t)
            if int(t["rc"]) == 0:
                assert (tmp_path / f"{name}t.dat").read_bytes() == (tmp_path / f"{name}0.dat").read_bytes()
        # (a failing BGZF member: the same error either way; the text path's read count is
        # what it had cut before the error)
        for k in ("rc", "bad") if name.startswith(("bad_crc", "slack")) else ("rc", "reads", "bases", "blocks", "bad"):
            assert got[0][k] == got[1][k], (name, k, got)
        if int(got[0]["rc"]) == 0:
            assert int(got[0]["reads"]) == (65536 + 400 if name.startswith("ragged") else n), name
            assert (tmp_path / f"{name}0.dat").read_bytes() == (tmp_path / f"{name}1.dat").read_bytes(), name
        else:
            assert name.startswith(("truncated", "bad_crc", "slack")), (name, got)


def _gzip_cases():
    """gzip inputs for the parallel inflater (pgzip.cpp): every deflate block type and zlib
    strategy, several members, headers with a name, trailing bytes, and damaged members."""
    import io
    import zlib
    rng = np.random.default_rng(3)
    seqs = _reads(3000, 300, 4)
    fq = b"".join(b"@r%d x\n%s\n+\n%s\n" % (i, s, b"I" * len(s)) for i, s in enumerate(seqs))
    homo = b"".join(b"@h%d\n%s\n+\n%s\n" % (i, b"A" * 5000, b"I" * 5000) for i in range(40))
    junk = bytes(rng.choice(list(b"ACGTNRYKMacgtn-"), 300_000))
    fa = b"".join(b">s%d\n%s\n" % (i, junk[j:j + 3000]) for i, j in enumerate(range(0, len(junk), 3000)))

    def strat(data, s):
        c = zlib.compressobj(6, zlib.DEFLATED, 31, 8, s)
        return c.compress(data) + c.flush()

    def named(data):
        b = io.BytesIO()
        with gzip.GzipFile(filename="reads.fq", mode="wb", fileobj=b, mtime=0) as g:
            g.write(data)
        return b.getvalue()

    h = len(fq) // 3
    ok = {"l1.fq.gz": gzip.compress(fq, 1), "l6.fq.gz": gzip.compress(fq, 6), "l9.fq.gz": gzip.compress(fq, 9),
          "stored.fq.gz": gzip.compress(fq, 0), "multi.fq.gz": gzip.compress(fq[:h], 6) + gzip.compress(fq[h:], 1),
          "empty_first.fq.gz": gzip.compress(b"") + gzip.compress(fq),
          "named.fq.gz": named(fq), "tail.fq.gz": gzip.compress(fq) + b"not gzip" * 9,
          "homo.fq.gz": gzip.compress(homo, 6), "fa.fa.gz": gzip.compress(fa, 6),
          "fixed.fq.gz": strat(fq, zlib.Z_FIXED), "huff.fq.gz": strat(fq, zlib.Z_HUFFMAN_ONLY),
          "rle.fq.gz": strat(fq, zlib.Z_RLE), "filtered.fa.gz": strat(fa, zlib.Z_FILTERED)}
    g6 = bytearray(ok["l6.fq.gz"])
    crc = bytearray(g6)
    crc[-6] ^= 1
    isz = bytearray(g6)
    isz[-2] ^= 1
    flip = bytearray(g6)
    flip[len(flip) // 2] ^= 0x5A
    bad = {"trunc.fq.gz": bytes(g6[:-100]), "crc.fq.gz": bytes(crc), "isize.fq.gz": bytes(isz),
           "flip.fq.gz": bytes(flip), "trunc_multi.fq.gz": ok["multi.fq.gz"][:-9]}
    # period-10 bases: 258-byte matches at distance 10 (8-symbol match copies) end on every
    # offset of the chunk buffers (the copy's slack past the reserved size)
    per = b"ACGTTGCAAC" * 600
    ok["period.fq.gz"] = gzip.compress(b"".join(b"@p%d\n%s\n+\n%s\n" % (i, per[i % 10:][:4000 + i], b"I" * (4000 + i))
                                                for i in range(60)), 9)

    def preset(data, dictionary):  # a member whose matches reach into a preset dictionary
        c = zlib.compressobj(6, zlib.DEFLATED, -15, 8, zlib.Z_DEFAULT_STRATEGY, zdict=dictionary)
        raw = c.compress(data) + c.flush()
        return (b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x00\xff" + raw
                + struct.pack("<II", zlib.crc32(data), len(data) & 0xFFFFFFFF))

    # distances that reach before the member's first byte: zlib / libdeflate refuse them
    # ("invalid distance too far back") even with a matching CRC; so must the parallel reader,
    # in its first chunk, in a later member (the stale window of the one before) and in a gap
    bad["farback.fq.gz"] = preset(fq, fq[:20000])
    bad["farback_multi.fq.gz"] = gzip.compress(fq[:h], 6) + preset(fq[h:], fq[h - 30000:h])
    return ok, bad


@pytest.mark.parametrize("maxout", [None, 4096])
def test_parallel_gzip_under_sanitizers(san, tmp_path, maxout):
    """Non-BGZF gzip through the parallel inflater (NTC_PGZ_MIN=0, 1-3 KiB chunks: hundreds
    of speculative chunk starts, false candidates and gaps) under ASan/UBSan and TSan: the
    same records as the production reader (libdeflate / zlib on one thread) for every block
    type, and the same error for damaged members.  maxout: a per-chunk output budget of 4 K
    symbols (NTC_PGZ_MAXOUT), so that true starts hit it and their chunks fall to the gaps."""
    ok, bad = _gzip_cases()
    for name, data in {**ok, **bad}.items():
        (tmp_path / name).write_bytes(data)
        exp = fastx_digest(str(tmp_path / name), 500)
        assert (exp[0] == 0) == (name in ok), (name, exp)
        for kind, chunk in (("asan", 1024), ("tsan", 3000)):
            env = dict(ENV, NTC_PGZ_MIN="0", NTC_PGZ_CHUNK=str(chunk))
            if maxout:
                env["NTC_PGZ_MAXOUT"] = str(maxout)
            r = subprocess.run([san[kind], "fastx", str(tmp_path / name), "4", "500", str(1 << 16), "1"], env=env,
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
            err = r.stderr.decode(errors="replace")
            assert r.returncode == 0 and "Sanitizer" not in err and "runtime error" not in err, err[-4000:]
            got = dict(x.split("=", 1) for x in r.stdout.decode().split())
            if exp[0]:
                assert int(got["rc"]) == exp[0], (name, kind, got)
            else:
                assert (int(got["rc"]), int(got["reads"]), int(got["bases"]), int(got["hash"], 16)) == exp, \
                    (name, kind)
