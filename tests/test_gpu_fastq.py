"""FASTQ parsed on the GPU (fastq.hip, ntc_fastq_parse / ntc_encode_pack_fastq) against the
host parser (fastx.cpp, ntc_fastx_*: needletail's records + normalize(true) as the CLI uses
them, src/main.rs:158-163), and the encode pipeline's text path (pipeline.cpp fill_text)
against its host-parse path: same bases and offsets, same metas and payload, same
encoded.dat bytes, same errors."""
import gzip
import os

import numpy as np
import pytest

import ntcomp_amd as nt

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = nt.GpuContext(0)
    yield c
    c.close()


def host_parse(path):
    rd = nt.FastxReader(str(path))
    bs, os_, base = [], [np.zeros(1, np.uint64)], 0
    while True:
        x = rd.batch(1 << 20)
        if x is None:
            break
        b, o = x
        bs.append(b[int(o[0]):int(o[-1])])
        os_.append((o[1:] - o[0] + base).astype(np.uint64))
        base += int(o[-1] - o[0])
    rd.close()
    return (np.concatenate(bs) if bs else np.zeros(0, np.uint8)), np.concatenate(os_)


def records(rng, n, lmin, lmax, alphabet=b"ACGT", crlf=False):
    nl = b"\r\n" if crlf else b"\n"
    out = []
    for i in range(n):
        L = int(rng.integers(lmin, lmax + 1))
        seq = bytes(rng.choice(np.frombuffer(alphabet, np.uint8), L)) if L else b""
        out.append(b"@read_%d some description" % i + nl + seq + nl + b"+" + nl + b"F" * len(seq) + nl)
    return out


def shapes():
    rng = np.random.default_rng(17)
    iupac = b"ACGTNacgtnRYSWKMBDHVrYswkmbdhvuU.~-xX*0"
    cases = {
        "acgt_150": b"".join(records(rng, 5000, 150, 150)),
        "ragged": b"".join(records(rng, 3000, 1, 700)),
        "iupac_and_junk": b"".join(records(rng, 2000, 20, 300, iupac)),
        "crlf": b"".join(records(rng, 2000, 50, 200, crlf=True)),
        "long_reads": b"".join(records(rng, 40, 5000, 40000)),
        "one_base": b"".join(records(rng, 100, 1, 1)),
    }
    # whitespace inside sequence lines is dropped (and not counted against the quality line,
    # which is compared by raw length, as parse_fq_range does)
    cases["spaces"] = b"".join(b"@s\nAC GT\tA\n+\nFFFFFFF\n" for _ in range(300))
    cases["no_final_newline"] = cases["acgt_150"][:-1]
    cases["empty_sequences"] = b"".join(records(rng, 500, 0, 3))
    return cases


@pytest.mark.parametrize("name", sorted(shapes()))
def test_gpu_fastq_parse_equals_host_parser(ctx, tmp_path, name):
    text = shapes()[name]
    (tmp_path / "x.fq").write_bytes(text)
    bases, offs = host_parse(tmp_path / "x.fq")
    n = len(offs) - 1
    gb, go = ctx.parse_fastq(text, n)
    assert np.array_equal(go, offs), name
    assert np.array_equal(gb, bases), name


def test_gpu_fastq_malformed_records(ctx):
    rng = np.random.default_rng(3)
    recs = records(rng, 1000, 30, 80)
    good = b"".join(recs)
    cases = {}
    r = bytearray(recs[517])
    r[0:1] = b">"  # header without '@'
    cases["header"] = (b"".join(recs[:517]) + bytes(r) + b"".join(recs[518:]), 1000, 517)
    r = recs[260].replace(b"\n+\n", b"\n-\n")  # no '+' line
    cases["plus"] = (b"".join(recs[:260]) + r + b"".join(recs[261:]), 1000, 260)
    r = recs[999][:-2] + b"\n"  # quality one shorter than the sequence
    cases["qual_len"] = (b"".join(recs[:999]) + r, 1000, 999)
    cases["too_few_lines"] = (good[:good.rindex(b"\n+\n")], 1000, 999)
    cases["junk_after"] = (good + b"@x", 1000, 999)
    cases["n_too_small"] = (good, 999, 998)
    for name, (text, n, bad) in cases.items():
        with pytest.raises(nt.NtcError) as e:
            ctx.parse_fastq(text, n)
        assert e.value.code == 8 and e.value.bad_read == bad, (name, e.value.bad_read)
    with pytest.raises(nt.NtcError):
        ctx.parse_fastq(b"@a\nAC\n+\nFF\n", 0)
    b, o = ctx.parse_fastq(b"", 0)
    assert len(b) == 0 and list(o) == [0]


def test_gpu_encode_pack_fastq_equals_encode_pack(ctx):
    """Same metas and payload as the host-parsed reads through ntc_encode_pack_batch, over
    three blocks and a partial one (k = 31 index of a 200 kbp genome)."""
    genome = nt.synth_genome(21, 200_000)
    ix = nt.Index.build([genome.tobytes()], 31)
    ctx.upload(ix)
    n, L = 3 * 65536 + 1234, 100
    reads = nt.synth_reads(genome, 22, 0, n, L, 10_000)
    body = reads.reshape(n, L)
    text = b"".join(b"@r\n" + body[i].tobytes().lower() + b"\n+\n" + b"#" * L + b"\n" for i in range(n))
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    m0, p0 = ctx.encode_pack(reads, offs)
    m1, p1, nb = ctx.encode_pack_fastq(text, n)
    assert nb == n * L and p1 == p0
    assert [bytes(x) for x in m1] == [bytes(x) for x in m0]


@pytest.mark.parametrize("bpb", [1, 4])
def test_encode_file_text_path_equals_host_parse(ctx, tmp_path, bpb):
    """ntc_encode_file on a FASTQ, mapped or through gzip / BGZF: GPU parse (default) and host
    parse write the same encoded.dat; a blank line mid-file hands the rest to the host parser;
    a truncated last record is NTC_ERR_FORMAT either way."""
    genome = nt.synth_genome(31, 100_000)
    ix = nt.Index.build([genome.tobytes()], 31)
    ctx.upload(ix)
    n, L = 5 * 65536 + 999, 75
    body = nt.synth_reads(genome, 32, 0, n, L, 10_000).reshape(n, L)
    recs = [b"@r%d\n" % i + body[i].tobytes() + b"\n+\n" + b"F" * L + b"\n" for i in range(n)]
    plain = b"".join(recs)
    from test_cli import _bgzf_member
    files = {"plain": plain, "crlf": plain.replace(b"\n", b"\r\n"),
             "mid_blank": b"".join(recs[:4 * 65536 + 5]) + b"\n" + b"".join(recs[4 * 65536 + 5:]),
             # through a decoder: the streamed text path (carried tails between batches)
             "plain_gz": gzip.compress(plain, 1),
             "plain_bgzf": b"".join(_bgzf_member(plain[i:i + 65000]) for i in range(0, len(plain), 65000))}
    for name, blob in files.items():
        (tmp_path / f"{name}.fq").write_bytes(blob)
        outs = {}
        for hp in (False, True):
            fd = os.open(tmp_path / f"{name}{int(hp)}.dat", os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
            try:
                st = nt.encode_file([ctx], str(tmp_path / f"{name}.fq"), fd, blocks_per_batch=bpb, host_parse=hp)
            finally:
                os.close(fd)
            outs[hp] = (tmp_path / f"{name}{int(hp)}.dat").read_bytes()
            assert st["reads"] == n and st["bases"] == n * L, (name, hp, st)
            assert (st["gpu_parsed"] > 0) == (not hp), (name, hp, st["gpu_parsed"])
        assert outs[False] == outs[True], name
    (tmp_path / "t.fq").write_bytes(plain[:-40])
    for hp in (False, True):
        fd = os.open(tmp_path / "t.dat", os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        try:
            with pytest.raises(nt.NtcError) as e:
                nt.encode_file([ctx], str(tmp_path / "t.fq"), fd, blocks_per_batch=bpb, host_parse=hp)
        finally:
            os.close(fd)
        assert e.value.code == 8, hp


def test_gpu_fastq_parse_does_not_leak_into_encode_status(ctx):
    """the parse reuses the context's status word and mailbox, so after
    encode_batch -> fastq_parse, encode_status must not report the parse's base count as
    the encode's record count: the parse was the last call, so there is no encode to
    report (NTC_ERR_INVALID_ARG), and a fresh encode reports its own count again."""
    g = nt.synth_genome(5, 20_000)
    ix = nt.Index.build([g.tobytes()], 31)
    ctx.upload(ix)
    n, L = 300, 150
    reads = nt.synth_reads(g, 6, 0, n, L, 10_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    recs, roff = ctx.encode(reads, offs)
    assert ctx.encode_status() == len(recs)
    text = b"".join(b"@r\n" + reads[i * L:(i + 1) * L].tobytes() + b"\n+\n" + b"F" * L + b"\n" for i in range(n))
    b, o = ctx.parse_fastq(text, n)
    assert len(b) == n * L
    with pytest.raises(nt.NtcError) as e:
        ctx.encode_status()
    assert e.value.code == 1
    recs2, _ = ctx.encode(reads, offs)
    assert np.array_equal(recs2, recs) and ctx.encode_status() == len(recs)
