"""The native encode pipeline (ntc_encode_file, include/ntcomp_pipeline.h) and the CLI's
multi-context paths: file bytes equal the container built block by block from
ntc_encode_batch records with the host codec (write_block_to per 65,536 reads, the last
block num_records % 65,536: src/main.rs:162-177), through the mapped FASTQ parser, buffer
growth and carries, several contexts on one GPU, and either deflate engine."""
import os
import subprocess
import sys

import numpy as np
import pytest

import ntcomp_amd as nt

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def setup(tmp_path_factory):
    d = tmp_path_factory.mktemp("pipe")
    genome = nt.synth_genome(12, 400_000)
    ix = nt.Index.build([genome.tobytes()], 31)
    ix.save(str(d / "idx"))
    return d, genome, ix


def write_fastq(path, reads, L):
    n = len(reads) // L
    body = reads.reshape(n, L)
    qual = np.full((n, L), ord("I"), np.uint8)
    nl = np.full((n, 1), 10, np.uint8)
    rec = np.concatenate([np.frombuffer(b"@r\n", np.uint8)[None, :].repeat(n, 0), body, nl,
                          np.frombuffer(b"+\n", np.uint8)[None, :].repeat(n, 0), qual, nl], axis=1)
    path.write_bytes(rec.tobytes())


def expected_file(ctx, reads, L):
    n = len(reads) // L
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    recs, roff = ctx.encode(reads, offs)
    out = nt.file_header()
    for b0 in range(0, n, 65536):
        b1 = min(n, b0 + 65536)
        try:
            out += nt.write_block(recs[int(roff[b0]):int(roff[b1])], b1 - b0)
        except nt.NtcError as e:
            assert e.code == 3  # dropped like the reference (App. B.3)
    return out


@pytest.mark.parametrize("n,L,bpb,batch_bases", [(140_000, 100, 1, 0), (200_000, 150, 16, 0),
                                                 (70_000, 100, 4, 1 << 20), (3, 150, 16, 0)])
def test_encode_file_equals_blockwise_host_codec(setup, tmp_path, n, L, bpb, batch_bases):
    d, genome, ix = setup
    ctx = nt.GpuContext(0)
    ctx.upload(ix)
    reads = nt.synth_reads(genome, 21, 0, n, L, 10_000)
    fq = tmp_path / "r.fq"
    write_fastq(fq, reads, L)
    out = tmp_path / "e.dat"
    with open(out, "wb") as f:
        st = nt.encode_file([ctx], str(fq), f.fileno(), threads=4, blocks_per_batch=bpb, batch_bases=batch_bases)
    assert st["reads"] == n and st["bases"] == n * L
    assert out.read_bytes() == expected_file(ctx, reads, L)
    ctx.close()


def test_encode_file_fasta_contigs_k255(tmp_path):
    """The reference's other input shape: a multi-contig FASTA (src/main.rs:158 reads any
    fastX), line-wrapped at 60 with lowercase stretches, normalised as needletail's
    normalize(true) does (main.rs:162), at k = 255: ntc_encode_file's bytes equal the
    container of the normalised contigs' records, and ntc_decode_file gives them back."""
    genome = nt.synth_genome(31, 300_000)
    ix = nt.Index.build([genome.tobytes()], 255)
    ix.save(str(tmp_path / "idx"))
    ctx = nt.GpuContext(0)
    ctx.upload(ix)
    rng = np.random.default_rng(4)
    g = genome.tobytes()
    contigs, text = [], bytearray()
    for i in range(300):
        L = int(rng.integers(1, 5000))
        st = int(rng.integers(0, len(g) - L))
        c = bytearray(g[st:st + L])
        if i % 3 == 0:  # a lowercase stretch
            a0 = int(rng.integers(0, L))
            c[a0:a0 + 200] = bytes(c[a0:a0 + 200]).lower()
        contigs.append(bytes(c).upper())
        text += b">contig_%d some description\n" % i
        text += b"".join(bytes(c[j:j + 60]) + b"\n" for j in range(0, L, 60))
    fa = tmp_path / "c.fa"
    fa.write_bytes(bytes(text))
    bases = np.frombuffer(b"".join(contigs), dtype=np.uint8)
    offs = np.cumsum([0] + [len(c) for c in contigs]).astype(np.uint64)
    recs, roff = ctx.encode(bases, offs)
    exp = nt.file_header() + nt.write_block(recs, len(contigs))
    with open(tmp_path / "e.dat", "wb") as f:
        st = nt.encode_file([ctx], str(fa), f.fileno(), threads=4)
    assert st["reads"] == len(contigs) and st["bases"] == len(bases)
    assert (tmp_path / "e.dat").read_bytes() == exp
    with open(tmp_path / "d.fa", "wb") as f:
        nt.decode_file([ctx], str(tmp_path / "e.dat"), f.fileno(), threads=4)
    assert (tmp_path / "d.fa").read_bytes() == b"".join(b">seq.%d\n%s\n" % (i + 1, c) for i, c in enumerate(contigs))
    ctx.close()


def test_encode_file_reports_bad_read(setup, tmp_path):
    d, genome, ix = setup
    ctx = nt.GpuContext(0)
    ctx.upload(ix)
    L = 100
    reads = nt.synth_reads(genome, 22, 0, 1000, L, 0).copy()
    reads[777 * L + 5] = ord("N")  # a base absent from the index: the reference never terminates
    fq = tmp_path / "bad.fq"
    write_fastq(fq, reads, L)
    with open(tmp_path / "x.dat", "wb") as f, pytest.raises(nt.NtcError) as e:
        nt.encode_file([ctx], str(fq), f.fileno(), threads=2)
    assert e.value.code == 2 and e.value.bad_read == 777
    ctx.close()


def _cli(*args, stdout=None):
    return subprocess.run([sys.executable, "-m", "ntcomp_amd", *args], cwd=REPO, stdout=stdout,
                          stderr=subprocess.PIPE, check=True)


def test_cli_two_contexts_on_one_gpu_and_deflate_engines(setup, tmp_path):
    """--devices 0,0: two contexts on device 0 take alternate batches; encoded.dat and the
    decoded FASTA are byte-identical to one context (no collective, blocks
    in file order).  --deflate libdeflate: other gzip bytes, identical blocks after inflate."""
    d, genome, ix = setup
    n, L = 300_000, 150
    reads = nt.synth_reads(genome, 23, 0, n, L, 10_000)
    fq = tmp_path / "r.fq"
    write_fastq(fq, reads, L)
    files = {}
    for tag, extra in (("one", ["--deflate", "zlib"]), ("two", ["--devices", "0,0", "--deflate", "zlib"]),
                       ("ld", ["--deflate", "libdeflate"])):
        with open(tmp_path / f"{tag}.dat", "wb") as f:
            _cli("encode", "-i", str(d / "idx"), str(fq), "--blocks-per-batch", "1", *extra, stdout=f)
        files[tag] = (tmp_path / f"{tag}.dat").read_bytes()
    assert files["one"] == files["two"]
    assert files["ld"] != files["one"]

    def blocks(data):
        pos, out = 32, []
        while pos < len(data):
            r, used, nrec = nt.read_block(data[pos:])
            out.append((r.tobytes(), nrec))
            pos += used
        return out

    assert blocks(files["ld"]) == blocks(files["one"])
    fa = {}
    for tag, extra in (("one", []), ("two", ["--devices", "0,0"])):
        with open(tmp_path / f"{tag}.fa", "wb") as f:
            _cli("decode", "-i", str(d / "idx"), str(tmp_path / "one.dat"), *extra, stdout=f)
        fa[tag] = (tmp_path / f"{tag}.fa").read_bytes()
    assert fa["one"] == fa["two"]
    lines = fa["one"].split(b"\n")
    assert b"".join(lines[1::2]) == reads.tobytes()


# ---- native decode pipeline (ntc_decode_file) ---------------------------------------------
def fasta_of(reads, offs, first=1):
    return b"".join(b">seq.%d\n" % (first + i) + reads[int(offs[i]):int(offs[i + 1])].tobytes() + b"\n"
                    for i in range(len(offs) - 1))


def encoded_file(ctx, tmp_path, reads, offs, name="e.dat"):
    """encoded.dat of ragged reads through the host codec, block by block (main.rs:162-177)."""
    n = len(offs) - 1
    recs, roff = ctx.encode(reads, offs)
    out, ends = nt.file_header(), []
    for b0 in range(0, n, 65536):
        b1 = min(n, b0 + 65536)
        out += nt.write_block(recs[int(roff[b0]):int(roff[b1])], b1 - b0)
        ends.append((len(out), b1))
    (tmp_path / name).write_bytes(out)
    return tmp_path / name, ends


def ragged(genome, n, seed, lo=1, hi=400):
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi, n)
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    starts = rng.integers(0, len(genome) - hi, n)
    reads = np.concatenate([genome[s:s + l] for s, l in zip(starts, lens)]).copy()
    flip = rng.random(len(reads)) < 0.01
    reads[flip] = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, int(flip.sum()))]
    return reads, offs


@pytest.fixture(params=["gpu", "host"])
def unpack(request, monkeypatch):
    """The decode pipeline's stream decode: on the GPU (default) or the host pool."""
    if request.param == "host":
        monkeypatch.setenv("NTC_HOST_UNPACK", "1")
    else:
        monkeypatch.delenv("NTC_HOST_UNPACK", raising=False)
    return request.param


@pytest.mark.parametrize("bpb,threads,nctx", [(1, 1, 1), (2, 4, 1), (16, 8, 1), (1, 3, 2)])
def test_decode_file_equals_reads(setup, tmp_path, bpb, threads, nctx, unpack):
    d, genome, ix = setup
    ctxs = [nt.GpuContext(0) for _ in range(nctx)]
    for c in ctxs:
        c.upload(ix)
    reads, offs = ragged(genome, 5 * 65536 + 321, 31)
    path, ends = encoded_file(ctxs[0], tmp_path, reads, offs)
    with open(tmp_path / "o.fa", "wb") as f:
        st = nt.decode_file(ctxs, str(path), f.fileno(), threads=threads, blocks_per_batch=bpb)
    exp = fasta_of(reads, offs)
    assert (tmp_path / "o.fa").read_bytes() == exp
    assert (st["reads"], st["bases"], st["blocks"], st["dropped_blocks"]) == (len(offs) - 1, len(reads), 6, 0)
    assert st["bytes_out"] == len(exp)
    for c in ctxs:
        c.close()


def test_decode_file_truncated_and_damaged_blocks(setup, tmp_path, unpack):
    """A truncated tail ends the input (read_exact, main.rs:199); a damaged gzip member ends
    the output after the blocks before it, without an error (main.rs:202)."""
    d, genome, ix = setup
    ctx = nt.GpuContext(0)
    ctx.upload(ix)
    reads, offs = ragged(genome, 4 * 65536 + 99, 32)
    path, ends = encoded_file(ctx, tmp_path, reads, offs)
    data = path.read_bytes()
    cases = {"trunc": (data[:-7], 4), "header_only": (data[:32], 0), "empty": (b"", 0)}
    bad = bytearray(data)
    a = ends[1][0]  # block 2 starts here: corrupt its first stream's deflate data
    bad[a + 32 + 12:a + 32 + 40] = b"\xff" * 28
    cases["damaged"] = (bytes(bad), 2)
    for name, (blob, keep) in cases.items():
        for bpb in (1, 3):
            p = tmp_path / f"{name}.dat"
            p.write_bytes(blob)
            with open(tmp_path / "o.fa", "wb") as f:
                st = nt.decode_file([ctx], str(p), f.fileno(), threads=4, blocks_per_batch=bpb)
            nr = ends[keep - 1][1] if keep else 0
            assert (tmp_path / "o.fa").read_bytes() == fasta_of(reads, offs[:nr + 1]), (name, bpb)
            assert st["blocks"] == keep and st["reads"] == nr, (name, bpb)
            if name == "damaged":
                assert st["dropped_blocks"] == 3 and "damaged" in st["error"]
    ctx.close()


def test_decode_file_stream_damage_found_after_inflate(setup, tmp_path, unpack):
    """A block whose gzip members are intact but whose streams are not (its flag stream's
    header claims 1000 more values than its codes hold) ends the output after the blocks
    before it, found by the GPU unpacker (default) or by the host pool alike, as
    decode_block's Err ends the reference's loop (main.rs:202)."""
    d, genome, ix = setup
    ctx = nt.GpuContext(0)
    ctx.upload(ix)
    reads, offs = ragged(genome, 4 * 65536 + 99, 33)
    path, ends = encoded_file(ctx, tmp_path, reads, offs)
    data = path.read_bytes()
    a, b = ends[1][0], ends[2][0]  # block 2
    meta, pay, used = nt.read_block_streams(data[a:b])
    assert used == b - a
    meta.stream[2].num_u64 += 1000
    p = tmp_path / "sd.dat"
    p.write_bytes(data[:a] + nt.deflate_block(meta, pay) + data[b:])
    nr = ends[1][1]
    for bpb in (1, 3):
        with open(tmp_path / "o.fa", "wb") as f:
            st = nt.decode_file([ctx], str(p), f.fileno(), threads=4, blocks_per_batch=bpb)
        assert (tmp_path / "o.fa").read_bytes() == fasta_of(reads, offs[:nr + 1]), (unpack, bpb)
        assert (st["blocks"], st["reads"], st["dropped_blocks"]) == (2, nr, 3), (unpack, bpb)
    ctx.close()


def test_cli_decode_to_a_pipe(setup, tmp_path):
    """stdout a pipe (not seekable): the writer falls back to write(2) in order."""
    d, genome, ix = setup
    ctx = nt.GpuContext(0)
    ctx.upload(ix)
    reads, offs = ragged(genome, 70_000, 33, 50, 3000)
    path, _ = encoded_file(ctx, tmp_path, reads, offs)
    ctx.close()
    r = _cli("decode", "-i", str(d / "idx"), str(path), "--blocks-per-batch", "1", stdout=subprocess.PIPE)
    assert r.stdout == fasta_of(reads, offs)


def test_cli_decode_appends_and_shares_a_redirect(setup, tmp_path):
    """`decode >> out` (O_APPEND: pwrite would ignore its offset) and `{ decode a; decode b; }
    > out` (one open file shared by two processes: the writer leaves the file offset past
    its text) keep every byte in order, as the reference's stdout does (main.rs:203-209).
    The batches hold > 8 MiB of text, so the parallel pwrite path is the one exercised."""
    d, genome, ix = setup
    ctx = nt.GpuContext(0)
    ctx.upload(ix)
    reads, offs = ragged(genome, 2 * 65536 + 7, 34, 100, 200)
    path, _ = encoded_file(ctx, tmp_path, reads, offs)
    ctx.close()
    exp = fasta_of(reads, offs)
    assert len(exp) > (8 << 20)
    out = tmp_path / "app.fa"
    out.write_bytes(b"head\n")
    with open(out, "ab") as f:
        _cli("decode", "-i", str(d / "idx"), str(path), "--blocks-per-batch", "2", stdout=f)
    assert out.read_bytes() == b"head\n" + exp
    shared = tmp_path / "shared.fa"
    with open(shared, "wb") as f:
        for _ in range(2):
            _cli("decode", "-i", str(d / "idx"), str(path), "--blocks-per-batch", "2", stdout=f)
    assert shared.read_bytes() == exp + exp


def test_contexts_share_one_index(setup, tmp_path):
    """ntc_index_share: a second context on the GPU uses the first one's device index (no
    second upload); both encode the same records, the shared index outlives the context that
    uploaded it, and the CLI's --contexts-per-gpu 2 writes the same file as one context."""
    d, genome, ix = setup
    a = nt.GpuContext(0).upload(ix)
    b = nt.GpuContext(0).share_index(a)
    reads = nt.synth_reads(genome, 41, 0, 30_000, 150, 10_000)
    offs = np.arange(0, len(reads) + 1, 150, dtype=np.uint64)
    ra, oa = a.encode(reads, offs)
    rb, ob = b.encode(reads, offs)
    assert np.array_equal(ra, rb) and np.array_equal(oa, ob)
    a.close()
    rc, oc = b.encode(reads, offs)
    assert np.array_equal(rc, ra)
    out, _ = b.decode(rc)
    assert np.array_equal(out, reads)
    b.close()
    fq = tmp_path / "r.fq"
    write_fastq(fq, reads, 150)
    outs = {}
    for c in (1, 2):
        with open(tmp_path / f"{c}.dat", "wb") as f:
            _cli("encode", "-i", str(d / "idx"), str(fq), "--contexts-per-gpu", str(c), "--blocks-per-batch", "1",
                 "--deflate", "zlib", stdout=f)
        outs[c] = (tmp_path / f"{c}.dat").read_bytes()
    assert outs[1] == outs[2]


def test_prepared_upload_equals_upload(setup):
    """ntc_index_prepare + ntc_index_upload_prepared (the native CLI derives the host tables
    while HIP starts): the same device index as ntc_index_upload -- same sizes, same records,
    exact round trip -- and one prepared index serves several contexts."""
    d, genome, ix = setup
    reads = nt.synth_reads(genome, 43, 0, 20_000, 150, 10_000)
    offs = np.arange(0, len(reads) + 1, 150, dtype=np.uint64)
    a = nt.GpuContext(0).upload(ix)
    prep = nt.IndexPrep(ix)
    b = nt.GpuContext(0).upload_prepared(prep)
    c = nt.GpuContext(0).upload_prepared(prep)
    prep.close()
    assert a.index_info() == b.index_info() == c.index_info()
    ra, oa = a.encode(reads, offs)
    for x in (b, c):
        r, o = x.encode(reads, offs)
        assert np.array_equal(r, ra) and np.array_equal(o, oa)
        out, _ = x.decode(r)
        assert np.array_equal(out, reads)
    for x in (a, b, c):
        x.close()


def test_decode_only_upload(setup):
    """ctx option decode_only: the upload builds the walk table alone (no path cover, suffix
    table or SCAN words, a smaller device index); decode is the same as on a full index, the
    option passes on through ntc_index_share, and encode calls fail with NTC_ERR_NO_INDEX."""
    d, genome, ix = setup
    reads = nt.synth_reads(genome, 44, 0, 20_000, 150, 10_000)
    offs = np.arange(0, len(reads) + 1, 150, dtype=np.uint64)
    full = nt.GpuContext(0).upload(ix)
    recs, _ = full.encode(reads, offs)
    dec = nt.GpuContext(0)
    dec.set_option("decode_only", 1)
    dec.upload(ix)
    assert dec.get_option("decode_only") == 1 and full.get_option("decode_only") == 0
    assert dec.index_info()[2] < full.index_info()[2]
    shared = nt.GpuContext(0)
    shared.share_index(dec)
    for x in (dec, shared):
        out, o2 = x.decode(recs)
        assert np.array_equal(out, reads) and np.array_equal(o2, offs)
        with pytest.raises(nt.NtcError) as e:
            x.encode(reads, offs)
        assert e.value.code == 7  # NTC_ERR_NO_INDEX
    dec.set_option("decode_only", 0)
    dec.upload(ix)  # a full upload again: encode works
    r2, _ = dec.encode(reads, offs)
    assert np.array_equal(r2, recs)
    for x in (full, dec, shared):
        x.close()


def test_warm_dma_option():
    """"warm_dma" copies that many bytes each way now (the CLI starts the DMA engines beside
    the index preparation); out-of-range sizes are NTC_ERR_INVALID_ARG."""
    ctx = nt.GpuContext(0)
    ctx.set_option("warm_dma", 4 << 20)
    for bad in (0, -1, (1 << 30) + 1):
        with pytest.raises(nt.NtcError):
            ctx.set_option("warm_dma", bad)
    ctx.close()
