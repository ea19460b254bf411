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
