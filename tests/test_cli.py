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
        _cli("encode", "-i", str(tmp_path / "idx"), "--blocks-per-batch", "1", str(fq), stdout=f)
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
