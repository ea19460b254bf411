"""GPU index build (ntc_build_index_device[_ex], build.hip) against the host builder
(sbwt_build.cpp, the stand-in for kbo::build, src/main.rs:111-134) and the brute-force
goldens: identical n, C, rows and LCS for every k-word width W = ceil(2k / 64) from 1 to 8,
with non-ACGT bytes, lower case, sequences shorter than k, empty sequences, many short
sequences and without reverse complements; in one pass and in memory-bounded passes (kbo's
BuildOpts { mem_gb, temp_dir }, src/cli.rs:56-61): forced partitions, a tiny device budget,
partitions spilled to files, a bucket heavier than a pass; an index built on the GPU encodes
and decodes like the host-built one."""
import numpy as np
import pytest

import ntcomp_amd as nt

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = nt.GpuContext(0)
    yield c
    c.close()


def same(a, b):
    assert (a.n, a.k) == (b.n, b.k)
    assert list(a.C) == list(b.C)
    assert np.array_equal(a.lcs, b.lcs)
    for c in range(4):
        assert np.array_equal(a.rows[c], b.rows[c]), c


def messy_seqs(seed, n, lo, hi):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        L = int(rng.integers(lo, hi))
        s = bytearray(rng.choice(list(b"ACGT"), L).astype(np.uint8).tobytes())
        if L > 10 and i % 3 == 0:
            s[int(rng.integers(0, L))] = ord("N")
        if i % 5 == 0:
            s = s.lower()
        out.append(bytes(s))
    return out + [b"", b"ACG", b"NNNNNNNN"]


@pytest.mark.parametrize("k", [1, 2, 3, 5, 11, 31, 32, 33, 63, 64, 65, 91, 96, 97, 160, 255])
def test_gpu_build_equals_host_build(ctx, k):
    seqs = messy_seqs(k, 40, 1, 600)
    same(nt.Index.build_gpu(ctx, seqs, k), nt.Index.build(seqs, k))
    same(nt.Index.build_gpu(ctx, seqs, k, add_revcomp=False), nt.Index.build(seqs, k, add_revcomp=False))


def test_gpu_build_genome_collection_and_reads(ctx):
    genome = nt.synth_genome(5, 1_000_000)
    strains = nt.synth_strains(genome, 3, 3, 10_000)
    texts = [genome.tobytes()] + [strains[i].tobytes() for i in range(3)]
    for k in (31, 91):
        same(nt.Index.build_gpu(ctx, texts, k), nt.Index.build(texts, k))
    reads = nt.synth_reads(genome, 3, 0, 20_000, 150, 10_000)
    many = [reads[i * 150:(i + 1) * 150].tobytes() for i in range(20_000)]
    same(nt.Index.build_gpu(ctx, many, 31), nt.Index.build(many, 31))


def test_gpu_built_index_encodes_like_host_built(ctx):
    genome = nt.synth_genome(6, 500_000)
    ix = nt.Index.build_gpu(ctx, [genome.tobytes()], 91)
    ref = nt.Index.build([genome.tobytes()], 91)
    same(ix, ref)
    ctx.upload(ix)
    n, L = 20_000, 150
    reads = nt.synth_reads(genome, 7, 0, n, L, 10_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    recs, roff = ctx.encode(reads, offs)
    out, o2 = ctx.decode(recs)
    assert np.array_equal(out, reads)
    from oracle_lib import OracleIndex
    exp, _ = OracleIndex(ref.n, 91, ref.rows, ref.C, ref.lcs).encode(reads[:500 * L], offs[:501])
    assert np.array_equal(recs[:len(exp)], exp)


def test_gpu_build_empty_inputs(ctx):
    for seqs in ([], [b""], [b"AC"], [b"NNNN"]):
        same(nt.Index.build_gpu(ctx, seqs, 5), nt.Index.build(seqs, 5))


def test_cli_build_gpu_writes_the_host_index(tmp_path):
    """`build --builder gpu` (main.rs:111-140 stand-in on the GPU) saves the same files as the
    host builder."""
    import subprocess
    import sys
    import os
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    g = nt.synth_genome(4, 50_000).tobytes().decode()
    fa = tmp_path / "g.fa"
    fa.write_text(">g\n" + "\n".join(g[i:i + 60] for i in range(0, len(g), 60)) + "\nACGTNNNNACGT\n")
    for b in ("host", "gpu"):
        subprocess.run([sys.executable, "-m", "ntcomp_amd", "build", "-o", str(tmp_path / b), "-k", "31",
                        "--builder", b, str(fa)], cwd=repo, check=True, stderr=subprocess.PIPE)
    for ext in (".sbwt", ".lcs"):
        assert (tmp_path / ("gpu" + ext)).read_bytes() == (tmp_path / ("host" + ext)).read_bytes()


def test_gpu_build_equals_goldens(ctx):
    """The GPU build against the brute-force SBWT of tests/golden/make_golden.py directly (one
    pass and forced partitions)."""
    from oracle_lib import golden_names, load_golden
    for name in golden_names():
        g = load_golden(name)
        for part in (0, 1024):
            st = {}
            ix = nt.Index.build_gpu(ctx, g["seqs"], g["k"], max_partition_keys=part, stats=st)
            assert (ix.n, ix.k, ix.C) == (g["n"], g["k"], g["C"]), (name, part)
            for c in range(4):
                assert np.array_equal(ix.row(c), g["rows_u64"][c]), (name, part, c)
            assert np.array_equal(ix.lcs, g["lcs_u8"]), (name, part)
            if part:
                assert st["kmer_partitions"] >= 2 or st["occurrences"] <= 1024, (name, st)


@pytest.mark.parametrize("k", [31, 91, 255])
def test_gpu_build_partitioned_equals_host(ctx, k, tmp_path):
    """Passes of at most ~1/8 of the occurrences (>= 4 k-mer and node partitions), with and
    without sorted partitions spilled to --temp-dir files: the host builder's index."""
    genome = nt.synth_genome(40 + k, 400_000)
    strains = nt.synth_strains(genome, 5, 2, 10_000)
    seqs = [genome.tobytes()] + [strains[i].tobytes() for i in range(2)] + messy_seqs(k, 30, 1, 700)
    ref = nt.Index.build(seqs, k)
    occ = 2 * sum(max(0, len(x) - k + 1) for x in seqs)
    for host_budget in (0, 1 << 16):
        st = {}
        ix = nt.Index.build_gpu(ctx, seqs, k, max_partition_keys=occ // 8, host_budget=host_budget,
                                temp_dir=tmp_path, stats=st)
        same(ix, ref)
        assert st["kmer_partitions"] >= 4 and st["node_partitions"] >= 4, st
        assert st["nodes"] == ref.n
        if host_budget:
            assert st["spilled_bytes"] > 0, st
        assert not list(tmp_path.iterdir())  # partition files are unlinked at creation


def test_gpu_build_tiny_device_budget(ctx):
    """A 12 MB device budget for a 3 Mbp collection: the sequence streams in chunks (a quarter
    of the budget each) and every pass fits the budget."""
    genome = nt.synth_genome(9, 1_000_000)
    strains = nt.synth_strains(genome, 7, 2, 5_000)
    seqs = [genome.tobytes()] + [strains[i].tobytes() for i in range(2)]
    st = {}
    ix = nt.Index.build_gpu(ctx, seqs, 31, device_budget=12 << 20, stats=st)
    same(ix, nt.Index.build(seqs, 31))
    assert st["peak_device_bytes"] <= 12 << 20, st
    assert st["seq_uploads"] > 1 and st["kmer_partitions"] > 1, st


@pytest.mark.parametrize("k", [2, 5, 31])
def test_gpu_build_heavy_bucket_compacts(ctx, k):
    """A low-complexity input (poly-A runs) puts most occurrences in one bucket, more than a
    pass holds: the accumulator is deduplicated in place and the chunk re-run."""
    rng = np.random.default_rng(k)
    seqs = [b"A" * 200_000, bytes(rng.choice(list(b"ACGT"), 5_000).astype(np.uint8)), b"A" * 3000 + b"C" * 3000]
    st = {}
    ix = nt.Index.build_gpu(ctx, seqs, k, max_partition_keys=4096, stats=st)
    same(ix, nt.Index.build(seqs, k))
    assert st["compactions"] >= 1, st


@pytest.mark.parametrize("k", [1, 3, 7, 8, 33])
def test_gpu_build_partitioned_small_k_and_reads(ctx, k):
    """Many short sequences (many sources, dummies in every partition) and k around the
    bucket width (m = min(7, k - 1) characters)."""
    seqs = messy_seqs(100 + k, 400, 1, 300)
    ref = nt.Index.build(seqs, k)
    same(nt.Index.build_gpu(ctx, seqs, k, max_partition_keys=2048), ref)
    same(nt.Index.build_gpu(ctx, seqs, k, max_partition_keys=2048, add_revcomp=False),
         nt.Index.build(seqs, k, add_revcomp=False))
