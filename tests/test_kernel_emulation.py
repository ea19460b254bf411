"""The kernels' lane logic (ntcomp_amd/csrc/encode_core.h: fast-contraction matching
statistics, O(1)-per-step extension, record packing, jump-table inverse walk), compiled
for the HOST by the test-only tests/emu library, against the golden vectors and against
the faithful CPU oracle on larger seeded inputs.  The same functions run on the GPU in
the -m gpu tests."""
import numpy as np
import pytest

import ntcomp_amd as nt
from emu_lib import emu_decode, emu_encode
from oracle_lib import OracleIndex, golden_names, load_golden, pack_reads


VARIANTS = [(4, True), (4, False), (1, False)]  # (kernel variant, path walk)


@pytest.mark.parametrize("variant,paths", VARIANTS)
@pytest.mark.parametrize("name", golden_names())
def test_emulated_kernel_matches_golden(name, variant, paths):
    g = load_golden(name)
    bases, offs = pack_reads(g["reads"])
    recs, roff, d, s = emu_encode(g["n"], g["k"], g["rows_u64"], g["C"], g["lcs_u8"], bases, offs, want_ms=True,
                                  variant=variant, use_paths=paths)
    exp_ms = np.array([x for r in g["ms"] for x in r], dtype=np.uint64).reshape(-1, 2)
    assert np.array_equal(d.astype(np.uint64), exp_ms[:, 0])
    assert np.array_equal(s.astype(np.uint64), exp_ms[:, 1])
    assert recs.tolist() == [w for r in g["records"] for w in r]
    out, o2 = emu_decode(g["n"], g["k"], g["rows_u64"], g["C"], g["lcs_u8"], recs)
    assert [out[o2[i]:o2[i + 1]].tobytes().decode() for i in range(len(o2) - 1)] == g["reads"]


@pytest.mark.parametrize("variant,paths", VARIANTS)
@pytest.mark.parametrize("k,err_ppm", [(31, 10_000), (91, 10_000), (91, 0), (15, 30_000), (255, 5_000), (11, 10_000)])
def test_emulated_kernel_matches_oracle_random(k, err_ppm, variant, paths):
    genome = nt.synth_genome(100 + k, 60_000)
    ix = nt.Index.build([genome.tobytes()], k, threads=4)
    rows, C, lcs = ix.rows, ix.C, ix.lcs
    L = 150 if k < 200 else 400
    reads = nt.synth_reads(genome, 5, 0, 600, L, err_ppm)
    offs = np.arange(0, 600 * L + 1, L, dtype=np.uint64)
    orc = OracleIndex(ix.n, k, rows, C, lcs)
    exp, eoff = orc.encode(reads, offs)
    got, goff = emu_encode(ix.n, k, rows, C, lcs, reads, offs, variant=variant, use_paths=paths)
    assert np.array_equal(goff, eoff)
    assert np.array_equal(got, exp)
    out, o2 = emu_decode(ix.n, k, rows, C, lcs, got)
    assert np.array_equal(out, reads)


@pytest.mark.parametrize("variant,paths", VARIANTS)
def test_emulated_ms_matches_oracle_unrelated_reads(variant, paths):
    # reads from a different genome: many contractions from short d
    genome = nt.synth_genome(3, 50_000)
    other = nt.synth_genome(4, 50_000)
    ix = nt.Index.build([genome.tobytes()], 31)
    reads = nt.synth_reads(other, 9, 0, 100, 150, 0)
    offs = np.arange(0, 100 * 150 + 1, 150, dtype=np.uint64)
    orc = OracleIndex(ix.n, 31, ix.rows, ix.C, ix.lcs)
    _, _, d, s = emu_encode(ix.n, 31, ix.rows, ix.C, ix.lcs, reads, offs, want_ms=True, variant=variant,
                            use_paths=paths)
    for r in range(100):
        od, olo = orc.ms(reads[r * 150:(r + 1) * 150].tobytes())
        assert np.array_equal(d[r * 150:(r + 1) * 150], od)
        assert np.array_equal(s[r * 150:(r + 1) * 150].astype(np.uint64), olo)


@pytest.mark.parametrize("k", [31, 91])
def test_emulated_v2_ms_on_repetitive_genome(k):
    # a genome built from repeated blocks: branching de Bruijn graph, many short paths,
    # non-singleton suffix groups -- the path walk must fall back correctly
    rng = np.random.default_rng(k)
    unit = nt.synth_genome(21, 400).tobytes()
    parts = []
    for _ in range(60):
        u = bytearray(unit)
        for _ in range(3):
            u[int(rng.integers(0, len(u)))] = b"ACGT"[int(rng.integers(0, 4))]
        parts.append(bytes(u) + nt.synth_genome(int(rng.integers(1, 1 << 30)), 97).tobytes())
    genome = np.frombuffer(b"".join(parts), dtype=np.uint8)
    ix = nt.Index.build([genome.tobytes()], k)
    reads = nt.synth_reads(genome, 8, 0, 800, 150, 10_000)
    offs = np.arange(0, 800 * 150 + 1, 150, dtype=np.uint64)
    orc = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs)
    exp, eoff = orc.encode(reads, offs)
    for variant in (4, 1):
        got, goff, d, s = emu_encode(ix.n, k, ix.rows, ix.C, ix.lcs, reads, offs, want_ms=True, variant=variant)
        assert np.array_equal(goff, eoff) and np.array_equal(got, exp)
    for r in range(0, 800, 37):
        od, olo = orc.ms(reads[r * 150:(r + 1) * 150].tobytes())
        assert np.array_equal(d[r * 150:(r + 1) * 150], od)
        assert np.array_equal(s[r * 150:(r + 1) * 150].astype(np.uint64), olo)


@pytest.mark.parametrize("k", [12, 31, 91])
def test_emulated_suffix_table_depth_is_invisible(k):
    """Records and matching statistics do not depend on the suffix-table depth U (U = 1
    walks every position through the SBWT; larger U reads more positions off the table)."""
    genome = nt.synth_genome(300 + k, 80_000)
    ix = nt.Index.build([genome.tobytes()], k)
    reads = nt.synth_reads(genome, 3, 0, 500, 150, 20_000)
    offs = np.arange(0, 500 * 150 + 1, 150, dtype=np.uint64)
    exp, eoff = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs).encode(reads, offs)
    base = None
    for u in (1, 2, 5, 9, 12, 14, 0):
        got, goff, d, s = emu_encode(ix.n, k, ix.rows, ix.C, ix.lcs, reads, offs, want_ms=True, tab_u=u)
        assert np.array_equal(got, exp) and np.array_equal(goff, eoff), u
        if base is None:
            base = (d, s)
        assert np.array_equal(d, base[0]) and np.array_equal(s, base[1]), u


def test_emulated_absent_character_is_an_invalid_base():
    # genome without 'T': a read holding T has d = 0 there (the reference never
    # terminates, lib.rs:207); the kernels report NTC_ERR_INVALID_BASE for that read
    ix = nt.Index.build(["ACGACGGACCAGACGAGGCAACGAGCACCGA" * 3], 7, add_revcomp=False)
    # (not b"ACGACGGAC": the reference panics on it, encode.rs:151-152 with len 9 > k = 7)
    reads = [b"CGGACCAGACGAGGCAACGA", b"ACGACGGACCAGACGAGG", b"ACGT"]
    bases, offs = pack_reads(reads)
    with pytest.raises(RuntimeError, match="rc=2 bad=2"):
        emu_encode(ix.n, 7, ix.rows, ix.C, ix.lcs, bases, offs)
    b2, o2 = pack_reads(reads[:2])
    got, goff = emu_encode(ix.n, 7, ix.rows, ix.C, ix.lcs, b2, o2)
    out, oo = emu_decode(ix.n, 7, ix.rows, ix.C, ix.lcs, got)
    assert np.array_equal(out, b2) and np.array_equal(oo, o2)


@pytest.mark.parametrize("k", [13, 31])
def test_emulated_periodic_genome_cycles(k):
    """Periodic contigs: with k above the period every k-mer lies on a pure cycle of the
    de Bruijn graph (no dummy leads in), so the path cover cuts each cycle at its smallest
    node.  Records stay bit-exact with and without paths."""
    from emu_lib import emu_path_cover
    unit_a, unit_b = b"ACGGTCATTC", b"TTGACCAGGATC"
    seqs = [unit_a * 20, unit_b * 15, nt.synth_genome(9, 3000).tobytes()]
    ix = nt.Index.build(seqs, k)
    h, tlen, npaths = emu_path_cover(ix.n, k, ix.rows, ix.C, ix.lcs)
    assert npaths >= 1 and tlen >= ix.n - 1
    genome = np.frombuffer(b"".join(seqs), dtype=np.uint8)
    reads = nt.synth_reads(genome, 4, 0, 400, 60, 20_000)
    offs = np.arange(0, 400 * 60 + 1, 60, dtype=np.uint64)
    exp, eoff = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs).encode(reads, offs)
    for paths in (True, False):
        got, goff = emu_encode(ix.n, k, ix.rows, ix.C, ix.lcs, reads, offs, use_paths=paths)
        assert np.array_equal(goff, eoff) and np.array_equal(got, exp)


@pytest.mark.parametrize("k", [23, 31, 91])
def test_emulated_linked_path_cover_strain_collection(k, monkeypatch):
    """Unitigs linked across branches (derived.cpp link_unitigs, the default): in a strain
    collection the shared sequence becomes a few long paths (fewer paths than unitigs), a
    read's runs leave them at its own variants and sequencing errors, and the records are
    the oracle's with linking on and off, with and without joint runs."""
    from emu_lib import emu_path_cover
    g = nt.synth_genome(21, 30_000)
    st = nt.synth_strains(g, 6, 60, 1500)
    texts = [g] + [st[i] for i in range(60)]
    ix = nt.Index.build([t.tobytes() for t in texts], k)
    monkeypatch.setenv("NTC_PATH_LINK", "0")
    _, tlen0, np0 = emu_path_cover(ix.n, k, ix.rows, ix.C, ix.lcs)
    monkeypatch.setenv("NTC_PATH_LINK", "1")
    _, tlen1, np1 = emu_path_cover(ix.n, k, ix.rows, ix.C, ix.lcs)
    assert np1 < np0 and tlen1 == tlen0 - k * (np0 - np1)  # a path takes its node count + k text positions
    reads = nt.synth_reads(np.concatenate(texts), 8, 0, 1500, 150, 10_000)
    offs = np.arange(0, 1500 * 150 + 1, 150, dtype=np.uint64)
    exp, eoff = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs).encode(reads, offs)
    for link in ("1", "0"):
        monkeypatch.setenv("NTC_PATH_LINK", link)
        for joint in ("1", "0"):
            monkeypatch.setenv("NTC_EMU_JOINT", joint)
            got, goff = emu_encode(ix.n, k, ix.rows, ix.C, ix.lcs, reads, offs)
            assert np.array_equal(goff, eoff) and np.array_equal(got, exp), (link, joint)


@pytest.mark.parametrize("block", [1, 3, 7, 256])
def test_emulated_staged_decode_block_sizes(block, monkeypatch):
    # k_dec_rec stages a block's output words in LDS and writes words shared with other
    # blocks character by character: tiny blocks make almost every word such a shared word
    monkeypatch.setenv("NTC_EMU_STAGE_BLOCK", str(block))
    genome = nt.synth_genome(8, 60_000)
    k = 31
    ix = nt.Index.build([genome.tobytes()], k)
    n, L = 300, 150
    reads = nt.synth_reads(genome, 6, 0, n, L, 20_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    got, _ = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs).encode(reads, offs)
    out, oo = emu_decode(ix.n, k, ix.rows, ix.C, ix.lcs, got)
    assert np.array_equal(out, reads)
    assert np.array_equal(oo, offs)


@pytest.mark.parametrize("block", [1, 4, 256])
def test_emulated_decode_direct_path_for_long_records(block, monkeypatch):
    # error-free 40 kb reads give ~one 40,000-base record each: more than kDecStageWords
    # (1024 words = 32 K bases) per block, so the decode writes ASCII directly
    monkeypatch.setenv("NTC_EMU_STAGE_BLOCK", str(block))
    genome = nt.synth_genome(18, 120_000)
    k = 31
    ix = nt.Index.build([genome.tobytes()], k)
    g = genome.tobytes()
    reads = [g[s:s + 40_000] for s in (0, 5_000, 31_000, 77_000)]
    bases = np.frombuffer(b"".join(reads), dtype=np.uint8).copy()
    offs = np.arange(0, 4 * 40_000 + 1, 40_000, dtype=np.uint64)
    got, _ = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs).encode(bases, offs)
    out, oo = emu_decode(ix.n, k, ix.rows, ix.C, ix.lcs, got)
    assert np.array_equal(out, bases)
    assert np.array_equal(oo, offs)


@pytest.mark.parametrize("k,glen", [(5, 300), (7, 20_000), (9, 2_000), (9, 20_000)])
def test_emulated_small_k_reference_panic_status(k, glen):
    """k <= 10: a short record with k < len <= 11 makes the reference panic
    (encode.rs:151-152, kmer[(k - len)..k]); the kernel returns NTC_ERR_REFERENCE_PANIC (11)
    for exactly the reads the oracle flags (ORC_ERR_PANIC), at the same first read of a batch,
    and bit-exact records for the others."""
    g = nt.synth_genome(50 + k, glen)
    ix = nt.Index.build([g.tobytes()], k)
    L, n = 150, 200
    reads = nt.synth_reads(g, 3, 0, n, L, 10_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    orc = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs)
    one = np.array([0, L], dtype=np.uint64)
    panics = [r for r in range(n) if orc.try_encode(reads[r * L:(r + 1) * L], one)[0] == -5]
    assert panics, "the case must occur"
    with pytest.raises(RuntimeError, match=f"rc=11 bad={panics[0]}"):
        emu_encode(ix.n, k, ix.rows, ix.C, ix.lcs, reads, offs)
    keep = [r for r in range(n) if r not in set(panics)]
    if keep:
        kr = np.concatenate([reads[r * L:(r + 1) * L] for r in keep])
        ko = np.arange(0, len(keep) * L + 1, L, dtype=np.uint64)
        got, goff = emu_encode(ix.n, k, ix.rows, ix.C, ix.lcs, kr, ko)
        exp, eoff = orc.encode(kr, ko)
        assert np.array_equal(got, exp) and np.array_equal(goff, eoff)


@pytest.mark.parametrize("joint", ["1", "0"])
@pytest.mark.parametrize("ext2", ["1", "0"])
@pytest.mark.parametrize("k", [31, 91])
def test_emulated_strain_collection(k, ext2, joint, monkeypatch):
    """A genome + 5 strains at 1 % substitutions (multi-node MS intervals over long climbs,
    short unitigs): records equal the oracle's with and without the two-character rank
    lines (NTC_EMU_EXT2), and decode back exactly.  The climbs run as joint path runs over
    the interval's first and last nodes (MsLane::note_single): (d, S) of every position of a
    read sample equals the oracle's matching statistics."""
    monkeypatch.setenv("NTC_EMU_EXT2", ext2)
    monkeypatch.setenv("NTC_EMU_JOINT", joint)
    g = nt.synth_genome(17, 150_000)
    st = nt.synth_strains(g, 3, 5, 10_000)
    texts = [g] + [st[i] for i in range(5)]
    ix = nt.Index.build([t.tobytes() for t in texts], k)
    n, L = 1500, 150
    reads = nt.synth_reads(np.concatenate(texts), 2, 0, n, L, 10_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    got, goff, d, s = emu_encode(ix.n, k, ix.rows, ix.C, ix.lcs, reads, offs, want_ms=True)
    orc = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs)
    exp, eoff = orc.encode(reads, offs)
    assert np.array_equal(goff, eoff) and np.array_equal(got, exp)
    for r in range(0, n, 11):
        od, olo = orc.ms(reads[r * L:(r + 1) * L].tobytes())
        assert np.array_equal(d[r * L:(r + 1) * L], od), r
        assert np.array_equal(s[r * L:(r + 1) * L].astype(np.uint64), olo), r
    out, oo = emu_decode(ix.n, k, ix.rows, ix.C, ix.lcs, got)
    assert np.array_equal(out, reads)


@pytest.mark.parametrize("win", ["1", "0"])
@pytest.mark.parametrize("k", [31, 91])
def test_emulated_run_breaks_without_joint_runs(k, win, monkeypatch):
    """k_ms4 as built for C91 (no joint runs) at U = 12 and 14, its SCAN on window words (the
    default) or on stride pair words behind the filter (win = 0).  Two strains make break
    positions long now and then (the mismatch is another copy's base), 3 % errors make breaks
    frequent; records and the (d, S) of a read sample equal the oracle's."""
    monkeypatch.setenv("NTC_EMU_JOINT", "0")
    monkeypatch.setenv("NTC_EMU_WIN", win)
    g = nt.synth_genome(41, 120_000)
    st = nt.synth_strains(g, 5, 2, 30_000)
    texts = [g] + [st[i] for i in range(2)]
    ix = nt.Index.build([t.tobytes() for t in texts], k)
    n, L = 1200, 150
    reads = nt.synth_reads(np.concatenate(texts), 6, 0, n, L, 30_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    orc = OracleIndex(ix.n, k, ix.rows, ix.C, ix.lcs)
    exp, eoff = orc.encode(reads, offs)
    for u in (12, 14):
        got, goff, d, s = emu_encode(ix.n, k, ix.rows, ix.C, ix.lcs, reads, offs, want_ms=True, tab_u=u)
        assert np.array_equal(goff, eoff) and np.array_equal(got, exp), u
        for r in range(0, n, 13):
            od, olo = orc.ms(reads[r * L:(r + 1) * L].tobytes())
            assert np.array_equal(d[r * L:(r + 1) * L], od), (u, r)
            assert np.array_equal(s[r * L:(r + 1) * L].astype(np.uint64), olo), (u, r)


def test_default_suffix_table_depth_follows_umer_density():
    """The upload's default depth (derived.cpp default_tab_u): U = min(k, 14, ceil(log4 n) + 2),
    one level deeper when the distinct 14-mers (nodes whose LCS with their colex predecessor is
    < 14) exceed 25 % of 4^14, as for a 100 Mbp genome (53 %); a strain collection of as many
    nodes that shares its 14-mers (S91: 8 %) keeps 14, and U never exceeds k."""
    from emu_lib import emu_default_tab_u
    n = 80_000_000  # > 0.25 * 4^14 = 67.1 M
    dense = np.zeros(n, dtype=np.uint8)  # every node its own 14-mer
    assert emu_default_tab_u(91, dense) == 15
    assert emu_default_tab_u(14, dense) == 14
    shared = np.full(n, 40, dtype=np.uint8)
    shared[::8] = 0  # 10 M distinct 14-mers: 15 %
    assert emu_default_tab_u(91, shared) == 14
    assert emu_default_tab_u(91, np.zeros(10_000_000, dtype=np.uint8)) == 14  # C91-sized: ceil(log4 n) + 2 = 14
    assert emu_default_tab_u(91, np.zeros(1000, dtype=np.uint8)) == 7
