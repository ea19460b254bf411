"""GPU block unpacker (unpack.hip: rice_decode / minimal_binary_decode / zip_block_contents,
src/decode.rs:51-149, on the device) against the independent codec restatement
(tests/golden/codec) and the host decoder (ntc_read_block): the same u64 records for every
fixture, for random blocks of 1 .. 70,000 records with Rice parameters from 0 to past 20,
and for full-size C91 blocks straight from the GPU packer; a damaged block ends the
output after the blocks before it (decode_block's Err, main.rs:202)."""
import numpy as np
import pytest

import ntcomp_amd as nt
from test_codec_golden import CASES, recs_of
from test_unpack import random_records

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = nt.GpuContext(0)
    yield c
    c.close()


def fixture_block(case):
    """(meta, payload) of a codec fixture: its four pre-deflate streams back to back"""
    meta = nt.BlockMeta()
    parts, off = [], 0
    for s in range(4):
        st = case["streams"][s]
        b = bytes.fromhex(st["payload"])
        assert len(b) == 8 * st["encoded_size"]
        meta.stream[s].num_u64, meta.stream[s].encoded_size, meta.stream[s].param = \
            st["num_u64"], st["encoded_size"], st["param"]
        meta.stream[s].offset = off
        parts.append(b)
        off += len(b)
    meta.n_recs = case["streams"][2]["num_u64"]
    return meta, b"".join(parts)


def test_gpu_unpack_codec_fixtures(ctx):
    names = [n for n in sorted(CASES) if not CASES[n]["dropped"]]
    blocks = [fixture_block(CASES[n]) for n in names]
    metas, payload = nt.concat_streams(blocks)
    ok, nr, nb = ctx.unpack(metas, payload, len(blocks))
    assert ok == len(names)
    exp = np.concatenate([recs_of(CASES[n]) for n in names])
    got = ctx.unpacked_records()
    assert np.array_equal(got, exp)
    flags = exp >> np.uint64(56)
    assert nr == int((flags & np.uint64(1)).sum())
    short = (flags & np.uint64(2)) != 0
    assert nb == int(np.where(short, flags >> np.uint64(2), (exp >> np.uint64(32)) & np.uint64(0xFFFFFF)).sum())
    for n in names:  # one at a time too (a stream far shorter than its 256 segments)
        ok, _, _ = ctx.unpack(*nt.concat_streams([fixture_block(CASES[n])]), 1)
        assert ok == 1 and np.array_equal(ctx.unpacked_records(), recs_of(CASES[n])), n


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_unpack_random_blocks(ctx, seed):
    rng = np.random.default_rng(seed)
    blocks, exp = [], []
    for i in range(12):
        n = int(rng.choice([2, 3, 50, 700, 4096, 20000, 70000]))
        recs = random_records(rng, n, colex_max=int(rng.choice([2, 1000, 1 << 20, 1 << 32])),
                              len_max=int(rng.choice([13, 100, 1 << 12, 1 << 24])),
                              short_frac=float(rng.choice([0.01, 0.3, 0.9])))
        recs[0] = np.uint64(5 | (12 << 32))  # one long record
        recs[-1] = np.uint64(1 | ((2 | (1 << 2)) << 56))  # and one short one (App. B.3)
        blob = nt.write_block(recs, n)
        blocks.append(nt.read_block_streams(blob)[:2])
        host, _, _ = nt.read_block(blob)
        assert np.array_equal(host, recs)
        exp.append(recs)
    metas, payload = nt.concat_streams(blocks)
    ok, _, _ = ctx.unpack(metas, payload, len(blocks))
    assert ok == len(blocks)
    assert np.array_equal(ctx.unpacked_records(), np.concatenate(exp))


def test_gpu_unpack_damaged_block_ends_output(ctx):
    rng = np.random.default_rng(5)
    blocks, exp = [], []
    for i in range(5):
        recs = random_records(rng, 3000)
        blocks.append(nt.read_block_streams(nt.write_block(recs, 3000))[:2])
        exp.append(recs)
    for damage in ("more_values", "short_stream", "flag_past_bases", "host_status"):
        metas, payload = nt.concat_streams(blocks)
        pay = bytearray(payload)
        m = metas[3]
        if damage == "more_values":  # the flag stream claims more codes than it holds
            m.stream[2].num_u64 += 40000
        elif damage == "short_stream":  # colex and length streams of different sizes
            m.stream[1].num_u64 -= 1
        elif damage == "flag_past_bases":  # more short bases than s4 holds
            m.stream[3].num_u64 += 1
        else:
            m.status = 8
        ok, nr, nb = ctx.unpack(metas, bytes(pay), len(blocks))
        assert ok == 3, damage
        got = ctx.unpacked_records()
        assert np.array_equal(got, np.concatenate(exp[:3])), damage


def test_gpu_unpack_full_blocks_from_the_gpu_packer(ctx):
    """C91-style reads: GPU packer -> deflate (host) -> inflate (host) -> GPU unpacker ->
    the encoder's records, and ntc_decode_fasta_unpacked -> the reads as FASTA."""
    genome = nt.synth_genome(11, 1_000_000)
    ix = nt.Index.build([genome.tobytes()], 91)
    ctx.upload(ix)
    n, L = 3 * 65536 + 1000, 150
    reads = nt.synth_reads(genome, 4, 0, n, L, 10_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    recs, _ = ctx.encode(reads, offs)
    metas, payload = ctx.encode_pack(reads, offs)
    blobs = [nt.deflate_block(m, payload, "libdeflate" if nt.libdeflate_available() else "zlib") for m in metas]
    blocks = [nt.read_block_streams(b)[:2] for b in blobs]
    um, up = nt.concat_streams(blocks)
    ok, nr, nb = ctx.unpack(um, up, len(blocks))
    assert (ok, nr, nb) == (len(blocks), n, n * L)
    assert np.array_equal(ctx.unpacked_records(), recs)
    text = ctx.decode_fasta_unpacked(first_id=1)
    lines = text.split(b"\n")
    assert lines[0] == b">seq.1" and lines[2 * (n - 1)] == b">seq.%d" % n
    assert b"".join(lines[1::2]) == reads.tobytes()
