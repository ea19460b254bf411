"""GPU block packer (pack.hip, ntc_pack_blocks_device / ntc_encode_pack_batch) against the
independent codec restatement (tests/golden/codec, tests/golden/make_codec_golden.py) and
against the host packer at full block size.  Parity level S of SURVEY.md Appendix C:
byte-exact pre-deflate streams and header fields of write_block_to (src/lib.rs:232-252)."""
import numpy as np
import pytest

import ntcomp_amd as nt
from test_codec_golden import CASES, recs_of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = nt.GpuContext(0)
    yield c
    c.close()


def device_pack(ctx, blocks, block_reads=1):
    """Pack a list of record arrays, one read each (block_reads = 1 -> one block per array)."""
    recs = np.concatenate([np.asarray(b, dtype=np.uint64) for b in blocks]) if blocks else np.zeros(0, np.uint64)
    roffs = np.zeros(len(blocks) + 1, dtype=np.uint64)
    roffs[1:] = np.cumsum([len(b) for b in blocks])
    d_recs, d_roffs = ctx.alloc(max(8, recs.nbytes)), ctx.alloc(roffs.nbytes)
    cap = max(1 << 16, 16 * len(recs) + 1024 * len(blocks))
    d_pay = ctx.alloc(cap)
    try:
        if len(recs):
            ctx.h2d(d_recs, recs)
        ctx.h2d(d_roffs, roffs)
        metas, used = ctx.pack_device(d_recs, d_roffs, len(blocks), block_reads, d_pay, cap)
        payload = np.zeros(max(used, 8), dtype=np.uint8)
        if used:
            ctx.d2h(payload, d_pay)
        return metas, payload[:used].tobytes()
    finally:
        for p in (d_recs, d_roffs, d_pay):
            ctx.free(p)


def test_gpu_pack_matches_codec_fixtures(ctx):
    names = sorted(CASES)
    metas, payload = device_pack(ctx, [recs_of(CASES[n]) for n in names])
    assert len(metas) == len(names)
    for n, m in zip(names, metas):
        c = CASES[n]
        if c["dropped"]:
            assert m.status == 3, n  # NTC_ERR_EMPTY_READ (App. B.3)
            continue
        assert m.status == 0, n
        got = nt.stream_payloads(m, payload)
        for s in range(4):
            exp = c["streams"][s]
            st = m.stream[s]
            assert (st.num_u64, st.encoded_size, st.param) == (exp["num_u64"], exp["encoded_size"], exp["param"]), (n, s)
            assert got[s].hex() == exp["payload"], (n, s)


def test_gpu_pack_fallback_tiles_equal_host_packer(ctx):
    """A tile whose codes overflow the LDS word buffers (s3 Rice parameter 0 with flag bytes
    of 253: 254 bits per code over 4096 records) goes through the global-atomic path."""
    rng = np.random.default_rng(3)
    n = 500_000
    recs = (rng.integers(0, 1 << 30, n, dtype=np.uint64) | (rng.integers(12, 200, n, dtype=np.uint64) << 32))
    recs[200_000:204_096] |= np.uint64(253) << np.uint64(56)  # long records (bit 1 clear) with flag 253
    recs[-1] = (np.uint64(2 | (5 << 2)) << np.uint64(56)) | np.uint64(0b1001110110)  # one short record
    hm, hp = nt.pack_block(recs, 1)
    assert hm.status == 0 and hm.stream[2].param == 0
    metas, payload = device_pack(ctx, [recs])
    assert metas[0].status == 0
    for s, (a, b) in enumerate(zip(nt.stream_payloads(hm, hp), nt.stream_payloads(metas[0], payload))):
        assert a == b, s


@pytest.mark.parametrize("k,err_ppm", [(91, 10_000), (31, 10_000), (91, 0)])
def test_gpu_encode_pack_equals_host_pack(ctx, k, err_ppm):
    """Full 65,536-read blocks plus a partial last block (main.rs:174-177): the fused
    encode + GPU pack path equals encode -> host records -> host packer, block by block,
    and the deflated container decodes back to the reads."""
    genome = nt.synth_genome(7 + k, 1_000_000)
    ix = nt.Index.build([genome.tobytes()], k)
    ctx.upload(ix)
    n, L = 3 * 65536 + 1234, 150
    reads = nt.synth_reads(genome, 11, 0, n, L, err_ppm)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    recs, roff = ctx.encode(reads, offs)
    metas, payload = ctx.encode_pack(reads, offs, 65536)
    assert len(metas) == 4
    blob = b""
    for b, m in enumerate(metas):
        r0, r1 = b * 65536, min(n, (b + 1) * 65536)
        assert m.num_records == r1 - r0
        hm, hp = nt.pack_block(recs[int(roff[r0]):int(roff[r1])], r1 - r0)
        assert m.status == hm.status
        if m.status:
            continue
        for s in range(4):
            assert (m.stream[s].num_u64, m.stream[s].encoded_size, m.stream[s].param) == \
                (hm.stream[s].num_u64, hm.stream[s].encoded_size, hm.stream[s].param), (b, s)
        assert nt.stream_payloads(m, payload) == nt.stream_payloads(hm, hp), b
        blob += nt.deflate_block(m, payload)
    pos, got = 0, []
    while pos < len(blob):
        r, used, _ = nt.read_block(blob[pos:])
        got.append(r)
        pos += used
    if all(m.status == 3 for m in metas):
        # error-free reads at k = 91 leave no short record: every block is dropped, as the
        # reference's write_block_to does (App. B.3), so the file holds no block
        assert err_ppm == 0 and not got
        return
    out, o2 = ctx.decode(np.concatenate(got))
    assert np.array_equal(out, reads) and np.array_equal(o2, offs)


def test_gpu_pack_empty_and_errors(ctx):
    metas, payload = device_pack(ctx, [])
    assert metas == [] and payload == b""
    # a short record past 32 bases -> NTC_ERR_FORMAT status for its block only
    good = recs_of(CASES["mixed_random"])
    bad = np.array([5 | (40 << 32) | (1 << 56), (2 | (40 << 2)) << 56], dtype=np.uint64)
    metas, _ = device_pack(ctx, [good, bad, good])
    assert [m.status for m in metas] == [0, 8, 0]


def test_gpu_pack_short_records_of_32_bases(ctx):
    """Short records at from_2bit's 32-base limit: a block of n of them fills ceil(32 n / 31)
    s4 chunks, more than n + 1, so neighbouring blocks' chunk regions must not overlap
    (pack.hip chunk_base).  Several such blocks side by side equal the host packer."""
    rng = np.random.default_rng(5)
    blocks = []
    for b in range(5):
        n = 64 + 37 * b
        short = rng.integers(0, 1 << 56, n, dtype=np.uint64) | (np.uint64(2 | (32 << 2)) << np.uint64(56))
        long_ = np.array([7 + b | (40 << 32) | (1 << 56)], dtype=np.uint64)
        blocks.append(np.concatenate([long_, short]))
    metas, payload = device_pack(ctx, blocks)
    for b, m in enumerate(metas):
        hm, hp = nt.pack_block(blocks[b], 1)
        assert m.status == hm.status == 0, b
        assert m.stream[3].num_u64 == hm.stream[3].num_u64 == -(-32 * (len(blocks[b]) - 1) // 31), b
        assert nt.stream_payloads(m, payload) == nt.stream_payloads(hm, hp), b
