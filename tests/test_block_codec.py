"""Host block container (ntcomp_amd/csrc/block_codec.cpp) -- write_block_to /
decode_block of src/lib.rs:232-368 and the codecs of src/encode.rs, src/decode.rs.
Records come from the CPU oracle so these tests need no GPU."""
import ctypes
import gzip

import numpy as np
import pytest

import ntcomp_amd as nt
from oracle_lib import OracleIndex, golden_names, load_golden, pack_reads


def _rec_arr(g):
    return np.array([w for r in g["records"] for w in r], dtype=np.uint64)


@pytest.mark.parametrize("name", golden_names())
def test_block_roundtrip_golden(name):
    g = load_golden(name)
    recs = _rec_arr(g)
    blob = nt.write_block(recs, len(g["reads"]))
    got, used, nrec = nt.read_block(blob)
    assert used == len(blob)
    assert np.array_equal(got, recs)
    assert nrec == len(g["reads"])


def test_block_layout_headers():
    g = load_golden("ecoli_like_k31")
    recs = _rec_arr(g)
    blob = nt.write_block(recs, 7)
    pos = 0
    flags = (recs >> np.uint64(56)).astype(np.uint64)
    n_long = int(((flags & np.uint64(2)) == 0).sum())
    expect_num_u64 = [n_long, n_long, len(recs), None]
    for s in range(4):
        h = blob[pos:pos + 32]
        block_size, num_records, num_u64, encoded_size = np.frombuffer(h[:16], dtype="<u4")
        rice_param = int(np.frombuffer(h[16:24], dtype="<u8")[0])
        assert h[24] == 8 and h[25:32] == b"\0" * 7  # bitpacker_exponent = 8, placeholders 0
        assert num_records == 7
        if expect_num_u64[s] is not None:
            assert num_u64 == expect_num_u64[s]
        payload = blob[pos + 32:pos + 32 + block_size]
        assert payload[:4] == b"\x1f\x8b\x08\x00" and payload[9] == 0xFF  # flate2-style gzip header
        raw = gzip.decompress(payload)
        assert len(raw) == 8 * encoded_size
        if s in (0, 3):  # minimal binary: param = max + 2
            assert rice_param >= 2
        pos += 32 + block_size
    assert pos == len(blob)


def test_short_stream_chunking_multiple_of_31():
    # decode.rs:114-118 takes T % 31 bases from the last chunk; T = 62 would panic in the
    # reference.  Here it must round-trip.
    short = []
    for j in range(62 // 2):
        w = (0b1001 & ((1 << 56) - 1)) | (((0 + 2) | (2 << 2)) << 56)  # 2 bases, not first
        short.append(w)
    long_first = (5 | (40 << 32) | (1 << 56))
    recs = np.array([long_first] + short, dtype=np.uint64)
    got, _, _ = nt.read_block(nt.write_block(recs, 1))
    assert np.array_equal(got, recs)


def test_block_without_short_records_is_dropped_like_reference():
    # minimal_binary_encode errors on an empty stream -> write_block_to writes nothing (B.3)
    recs = np.array([5 | (40 << 32) | (1 << 56)], dtype=np.uint64)
    with pytest.raises(nt.NtcError) as e:
        nt.write_block(recs, 1)
    assert e.value.code == 3


def test_multi_block_stream_and_eof():
    g = load_golden("k91_err")
    ix = OracleIndex(g["n"], g["k"], g["rows_u64"], g["C"], g["lcs_u8"])
    blob = b"\0" * 32
    per_read = g["records"]
    for a in range(0, len(per_read), 5):
        chunk = np.array([w for r in per_read[a:a + 5] for w in r], dtype=np.uint64)
        try:
            blob += nt.write_block(chunk, len(per_read[a:a + 5]))
        except nt.NtcError:
            pass
    pos, allrecs = 32, []
    while True:
        try:
            recs, used, _ = nt.read_block(blob[pos:])
        except nt.NtcError as e:
            assert e.code == 9  # clean EOF
            break
        allrecs.append(recs)
        pos += used
    out, offs = ix.decode(np.concatenate(allrecs))
    got = [out[offs[i]:offs[i + 1]].tobytes().decode() for i in range(len(offs) - 1)]
    assert len(got) > 0 and all(r in g["reads"] for r in got)


def test_stream_bytes_hand_derived_fixture():
    """Byte order of the stream words, pinned by hand (parity unpinned vs the reference: no
    reference-written encoded.dat exists offline).  One read of 3 long records with colex
    0, 1, 2 (lengths 12, 13, 14) and a short one: s1 = [0, 1, 2] -> minimal binary with max = 2 + 2 = 4
    (encode.rs:77-94): v + 1 = 1, 2, 3 in 2 bits = 01 10 11 -> 0b011011 then zero padding,
    so the inflated s1 payload is 6C 00 00 00 00 00 00 00 (MSB-first bitstream on disk,
    SURVEY.md A.4).  s2 = lengths [12, 13, 14] with Rice and s3 = flags follow."""
    recs = np.array([(1 << 56) | (12 << 32) | 0, (13 << 32) | 1, (14 << 32) | 2, (2 | 1 << 2) << 56],
                    dtype=np.uint64)  # + one short record "A" (a block without one is dropped, App. B.3)
    blob = nt.write_block(recs, 1)
    h = blob[:32]
    block_size, _, num_u64, encoded_size = np.frombuffer(h[:16], dtype="<u4")
    assert (num_u64, encoded_size, int(np.frombuffer(h[16:24], dtype="<u8")[0])) == (3, 1, 4)
    payload = gzip.decompress(blob[32:32 + int(block_size)])
    assert payload == bytes([0x6C, 0, 0, 0, 0, 0, 0, 0])
    got, used, _ = nt.read_block(blob)
    assert np.array_equal(got, recs)
