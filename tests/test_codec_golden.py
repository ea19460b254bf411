"""Block codec vs the independent restatement (tests/golden/make_codec_golden.py).

The fixtures hold, per case, the u64 records of a block and the four streams that
write_block_to (src/lib.rs:232-252) hands to deflate: header fields (num_u64,
encoded_size, rice_param) and the pre-deflate bytes (split_encoded_dictionary +
rice / minimal-binary coding, src/encode.rs:59-127,168-229), restated from the published
dsi-bitstream / bitnuc / flate2 algorithms on '0'/'1' strings -- no code shared with
ntcomp_amd/csrc/block_codec.cpp or pack.hip.  Parity level S of SURVEY.md Appendix C;
the deflate bytes themselves (zlib-rs in the reference) stay unpinned, only what
inflates out of them is checked.  The GPU packer is checked against the same fixtures in
tests/test_gpu_pack.py (-m gpu)."""
import gzip
import json
import os
import struct
import zlib

import numpy as np
import pytest

import ntcomp_amd as nt

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "codec", "codec_fixtures.json.gz")


def load_cases():
    with gzip.open(FIX, "rt") as f:
        return json.load(f)


DOC = load_cases()
CASES = {c["name"]: c for c in DOC["cases"]}


def recs_of(case):
    return np.array([int(x, 16) for x in case["records"]], dtype=np.uint64)


def parse_container(blob):
    """-> list of 4 (header dict, gzip member bytes); asserts the block is fully consumed."""
    out, pos = [], 0
    for _ in range(4):
        block_size, num_records, num_u64, encoded_size, rice_param = struct.unpack_from("<IIIIQ", blob, pos)
        tail = blob[pos + 24:pos + 32]
        assert tail == b"\x08" + b"\0" * 7  # bitpacker_exponent = 8, placeholders 0 (encode.rs:113-120)
        member = blob[pos + 32:pos + 32 + block_size]
        out.append(({"num_records": num_records, "num_u64": num_u64, "encoded_size": encoded_size,
                     "param": rice_param}, member))
        pos += 32 + block_size
    assert pos == len(blob)
    return out


def test_fixture_shape():
    assert DOC["gzip_header_hex"] == "1f8b08000000000000ff"
    names = set(CASES)
    for need in ("rice_param0_flags", "rice_quotient_ge64", "minimal_binary_pow2", "short_bases_multiple_of_31",
                 "dropped_no_short", "dropped_no_long", "last_block_num_records", "extreme_fields"):
        assert need in names
    c = CASES["rice_param0_flags"]
    assert c["streams"][2]["param"] == 0
    c = CASES["rice_quotient_ge64"]
    p = c["streams"][1]["param"]
    assert max((int(r, 16) >> 32) & 0xFFFFFF for r in c["records"]) >> p >= 64
    c = CASES["minimal_binary_pow2"]
    for s in (0, 3):
        m = c["streams"][s]["param"]
        assert m & (m - 1) == 0  # max + 2 is a power of two
    assert CASES["short_bases_multiple_of_31"]["short_bases"] % 31 == 0
    assert CASES["last_block_num_records"]["num_records"] == 70000 % 65536


def test_restatement_hand_vector():
    """one_long_one_short by hand: s1 = [0] -> max = 2, l = 1, limit = 2, value 1 -> '1';
    s4 = one chunk "A" = 0 -> max 2 -> '1'; so both payloads are 0x80 00.. (one word)."""
    c = CASES["one_long_one_short"]
    assert c["streams"][0]["payload"] == "8000000000000000"
    assert c["streams"][3]["payload"] == "8000000000000000"
    # s2 = [12]: p = log2_b(1/12) = 3, rice(12, 3) = unary(1) 100 = '01' '100' -> 0110 0...
    assert c["streams"][1]["param"] == 3 and c["streams"][1]["payload"] == "6000000000000000"


@pytest.mark.parametrize("name", sorted(CASES))
def test_host_pack_matches_fixture(name):
    c = CASES[name]
    meta, payload = nt.pack_block(recs_of(c), c["num_records"])
    if c["dropped"]:
        assert meta.status == 3  # NTC_ERR_EMPTY_READ: write_block_to errs (App. B.3)
        return
    assert meta.status == 0 and meta.num_records == c["num_records"]
    got = nt.stream_payloads(meta, payload)
    for s in range(4):
        exp = c["streams"][s]
        m = meta.stream[s]
        assert (m.num_u64, m.encoded_size, m.param) == (exp["num_u64"], exp["encoded_size"], exp["param"]), (name, s)
        assert got[s].hex() == exp["payload"], (name, s)


@pytest.mark.parametrize("engine", ["zlib", "libdeflate"])
@pytest.mark.parametrize("name", sorted(CASES))
def test_write_block_container_matches_fixture(name, engine):
    c = CASES[name]
    recs = recs_of(c)
    if c["dropped"]:
        with pytest.raises(nt.NtcError) as e:
            nt.write_block(recs, c["num_records"])
        assert e.value.code == 3
        return
    if engine == "zlib":
        blob = nt.write_block(recs, c["num_records"])
    else:
        meta, payload = nt.pack_block(recs, c["num_records"])
        try:
            blob = nt.deflate_block(meta, payload, engine)
        except nt.NtcError as e:
            if e.code == 10:
                pytest.skip("libdeflate.so.0 not on this host")
            raise
    for s, (h, member) in enumerate(parse_container(blob)):
        exp = c["streams"][s]
        assert h == {"num_records": c["num_records"], "num_u64": exp["num_u64"],
                     "encoded_size": exp["encoded_size"], "param": exp["param"]}
        assert member[:10].hex() == DOC["gzip_header_hex"]  # flate2 GzEncoder header (OS 255)
        raw = zlib.decompress(member, 31)
        assert raw.hex() == exp["payload"]
        crc, isize = struct.unpack("<II", member[-8:])
        assert crc == zlib.crc32(raw) and isize == len(raw)


@pytest.mark.parametrize("name", sorted(CASES))
def test_read_block_of_independently_built_container(name):
    """A container assembled here from the fixture streams (Python's zlib, not the
    library's deflate) decodes to the fixture records (decode_block, lib.rs:320-363)."""
    c = CASES[name]
    if c["dropped"]:
        return
    blob = b""
    for exp in c["streams"]:
        raw = bytes.fromhex(exp["payload"])
        co = zlib.compressobj(6, zlib.DEFLATED, 31)
        member = co.compress(raw) + co.flush()
        blob += struct.pack("<IIIIQ", len(member), c["num_records"], exp["num_u64"], exp["encoded_size"],
                            exp["param"]) + b"\x08" + b"\0" * 7 + member
    got, used, nrec = nt.read_block(blob)
    assert used == len(blob) and nrec == c["num_records"]
    assert np.array_equal(got, recs_of(c))


def test_short_record_past_32_bases_is_malformed():
    # from_2bit panics past 32 bases (encode.rs:220): the packer reports NTC_ERR_FORMAT
    recs = np.array([5 | (40 << 32) | (1 << 56), (2 | (40 << 2)) << 56], dtype=np.uint64)
    with pytest.raises(nt.NtcError) as e:
        nt.pack_block(recs, 1)
    assert e.value.code == 8


@pytest.mark.parametrize("engine", ["zlib", "libdeflate"])
@pytest.mark.parametrize("name", sorted(n for n in CASES if not CASES[n]["dropped"]))
def test_deflate_streams_concatenate_to_the_block(name, engine):
    """ntc_deflate_stream (the pipeline deflates a block's four streams in parallel): the four
    parts back to back are ntc_deflate_block's bytes; a dropped block's status comes back."""
    c = CASES[name]
    meta, payload = nt.pack_block(recs_of(c), c["num_records"])
    try:
        whole = nt.deflate_block(meta, payload, engine)
    except nt.NtcError as e:
        if e.code == 10:
            pytest.skip("libdeflate.so.0 not on this host")
        raise
    assert b"".join(nt.deflate_stream(meta, s, payload, engine) for s in range(4)) == whole
    with pytest.raises(nt.NtcError):
        nt.deflate_stream(meta, 4, payload, engine)


def test_adaptive_deflate_stores_incompressible_streams():
    """NTC_DEFLATE_ADAPTIVE: a stream of >= 7.9 bits of order-0 entropy per byte (checked on
    its first 32 KiB) goes out as stored deflate blocks (5 bytes per <= 65,535, so the member
    is 18 bytes of gzip framing longer than the data plus those), anything else as
    libdeflate level 6 -- the same bytes as NTC_DEFLATE_LIBDEFLATE.  Both inflate to the
    streams (Python's zlib checks the CRC and ISIZE too)."""
    if not nt.libdeflate_available():
        pytest.skip("libdeflate.so.0 not on this host")
    rng = np.random.default_rng(5)
    # long records with random colex ids (s1 near 8 bits/byte) and short ones with random bases
    n = 20000
    recs = np.zeros(2 * n, dtype=np.uint64)
    ids = rng.integers(0, 1 << 31, n, dtype=np.uint64)
    lens = rng.integers(12, 40, n, dtype=np.uint64)
    recs[0::2] = ids | (lens << np.uint64(32)) | (np.uint64(1) << np.uint64(56))
    sl = rng.integers(1, 12, n, dtype=np.uint64)
    bases = rng.integers(0, 1 << 22, n, dtype=np.uint64) & ((np.uint64(1) << (np.uint64(2) * sl)) - np.uint64(1))
    recs[1::2] = bases | (((np.uint64(2) | (sl << np.uint64(2)))) << np.uint64(56))
    meta, payload = nt.pack_block(recs, n)
    streams = nt.stream_payloads(meta, payload)
    ad = parse_container(nt.deflate_block(meta, payload, "adaptive"))
    ld = parse_container(nt.deflate_block(meta, payload, "libdeflate"))
    stored = 0
    for s, ((h, m), (_, m_ld)) in enumerate(zip(ad, ld)):
        raw = streams[s]
        assert zlib.decompress(m, 31) == raw and zlib.decompress(m_ld, 31) == raw
        if len(raw) >= 4096 and entropy0(raw[:32768]) >= 7.9:
            stored += 1
            assert len(m) == 18 + len(raw) + 5 * max(1, -(-len(raw) // 65535)), s
            assert len(m) <= len(m_ld) * 1.001 + 64, s
        else:
            assert m == m_ld, s
    assert stored >= 1


def entropy0(b):
    c = np.bincount(np.frombuffer(b, dtype=np.uint8), minlength=256).astype(float)
    p = c[c > 0] / len(b)
    return float(-(p * np.log2(p)).sum())
