#!/usr/bin/env python3
"""Golden vectors for the encoded.dat block codec -- an INDEPENDENT restatement.

Test infrastructure only.  This file shares no code with ntcomp_amd/csrc/block_codec.cpp
(or the GPU packer): it restates, from the published algorithms, what the reference's
write_block_to (src/lib.rs:232-252) computes before deflate, using explicit '0'/'1'
strings rather than word arithmetic:

  split_encoded_dictionary  src/encode.rs:168-229   four streams per block
      s1 = colex (bits 0-31) of every long record (flag bit 1 clear)
      s2 = length (bits 32-55) of every long record
      s3 = flag byte (bits 56-63) of every record
      s4 = the 2-bit bases of every short record, concatenated in record order, cut into
           31-base chunks (`chunks(31)`), each chunk bitnuc::as_2bit
  rice_encode               src/encode.rs:59-75     s2, s3
  minimal_binary_encode     src/encode.rs:77-94     s1, s4 (writes v + 1, max = maxval + 2)
  compress_block            src/encode.rs:96-127    header fields + to_ne_bytes of the words
  deflate_bytes             src/encode.rs:49-57     flate2 GzEncoder, Compression::default()

Third-party pieces, restated from their published descriptions ([ext, recalled]: the
crates are not in this container):

  dsi-bitstream 0.5.0 (Cargo.lock:462-465)
    * BufBitWriter<BE, MemWordWriterVec<u64>>: the code bits form one MSB-first bit
      string; it is cut into 64-bit words, the last word zero-padded, no word for an empty
      string.  The writer hands each word to the word writer as `to_be()`, so the native
      (little-endian) bytes encode.rs:107-109 takes of it are the bit string's bytes in order.
    * write_unary(n): n zeros, then a one.
    * write_rice(n, log2_b): unary(n >> log2_b), then the low log2_b bits of n.
    * write_minimal_binary(n, max): l = floor(log2 max), limit = 2^(l+1) - max;
      n < limit -> n in l bits; else n + limit in l + 1 bits.
    * rice::log2_b(p) = ceil(log2(-ln(phi) / ln_1p(-p))) cast `as usize` (Rust: NaN and
      negatives -> 0), phi = (sqrt 5 + 1) / 2.
  bitnuc 0.2.11 (Cargo.lock:145-148): as_2bit packs base i into bits 2i..2i+1,
      A = 0, C = 1, G = 2, T = 3 (as_2bit(b"ACGT") == 0b11100100).
  flate2 1.1.2 GzEncoder: 10-byte member header 1f 8b 08 00 | mtime 0 | XFL 0 | OS 255,
      then raw deflate (level 6 = Compression::default()), CRC-32, ISIZE.  The deflate
      bytes come from zlib-rs 0.5.1 in the reference and are NOT pinned here (only what
      inflates out of them is).

Reference behaviours the fixtures pin:
  * B.3  a block with no long record (empty s1) or no short record (empty s4) makes
         minimal_binary_encode err; write_block_to writes nothing ("dropped": true).
  * B.4  T (short bases of the block) % 31 == 0: the reference decoder would slice past
         the last chunk; the encoder side is well defined and pinned here.
  * B.6  the last block's num_records is num_records % 65536 (main.rs:176): the header
         carries whatever the caller passes.

Run: python tests/golden/make_codec_golden.py  ->  tests/golden/codec/codec_fixtures.json.gz
"""
import gzip
import json
import math
import os
import random

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "codec", "codec_fixtures.json.gz")

# ---- dsi-bitstream, restated on bit strings ----------------------------------------------
class BitString:
    def __init__(self):
        self.parts = []

    def bits(self, value, n):  # write_bits: the low n bits of value, MSB first
        if n:
            assert 0 <= value < (1 << n)
            self.parts.append(format(value, "0%db" % n))

    def unary(self, n):
        self.parts.append("0" * n + "1")

    def rice(self, n, log2_b):
        self.unary(n >> log2_b)
        self.bits(n & ((1 << log2_b) - 1), log2_b)

    def minimal_binary(self, n, mx):
        assert 0 <= n < mx
        l = mx.bit_length() - 1
        limit = (1 << (l + 1)) - mx
        if n < limit:
            self.bits(n, l)
        else:
            self.bits(n + limit, l + 1)

    def words(self):
        s = "".join(self.parts)
        if len(s) % 64:
            s += "0" * (64 - len(s) % 64)
        return [int(s[i:i + 64], 2) for i in range(0, len(s), 64)]


def rust_as_usize(x):
    if math.isnan(x) or x <= 0:
        return 0
    if math.isinf(x):
        return (1 << 64) - 1
    return int(x)


def log2_b(p):
    with np.errstate(all="ignore"):
        phi = (np.sqrt(np.float64(5.0)) + np.float64(1.0)) / np.float64(2.0)
        x = np.ceil(np.log2(-np.log(phi) / np.log1p(-np.float64(p))))
    return rust_as_usize(float(x))


def rice_stream(values):
    # encode.rs:62: inv_mean = exp(ln(len) - ln(sum)) in f64 (sum as u64 -> f64)
    with np.errstate(all="ignore"):
        inv_mean = np.exp(np.log(np.float64(len(values))) - np.log(np.float64(sum(values))))
    param = log2_b(float(inv_mean))
    w = BitString()
    for v in values:
        w.rice(v, param)
    return w.words(), param


def minimal_binary_stream(values):
    if not values:
        return None, None  # encode.rs:80: max() of an empty stream -> EncodeError
    mx = max(values) + 2
    w = BitString()
    for v in values:
        w.minimal_binary(v + 1, mx)
    return w.words(), mx


# ---- bitnuc + split_encoded_dictionary --------------------------------------------------
def as_2bit(codes):
    assert len(codes) <= 32
    return sum(c << (2 * i) for i, c in enumerate(codes))


def split(records):
    s1, s2, s3, bases = [], [], [], []
    for w in records:
        flag = w >> 56
        s3.append(flag)
        if flag & 2 == 0:
            s1.append(w & 0xFFFFFFFF)
            s2.append((w >> 32) & 0xFFFFFF)
        else:
            n = (flag & 0xFC) >> 2
            bases += [(w >> (2 * i)) & 3 for i in range(n)]
    s4 = [as_2bit(bases[i:i + 31]) for i in range(0, len(bases), 31)]
    return s1, s2, s3, s4, len(bases)


def payload_hex(words):
    return "".join(w.to_bytes(8, "big").hex() for w in words)  # to_be() then to_ne_bytes (LE)


def case(name, records, num_records, note=""):
    s1, s2, s3, s4, T = split(records)
    streams = []
    dropped = False
    for vals, codec in ((s1, "minimal_binary"), (s2, "rice"), (s3, "rice"), (s4, "minimal_binary")):
        if codec == "rice":
            words, param = rice_stream(vals) if vals else (None, None)
        else:
            words, param = minimal_binary_stream(vals)
        if words is None:
            dropped = True
            streams.append(None)
            continue
        streams.append({"codec": codec, "num_u64": len(vals), "encoded_size": len(words), "param": param,
                        "payload": payload_hex(words)})
    if dropped:
        streams = None  # write_block_to returns Err before writing anything (B.3)
    return {"name": name, "note": note, "num_records": num_records,
            "records": [format(w, "016x") for w in records], "short_bases": T, "dropped": dropped,
            "streams": streams}


# ---- record builders ---------------------------------------------------------------------
def long_rec(colex, length, first):
    assert 11 < length < (1 << 24) and 0 <= colex < (1 << 32)
    return colex | (length << 32) | (int(first) << 56)


def short_rec(codes, first):
    assert 1 <= len(codes) <= 11
    return as_2bit(codes) | (((int(first) + 2) | (len(codes) << 2)) << 56)


def random_block(rng, n_reads, colex_bits=32, p_long=0.75):
    recs = []
    for _ in range(n_reads):
        nr = rng.randint(1, 8)
        for j in range(nr):
            first = j == 0
            if rng.random() < p_long:
                length = min((1 << 24) - 1, 12 + int(rng.expovariate(1 / 40.0)))
                recs.append(long_rec(rng.getrandbits(colex_bits), length, first))
            else:
                recs.append(short_rec([rng.randrange(4) for _ in range(rng.randint(1, 11))], first))
    return recs


def golden_index_records(name):
    with gzip.open(os.path.join(HERE, name + ".json.gz"), "rt") as f:
        g = json.load(f)
    return [w for r in g["records"] for w in r], len(g["reads"])


def main():
    rng = random.Random(20260917)
    cases = []
    for name in ("k91_err", "ecoli_like_k31", "fasta_data_k255"):
        recs, nreads = golden_index_records(name)
        cases.append(case("records_of_" + name, recs, nreads, "records of the index golden " + name))
    cases.append(case("mixed_random", random_block(rng, 600), 600, "random fields; codes cross u64 words"))
    cases.append(case("mixed_random_small_colex", random_block(rng, 300, colex_bits=12), 300,
                      "minimal binary with a short code width"))
    # Rice parameter 0 on s3: mean flag <= 2.618 (mostly long records, flag 0 / 1)
    recs = [long_rec(rng.getrandbits(20), 40 + i, i % 7 == 0) for i in range(300)] + [short_rec([1], False)]
    cases.append(case("rice_param0_flags", recs, 43, "s3 Rice parameter 0"))
    # Rice quotients >= 64 on s2 (a few lengths near 2^24 among short ones)
    recs = [long_rec(i, 12 + (i % 5), i % 3 == 0) for i in range(200)]
    recs[17] = long_rec(17, (1 << 24) - 1, False)
    recs[150] = long_rec(150, 5_000_000, True)
    recs.append(short_rec([0, 1, 2], True))
    cases.append(case("rice_quotient_ge64", recs, 68, "s2 unary parts of >= 64 zeros"))
    # minimal binary with max + 2 a power of two (s1: max colex 2^20 - 2; s4: max chunk 2^62 - 2)
    recs = [long_rec(rng.randrange((1 << 20) - 2), 50, True) for _ in range(40)] + [long_rec((1 << 20) - 2, 60, False)]
    recs += [short_rec([2] + [3] * 10, False), short_rec([3] * 11, False), short_rec([3] * 9, True)]
    recs += [short_rec([rng.randrange(4) for _ in range(11)], False) for _ in range(3)]
    recs += [short_rec([1], False)] * 3  # T = 31 + 33 + 3 = 64 bases -> 3 chunks
    cases.append(case("minimal_binary_pow2", recs, 41, "s1 max+2 = 2^20; s4 first chunk = 2^62 - 2 (GTTT...T)"))
    # s4 with T % 31 == 0 (App. B.4)
    recs = [long_rec(5, 40, True)] + [short_rec([(i + j) % 4 for j in range(11)], i == 3)
                                      for i in range(8)] + [short_rec([0, 1, 2, 3, 0], False)]
    assert sum(((r >> 58) & 63) for r in recs if (r >> 57) & 1) % 31 == 0
    cases.append(case("short_bases_multiple_of_31", recs, 2, "T = 93: the reference decoder's T % 31 quirk"))
    # extreme values: colex 2^32 - 1 (33-bit minimal binary code), length 2^24 - 1, colex 0
    recs = [long_rec(0xFFFFFFFF, (1 << 24) - 1, True), long_rec(0, 12, False), short_rec([3] * 11, False),
            long_rec(0xFFFFFFFE, 13, True), short_rec([0], True)]
    cases.append(case("extreme_fields", recs, 3, "minimal binary width 32/33, max length"))
    # a single long and a single short record (s1 max + 2 = 2 -> 1-bit codes)
    cases.append(case("one_long_one_short", [long_rec(0, 12, True), short_rec([0], False)], 1,
                      "s1 = [0]: max = 2, l = 1"))
    # last block of a file: num_records = 70000 % 65536 (main.rs:176)
    cases.append(case("last_block_num_records", random_block(rng, 40), 70000 % 65536,
                      "header num_records as main.rs:176 passes it"))
    # dropped blocks (B.3)
    cases.append(case("dropped_no_short", [long_rec(9, 30, True), long_rec(10, 31, True)], 2,
                      "s4 empty -> write_block_to errs, block not written"))
    cases.append(case("dropped_no_long", [short_rec([1, 2], True), short_rec([0], True)], 2,
                      "s1 empty -> write_block_to errs, block not written"))
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    doc = {"generator": "tests/golden/make_codec_golden.py", "gzip_header_hex": "1f8b08000000000000ff",
           "cases": cases}
    with gzip.GzipFile(OUT, "wb", mtime=0) as f:
        f.write(json.dumps(doc, sort_keys=True).encode())
    print(f"{len(cases)} cases -> {OUT} ({os.path.getsize(OUT)} bytes)")
    for c in cases:
        if c["dropped"]:
            print(f"  {c['name']}: dropped")
        else:
            print(f"  {c['name']}: {len(c['records'])} records, params "
                  f"{[s['param'] for s in c['streams']]}, words {[s['encoded_size'] for s in c['streams']]}")


if __name__ == "__main__":
    main()
