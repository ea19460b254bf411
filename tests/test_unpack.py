"""Host half of the GPU unpacker (ntc_read_block_streams): a block's stream headers and its
four inflated streams, exactly the pre-deflate words the packer wrote (src/lib.rs:320-363
up to rice_decode / minimal_binary_decode), for containers written by the host codec."""
import numpy as np
import pytest

import ntcomp_amd as nt


def random_records(rng, n, colex_max=1 << 32, len_max=1 << 24, short_frac=0.3):
    recs = np.zeros(n, dtype=np.uint64)
    first = rng.random(n) < 0.3
    short = rng.random(n) < short_frac
    for i in range(n):
        f = int(first[i])
        if short[i]:
            L = int(rng.integers(1, 12))
            bases = int(rng.integers(0, 1 << (2 * L)))
            recs[i] = bases | (((f + 2) | (L << 2)) << 56)
        else:
            L = int(rng.integers(12, len_max))
            recs[i] = int(rng.integers(0, colex_max)) | (L << 32) | (f << 56)
    return recs


@pytest.mark.parametrize("seed,n", [(1, 1), (2, 37), (3, 5000), (4, 70000)])
def test_read_block_streams_equal_packer_payload(seed, n):
    rng = np.random.default_rng(seed)
    recs = random_records(rng, n, len_max=1 << (6 + seed * 4), short_frac=0.5 if n > 1 else 0.0)
    if n == 1:  # a block needs a long and a short record (App. B.3)
        recs = np.concatenate([recs, random_records(rng, 1, short_frac=1.0)])
    blob = nt.write_block(recs, 7)
    meta, pay = nt.pack_block(recs, 7)
    got, gpay, used = nt.read_block_streams(blob)
    assert used == len(blob)
    assert (got.n_recs, got.num_records, got.status) == (len(recs), 7, 0)
    for s in range(4):
        a, b = meta.stream[s], got.stream[s]
        assert (a.num_u64, a.encoded_size, a.param) == (b.num_u64, b.encoded_size, b.param), s
    assert nt.stream_payloads(got, gpay) == nt.stream_payloads(meta, pay)


def test_read_block_streams_errors():
    rng = np.random.default_rng(9)
    recs = random_records(rng, 300)
    blob = nt.write_block(recs, 1)
    with pytest.raises(nt.NtcError) as e:
        nt.read_block_streams(b"")
    assert e.value.code == 9  # NTC_ERR_IO: a clean end of input
    for cut in (10, 40, len(blob) - 3):
        with pytest.raises(nt.NtcError) as e:
            nt.read_block_streams(blob[:cut])
        assert e.value.code == 8, cut  # NTC_ERR_FORMAT
    bad = bytearray(blob)
    bad[32 + 20] ^= 0xFF  # inside the first gzip member
    with pytest.raises(nt.NtcError) as e:
        nt.read_block_streams(bytes(bad))
    assert e.value.code == 8
