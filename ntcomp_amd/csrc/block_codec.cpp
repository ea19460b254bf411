// Block container of encoded.dat: the host-side steps on either side of the GPU kernels.
//
//   split_encoded_dictionary  encode.rs:168-229  (4 streams: colex ranks, match lengths,
//                                                 flag bytes, short-record bases in 31-base
//                                                 as_2bit chunks)
//   rice_encode / minimal_binary_encode         encode.rs:59-94   [ext dsi-bitstream 0.5.0]
//   deflate_bytes (gzip, level 6)               encode.rs:49-57   [ext flate2 1.1.2]
//   compress_block + BlockHeader (32 B)         encode.rs:96-127, lib.rs:37-50,75-86
//   write_block_to                              lib.rs:232-252
//   decode_block / decompress_block /
//   zip_block_contents                          lib.rs:320-368, decode.rs:41-149
//   file header (4 x u64 = 32 zero bytes)       lib.rs:29-35,52-73
//
// Restated dsi-bitstream semantics (not in the container; recalled):
//   * BufBitWriter<BE, u64 words>: bits MSB-first into u64 words, last word zero-padded;
//     words stored with to_ne_bytes (little-endian) (encode.rs:107-109).
//   * unary(n) = n zeros then a one; rice(n, b) = unary(n >> b) then the low b bits.
//   * rice::log2_b(p) = ceil(log2(ln(phi) / -ln(1-p))), saturating at 0 (Rust `as usize`).
//   * minimal_binary(v, max): l = floor(log2 max), limit = 2^(l+1) - max;
//     v < limit -> v in l bits, else v + limit in l+1 bits.
//   * gzip member like flate2's GzEncoder: 10-byte header (mtime 0, XFL 0, OS 255), raw
//     deflate at level 6, CRC32 + ISIZE trailer.  Deflate bytes come from system zlib, so
//     they inflate identically but are not byte-identical to zlib-rs (parity level F is
//     unpinned).
#include <zlib.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ntcomp_codec.h"

namespace {

// ---- bit writer / reader (big-endian bit order in u64 words) -------------------------
struct BitWriter {
    std::vector<uint64_t> words;
    uint64_t cur = 0;
    int used = 0;  // bits used in cur (from the MSB)
    void put(uint64_t v, int nbits) {  // the low nbits (<= 64) of v, most significant first
        if (nbits <= 0) return;
        if (nbits < 64) v &= (1ULL << nbits) - 1;
        const int room = 64 - used;
        if (nbits <= room) {
            cur |= (room == nbits) ? v : (v << (room - nbits));
            used += nbits;
        } else {
            const int lo = nbits - room;  // 1..63
            cur |= v >> lo;
            words.push_back(cur);
            cur = v << (64 - lo);
            used = lo;
        }
        if (used == 64) {
            words.push_back(cur);
            cur = 0;
            used = 0;
        }
    }
    void unary(uint64_t n) {
        while (n >= 64) {
            put(0, 64);
            n -= 64;
        }
        if (n) put(0, (int)n);
        put(1, 1);
    }
    std::vector<uint64_t> finish() {
        if (used) {
            words.push_back(cur);
            cur = 0;
            used = 0;
        }
        return words;
    }
};

struct BitReader {
    const uint64_t *w;
    uint64_t nw, pos = 0;  // bit position
    BitReader(const uint64_t *words, uint64_t n) : w(words), nw(n) {}
    // the next 64 bits from pos, MSB first (zero past the end)
    uint64_t peek64() const {
        const uint64_t i = pos >> 6, sh = pos & 63;
        const uint64_t hi = i < nw ? w[i] : 0;
        if (!sh) return hi;
        const uint64_t lo = i + 1 < nw ? w[i + 1] : 0;
        return (hi << sh) | (lo >> (64 - sh));
    }
    bool bit(int &b) {
        if (pos >= nw * 64) return false;
        b = (int)((w[pos >> 6] >> (63 - (pos & 63))) & 1);
        pos++;
        return true;
    }
    bool get(int nbits, uint64_t &v) {
        if (nbits == 0) {
            v = 0;
            return true;
        }
        if (pos + (uint64_t)nbits > nw * 64) return false;
        v = peek64() >> (64 - nbits);
        pos += (uint64_t)nbits;
        return true;
    }
    bool unary(uint64_t &n) {  // zeros up to and including the terminating one
        n = 0;
        for (;;) {
            if (pos >= nw * 64) return false;
            const uint64_t x = peek64();
            if (x) {
                const int z = __builtin_clzll(x);
                if (pos + (uint64_t)z >= nw * 64) return false;
                n += (uint64_t)z;
                pos += (uint64_t)z + 1;
                return true;
            }
            n += 64;
            pos += 64;
        }
    }
};

int ilog2(uint64_t x) { return 63 - __builtin_clzll(x); }

uint64_t rice_log2_b(double p) {
    const double phi = (std::sqrt(5.0) + 1.0) / 2.0;
    double v = std::ceil(std::log2(std::log(phi) / -std::log1p(-p)));
    if (!(v > 0)) return 0;  // NaN and negatives saturate to 0 like Rust's `as usize`
    if (v > 63) return 63;
    return (uint64_t)v;
}

std::vector<uint64_t> rice_encode(const std::vector<uint64_t> &ints, uint64_t &param) {
    long double sum = 0;
    for (uint64_t x : ints) sum += (long double)x;
    // encode.rs:62: inv_mean = exp(ln(len) - ln(sum))
    double inv_mean = std::exp(std::log((double)ints.size()) - std::log((double)sum));
    param = rice_log2_b(inv_mean);
    BitWriter bw;
    for (uint64_t n : ints) {
        bw.unary(n >> param);
        if (param) bw.put(n & ((1ULL << param) - 1), (int)param);
    }
    return bw.finish();
}

bool minimal_binary_encode(const std::vector<uint64_t> &ints, std::vector<uint64_t> &out, uint64_t &param) {
    if (ints.empty()) return false;  // encode.rs:80 EncodeError (block dropped, Appendix B.3)
    uint64_t mx = 0;
    for (uint64_t x : ints) mx = x > mx ? x : mx;
    param = mx + 2;
    const int l = ilog2(param);
    const uint64_t limit = (2ULL << l) - param;
    BitWriter bw;
    for (uint64_t x : ints) {
        uint64_t v = x + 1;
        if (v < limit) bw.put(v, l);
        else bw.put(v + limit, l + 1);
    }
    out = bw.finish();
    return true;
}

bool rice_decode(const std::vector<uint64_t> &w, uint64_t n, uint64_t param, std::vector<uint64_t> &out) {
    BitReader br(w.data(), w.size());
    out.resize(n);
    for (uint64_t i = 0; i < n; i++) {
        uint64_t q, r = 0;
        if (!br.unary(q) || (param && !br.get((int)param, r))) return false;
        out[i] = (q << param) | r;
    }
    return true;
}

bool minimal_binary_decode(const std::vector<uint64_t> &w, uint64_t n, uint64_t param, std::vector<uint64_t> &out) {
    if (param < 1) return n == 0;
    BitReader br(w.data(), w.size());
    const int l = ilog2(param);
    const uint64_t limit = (2ULL << l) - param;
    out.resize(n);
    for (uint64_t i = 0; i < n; i++) {
        uint64_t v;
        if (!br.get(l, v)) return false;
        if (v >= limit) {
            int b;
            if (!br.bit(b)) return false;
            v = ((v << 1) | (uint64_t)b) - limit;
        }
        if (v == 0) return false;
        out[i] = v - 1;
    }
    return true;
}

// ---- gzip (flate2 GzEncoder-shaped member) ---------------------------------------------
bool gzip_bytes(const uint8_t *data, size_t n, std::vector<uint8_t> &out) {
    const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 0xff};
    out.assign(hdr, hdr + 10);
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (deflateInit2(&zs, 6, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
    size_t bound = deflateBound(&zs, (uLong)n) + 16;
    out.resize(10 + bound);
    zs.next_in = const_cast<Bytef *>(data);
    zs.avail_in = (uInt)n;
    zs.next_out = out.data() + 10;
    zs.avail_out = (uInt)bound;
    int rc = deflate(&zs, Z_FINISH);
    size_t produced = bound - zs.avail_out;
    deflateEnd(&zs);
    if (rc != Z_STREAM_END) return false;
    out.resize(10 + produced);
    uint32_t crc = (uint32_t)crc32(0L, data, (uInt)n), isize = (uint32_t)n;
    for (int i = 0; i < 4; i++) out.push_back((uint8_t)(crc >> (8 * i)));
    for (int i = 0; i < 4; i++) out.push_back((uint8_t)(isize >> (8 * i)));
    return true;
}

bool gunzip_bytes(const uint8_t *data, size_t n, std::vector<uint8_t> &out) {
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (inflateInit2(&zs, 15 + 16) != Z_OK) return false;
    out.clear();
    zs.next_in = const_cast<Bytef *>(data);
    zs.avail_in = (uInt)n;
    uint8_t buf[1 << 16];
    int rc;
    do {
        zs.next_out = buf;
        zs.avail_out = sizeof(buf);
        rc = inflate(&zs, Z_NO_FLUSH);
        if (rc != Z_OK && rc != Z_STREAM_END) {
            inflateEnd(&zs);
            return false;
        }
        out.insert(out.end(), buf, buf + (sizeof(buf) - zs.avail_out));
    } while (rc != Z_STREAM_END);
    inflateEnd(&zs);
    return true;
}

// ---- block header: bincode fixed-int little-endian, 32 bytes (lib.rs:37-50) ------------
struct BlockHeader {
    uint32_t block_size, num_records, num_u64, encoded_size;
    uint64_t rice_param;
    uint8_t bitpacker_exponent, placeholder1;
    uint32_t placeholder2;
    uint16_t placeholder3;
};

void put_le(std::vector<uint8_t> &o, uint64_t v, int bytes) {
    for (int i = 0; i < bytes; i++) o.push_back((uint8_t)(v >> (8 * i)));
}
uint64_t get_le(const uint8_t *p, int bytes) {
    uint64_t v = 0;
    for (int i = 0; i < bytes; i++) v |= (uint64_t)p[i] << (8 * i);
    return v;
}
void write_header(std::vector<uint8_t> &o, const BlockHeader &h) {
    put_le(o, h.block_size, 4);
    put_le(o, h.num_records, 4);
    put_le(o, h.num_u64, 4);
    put_le(o, h.encoded_size, 4);
    put_le(o, h.rice_param, 8);
    put_le(o, h.bitpacker_exponent, 1);
    put_le(o, h.placeholder1, 1);
    put_le(o, h.placeholder2, 4);
    put_le(o, h.placeholder3, 2);
}
BlockHeader read_header(const uint8_t *p) {
    BlockHeader h;
    h.block_size = (uint32_t)get_le(p, 4);
    h.num_records = (uint32_t)get_le(p + 4, 4);
    h.num_u64 = (uint32_t)get_le(p + 8, 4);
    h.encoded_size = (uint32_t)get_le(p + 12, 4);
    h.rice_param = get_le(p + 16, 8);
    h.bitpacker_exponent = p[24];
    h.placeholder1 = p[25];
    h.placeholder2 = (uint32_t)get_le(p + 26, 4);
    h.placeholder3 = (uint16_t)get_le(p + 30, 2);
    return h;
}

uint64_t as_2bit(const uint8_t *codes, size_t n) {
    uint64_t v = 0;
    for (size_t j = 0; j < n; j++) v |= (uint64_t)codes[j] << (2 * j);
    return v;
}

// encode.rs:96-127
bool compress_block(const std::vector<uint64_t> &data, uint64_t num_records, bool rice, std::vector<uint8_t> &out) {
    std::vector<uint64_t> words;
    uint64_t param = 0;
    if (rice) {
        words = rice_encode(data, param);
    } else if (!minimal_binary_encode(data, words, param)) {
        return false;
    }
    // Words hold the bitstream MSB-first.  dsi-bitstream's BE BufBitWriter hands each word to
    // the word writer as to_be(), and encode.rs:107-109 then emits to_ne_bytes (little-endian
    // on x86): the bytes on disk are the MSB-first bitstream, i.e. each word big-endian
    // [ext dsi-bitstream 0.5.0, recalled; SURVEY.md A.4].  Parity unpinned vs the reference
    // (no reference-written encoded.dat exists offline).
    std::vector<uint8_t> bytes(words.size() * 8);
    for (size_t i = 0; i < words.size(); i++)
        for (int b = 0; b < 8; b++) bytes[i * 8 + b] = (uint8_t)(words[i] >> (8 * (7 - b)));
    std::vector<uint8_t> gz;
    if (!gzip_bytes(bytes.data(), bytes.size(), gz)) return false;
    BlockHeader h{};
    h.block_size = (uint32_t)gz.size();
    h.num_records = (uint32_t)num_records;
    h.num_u64 = (uint32_t)data.size();
    h.encoded_size = (uint32_t)words.size();
    h.rice_param = param;
    h.bitpacker_exponent = 8;
    out.clear();
    write_header(out, h);
    out.insert(out.end(), gz.begin(), gz.end());
    return true;
}

bool decompress_block(const uint8_t *payload, const BlockHeader &h, bool rice, std::vector<uint64_t> &out) {
    std::vector<uint8_t> bytes;
    if (!gunzip_bytes(payload, h.block_size, bytes)) return false;
    std::vector<uint64_t> words(bytes.size() / 8);
    for (size_t i = 0; i < words.size(); i++) {  // big-endian words (see compress_block)
        uint64_t w = 0;
        for (int b = 0; b < 8; b++) w = (w << 8) | bytes[8 * i + b];
        words[i] = w;
    }
    if (words.size() != h.encoded_size) return false;  // decode.rs:319-321
    return rice ? rice_decode(words, h.num_u64, h.rice_param, out)
                : minimal_binary_decode(words, h.num_u64, h.rice_param, out);
}

}  // namespace

extern "C" {

void ntc_file_header(uint8_t out[32]) { std::memset(out, 0, 32); }

int ntc_write_block(const uint64_t *recs, uint64_t n_recs, uint64_t num_records, uint8_t **out, uint64_t *out_len) {
    if (!out || !out_len || (n_recs && !recs)) return NTC_ERR_INVALID_ARG;
    *out = nullptr;
    *out_len = 0;
    if (n_recs == 0) return NTC_ERR_EMPTY_READ;  // split_encoded_dictionary EncodeError
    // split_encoded_dictionary (encode.rs:168-229)
    std::vector<uint64_t> d1, d2, d3;
    std::vector<uint8_t> tmp;
    d3.reserve(n_recs);
    for (uint64_t i = 0; i < n_recs; i++) {
        const uint64_t w = recs[i];
        const uint8_t flag = (uint8_t)(w >> 56);
        d3.push_back(flag);
        if ((flag & 2) == 0) {
            d1.push_back(w & 0xFFFFFFFFULL);
            d2.push_back((w >> 32) & 0xFFFFFFULL);
        } else {
            const uint32_t len = flag >> 2;
            for (uint32_t j = 0; j < len; j++) tmp.push_back((uint8_t)((w >> (2 * j)) & 3));
        }
    }
    std::vector<uint64_t> d4;
    for (size_t a = 0; a < tmp.size(); a += 31) d4.push_back(as_2bit(tmp.data() + a, std::min<size_t>(31, tmp.size() - a)));
    std::vector<uint8_t> b1, b2, b3, b4;
    // write_block_to (lib.rs:232-252): all four are built before anything is written; an
    // empty minimal-binary stream is an error and the whole block is dropped (B.3)
    if (!compress_block(d1, num_records, false, b1)) return NTC_ERR_EMPTY_READ;
    if (!compress_block(d2, num_records, true, b2)) return NTC_ERR_FORMAT;
    if (!compress_block(d3, num_records, true, b3)) return NTC_ERR_FORMAT;
    if (!compress_block(d4, num_records, false, b4)) return NTC_ERR_EMPTY_READ;
    const uint64_t total = b1.size() + b2.size() + b3.size() + b4.size();
    uint8_t *buf = (uint8_t *)std::malloc(total ? total : 1);
    if (!buf) return NTC_ERR_CAPACITY;
    uint64_t o = 0;
    for (auto *b : {&b1, &b2, &b3, &b4}) {
        std::memcpy(buf + o, b->data(), b->size());
        o += b->size();
    }
    *out = buf;
    *out_len = total;
    return NTC_OK;
}

int ntc_read_block(const uint8_t *data, uint64_t len, uint64_t *consumed, uint64_t **recs, uint64_t *n_recs,
                   uint64_t *num_records) {
    if (!data || !consumed || !recs || !n_recs) return NTC_ERR_INVALID_ARG;
    *recs = nullptr;
    *n_recs = 0;
    *consumed = 0;
    uint64_t pos = 0;
    std::vector<uint64_t> parts[4];
    BlockHeader hs[4];
    for (int s = 0; s < 4; s++) {
        if (pos + 32 > len) return s == 0 && pos == len ? NTC_ERR_IO : NTC_ERR_FORMAT;  // IO = clean EOF
        hs[s] = read_header(data + pos);
        pos += 32;
        if (pos + hs[s].block_size > len) return NTC_ERR_FORMAT;
        if (!decompress_block(data + pos, hs[s], s == 1 || s == 2, parts[s])) return NTC_ERR_FORMAT;
        pos += hs[s].block_size;
    }
    // zip_block_contents (decode.rs:102-149)
    const auto &c1 = parts[0], &c2 = parts[1], &fl = parts[2], &bn = parts[3];
    if (c1.size() != c2.size()) return NTC_ERR_FORMAT;
    uint64_t T = 0;
    for (uint64_t f : fl) T += (f & 0xFC) >> 2;
    std::vector<uint8_t> vals;
    vals.reserve(T);
    for (size_t i = 0; i < bn.size(); i++) {
        // decode.rs:114-118 uses T % 31 for the last chunk, which panics whenever T is a
        // positive multiple of 31 (Appendix B.4); ((T-1) % 31) + 1 agrees everywhere else
        uint64_t l = (i + 1 == bn.size()) ? ((T - 1) % 31) + 1 : 31;
        for (uint64_t j = 0; j < l; j++) vals.push_back((uint8_t)((bn[i] >> (2 * j)) & 3));
    }
    std::vector<uint64_t> out(fl.size());
    size_t i = 0, j = 0;
    for (size_t r = 0; r < fl.size(); r++) {
        const uint8_t flag = (uint8_t)fl[r];
        uint64_t w;
        if ((flag & 2) == 0) {
            if (i >= c1.size()) return NTC_ERR_FORMAT;
            w = (c1[i] & 0xFFFFFFFFULL) | ((c2[i] & 0xFFFFFFULL) << 32);
            i++;
        } else {
            const uint32_t l = flag >> 2;
            if (j + l > vals.size()) return NTC_ERR_FORMAT;
            w = as_2bit(vals.data() + j, l) & 0x00FFFFFFFFFFFFFFULL;
            j += l;
        }
        out[r] = w | ((uint64_t)flag << 56);
    }
    uint64_t *buf = (uint64_t *)std::malloc((out.size() ? out.size() : 1) * 8);
    if (!buf) return NTC_ERR_CAPACITY;
    std::memcpy(buf, out.data(), out.size() * 8);
    *recs = buf;
    *n_recs = out.size();
    *consumed = pos;
    if (num_records) *num_records = hs[0].num_records;
    return NTC_OK;
}

void ntc_buffer_free(void *p) { std::free(p); }

}  // extern "C"
