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
// write_block_to = pack (everything before deflate: ntc_pack_block here, or the GPU packer
// ntc_pack_blocks_device in pack.hip) + deflate (ntc_deflate_block).  The packed streams
// are pinned by tests/golden/make_codec_golden.py, an independent restatement.
//
// Restated dsi-bitstream semantics (not in the container; recalled):
//   * BufBitWriter<BE, u64 words>: bits MSB-first into u64 words, last word zero-padded;
//     the writer hands words over as to_be(), encode.rs:107-109 emits to_ne_bytes
//     (little-endian): on disk each word is big-endian, i.e. the MSB-first bit stream.
//   * unary(n) = n zeros then a one; rice(n, b) = unary(n >> b) then the low b bits.
//   * rice::log2_b(p) = ceil(log2(ln(phi) / -ln(1-p))), saturating at 0 (Rust `as usize`).
//   * minimal_binary(v, max): l = floor(log2 max), limit = 2^(l+1) - max;
//     v < limit -> v in l bits, else v + limit in l+1 bits.
//   * gzip member like flate2's GzEncoder: 10-byte header (mtime 0, XFL 0, OS 255), raw
//     deflate at level 6, CRC32 + ISIZE trailer.  Deflate bytes come from system zlib (or
//     libdeflate), so they inflate identically but are not byte-identical to zlib-rs
//     (parity level F is unpinned).
#include <dlfcn.h>
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ntcomp_codec.h"
#include "ntc_internal.h"
#include "codec_params.h"

namespace {

// ---- bit writer / reader (big-endian bit order in u64 words) -------------------------
// Writes into a caller-sized word array (exact sizes come from a counting pass).
struct BitSink {
    uint64_t *w;
    uint64_t n = 0;    // complete words written
    uint64_t acc = 0;  // bits in progress, from the MSB
    int used = 0;      // 0..63
    explicit BitSink(uint64_t *words) : w(words) {}
    inline void put(uint64_t v, int nb) {  // v < 2^nb, nb <= 64
        if (nb <= 0) return;
        const int room = 64 - used;
        if (nb < room) {
            acc |= v << (room - nb);
            used += nb;
        } else {
            const int lo = nb - room;  // 0..63 bits spill into the next word
            w[n++] = acc | (lo ? v >> lo : v);
            acc = lo ? v << (64 - lo) : 0;
            used = lo;
        }
    }
    inline void zeros(uint64_t z) {  // z zero bits
        uint64_t t = (uint64_t)used + z;
        if (t >= 64) {
            w[n++] = acc;
            acc = 0;
            t -= 64;
            while (t >= 64) {
                w[n++] = 0;
                t -= 64;
            }
        }
        used = (int)t;
    }
    uint64_t finish() {
        if (used) {
            w[n++] = acc;
            acc = 0;
            used = 0;
        }
        return n;
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

bool rice_decode(const std::vector<uint64_t> &w, uint64_t n, uint64_t param, std::vector<uint64_t> &out) {
    if (param > 63) return false;
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
    const uint64_t limit = (l == 63 ? 0 : (2ULL << l)) - param;
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

// ---- deflate engines -------------------------------------------------------------------
bool zlib_deflate(const uint8_t *data, size_t n, std::vector<uint8_t> &out, size_t at) {
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (deflateInit2(&zs, 6, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
    const size_t bound = deflateBound(&zs, (uLong)n) + 16;
    out.resize(at + bound);
    zs.next_in = const_cast<Bytef *>(data);
    zs.avail_in = (uInt)n;
    zs.next_out = out.data() + at;
    zs.avail_out = (uInt)bound;
    const int rc = deflate(&zs, Z_FINISH);
    const size_t produced = bound - zs.avail_out;
    deflateEnd(&zs);
    if (rc != Z_STREAM_END) return false;
    out.resize(at + produced);
    return true;
}

// libdeflate.so.0 (dlopen; the image ships the runtime library without headers).  One
// compressor per thread: libdeflate compressors are not thread-safe.
struct LibDeflate {
    void *(*alloc_c)(int) = nullptr;
    void (*free_c)(void *) = nullptr;
    size_t (*deflate_c)(void *, const void *, size_t, void *, size_t) = nullptr;
    size_t (*bound_c)(void *, size_t) = nullptr;
    uint32_t (*crc32_c)(uint32_t, const void *, size_t) = nullptr;  // libdeflate_crc32 (optional)
    bool ok = false;
    LibDeflate() {
        void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc_c = (void *(*)(int))dlsym(h, "libdeflate_alloc_compressor");
        free_c = (void (*)(void *))dlsym(h, "libdeflate_free_compressor");
        deflate_c = (size_t(*)(void *, const void *, size_t, void *, size_t))dlsym(h, "libdeflate_deflate_compress");
        bound_c = (size_t(*)(void *, size_t))dlsym(h, "libdeflate_deflate_compress_bound");
        crc32_c = (uint32_t(*)(uint32_t, const void *, size_t))dlsym(h, "libdeflate_crc32");
        ok = alloc_c && free_c && deflate_c && bound_c;
    }
};
LibDeflate &libdeflate() {
    static LibDeflate L;
    return L;
}
struct ThreadCompressor {
    void *c = nullptr;
    ~ThreadCompressor() {
        if (c) libdeflate().free_c(c);
    }
};
thread_local ThreadCompressor tl_compressor;

bool libdeflate_deflate(const uint8_t *data, size_t n, std::vector<uint8_t> &out, size_t at) {
    LibDeflate &L = libdeflate();
    if (!L.ok) return false;
    if (!tl_compressor.c && !(tl_compressor.c = L.alloc_c(6))) return false;
    const size_t bound = L.bound_c(tl_compressor.c, n);
    out.resize(at + bound);
    const size_t got = L.deflate_c(tl_compressor.c, data, n, out.data() + at, bound);
    if (!got && n) return false;
    out.resize(at + got);
    return true;
}

// order-0 entropy of p[0, n) in bits per byte
double entropy0(const uint8_t *p, size_t n) {
    if (!n) return 0;
    uint32_t h[4][256] = {};
    size_t i = 0;
    for (; i + 4 <= n; i += 4) h[0][p[i]]++, h[1][p[i + 1]]++, h[2][p[i + 2]]++, h[3][p[i + 3]]++;
    for (; i < n; i++) h[0][p[i]]++;
    double e = 0;
    for (int c = 0; c < 256; c++) {
        const uint32_t k = h[0][c] + h[1][c] + h[2][c] + h[3][c];
        if (k) e -= (double)k * std::log2((double)k / (double)n);
    }
    return e / (double)n;
}

// raw deflate of stored blocks (BTYPE 00, at most 65,535 bytes each; one empty final block
// for n = 0), appended to out
void stored_deflate(const uint8_t *data, size_t n, std::vector<uint8_t> &out) {
    size_t i = 0;
    do {
        const size_t len = std::min<size_t>(n - i, 65535);
        const bool last = i + len == n;
        const uint8_t h[5] = {(uint8_t)(last ? 1 : 0), (uint8_t)len, (uint8_t)(len >> 8), (uint8_t)~len,
                              (uint8_t)(~len >> 8)};
        out.insert(out.end(), h, h + 5);
        out.insert(out.end(), data + i, data + i + len);
        i += len;
    } while (i < n);
}

constexpr size_t kEntropySample = 32u << 10;
constexpr double kStoreEntropy = 7.9;

// one gzip member (flate2 GzEncoder shape) appended to out
bool gzip_append(const uint8_t *data, size_t n, int engine, std::vector<uint8_t> &out) {
    static const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 0xff};
    const size_t start = out.size();
    out.insert(out.end(), hdr, hdr + 10);
    bool ok = true;
    if (engine == NTC_DEFLATE_ADAPTIVE && n >= 4096 && entropy0(data, std::min(n, kEntropySample)) >= kStoreEntropy)
        stored_deflate(data, n, out);
    else if (engine == NTC_DEFLATE_LIBDEFLATE || engine == NTC_DEFLATE_ADAPTIVE)
        ok = libdeflate_deflate(data, n, out, start + 10);
    else
        ok = zlib_deflate(data, n, out, start + 10);
    if (!ok) return false;
    LibDeflate &L = libdeflate();  // the same CRC-32 either way; libdeflate's is ~10x faster
    const uint32_t crc = L.ok && L.crc32_c ? L.crc32_c(0, data, n) : (uint32_t)crc32(0L, data, (uInt)n),
                   isize = (uint32_t)n;
    for (int i = 0; i < 4; i++) out.push_back((uint8_t)(crc >> (8 * i)));
    for (int i = 0; i < 4; i++) out.push_back((uint8_t)(isize >> (8 * i)));
    return true;
}

// libdeflate gzip inflate (one decompressor per thread) into a buffer of the expected size
struct LibInflate {
    void *(*alloc_d)() = nullptr;
    void (*free_d)(void *) = nullptr;
    int (*gz_d)(void *, const void *, size_t, void *, size_t, size_t *) = nullptr;
    bool ok = false;
    LibInflate() {
        void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc_d = (void *(*)())dlsym(h, "libdeflate_alloc_decompressor");
        free_d = (void (*)(void *))dlsym(h, "libdeflate_free_decompressor");
        gz_d = (int (*)(void *, const void *, size_t, void *, size_t, size_t *))dlsym(h, "libdeflate_gzip_decompress");
        ok = alloc_d && free_d && gz_d;
    }
};
LibInflate &libinflate() {
    static LibInflate L;
    return L;
}
struct ThreadDecompressor {
    void *d = nullptr;
    ~ThreadDecompressor() {
        if (d) libinflate().free_d(d);
    }
};
thread_local ThreadDecompressor tl_decompressor;

// exactly `want` bytes out of one gzip member, or false (libdeflate when present, else zlib)
bool gunzip_exact(const uint8_t *data, size_t n, size_t want, std::vector<uint8_t> &out);

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

inline uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

bool gunzip_exact(const uint8_t *data, size_t n, size_t want, std::vector<uint8_t> &out) {
    LibInflate &L = libinflate();
    if (L.ok && (tl_decompressor.d || (tl_decompressor.d = L.alloc_d()))) {
        out.resize(want);
        size_t got = 0;
        // libdeflate needs the whole member; a longer (corrupt) one fails with short output
        if (L.gz_d(tl_decompressor.d, data, n, out.data(), want, &got) == 0) return got == want;
        return false;
    }
    if (!gunzip_bytes(data, n, out)) return false;
    return out.size() == want;
}

bool decompress_block(const uint8_t *payload, const BlockHeader &h, bool rice, std::vector<uint64_t> &out) {
    std::vector<uint8_t> bytes;
    if (!gunzip_exact(payload, h.block_size, (size_t)h.encoded_size * 8, bytes)) return false;
    std::vector<uint64_t> words(bytes.size() / 8);
    for (size_t i = 0; i < words.size(); i++) {  // big-endian words (see pack_block)
        uint64_t w;
        std::memcpy(&w, bytes.data() + 8 * i, 8);
        words[i] = bswap64(w);
    }
    if (words.size() != h.encoded_size) return false;  // decode.rs:90-92
    return rice ? rice_decode(words, h.num_u64, h.rice_param, out)
                : minimal_binary_decode(words, h.num_u64, h.rice_param, out);
}

// Rice code length of v with parameter p
inline uint64_t rice_bits(uint64_t v, int p) { return (v >> p) + 1 + (uint64_t)p; }

}  // namespace

extern "C" {

void ntc_file_header(uint8_t out[32]) { std::memset(out, 0, 32); }

// split_encoded_dictionary (encode.rs:168-229) + rice / minimal binary coding
// (encode.rs:59-94), words written as compress_block hands them to deflate.
int ntc_pack_block(const uint64_t *recs, uint64_t n_recs, uint64_t num_records, ntc_block_meta *meta,
                   uint8_t **payload, uint64_t *payload_len) {
    if (!meta || !payload || !payload_len || (n_recs && !recs)) return NTC_ERR_INVALID_ARG;
    *payload = nullptr;
    *payload_len = 0;
    std::memset(meta, 0, sizeof(*meta));
    meta->num_records = num_records;
    meta->n_recs = n_recs;
    if (n_recs == 0) return meta->status = NTC_ERR_EMPTY_READ;  // split_encoded_dictionary EncodeError
    // pass 1: stream totals
    uint64_t n_long = 0, max1 = 0, sum2 = 0, sum3 = 0, T = 0;
    for (uint64_t i = 0; i < n_recs; i++) {
        const uint64_t w = recs[i], flag = w >> 56;
        sum3 += flag;
        if ((flag & 2) == 0) {
            n_long++;
            const uint64_t c = w & 0xFFFFFFFFULL;
            max1 = c > max1 ? c : max1;
            sum2 += (w >> 32) & 0xFFFFFFULL;
        } else {
            T += flag >> 2;
        }
    }
    // s4 chunk values: the short bases in 31-base as_2bit chunks.  A short record's bases
    // are bits 0-55 (encode.rs:216-221: from_2bit of bytes 0..7); from_2bit panics past 32
    // bases, so a longer length is a malformed block here.
    std::vector<uint64_t> s4((T + 30) / 31);
    uint64_t max4 = 0;
    {
        uint64_t chunk = 0, nchunk = 0;
        int have = 0;  // bases in chunk
        for (uint64_t i = 0; i < n_recs; i++) {
            const uint64_t w = recs[i], flag = w >> 56;
            if ((flag & 2) == 0) continue;
            int len = (int)(flag >> 2);
            if (len > 32) return meta->status = NTC_ERR_FORMAT;
            uint64_t bits = w & 0x00FFFFFFFFFFFFFFULL;
            if (len < 28) bits &= (1ULL << (2 * len)) - 1;
            while (len) {
                const int take = len < 31 - have ? len : 31 - have;  // <= 31
                chunk |= (bits & ((1ULL << (2 * take)) - 1)) << (2 * have);
                bits >>= 2 * take;
                have += take;
                len -= take;
                if (have == 31) {
                    s4[nchunk++] = chunk;
                    max4 = chunk > max4 ? chunk : max4;
                    chunk = 0;
                    have = 0;
                }
            }
        }
        if (have) {
            s4[nchunk++] = chunk;
            max4 = chunk > max4 ? chunk : max4;
        }
    }
    // write_block_to computes all four before writing: an empty minimal-binary stream errs
    // and the block is dropped (lib.rs:242-250, App. B.3)
    if (n_long == 0 || T == 0) return meta->status = NTC_ERR_EMPTY_READ;
    const int p2 = ntc_rice_log2_b(n_long, sum2), p3 = ntc_rice_log2_b(n_recs, sum3);
    const uint64_t m1 = max1 + 2, m4 = max4 + 2;
    const int l1 = ilog2(m1), l4 = ilog2(m4);
    const uint64_t lim1 = (2ULL << l1) - m1, lim4 = (l4 == 63 ? 0 : (2ULL << l4)) - m4;
    // pass 2: exact code lengths
    uint64_t b1 = 0, b2 = 0, b3 = 0, b4 = 0;
    for (uint64_t i = 0; i < n_recs; i++) {
        const uint64_t w = recs[i], flag = w >> 56;
        b3 += rice_bits(flag, p3);
        if ((flag & 2) == 0) {
            b1 += (uint64_t)l1 + ((w & 0xFFFFFFFFULL) + 1 >= lim1);
            b2 += rice_bits((w >> 32) & 0xFFFFFFULL, p2);
        }
    }
    for (uint64_t v : s4) b4 += (uint64_t)l4 + (v + 1 >= lim4);
    const uint64_t wn[4] = {(b1 + 63) / 64, (b2 + 63) / 64, (b3 + 63) / 64, (b4 + 63) / 64};
    const uint64_t total_words = wn[0] + wn[1] + wn[2] + wn[3];
    uint64_t *words = (uint64_t *)std::malloc(total_words * 8 + 8);
    if (!words) return NTC_ERR_CAPACITY;
    uint64_t off = 0;
    const uint64_t params[4] = {m1, (uint64_t)p2, (uint64_t)p3, m4};
    const uint64_t counts[4] = {n_long, n_long, n_recs, (uint64_t)s4.size()};
    for (int s = 0; s < 4; s++) {
        meta->stream[s].num_u64 = counts[s];
        meta->stream[s].encoded_size = wn[s];
        meta->stream[s].param = params[s];
        meta->stream[s].offset = off * 8;
        off += wn[s];
    }
    // pass 3: codes
    BitSink o1(words), o2(words + wn[0]), o3(words + wn[0] + wn[1]), o4(words + wn[0] + wn[1] + wn[2]);
    const uint64_t mask2 = (1ULL << p2) - 1, mask3 = (1ULL << p3) - 1;
    for (uint64_t i = 0; i < n_recs; i++) {
        const uint64_t w = recs[i], flag = w >> 56;
        o3.zeros(flag >> p3);
        o3.put(((uint64_t)1 << p3) | (flag & mask3), p3 + 1);
        if ((flag & 2) == 0) {
            const uint64_t v = (w & 0xFFFFFFFFULL) + 1;
            if (v < lim1) o1.put(v, l1);
            else o1.put(v + lim1, l1 + 1);
            const uint64_t len = (w >> 32) & 0xFFFFFFULL;
            o2.zeros(len >> p2);
            o2.put(((uint64_t)1 << p2) | (len & mask2), p2 + 1);
        }
    }
    for (uint64_t c : s4) {
        const uint64_t v = c + 1;
        if (v < lim4) o4.put(v, l4);
        else o4.put(v + lim4, l4 + 1);  // v + lim4 < 2^(l4+1) <= 2^63: fits
    }
    const uint64_t got[4] = {o1.finish(), o2.finish(), o3.finish(), o4.finish()};
    for (int s = 0; s < 4; s++)
        if (got[s] != wn[s]) {
            std::free(words);
            return NTC_ERR_FORMAT;  // internal size mismatch (never expected)
        }
    for (uint64_t i = 0; i < total_words; i++) words[i] = bswap64(words[i]);  // on-disk byte order
    *payload = (uint8_t *)words;
    *payload_len = total_words * 8;
    return meta->status = NTC_OK;
}

// compress_block's header + deflate_bytes for each stream (encode.rs:96-127)
}  // extern "C"

namespace {
// stream s of a block: its 32-byte header (write_block_to's fields) + gzip member, appended
int deflate_stream_into(const ntc_block_meta *meta, int s, const uint8_t *payload, int engine,
                        std::vector<uint8_t> &buf) {
    const ntc_stream_meta &m = meta->stream[s];
    const size_t hpos = buf.size();
    buf.resize(hpos + 32);
    if (!gzip_append(payload + m.offset, m.encoded_size * 8, engine, buf)) return NTC_ERR_FORMAT;
    BlockHeader h{};
    h.block_size = (uint32_t)(buf.size() - hpos - 32);
    h.num_records = (uint32_t)meta->num_records;
    h.num_u64 = (uint32_t)m.num_u64;
    h.encoded_size = (uint32_t)m.encoded_size;
    h.rice_param = m.param;
    h.bitpacker_exponent = 8;
    std::vector<uint8_t> hb;
    write_header(hb, h);
    std::memcpy(buf.data() + hpos, hb.data(), 32);
    return NTC_OK;
}

int deflate_checks(const ntc_block_meta *meta, const uint8_t *payload, int engine, uint8_t **out, uint64_t *out_len) {
    if (!meta || !out || !out_len) return NTC_ERR_INVALID_ARG;
    *out = nullptr;
    *out_len = 0;
    if (meta->status != NTC_OK) return meta->status;
    if (!payload) return NTC_ERR_INVALID_ARG;
    if (engine != NTC_DEFLATE_ZLIB && engine != NTC_DEFLATE_LIBDEFLATE && engine != NTC_DEFLATE_ADAPTIVE)
        return NTC_ERR_INVALID_ARG;
    if (engine != NTC_DEFLATE_ZLIB && !libdeflate().ok) return NTC_ERR_UNSUPPORTED;
    return NTC_OK;
}

int hand_out(const std::vector<uint8_t> &buf, uint8_t **out, uint64_t *out_len) {
    uint8_t *o = (uint8_t *)std::malloc(buf.size() ? buf.size() : 1);
    if (!o) return NTC_ERR_CAPACITY;
    std::memcpy(o, buf.data(), buf.size());
    *out = o;
    *out_len = buf.size();
    return NTC_OK;
}
}  // namespace

extern "C" {

int ntc_deflate_block(const ntc_block_meta *meta, const uint8_t *payload, int engine, uint8_t **out,
                      uint64_t *out_len) {
    int rc = deflate_checks(meta, payload, engine, out, out_len);
    if (rc) return rc;
    std::vector<uint8_t> buf;
    uint64_t est = 0;
    for (int s = 0; s < 4; s++) est += meta->stream[s].encoded_size * 8 + 64;
    buf.reserve(est + est / 16);
    for (int s = 0; s < 4; s++)
        if ((rc = deflate_stream_into(meta, s, payload, engine, buf))) return rc;
    return hand_out(buf, out, out_len);
}

int ntc_deflate_stream(const ntc_block_meta *meta, int stream, const uint8_t *payload, int engine, uint8_t **out,
                       uint64_t *out_len) {
    if (stream < 0 || stream > 3) return NTC_ERR_INVALID_ARG;
    int rc = deflate_checks(meta, payload, engine, out, out_len);
    if (rc) return rc;
    std::vector<uint8_t> buf;
    buf.reserve(meta->stream[stream].encoded_size * 8 + meta->stream[stream].encoded_size / 2 + 128);
    if ((rc = deflate_stream_into(meta, stream, payload, engine, buf))) return rc;
    return hand_out(buf, out, out_len);
}

int ntc_write_block(const uint64_t *recs, uint64_t n_recs, uint64_t num_records, uint8_t **out, uint64_t *out_len) {
    if (!out || !out_len || (n_recs && !recs)) return NTC_ERR_INVALID_ARG;
    *out = nullptr;
    *out_len = 0;
    ntc_block_meta meta;
    uint8_t *payload = nullptr;
    uint64_t plen = 0;
    int rc = ntc_pack_block(recs, n_recs, num_records, &meta, &payload, &plen);
    if (rc == NTC_OK) rc = ntc_deflate_block(&meta, payload, NTC_DEFLATE_ZLIB, out, out_len);
    std::free(payload);
    return rc;
}

}  // extern "C"

namespace {
// zip_block_contents (decode.rs:102-149): the four decoded streams -> u64 records, into vec
// (resized) or out (cap records; NTC_ERR_CAPACITY if more).  *n_recs = the block's records.
int zip_parts(const std::vector<uint64_t> (&parts)[4], std::vector<uint64_t> *vec, uint64_t *out, uint64_t cap,
              uint64_t *n_recs) {
    const auto &c1 = parts[0], &c2 = parts[1], &fl = parts[2], &bn = parts[3];
    if (c1.size() != c2.size()) return NTC_ERR_FORMAT;
    uint64_t T = 0;
    for (uint64_t f : fl) T += (f & 0xFC) >> 2;
    // short-record bases: chunk i holds 31 bases, the last one the rest.  decode.rs:114-118
    // uses T % 31 for the last chunk, which panics whenever T is a positive multiple of 31
    // (Appendix B.4); ((T-1) % 31) + 1 agrees everywhere else
    if (T ? bn.size() != (T + 30) / 31 : false) return NTC_ERR_FORMAT;
    *n_recs = fl.size();
    if (vec) {
        vec->resize(fl.size());
        out = vec->data();
    } else if (fl.size() > cap) {
        return NTC_ERR_CAPACITY;
    }
    size_t i = 0;
    uint64_t j = 0;  // next short base
    for (size_t r = 0; r < fl.size(); r++) {
        const uint8_t flag = (uint8_t)fl[r];
        uint64_t w;
        if ((flag & 2) == 0) {
            if (i >= c1.size()) return NTC_ERR_FORMAT;
            w = (c1[i] & 0xFFFFFFFFULL) | ((c2[i] & 0xFFFFFFULL) << 32);
            i++;
        } else {
            const uint32_t l = flag >> 2;
            if (j + l > T) return NTC_ERR_FORMAT;
            // bases j .. j + l - 1 of the concatenation: from chunk j / 31 (and the next)
            w = 0;
            for (uint32_t t = 0; t < l; t++) {
                const uint64_t q = j + t;
                w |= ((bn[q / 31] >> (2 * (q % 31))) & 3ULL) << (2 * t);
            }
            w &= 0x00FFFFFFFFFFFFFFULL;
            j += l;
        }
        out[r] = w | ((uint64_t)flag << 56);
    }
    return NTC_OK;
}

// decode_block's container half (lib.rs:320-363): the block's four streams, decompressed and
// zipped back into u64 records (zip_block_contents, decode.rs:102-149), into vec (resized)
// or out (cap records; NTC_ERR_CAPACITY if more).  *n_recs = the block's record count.
int read_block_impl(const uint8_t *data, uint64_t len, uint64_t *consumed, std::vector<uint64_t> *vec, uint64_t *out,
                    uint64_t cap, uint64_t *n_recs, uint64_t *num_records) {
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
    const int rc = zip_parts(parts, vec, out, cap, n_recs);
    if (rc == NTC_OK || rc == NTC_ERR_CAPACITY) {
        *consumed = pos;
        if (num_records) *num_records = hs[0].num_records;
    }
    return rc;
}
}  // namespace

namespace ntc {
// The GPU unpacker's work on the host (the sanitizer builds' stand-in for the device): one
// block's inflated streams (payload at meta's offsets) -> records; NTC_ERR_FORMAT if damaged.
int unpack_block_host(const ntc_block_meta &m, const uint8_t *payload, std::vector<uint64_t> &recs) {
    std::vector<uint64_t> parts[4];
    for (int s = 0; s < 4; s++) {
        const ntc_stream_meta &st = m.stream[s];
        std::vector<uint64_t> words(st.encoded_size);
        for (uint64_t i = 0; i < st.encoded_size; i++) {
            uint64_t w;
            std::memcpy(&w, payload + st.offset + 8 * i, 8);
            words[i] = bswap64(w);
        }
        const bool ok = (s == 1 || s == 2) ? rice_decode(words, st.num_u64, st.param, parts[s])
                                           : minimal_binary_decode(words, st.num_u64, st.param, parts[s]);
        if (!ok) return NTC_ERR_FORMAT;
    }
    uint64_t n = 0;
    return zip_parts(parts, &recs, nullptr, 0, &n);
}
}  // namespace ntc

extern "C" {

int ntc_read_block(const uint8_t *data, uint64_t len, uint64_t *consumed, uint64_t **recs, uint64_t *n_recs,
                   uint64_t *num_records) {
    if (!data || !consumed || !recs || !n_recs) return NTC_ERR_INVALID_ARG;
    *recs = nullptr;
    std::vector<uint64_t> v;
    uint64_t used = 0;
    const int rc = read_block_impl(data, len, &used, &v, nullptr, 0, n_recs, num_records);
    if (rc) {
        *n_recs = 0;
        *consumed = 0;
        return rc;
    }
    uint64_t *buf = (uint64_t *)std::malloc((v.size() ? v.size() : 1) * 8);
    if (!buf) return NTC_ERR_CAPACITY;
    std::memcpy(buf, v.data(), v.size() * 8);
    *recs = buf;
    *consumed = used;
    return NTC_OK;
}

int ntc_read_block_streams(const uint8_t *data, uint64_t len, uint64_t *consumed, uint8_t *payload,
                           uint64_t capacity, ntc_block_meta *meta) {
    if (!data || !consumed || !meta || (capacity && !payload)) return NTC_ERR_INVALID_ARG;
    *consumed = 0;
    std::memset(meta, 0, sizeof(*meta));
    uint64_t pos = 0, off = 0;
    BlockHeader hs[4];
    for (int s = 0; s < 4; s++) {
        if (pos + 32 > len) return s == 0 && pos == len ? NTC_ERR_IO : NTC_ERR_FORMAT;  // IO = clean EOF
        hs[s] = read_header(data + pos);
        pos += 32;
        if (pos + hs[s].block_size > len) return NTC_ERR_FORMAT;
        const uint64_t want = (uint64_t)hs[s].encoded_size * 8;
        if (off + want > capacity) return NTC_ERR_CAPACITY;
        // libdeflate straight into the payload; zlib through a vector
        LibInflate &L = libinflate();
        bool ok = false;
        if (L.ok && (tl_decompressor.d || (tl_decompressor.d = L.alloc_d()))) {
            size_t got = 0;
            ok = L.gz_d(tl_decompressor.d, data + pos, hs[s].block_size, payload + off, want, &got) == 0 && got == want;
        } else {
            std::vector<uint8_t> v;
            ok = gunzip_bytes(data + pos, hs[s].block_size, v) && v.size() == want;
            if (ok && want) std::memcpy(payload + off, v.data(), want);
        }
        if (!ok) return NTC_ERR_FORMAT;
        meta->stream[s].num_u64 = hs[s].num_u64;
        meta->stream[s].encoded_size = hs[s].encoded_size;
        meta->stream[s].param = hs[s].rice_param;
        meta->stream[s].offset = off;
        off += want;
        pos += hs[s].block_size;
    }
    meta->num_records = hs[0].num_records;
    meta->n_recs = hs[2].num_u64;
    *consumed = pos;
    return NTC_OK;
}

int ntc_read_block_into(const uint8_t *data, uint64_t len, uint64_t *consumed, uint64_t *recs, uint64_t capacity,
                        uint64_t *n_recs, uint64_t *num_records) {
    if (!data || !consumed || !n_recs || (capacity && !recs)) return NTC_ERR_INVALID_ARG;
    return read_block_impl(data, len, consumed, nullptr, recs, capacity, n_recs, num_records);
}

void ntc_buffer_free(void *p) { std::free(p); }

}  // extern "C"
