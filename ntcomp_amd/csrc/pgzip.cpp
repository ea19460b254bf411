// Parallel inflate of one (or several concatenated) non-BGZF gzip members: the reference's
// documented input, a plain `.fastq.gz` (README.md:30), is read by needletail through one
// flate2 stream (src/main.rs:158), and a single-member gzip cannot be split at member
// boundaries the way BGZF can (fastx.cpp DeflateReader).
//
// The compressed bytes are cut into chunks of kChunkBytes.  Per chunk, a worker finds the
// first deflate block that starts at or after the chunk's first bit (dynamic-Huffman headers
// are validated the way zlib's inflate_table validates them -- complete code-length code,
// no over-subscribed or (beyond one code of length 1) incomplete literal/length or distance
// code, an end-of-block code -- and stored headers by LEN == ~NLEN), then inflates from there
// to the first block boundary at or after the next chunk's first bit WITHOUT knowing the
// 32 KiB window before it: output symbols are 16 bits wide, and a match reaching back into
// the unknown window copies marker values 0x8000 + (window offset) instead of bytes.  A
// resolver then walks the chunks in order: a chunk whose start is exactly where the previous
// one ended is real (the first chunk starts at the member's first block), and its markers
// are replaced from the previous chunk's last 32 KiB; a chunk whose start was a false
// candidate, or whose search found nothing, is covered by a sequential "gap" inflate from the
// last true position with the window known.  Output = exactly the member's inflated bytes;
// the CRC-32 and ISIZE of every member's trailer are checked (zlib's gzread does the same),
// so a corrupt or truncated member is an error.  Bytes after the last member that are not a
// gzip header end the input (as gzread does).
//
// Workers run ahead of the consumer by a bounded number of chunks; the consumer's
// pgz_read converts the 16-bit symbols to bytes and computes the CRC in parallel slices.
#include <dlfcn.h>
#include <fcntl.h>
#include <emmintrin.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "ntc_internal.h"

namespace {

constexpr uint32_t kWin = 32768;           // deflate window
// compressed bytes per speculative chunk (NTC_PGZ_CHUNK overrides, for tests)
uint64_t chunk_bytes() {
    static const uint64_t c = [] {
        const char *e = std::getenv("NTC_PGZ_CHUNK");
        const long long v = e ? std::atoll(e) : 0;
        return v >= 64 ? (uint64_t)v : (uint64_t)(2u << 20);
    }();
    return c;
}
constexpr uint64_t kMaxChunkSymbols = 32u << 20;  // past it a chunk is left to the sequential path
constexpr uint16_t kMarker = 0x8000;        // 0x8000 + j: byte j of the unknown window

// ---- Huffman tables ----------------------------------------------------------------------
// entry: bits 0-3 bits consumed by this level, 4-7 kind, 8-15 extra bits (or subtable bits),
// 16-31 value (literal byte, length / distance base, subtable offset)
enum : uint32_t { kLit = 0, kLen = 1, kEob = 2, kSub = 3, kBad = 4 };
constexpr uint32_t kLitBits = 10, kDistBits = 8;

inline uint32_t ent(uint32_t nb, uint32_t kind, uint32_t extra, uint32_t val) {
    return nb | kind << 4 | extra << 8 | val << 16;
}

const uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                               31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
const uint16_t kDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

inline uint32_t rev_bits(uint32_t c, uint32_t n) {
    uint32_t r = 0;
    for (uint32_t i = 0; i < n; i++) r |= ((c >> i) & 1u) << (n - 1 - i);
    return r;
}

struct Table {
    std::vector<uint32_t> e;
    uint32_t bits = 0;
};

// canonical Huffman code from lengths, kind 0 literal/length, 1 distance, 2 code lengths
// (zlib inflate_table's checks): false when over-subscribed, or incomplete unless it is one
// code of length 1 (not for code lengths), or no code at all (distances only)
bool build_table(const uint8_t *len, uint32_t n, uint32_t tbits, int kind, Table &t) {
    uint32_t count[16] = {0};
    for (uint32_t s = 0; s < n; s++) count[len[s]]++;
    uint32_t maxl = 0;
    for (uint32_t l = 15; l >= 1; l--)
        if (count[l]) { maxl = l; break; }
    t.bits = tbits;
    if (maxl == 0) {  // no codes: every lookup is invalid (a block of literals only, for distances)
        if (kind != 1) return false;
        t.e.assign(1u << tbits, ent(1, kBad, 0, 0));
        return true;
    }
    int left = 1;
    for (uint32_t l = 1; l <= 15; l++) {
        left <<= 1;
        left -= (int)count[l];
        if (left < 0) return false;  // over-subscribed
    }
    if (left > 0 && (kind == 2 || maxl != 1)) return false;  // incomplete
    uint32_t next[16];
    next[1] = 0;
    for (uint32_t l = 1; l < 15; l++) next[l + 1] = (next[l] + count[l]) << 1;
    const uint32_t sub = maxl > tbits ? maxl - tbits : 0;
    t.e.assign(1u << tbits, ent(1, kBad, 0, 0));
    // subtables: one per tbits-prefix that has longer codes, 2^sub entries each
    std::vector<int32_t> subof(1u << tbits, -1);
    for (uint32_t s = 0; s < n; s++) {
        const uint32_t l = len[s];
        if (!l) continue;
        const uint32_t code = next[l]++;
        uint32_t v;
        if (kind == 0) {
            v = s < 256 ? ent(0, kLit, 0, s) : s == 256 ? ent(0, kEob, 0, 0)
                : s < 286 ? ent(0, kLen, kLenExtra[s - 257], kLenBase[s - 257]) : ent(0, kBad, 0, 0);
        } else if (kind == 1) {
            v = s < 30 ? ent(0, kLen, kDistExtra[s], kDistBase[s]) : ent(0, kBad, 0, 0);
        } else {
            v = ent(0, kLit, 0, s);
        }
        const uint32_t r = rev_bits(code, l);  // the stream sends codes MSB first; we read LSB first
        if (l <= tbits) {
            for (uint32_t x = r; x < (1u << tbits); x += 1u << l) t.e[x] = v | l;
        } else {
            const uint32_t pre = r & ((1u << tbits) - 1);
            if (subof[pre] < 0) {
                subof[pre] = (int32_t)t.e.size();
                t.e.resize(t.e.size() + (1u << sub), ent(1, kBad, 0, 0));
                t.e[pre] = ent(tbits, kSub, sub, (uint32_t)subof[pre]);
            }
            const uint32_t rl = l - tbits, hi = r >> tbits;
            for (uint32_t x = hi; x < (1u << sub); x += 1u << rl) t.e[(uint32_t)subof[pre] + x] = v | rl;
        }
    }
    return t.e.size() < (1u << 16);
}

// The fixed tables are never destroyed: a reader closed on a detached thread (pgz_close) may
// still have a worker inflating when the process runs its static destructors at exit.
const Table &fixed_lit() {
    static const Table *t = new Table([] {
        uint8_t l[288];
        for (int i = 0; i < 144; i++) l[i] = 8;
        for (int i = 144; i < 256; i++) l[i] = 9;
        for (int i = 256; i < 280; i++) l[i] = 7;
        for (int i = 280; i < 288; i++) l[i] = 8;
        Table x;
        build_table(l, 288, kLitBits, 0, x);
        return x;
    }());
    return *t;
}
const Table &fixed_dist() {
    static const Table *t = new Table([] {
        uint8_t l[32];  // 30 and 31 complete the code and decode as invalid
        for (int i = 0; i < 32; i++) l[i] = 5;
        Table x;
        build_table(l, 32, kDistBits, 1, x);
        return x;
    }());
    return *t;
}

// ---- bit input ---------------------------------------------------------------------------
struct Bits {
    const uint8_t *in;
    uint64_t n;       // bytes
    uint64_t ip = 0;  // next byte to load
    uint64_t buf = 0;
    uint32_t cnt = 0;
    uint64_t over = 0;  // zero bytes fed past the end
    Bits(const uint8_t *p, uint64_t size, uint64_t bit) : in(p), n(size) {
        ip = bit >> 3;
        refill();
        const uint32_t s = (uint32_t)(bit & 7);
        buf >>= s;
        cnt -= s;
    }
    inline void refill() {
        if (ip + 8 <= n) {
            uint64_t w;
            std::memcpy(&w, in + ip, 8);
            buf |= w << cnt;
            ip += (63 - cnt) >> 3;
            cnt |= 56;
        } else {
            while (cnt <= 55) {
                const uint64_t b = ip < n ? in[ip] : 0;
                if (ip >= n) over++;
                ip++;
                buf |= b << cnt;
                cnt += 8;
            }
        }
    }
    inline uint32_t peek(uint32_t k) const { return (uint32_t)(buf & ((1ull << k) - 1)); }
    inline void drop(uint32_t k) {
        buf >>= k;
        cnt -= k;
    }
    inline uint32_t get(uint32_t k) {
        const uint32_t v = peek(k);
        drop(k);
        return v;
    }
    uint64_t pos() const { return ip * 8 - cnt; }  // bit offset of the next unread bit
    bool overrun() const { return pos() > n * 8; }
};

// ---- one block header ------------------------------------------------------------------
// Reads the dynamic header after BFINAL/BTYPE into lit/dist tables; false when invalid.
bool read_dynamic(Bits &b, Table &lit, Table &dist) {
    b.refill();
    const uint32_t nlit = b.get(5) + 257, ndist = b.get(5) + 1, nclen = b.get(4) + 4;
    if (nlit > 286 || ndist > 30) return false;
    static const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    uint8_t cl[19] = {0};
    for (uint32_t i = 0; i < nclen; i++) {
        if (b.cnt < 3) b.refill();
        cl[order[i]] = (uint8_t)b.get(3);
    }
    Table ct;
    if (!build_table(cl, 19, 7, 2, ct)) return false;
    uint8_t lens[286 + 30];
    uint32_t i = 0;
    while (i < nlit + ndist) {
        b.refill();
        const uint32_t e = ct.e[b.peek(7)];
        if (((e >> 4) & 0xF) != kLit) return false;
        b.drop(e & 0xF);
        const uint32_t s = e >> 16;
        if (s < 16) {
            lens[i++] = (uint8_t)s;
        } else if (s == 16) {
            if (i == 0) return false;
            const uint32_t r = 3 + b.get(2);
            if (i + r > nlit + ndist) return false;
            const uint8_t p = lens[i - 1];
            for (uint32_t k = 0; k < r; k++) lens[i++] = p;
        } else {
            const uint32_t r = s == 17 ? 3 + b.get(3) : 11 + b.get(7);
            if (i + r > nlit + ndist) return false;
            for (uint32_t k = 0; k < r; k++) lens[i++] = 0;
        }
    }
    if (lens[256] == 0) return false;  // no end-of-block code
    if (!build_table(lens, nlit, kLitBits, 0, lit)) return false;
    if (!build_table(lens + nlit, ndist, kDistBits, 1, dist)) return false;
    return !b.overrun();
}

// ---- inflate ----------------------------------------------------------------------------
// kInfLimit: the output passed max_out (a true start in data that compresses better than
// the chunk budget assumes): not evidence of a false candidate, so speculation stops there
enum InfRc { kInfBoundary = 0, kInfFinal = 1, kInfError = -1, kInfLimit = -2 };

// 16-bit symbol output: p[0 .. kWin) is the window (markers or bytes), symbols follow; grown
// with realloc (no zero fill: a chunk's buffer is written once).  Every allocation holds
// kSlack symbols past cap: a match copies 8 symbols a step, so a 258-symbol match admitted at
// x + 262 <= cap may store up to x + 264.
//
// The buffers are anonymous mappings in 2 MiB units with transparent huge pages requested
// (NTC_PGZ_THP=0: malloc/realloc): a reader keeps ~T + 4 chunk buffers of ~26 MB, and with
// 4 KiB pages faulting them in and unmapping them at the end cost the pipeline tens of
// milliseconds.
constexpr size_t kSlack = 8;
bool thp_on() {
    static const bool on = [] {
        const char *e = std::getenv("NTC_PGZ_THP");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}
size_t map_bytes(size_t symbols) { return (((symbols + kSlack) * 2) + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1); }
void sym_free(uint16_t *p, size_t cap) {
    if (!p) return;
    if (thp_on()) munmap(p, map_bytes(cap));
    else std::free(p);
}
struct Out {
    uint16_t *p = nullptr;
    size_t n = 0, cap = 0;
    size_t min_ref = SIZE_MAX;  // lowest symbol index a match copied from (window reach check)
    Out() = default;
    Out(const Out &) = delete;
    Out &operator=(const Out &) = delete;
    ~Out() { sym_free(p, cap); }
    bool reserve(size_t c) {
        if (c <= cap) return true;
        if (!thp_on()) {
            void *q = std::realloc(p, (c + kSlack) * 2);
            if (!q) return false;
            p = (uint16_t *)q;
            cap = c;
            return true;
        }
        const size_t nb = map_bytes(c);
        void *q = p ? mremap(p, map_bytes(cap), nb, MREMAP_MAYMOVE)
                    : mmap(nullptr, nb, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (q == MAP_FAILED) return false;
        madvise(q, nb, MADV_HUGEPAGE);
        p = (uint16_t *)q;
        cap = nb / 2 - kSlack;
        return true;
    }
};

// Inflate blocks from bit `start` into o (symbols appended after o.n), stopping at the first
// block boundary at or after stop_bit (kInfBoundary), after the final block (kInfFinal), on
// invalid data (kInfError) or on an output past max_out symbols (kInfLimit).  Symbols below
// index lo are not part of the member (the window in front of a member's start): a distance
// reaching them is invalid, "invalid distance too far back" in zlib.  o.min_ref records the
// lowest index any match copied from, so that a speculative chunk (lo = 0, its window is
// markers) can be checked once the member's valid window is known.  *end = the bit reached.
int inflate_blocks(const uint8_t *in, uint64_t n, uint64_t start, uint64_t stop_bit, Out &o, uint64_t max_out,
                   uint64_t lo, uint64_t *end) {
    Bits b(in, n, start);
    Table dl, dd;
    if (!o.reserve(o.n + (1u << 20))) return kInfError;
    int rc = kInfError;
    for (;;) {
        if (b.pos() >= stop_bit) {
            rc = kInfBoundary;
            break;
        }
        b.refill();
        const uint32_t hdr = b.get(3);
        const uint32_t final = hdr & 1, type = hdr >> 1;
        const Table *lt, *dt;
        if (type == 0) {  // stored
            b.drop(b.cnt & 7);  // to the byte boundary
            b.refill();
            const uint32_t len = b.get(16), nlen = b.get(16);
            if ((len ^ 0xFFFF) != nlen) break;
            if (o.n + len > max_out) {
                rc = kInfLimit;
                break;
            }
            if (!o.reserve(o.n + len + 4096)) break;
            uint32_t left = len;
            while (left && b.cnt >= 8) {  // whole bytes still in the bit buffer
                o.p[o.n++] = (uint16_t)b.get(8);
                left--;
            }
            if (left) {  // the buffer is empty and byte-aligned: copy from the input
                const uint64_t q = b.pos() >> 3;
                if (q + left > n) break;
                for (uint32_t k = 0; k < left; k++) o.p[o.n++] = in[q + k];
                b = Bits(in, n, (q + left) * 8);
            }
            if (b.overrun()) break;
            if (final) {
                rc = kInfFinal;
                break;
            }
            continue;
        } else if (type == 1) {
            lt = &fixed_lit();
            dt = &fixed_dist();
        } else if (type == 2) {
            if (!read_dynamic(b, dl, dd)) break;
            lt = &dl;
            dt = &dd;
        } else {
            break;
        }
        // the symbol loop on local copies of the bit state and the output
        const uint32_t *L = lt->e.data(), *D = dt->e.data();
        uint64_t bb = b.buf, ip = b.ip;
        uint32_t bc = b.cnt;
        uint16_t *op = o.p;
        size_t x = o.n, cap = o.cap, mref = o.min_ref;
        bool ok = true, limit = false;
        for (;;) {
            if (bc < 48) {
                if (ip + 8 <= n) {
                    uint64_t w;
                    std::memcpy(&w, in + ip, 8);
                    bb |= w << bc;
                    ip += (63 - bc) >> 3;
                    bc |= 56;
                } else {
                    b.buf = bb; b.cnt = bc; b.ip = ip;
                    b.refill();
                    bb = b.buf; bc = b.cnt; ip = b.ip;
                    if (b.over > 16) {  // past the input's end (zeros fed in): truncated or garbage
                        ok = false;
                        break;
                    }
                }
            }
            if (x + 262 > cap) {  // room for one match (258) or literals
                o.n = x;
                if (x + 262 > max_out) {
                    ok = false;
                    limit = true;
                    break;
                }
                if (!o.reserve(std::min<size_t>(max_out, std::max<size_t>(2 * cap, x + 4096)))) {
                    ok = false;
                    break;
                }
                op = o.p;
                cap = o.cap;
            }
            uint32_t e = L[bb & ((1u << kLitBits) - 1)];
            if (((e >> 4) & 0xF) == kSub) {
                bb >>= kLitBits;
                bc -= kLitBits;
                e = L[(e >> 16) + (bb & ((1u << ((e >> 8) & 0xFF)) - 1))];
            }
            bb >>= e & 0xF;
            bc -= e & 0xF;
            const uint32_t kind = (e >> 4) & 0xF;
            if (kind == kLit) {
                op[x++] = (uint16_t)(e >> 16);
                // a second literal without a refill when the bits allow (>= 15 left)
                const uint32_t e2 = L[bb & ((1u << kLitBits) - 1)];
                if (((e2 >> 4) & 0xF) == kLit && bc >= 15) {
                    bb >>= e2 & 0xF;
                    bc -= e2 & 0xF;
                    op[x++] = (uint16_t)(e2 >> 16);
                }
                continue;
            }
            if (kind == kEob) break;
            if (kind != kLen) {
                ok = false;
                break;
            }
            const uint32_t le = (e >> 8) & 0xFF;
            const uint32_t len = (e >> 16) + (uint32_t)(bb & ((1u << le) - 1));
            bb >>= le;
            bc -= le;
            uint32_t f = D[bb & ((1u << kDistBits) - 1)];
            if (((f >> 4) & 0xF) == kSub) {
                bb >>= kDistBits;
                bc -= kDistBits;
                f = D[(f >> 16) + (bb & ((1u << ((f >> 8) & 0xFF)) - 1))];
            }
            bb >>= f & 0xF;
            bc -= f & 0xF;
            if (((f >> 4) & 0xF) != kLen) {
                ok = false;
                break;
            }
            const uint32_t de = (f >> 8) & 0xFF;
            const uint32_t dist = (f >> 16) + (uint32_t)(bb & ((1u << de) - 1));
            bb >>= de;
            bc -= de;
            if (dist > x - lo) {  // o holds the kWin window in front, valid from lo
                ok = false;
                break;
            }
            if (x - dist < mref) mref = x - dist;
            const uint16_t *src = op + x - dist;
            uint16_t *d = op + x;
            if (dist >= 8) {  // 8 symbols (16 bytes) a step; the buffer has 8 symbols of slack
                for (uint32_t k = 0; k < len; k += 8) std::memcpy(d + k, src + k, 16);
            } else if (dist == 1) {
                const uint16_t v = src[0];
                for (uint32_t k = 0; k < len; k++) d[k] = v;
            } else {
                for (uint32_t k = 0; k < len; k++) d[k] = src[k];
            }
            x += len;
        }
        b.buf = bb;
        b.cnt = bc;
        b.ip = ip;
        o.n = x;
        o.min_ref = mref;
        if (limit) {
            rc = kInfLimit;
            break;
        }
        if (!ok || b.overrun()) break;
        if (final) {
            rc = kInfFinal;
            break;
        }
    }
    *end = b.pos();
    return rc;
}

// candidate block start at bit p: a dynamic header that builds valid tables, or a stored
// header (LEN == ~NLEN, BFINAL 0)
bool plausible_block(const uint8_t *in, uint64_t n, uint64_t p) {
    if ((p >> 3) + 32 > n) return false;
    Bits b(in, n, p);
    const uint32_t hdr = b.peek(3);
    if (hdr & 1) return false;  // the final block: found by the chain, not searched for
    const uint32_t type = hdr >> 1;
    if (type == 2) {
        const uint64_t h = b.peek(17);
        if (((h >> 3) & 31) > 29 || ((h >> 8) & 31) > 29) return false;
        // the code-length code must be complete: checked from its 3-bit lengths before any
        // table is built (most candidates fail here)
        const uint32_t nclen = (uint32_t)((h >> 13) & 15) + 4;
        b.drop(17);
        uint32_t count[8] = {0};
        b.refill();
        for (uint32_t i = 0; i < nclen; i++) {
            if (b.cnt < 3) b.refill();
            count[b.get(3)]++;
        }
        int left = 1;
        for (uint32_t l = 1; l <= 7; l++) {
            left = (left << 1) - (int)count[l];
            if (left < 0) return false;
        }
        if (left != 0) return false;
        Bits c(in, n, p + 3);
        Table l, d;
        return read_dynamic(c, l, d);
    }
    if (type == 0) {
        b.drop(3);
        const uint32_t pad = b.cnt & 7;
        if (b.peek(pad)) return false;  // zlib pads with zero bits
        b.drop(pad);
        b.refill();
        const uint32_t len = b.get(16), nlen = b.get(16);
        return (len ^ 0xFFFF) == nlen && len > 0;
    }
    return false;
}

uint64_t find_block(const uint8_t *in, uint64_t n, uint64_t from, uint64_t to) {
    for (uint64_t p = from; p < to; p++) {
        // quick filter on the 3 header bits: BFINAL 0, BTYPE 10 or 00
        const uint32_t v = (in[p >> 3] | (uint32_t)((p >> 3) + 1 < n ? in[(p >> 3) + 1] : 0) << 8) >> (p & 7);
        const uint32_t h = v & 7;
        if (h != 4 && h != 0) continue;
        if (plausible_block(in, n, p)) return p;
    }
    return UINT64_MAX;
}

// gzip member header at byte h: the first deflate byte, or 0 when not a member header
uint64_t member_header(const uint8_t *in, uint64_t n, uint64_t h) {
    if (h + 18 > n || in[h] != 0x1F || in[h + 1] != 0x8B || in[h + 2] != 8) return 0;
    const uint8_t flg = in[h + 3];
    if (flg & 0xE0) return 0;
    uint64_t p = h + 10;
    if (flg & 4) {
        if (p + 2 > n) return 0;
        p += 2 + (in[p] | (uint32_t)in[p + 1] << 8);
    }
    for (int f = 8; f <= 16; f <<= 1)
        if (flg & f) {
            while (p < n && in[p]) p++;
            p++;
        }
    if (flg & 2) p += 2;
    return p < n ? p : 0;
}

using CrcFn = uint32_t (*)(uint32_t, const void *, size_t);
CrcFn crc_impl() {
    static CrcFn f = [] {
        void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        CrcFn g = h ? (CrcFn)dlsym(h, "libdeflate_crc32") : nullptr;
        if (!g) g = [](uint32_t c, const void *p, size_t len) -> uint32_t {
            while (len) {
                const uInt t = (uInt)std::min<size_t>(len, 1u << 30);
                c = (uint32_t)crc32(c, (const Bytef *)p, t);
                p = (const char *)p + t;
                len -= t;
            }
            return c;
        };
        return g;
    }();
    return f;
}

// ---- the reader -------------------------------------------------------------------------
struct Chunk {
    uint64_t b0 = 0, b1 = 0;    // bit range [b0, b1) of the compressed data
    uint64_t start = UINT64_MAX, end = 0;  // block found at start, inflated to end
    int rc = kInfError;         // kInfBoundary / kInfFinal, or kInfError (no usable start)
    Out out;                    // kWin window markers, then the symbols
    bool done = false;
};

// a run of output the consumer copies: chunk symbols (markers resolved with win) or bytes
struct Piece {
    std::shared_ptr<Chunk> ch;  // symbols ch->out[kWin + off ...]
    std::vector<uint8_t> bytes; // (gap) inflated with the window known
    std::vector<uint8_t> win;   // kWin bytes: marker j -> win[j]
    uint64_t off = 0, len = 0;  // consumed so far, total
    bool member_end = false;    // after this piece: the member's trailer
    uint32_t crc = 0, isize = 0;
};

}  // namespace

namespace ntc {

struct PgzReader {
    const uint8_t *in = nullptr;
    uint64_t n = 0;
    int fd = -1;
    unsigned T = 1;
    uint64_t nchunks = 0;
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::shared_ptr<Chunk>> ring;  // chunks next_res .. next_res + ring.size() - 1
    uint64_t next_claim = 0, next_res = 0;    // chunk indices
    bool stop = false;
    unsigned ahead = 0;
    // resolver state
    uint64_t first_bit = 0;        // the first member's first block
    uint64_t pos = 0;              // true bit position (a block boundary of the current member)
    std::vector<uint8_t> win;      // the last kWin bytes of the current member's output
    uint64_t win_valid = 0;        // bytes of win that belong to the member
    bool ended = false, failed = false, in_member = true;
    std::deque<Piece> pieces;
    uint32_t mcrc = 0;             // CRC of the member's bytes delivered so far
    uint64_t msize = 0;
    uint64_t max_out_per_chunk = 0;
    // chunk output buffers kept for reuse (fresh ones fault their pages in under the process's
    // memory-map lock, which serialised the workers)
    std::vector<std::pair<uint16_t *, size_t>> pool;
    std::unique_ptr<Gang> conv;  // pgz_read's conversion + CRC threads
    // Once every chunk is claimed no worker needs a buffer again: recycled buffers go to a
    // reaper thread that unmaps them while the last chunks are still read (~2 ms per 26 MB
    // buffer on the box, 28 buffers: 50 ms that otherwise fell on the close)
    std::vector<std::pair<uint16_t *, size_t>> grave;
    std::thread reaper;
    bool reaper_on = false;
    void recycle(Chunk &c) {
        if (!c.out.p) return;
        std::lock_guard<std::mutex> g(mu);
        if (next_claim >= nchunks && !stop) {
            grave.push_back({c.out.p, c.out.cap});
            if (!reaper_on) {
                reaper_on = true;
                reaper = std::thread([this] { reap(); });
            }
            cv.notify_all();
        } else {
            pool.push_back({c.out.p, c.out.cap});
        }
        c.out.p = nullptr;
        c.out.cap = c.out.n = 0;
    }
    void reap() {
        for (;;) {
            std::pair<uint16_t *, size_t> b;
            {
                std::unique_lock<std::mutex> g(mu);
                cv.wait(g, [&] { return stop || !grave.empty() || !pool.empty(); });
                if (!grave.empty()) {
                    b = grave.back();
                    grave.pop_back();
                } else if (!pool.empty()) {  // the spare buffers no worker will take again
                    b = pool.back();
                    pool.pop_back();
                } else {
                    return;  // stop, nothing left
                }
            }
            sym_free(b.first, b.second);
        }
    }
    uint64_t st_wait_ns = 0, st_conv_ns = 0;
    std::atomic<uint64_t> st_gap_bits{0}, st_chunks_ok{0}, st_false{0}, st_spec_ns{0}, st_find_ns{0};

    ~PgzReader() {
        if (std::getenv("NTC_PGZ_STATS"))
            std::fprintf(stderr, "pgz: %llu chunks, %llu accepted, %llu false starts, gap %.1f MB, spec %.3f s, find %.3f s, "
                                 "read: wait %.3f s, convert %.3f s\n",
                         (unsigned long long)nchunks, (unsigned long long)st_chunks_ok.load(),
                         (unsigned long long)st_false.load(), st_gap_bits.load() / 8e6, st_spec_ns.load() / 1e9,
                         st_find_ns.load() / 1e9, st_wait_ns / 1e9, st_conv_ns / 1e9);
        const auto c0 = std::chrono::steady_clock::now();
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto &t : th) t.join();
        if (reaper.joinable()) reaper.join();  // it frees what is left of grave and pool first
        for (auto &b : grave) sym_free(b.first, b.second);
        const auto c1 = std::chrono::steady_clock::now();
        for (auto &b : pool) sym_free(b.first, b.second);
        const auto c2 = std::chrono::steady_clock::now();
        if (in) munmap((void *)in, n);
        if (fd >= 0) close(fd);
        if (std::getenv("NTC_PGZ_STATS")) {
            const auto c3 = std::chrono::steady_clock::now();
            auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
                return std::chrono::duration<double, std::milli>(b - a).count();
            };
            std::fprintf(stderr, "pgz close: join %.2f ms, free %zu buffers %.2f ms, unmap %.2f ms\n", ms(c0, c1),
                         pool.size(), ms(c1, c2), ms(c2, c3));
        }
    }

    void worker() {
        for (;;) {
            std::shared_ptr<Chunk> c;
            {
                std::unique_lock<std::mutex> g(mu);
                cv.wait(g, [&] { return stop || (next_claim < nchunks && next_claim < next_res + ahead); });
                if (stop) return;
                c = std::make_shared<Chunk>();
                if (!pool.empty()) {
                    c->out.p = pool.back().first;
                    c->out.cap = pool.back().second;
                    pool.pop_back();
                }
                c->b0 = next_claim * chunk_bytes() * 8;
                c->b1 = std::min(n * 8, (next_claim + 1) * chunk_bytes() * 8);
                ring.push_back(c);
                next_claim++;
            }
            const auto t0 = std::chrono::steady_clock::now();
            speculate(*c);
            const uint64_t dt = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
            st_spec_ns += dt;
            if (std::getenv("NTC_PGZ_STATS")) std::fprintf(stderr, "chunk b0 %llu start %llu end %llu rc %d out %zu %.3f s\n", (unsigned long long)c->b0, (unsigned long long)c->start, (unsigned long long)c->end, c->rc, c->out.n, dt / 1e9);
            {
                std::lock_guard<std::mutex> g(mu);
                c->done = true;
            }
            cv.notify_all();
        }
    }
    void speculate(Chunk &c) {
        uint64_t from = c.b0 == 0 ? first_bit : c.b0;  // chunk 0: the first member's first block
        for (;;) {
            const auto t0 = std::chrono::steady_clock::now();
            const uint64_t p = c.b0 == 0 ? from : find_block(in, n, from, c.b1);
            st_find_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
            if (p == UINT64_MAX || p >= c.b1) return;
            if (!c.out.reserve(kWin + chunk_bytes() * 6)) return;  // ~ a FASTQ chunk's output
            for (uint32_t j = 0; j < kWin; j++) c.out.p[j] = (uint16_t)(kMarker + j);
            c.out.n = kWin;
            c.out.min_ref = SIZE_MAX;
            uint64_t end = 0;
            const int rc = inflate_blocks(in, n, p, c.b1, c.out, max_out_per_chunk, 0, &end);
            if (rc >= 0) {
                c.start = p;
                c.end = end;
                c.rc = rc;
                return;
            }
            c.out.n = 0;
            // past the output budget: a start this well compressed is likely true, and every
            // later candidate in the chunk would inflate as far again -- leave the chunk to the
            // resolver's sequential gap
            if (rc == kInfLimit) return;
            st_false++;
            if (c.b0 == 0) return;
            from = p + 1;
        }
    }

    // member trailer at the byte after bit pos; then the next member or the end
    void end_member(uint64_t bitpos) {
        const uint64_t t = (bitpos + 7) >> 3;
        Piece pc;
        pc.member_end = true;
        if (t + 8 > n) {
            failed = true;
            return;
        }
        pc.crc = in[t] | in[t + 1] << 8 | in[t + 2] << 16 | (uint32_t)in[t + 3] << 24;
        pc.isize = in[t + 4] | in[t + 5] << 8 | in[t + 6] << 16 | (uint32_t)in[t + 7] << 24;
        pieces.push_back(std::move(pc));
        const uint64_t h = member_header(in, n, t + 8);
        if (!h) {
            ended = true;  // no further member: trailing bytes are ignored (gzread)
            return;
        }
        pos = h * 8;
        win_valid = 0;
    }

    void push_window(const uint8_t *p, uint64_t len) {  // the member's output grew by p[0..len)
        if (len == 0) return;
        if (len >= kWin) {
            std::memcpy(win.data(), p + len - kWin, kWin);
        } else {
            std::memmove(win.data(), win.data() + len, kWin - len);
            std::memcpy(win.data() + kWin - len, p, len);
        }
        win_valid = std::min<uint64_t>(kWin, win_valid + len);
    }

    // inflate sequentially from pos (window known) to the first block boundary >= stop
    bool gap(uint64_t stop) {
        Out o;
        if (!o.reserve(kWin + (1u << 20))) {
            failed = true;
            return false;
        }
        for (uint32_t j = 0; j < kWin; j++) o.p[j] = win[j];
        o.n = kWin;
        uint64_t end = 0;
        const int rc = inflate_blocks(in, n, pos, stop, o, UINT64_MAX, kWin - win_valid, &end);
        st_gap_bits += end - pos;
        if (rc < 0) {
            failed = true;
            return false;
        }
        Piece pc;
        pc.bytes.resize(o.n - kWin);
        for (size_t i = 0; i < pc.bytes.size(); i++) pc.bytes[i] = (uint8_t)o.p[kWin + i];
        pc.len = pc.bytes.size();
        push_window(pc.bytes.data(), pc.len);
        pieces.push_back(std::move(pc));
        pos = end;
        if (rc == kInfFinal) end_member(end);
        return true;
    }

    // resolve chunks until at least `want` bytes are queued, or the end
    void resolve(uint64_t want) {
        auto queued = [&] {
            uint64_t q = 0;
            for (auto &p : pieces) q += p.len - p.off;
            return q;
        };
        while (!ended && !failed && queued() < want) {
            std::shared_ptr<Chunk> c;
            {
                std::unique_lock<std::mutex> g(mu);
                if (next_res >= nchunks) {
                    c = nullptr;
                } else {
                    cv.wait(g, [&] { return !ring.empty() && ring.front()->done; });
                    c = ring.front();
                    ring.pop_front();
                    next_res++;
                }
            }
            cv.notify_all();
            if (!c) {  // past the last chunk: the rest sequentially
                if (!gap(UINT64_MAX)) return;
                if (!ended && pos >= n * 8) failed = true;
                continue;
            }
            // a true boundary before this chunk's start: inflate the gap up to it (again after
            // a member that ends inside the gap)
            while (c->rc != kInfError && pos < c->start && !ended && !failed)
                if (!gap(c->start)) return;
            if (ended || failed) return;
            if (c->rc != kInfError && pos == c->start) {
                // the chunk's matches may only reach the member's own bytes in the window
                if (c->out.min_ref != SIZE_MAX && c->out.min_ref < kWin - win_valid) {
                    failed = true;
                    return;
                }
                Piece pc;
                pc.len = c->out.n - kWin;
                pc.win = win;  // markers resolve against the member's window before the chunk
                // the member's window after the chunk: its last kWin symbols, resolved
                const uint64_t tail = std::min<uint64_t>(pc.len, kWin);
                std::vector<uint8_t> tb(tail);
                const uint16_t *s = c->out.p + c->out.n - tail;
                for (uint64_t i = 0; i < tail; i++) tb[i] = s[i] >= kMarker ? win[s[i] - kMarker] : (uint8_t)s[i];
                pc.ch = c;
                st_chunks_ok++;
                pieces.push_back(std::move(pc));
                push_window(tb.data(), tail);
                pos = c->end;
                if (c->rc == kInfFinal) end_member(c->end);
            }
            // else: a false candidate, or no start found here -- covered by the next gap
            else recycle(*c);
        }
    }
};

PgzReader *pgz_open(const char *path, int threads) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return nullptr;
    struct stat sb;
    if (fstat(fd, &sb) != 0 || sb.st_size < 18) {
        close(fd);
        return nullptr;
    }
    void *m = mmap(nullptr, (size_t)sb.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) {
        close(fd);
        return nullptr;
    }
    madvise(m, (size_t)sb.st_size, MADV_SEQUENTIAL);
    auto *r = new PgzReader;
    r->in = (const uint8_t *)m;
    r->n = (uint64_t)sb.st_size;
    r->fd = fd;
    const uint64_t h = member_header(r->in, r->n, 0);
    if (!h) {
        delete r;
        return nullptr;
    }
    r->pos = r->first_bit = h * 8;
    r->win.assign(kWin, 0);
    r->T = (unsigned)std::max(1, threads);
    r->ahead = r->T + 4;
    r->nchunks = (r->n + chunk_bytes() - 1) / chunk_bytes();
    // NTC_PGZ_MAXOUT (symbols, for tests) lowers the per-chunk output budget
    const char *mo = std::getenv("NTC_PGZ_MAXOUT");
    const long long mov = mo ? std::atoll(mo) : 0;
    r->max_out_per_chunk = kWin + (mov >= 1024 ? (uint64_t)mov : kMaxChunkSymbols);
    for (unsigned t = 0; t < r->T; t++) r->th.emplace_back([r] { r->worker(); });
    return r;
}

// The reader's teardown (its workers joined, ~T + 4 chunk buffers of ~26 MB unmapped, the
// input unmapped) took 43-50 ms on the box, at the end of the encode pipeline's critical
// path; it runs on a detached thread instead (synchronously under the sanitizers, whose
// leak and thread checks run at exit).  NTC_PGZ_SYNC_CLOSE=1 restores the synchronous close.
void pgz_close(PgzReader *r) {
    if (!r) return;
#if defined(__SANITIZE_ADDRESS__) || defined(__SANITIZE_THREAD__)
    delete r;
#else
    static const bool sync = [] {
        const char *e = std::getenv("NTC_PGZ_SYNC_CLOSE");
        return e && std::atoi(e) != 0;
    }();
    if (sync) {
        delete r;
        return;
    }
    try {
        std::thread([r] { delete r; }).detach();
    } catch (...) {
        delete r;
    }
#endif
}

// cap bytes into dst (fewer only at the end): 1 filled, 0 the end was met, -1 error
int pgz_read(PgzReader *r, char *dst, size_t cap, size_t *got) {
    *got = 0;
    if (r->failed) return -1;
    const auto t0 = std::chrono::steady_clock::now();
    r->resolve(cap);
    const auto t1 = std::chrono::steady_clock::now();
    r->st_wait_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
    // the copy plan: pieces' ranges into dst, converted and CRC'd in parallel slices
    struct Seg {
        Piece *p;
        uint64_t off, len, at;
    };
    std::vector<Seg> segs;
    uint64_t filled = 0;
    size_t visited = 0;  // leading pieces taken into segs (member ends included)
    for (auto &p : r->pieces) {
        if (filled >= cap) break;
        visited++;
        if (p.member_end) {
            segs.push_back({&p, 0, 0, filled});
            continue;
        }
        const uint64_t t = std::min<uint64_t>(p.len - p.off, cap - filled);
        if (t) segs.push_back({&p, p.off, t, filled});
        filled += t;
    }
    // split big segments into slices of <= 4 MB for the threads
    struct Slice {
        size_t seg;
        uint64_t off, len, at;
        uint32_t crc;
    };
    std::vector<Slice> sl;
    for (size_t i = 0; i < segs.size(); i++)
        for (uint64_t o = 0; o < segs[i].len; o += 4u << 20)
            sl.push_back({i, segs[i].off + o, std::min<uint64_t>(4u << 20, segs[i].len - o), segs[i].at + o, 0});
    const CrcFn crcf = crc_impl();
    std::atomic<size_t> next{0};
    auto work = [&] {
        for (size_t i; (i = next.fetch_add(1)) < sl.size();) {
            Slice &s = sl[i];
            Piece &p = *segs[s.seg].p;
            uint8_t *d = (uint8_t *)dst + s.at;
            if (p.ch) {
                const uint16_t *src = p.ch->out.p + kWin + s.off;
                const uint8_t *w = p.win.data();
                uint64_t k = 0;
                // 16 symbols a step: no marker among them (the usual case once the chunk is
                // past its first window's reach) -> one pack; else one by one
                for (; k + 16 <= s.len; k += 16) {
                    const __m128i a = _mm_loadu_si128((const __m128i *)(src + k));
                    const __m128i c = _mm_loadu_si128((const __m128i *)(src + k + 8));
                    const __m128i hi = _mm_and_si128(_mm_or_si128(a, c), _mm_set1_epi16((short)0xFF00));
                    if (_mm_movemask_epi8(_mm_cmpeq_epi8(hi, _mm_setzero_si128())) == 0xFFFF) {
                        _mm_storeu_si128((__m128i *)(d + k), _mm_packus_epi16(a, c));
                    } else {
                        for (uint64_t q = k; q < k + 16; q++) {
                            const uint16_t v = src[q];
                            d[q] = v < 256 ? (uint8_t)v : w[(v - kMarker) & (kWin - 1)];
                        }
                    }
                }
                for (; k < s.len; k++) {
                    const uint16_t v = src[k];
                    d[k] = v < 256 ? (uint8_t)v : w[(v - kMarker) & (kWin - 1)];
                }
            } else {
                std::memcpy(d, p.bytes.data() + s.off, s.len);
            }
            s.crc = crcf(0, d, s.len);
        }
    };
    if (sl.size() > 1) {  // the reader's conversion gang (created at the first read that needs it)
        if (!r->conv) r->conv.reset(new Gang((int)r->T));
        r->conv->run([&](int) { work(); });
    } else {
        work();
    }
    r->st_conv_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t1).count();
    // CRC per member, in order; the pieces consumed
    size_t si = 0;
    for (size_t i = 0; i < segs.size(); i++) {
        Piece &p = *segs[i].p;
        if (p.member_end) {
            if (p.crc != r->mcrc || p.isize != (uint32_t)r->msize) {
                r->failed = true;
                return -1;
            }
            r->mcrc = 0;
            r->msize = 0;
            continue;
        }
        for (; si < sl.size() && sl[si].seg == i; si++) {
            r->mcrc = (uint32_t)crc32_combine(r->mcrc, sl[si].crc, (z_off_t)sl[si].len);
            r->msize += sl[si].len;
        }
        p.off += segs[i].len;
    }
    for (size_t i = 0; i < visited; i++) {
        const Piece &p = r->pieces.front();
        if (!p.member_end && p.off < p.len) break;
        if (p.ch && p.ch.use_count() == 1) r->recycle(*p.ch);
        r->pieces.pop_front();
    }
    *got = filled;
    if (r->failed) return -1;
    if (filled < cap) return r->pieces.empty() && r->ended ? 0 : (r->failed ? -1 : 0);
    return 1;
}

}  // namespace ntc
