// GPU block unpacker: decode_block (src/lib.rs:320-368) after inflate -- the inverse of
// pack.hip.  The host inflates each block's four gzip'd streams into one buffer (the
// big-endian words compress_block wrote, src/encode.rs:107-109); everything after that runs
// here, and the records never exist in host memory:
//
//   rice_decode / minimal_binary_decode   src/decode.rs:51-99   [ext dsi-bitstream 0.5.0]
//   zip_block_contents                    src/decode.rs:102-149 (short-record bases from the
//                                         31-base 2-bit chunks of s4, App. B.4's ((T-1) % 31) + 1)
//
// A code stream is a chain of variable-length codes (Rice: unary quotient + p bits; minimal
// binary: l or l + 1 bits), so its code boundaries are found in parallel, segment by segment,
// with every stream cut into tiles (a workgroup each) so a call's streams fill the GPU:
// Rice streams (s2, s3; k_rice_*) synchronise the way a self-synchronising prefix code does:
//   every segment is decoded from its first bit as if a code started there, its starts
//   marked in a bitmap; each chain then goes on past its segment's end until it meets a
//   start a later segment's chain marked (nearly always the next one's, within a few codes),
//   from where both agree.  Segment 0's chain is the true one (the stream starts with a
//   code), so the true chain is: segment 0's chain, its codes past the end up to the meeting
//   point, the met segment's marked starts from there, and so on -- true codes per segment
//   (a popcount + the codes up to the meeting point), a scan, a decode into place.  A chain
//   that meets none within 8 segments makes one lane decode the stream.
// Minimal-binary streams (s1, s4; k_mb_*) are l- or (l + 1)-bit codes, nearly all of one
//   length, and such chains need not ever meet: there every segment's transfer is computed
//   for each of the l + 1 offsets a code can start at, and the true entries follow from
//   composed tile transfers.
//
// k_zip_count + k_zip_write (a workgroup per 4,096 records of a block) zip the four value
// streams back into u64 records with two block scans (long records -> s1/s2 index, short
// records -> base offset; each segment starts from the counts of the ones before it), check
// what read_block_impl checks (stream sizes, flags past the streams), and sums the reads
// (first flags) and bases the FASTA writer needs.
//
// Work: Rice bits are decoded ~2x (speculative + final, the continuations are short),
// minimal-binary bits l + 2 times; the payload (~1 B per record at C91) is L2-resident.
#include <hip/hip_runtime.h>

#include "../../include/ntcomp_gpu.h"
#include "kernels.h"

namespace ntc {

namespace {

constexpr int kZipThreads = 256;   // threads per block in the zip
constexpr int kZipPer = 4;         // records per thread per zip tile

__device__ __forceinline__ uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

// The 64 stream bits from bit position pos (MSB first), zero past the stream's end.  The
// cursor keeps the two words under the last position: a thread's positions only grow, so a
// code costs a load only when it crosses into the next word.
// A workgroup's words may be staged in LDS (sw: words w0 .. w0 + nl - 1, byte-swapped);
// positions outside that window read global memory.
struct Bits64 {
    const uint64_t *w;
    uint64_t nwords;
    uint64_t wi = ~0ull - 1, hi = 0, lo = 0;  // (not ~0: ~0 + 1 would look like "the next word" of word 0)
    const uint64_t *sw = nullptr;
    uint64_t w0 = 0, nl = 0;
    __device__ __forceinline__ uint64_t load(uint64_t i) const {
        if (i - w0 < nl) return sw[i - w0];
        return i < nwords ? bswap64(w[i]) : 0;
    }
    __device__ __forceinline__ uint64_t peek(uint64_t pos) {
        const uint64_t i = pos >> 6;
        if (i != wi) {
            if (i == wi + 1) {
                hi = lo;
                lo = load(i + 1);
            } else {
                hi = load(i);
                lo = load(i + 1);
            }
            wi = i;
        }
        const uint32_t sh = (uint32_t)(pos & 63);
        return sh ? (hi << sh) | (lo >> (64 - sh)) : hi;
    }
};

// The workgroup's words staged in LDS (sw: words w0 .. w0 + nl - 1, byte-swapped), positions
// outside the window read global memory; no cursor: a peek is two LDS loads issued together
// and no branch on the lane's position history (the lanes of a wave decode different codes).
struct WinBits {
    const uint64_t *w;
    uint64_t nwords;
    const uint64_t *sw;
    uint64_t w0, nl;
    __device__ __forceinline__ uint64_t peek(uint64_t pos) const {
        const uint64_t i = pos >> 6, rel = i - w0;
        uint64_t hi, lo;
        if (rel + 1 < nl) {
            hi = sw[rel];
            lo = sw[rel + 1];
        } else {
            hi = i < nwords ? bswap64(w[i]) : 0;
            lo = i + 1 < nwords ? bswap64(w[i + 1]) : 0;
        }
        const uint32_t sh = (uint32_t)(pos & 63);
        return sh ? (hi << sh) | (lo >> (64 - sh)) : hi;
    }
};

struct Code {
    uint64_t len;  // bits (0: no code here -- it runs past the end of the stream)
    uint64_t val;  // the value the reference's decoder returns (minimal binary: v - 1)
    bool bad;      // minimal binary v == 0 (decode.rs's check)
};

// Rice (param p): zeros up to a one, then p bits
template <class Bits>
__device__ __forceinline__ Code rice_at(Bits &bt, uint64_t pos, uint32_t p) {
    const uint64_t nbits = bt.nwords * 64;
    uint64_t q = 0, at = pos;
    if (pos < nbits) {  // the usual code: unary part, stop bit and p bits within one peek
        const uint64_t x = bt.peek(pos);
        const uint32_t z = x ? (uint32_t)__builtin_clzll(x) : 64u;
        if (z + 1 + p <= 64 && pos + z + 1 + p <= nbits) {
            const uint64_t rest = z + 1 < 64 ? x << (z + 1) : 0;
            return {z + 1 + p, ((uint64_t)z << p) | (p ? rest >> (64 - p) : 0), false};
        }
    }
    for (;;) {
        if (at >= nbits) return {0, 0, false};
        const uint64_t x = bt.peek(at);
        if (x) {
            const uint32_t z = (uint32_t)__builtin_clzll(x);
            if (at + z >= nbits) return {0, 0, false};
            q += z;
            at += z + 1;
            break;
        }
        q += 64;
        at += 64;
    }
    uint64_t r = 0;
    if (p) {
        if (at + p > nbits) return {0, 0, false};
        r = bt.peek(at) >> (64 - p);
        at += p;
    }
    return {at - pos, (q << p) | r, false};
}

// minimal binary (max = param): l = floor(log2 param), limit = 2^(l+1) - param
template <class Bits>
__device__ __forceinline__ Code mb_at(Bits &bt, uint64_t pos, uint32_t l, uint64_t limit) {
    const uint64_t nbits = bt.nwords * 64;
    if (pos + l > nbits) return {0, 0, false};
    const uint64_t x = bt.peek(pos);
    uint64_t v = l ? x >> (64 - l) : 0;
    uint64_t len = l;
    if (v >= limit) {
        if (pos + l + 1 > nbits) return {0, 0, false};
        v = (x >> (63 - l)) - limit;
        len = l + 1;
    }
    return {len, v ? v - 1 : 0, v == 0};
}


// the workgroup's window of a stream's words into LDS (zero past the stream's end)
__device__ __forceinline__ void stage_words(uint64_t *sw, const uint64_t *w, uint64_t nwords, uint64_t w0, uint32_t n) {
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) sw[i] = w0 + i < nwords ? bswap64(w[w0 + i]) : 0;
    __syncthreads();
}

__device__ __forceinline__ bool marked(const uint64_t *m, uint64_t pos) { return (m[pos >> 6] >> (pos & 63)) & 1u; }

// marks in [a, b) of the bitmap
__device__ uint64_t count_marks(const uint64_t *m, uint64_t a, uint64_t b) {
    uint64_t c = 0;
    while (a < b) {
        const uint64_t i = a >> 6;
        const uint32_t s = (uint32_t)(a & 63);
        const uint64_t e = ((i + 1) << 6) < b ? ((i + 1) << 6) : b;
        uint64_t x = m[i] >> s;
        const uint32_t nb = (uint32_t)(e - a);
        if (nb < 64) x &= (1ull << nb) - 1;
        c += (uint64_t)__popcll(x);
        a = e;
    }
    return c;
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
    for (int d = 32; d; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

// exclusive block scan (kThreads threads), through sh (>= threads / 64 words)
template <int kThreads>
__device__ __forceinline__ uint64_t block_exscan(uint64_t v, uint64_t *tot, uint64_t *sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t t = __shfl_up(inc, d, 64);
        if (lane >= d) inc += t;
    }
    if (lane == 63) sh[wid] = inc;
    __syncthreads();
    uint64_t base = 0, all = 0;
    for (int k = 0; k < kThreads / 64; k++) {
        const uint64_t x = sh[k];
        base += k < wid ? x : 0;
        all += x;
    }
    __syncthreads();
    *tot = all;
    return base + inc - v;
}

// ---- Rice streams (s2, s3) ------------------------------------------------------------------
// Segments of kRiceSegBits bits (whole bitmap words), a wave per tile of kRiceTileSegs
// segments, so a call's streams spread over the whole GPU.  Per segment (g = the call's
// segment index; the arrays below are indexed by it):
//   k_rice_a      the speculative chain from the segment's first bit: its code starts marked
//                 in the bitmap, END = its first start past the segment (kDeadPos: it ran past
//                 the stream's end);
//   k_rice_b      on from END until a start some later segment's chain marked: NEXT = that
//                 segment, Y = the meeting point, PRE = the codes before it.  Nearly always
//                 the next segment, within a few codes; otherwise the stream's flags get
//                 kNotSimple (its true chain is followed by k_rice_walk), and a chain that met
//                 none within 8 segments gets kSerial (one lane decodes the stream);
//   k_rice_walk   a wave per stream: the serial decode, or the true chain's segments and the
//                 points it joins them at (ENTRY, kNoEntry for the segments it runs through);
//                 a simple stream's segment g is joined at Y[g - 1];
//   k_rice_count  true codes per segment (marks from its entry to its end + PRE), per tile;
//   k_rice_scan   a wave per stream: the tiles' first value indices, the stream's status;
//   k_rice_decode each segment's true codes into place.
#ifndef NTC_RICE_SEG_BITS
#define NTC_RICE_SEG_BITS 512
#endif
constexpr int kRiceSegBits = NTC_RICE_SEG_BITS;  // a multiple of 64
constexpr int kRiceTileSegs = 64;
constexpr uint64_t kDeadPos = ~0ull, kNoEntry = ~0ull;
constexpr uint32_t kNoNext = 0xFFFFFFFFu;
constexpr uint32_t kNotSimple = 1, kSerial = 2, kBadParam = 4;
constexpr uint32_t kRiceWin = kRiceTileSegs * kRiceSegBits / 64 + 16;  // LDS words: the tile + 1024 bits

struct RiceWs {
    uint64_t *Y, *E, *END;
    uint32_t *NEXT, *PRE, *CNT;
    uint64_t *TSUM, *TOFF;
    uint32_t *flags;
};
__host__ __device__ inline RiceWs rice_ws(void *base, uint64_t n_tiles, uint64_t n_streams) {
    const uint64_t ns = n_tiles * kRiceTileSegs;
    RiceWs w;
    uint64_t *q = (uint64_t *)base;
    w.Y = q;
    w.E = q + ns;
    w.END = q + 2 * ns;
    w.TSUM = q + 3 * ns;
    w.TOFF = w.TSUM + n_tiles;
    uint32_t *r = (uint32_t *)(w.TOFF + n_tiles);
    w.NEXT = r;
    w.PRE = r + ns;
    w.CNT = r + 2 * ns;
    w.flags = r + 3 * ns;
    (void)n_streams;
    return w;
}
static uint64_t rice_ws_bytes(uint64_t n_tiles, uint64_t n_streams) {
    return n_tiles * kRiceTileSegs * 36 + n_tiles * 16 + n_streams * 4 + 64;
}

struct RiceSeg {
    UnpackStream s;
    uint64_t seg, a, b, g, nbits;
    uint32_t r;
    bool active;
};
__device__ __forceinline__ RiceSeg rice_seg(const UnpackStream *st, const UnpTile *tiles) {
    const UnpTile tl = tiles[blockIdx.x];
    RiceSeg x;
    x.s = st[tl.si];
    x.r = tl.stream;
    x.nbits = x.s.nwords * 64;
    x.seg = (uint64_t)tl.tile * kRiceTileSegs + threadIdx.x;
    x.a = x.seg * kRiceSegBits;
    x.b = x.a + kRiceSegBits < x.nbits ? x.a + kRiceSegBits : x.nbits;
    x.g = (uint64_t)blockIdx.x * kRiceTileSegs + threadIdx.x;
    x.active = x.a < x.nbits;
    return x;
}

__global__ __launch_bounds__(kRiceTileSegs) void k_rice_a(const uint64_t *payload, const UnpackStream *st,
                                                         const UnpTile *tiles, uint64_t *marks, RiceWs w) {
    const RiceSeg x = rice_seg(st, tiles);
    __shared__ uint64_t sw[kRiceWin];
    const uint64_t w0 = (uint64_t)tiles[blockIdx.x].tile * kRiceTileSegs * kRiceSegBits / 64;
    stage_words(sw, payload + x.s.word_off, x.s.nwords, w0, kRiceWin);
    if (!x.active) return;
    uint64_t *m = marks + x.s.word_off;
    WinBits bt{payload + x.s.word_off, x.s.nwords, sw, w0, kRiceWin};
    const uint32_t p = (uint32_t)x.s.param;
    uint64_t pos = x.a, word = 0, wi = x.a >> 6;
    bool dead = false;
    while (pos < x.b) {
        const Code c = rice_at(bt, pos, p);
        if (!c.len) {
            dead = true;
            break;
        }
        while ((pos >> 6) != wi) {  // (a code may skip whole words: they hold no start)
            m[wi] = word;
            wi++;
            word = 0;
        }
        word |= 1ull << (pos & 63);
        pos += c.len;
    }
    for (; wi < (x.b + 63) >> 6; wi++) {
        m[wi] = word;
        word = 0;
    }
    w.END[x.g] = dead ? kDeadPos : pos;
}

__global__ __launch_bounds__(kRiceTileSegs) void k_rice_b(const uint64_t *payload, const UnpackStream *st,
                                                         const UnpTile *tiles, const uint64_t *marks, RiceWs w) {
    const RiceSeg x = rice_seg(st, tiles);
    __shared__ uint64_t sw[kRiceWin];
    const uint64_t w0 = (uint64_t)tiles[blockIdx.x].tile * kRiceTileSegs * kRiceSegBits / 64;
    stage_words(sw, payload + x.s.word_off, x.s.nwords, w0, kRiceWin);
    if (!x.active) return;
    const uint64_t *m = marks + x.s.word_off;
    const uint64_t e = w.END[x.g];
    uint64_t q = e, pre = 0;
    uint32_t nx = kNoNext, fl = 0;
    if (e == kDeadPos) {
        q = x.nbits;
        if (x.b < x.nbits) fl |= kNotSimple;  // the stream's codes end inside it
    } else {
        WinBits bt{payload + x.s.word_off, x.s.nwords, sw, w0, kRiceWin};
        const uint32_t p = (uint32_t)x.s.param;
        const uint64_t lim = x.b + 8ull * kRiceSegBits;
        while (q < x.nbits) {
            if (marked(m, q)) {
                nx = (uint32_t)(q / kRiceSegBits);
                break;
            }
            if (q >= lim) {
                fl |= kSerial;
                break;
            }
            const Code c = rice_at(bt, q, p);
            if (!c.len) break;
            q += c.len;
            pre++;
        }
        if (x.b < x.nbits && nx != (uint32_t)(x.seg + 1)) fl |= kNotSimple;
    }
    w.NEXT[x.g] = nx;
    w.Y[x.g] = q;
    w.PRE[x.g] = (uint32_t)pre;
    if (fl) atomicOr(&w.flags[x.r], fl);
}

__global__ __launch_bounds__(64) void k_rice_walk(const uint64_t *payload, const UnpackStream *st,
                                                 const UnpStreamRef *rs, uint64_t *vals, int32_t *status, RiceWs w) {
    const UnpStreamRef ref = rs[blockIdx.x];
    const UnpackStream s = st[ref.si];
    const int t = threadIdx.x;
    if (s.param > 63) {
        if (t == 0) {
            status[ref.si] = NTC_ERR_FORMAT;
            w.flags[blockIdx.x] = kBadParam;
        }
        return;
    }
    if (s.n == 0 || ref.n_tiles == 0) {
        if (t == 0) status[ref.si] = s.n == 0 ? 0 : NTC_ERR_FORMAT;
        return;
    }
    const uint32_t fl = w.flags[blockIdx.x];
    if (fl & kSerial) {  // one lane decodes the whole stream
        if (t == 0) {
            Bits64 bt{payload + s.word_off, s.nwords};
            uint64_t p = 0;
            int err = 0;
            for (uint64_t i = 0; i < s.n; i++) {
                const Code c = rice_at(bt, p, (uint32_t)s.param);
                if (!c.len) {
                    err = NTC_ERR_FORMAT;
                    break;
                }
                vals[s.val_off + i] = c.val;
                p += c.len;
            }
            status[ref.si] = err;
        }
        return;
    }
    if (!(fl & kNotSimple)) return;
    const uint64_t g0 = (uint64_t)ref.first_tile * kRiceTileSegs, ns = (uint64_t)ref.n_tiles * kRiceTileSegs;
    for (uint64_t i = t; i < ns; i += 64) w.E[g0 + i] = kNoEntry;
    // the chain's segments in increasing order (NEXT > the segment): their NEXT / Y staged in
    // LDS a chunk at a time, lane 0 following the chain through each chunk
    constexpr uint32_t kChunk = 512;
    __shared__ uint32_t s_nx[kChunk];
    __shared__ uint64_t s_y[kChunk];
    __shared__ uint64_t s_v, s_yy;
    __shared__ int s_end;
    if (t == 0) {
        s_v = 0;
        s_yy = 0;
        s_end = 0;
    }
    __syncthreads();
    for (uint64_t c0 = 0; c0 < ns; c0 += kChunk) {
        if (s_end) break;  // (uniform: read after a barrier)
        const uint64_t nc = ns - c0 < kChunk ? ns - c0 : kChunk;
        if (s_v >= c0 + nc) continue;  // the chain skips this chunk
        for (uint32_t i = t; i < nc; i += 64) {
            s_nx[i] = w.NEXT[g0 + c0 + i];
            s_y[i] = w.Y[g0 + c0 + i];
        }
        __syncthreads();
        if (t == 0) {
            uint64_t v = s_v, y = s_yy;
            while (v < c0 + nc) {
                w.E[g0 + v] = y;
                const uint32_t nx = s_nx[v - c0];
                if (nx == kNoNext) {
                    s_end = 1;
                    break;
                }
                y = s_y[v - c0];
                v = nx;
            }
            s_v = v;
            s_yy = y;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(kRiceTileSegs) void k_rice_count(const UnpackStream *st, const UnpTile *tiles,
                                                             const uint64_t *marks, RiceWs w) {
    const RiceSeg x = rice_seg(st, tiles);
    const uint32_t fl = w.flags[x.r];
    if (fl & (kSerial | kBadParam)) return;
    uint64_t y = kNoEntry;
    if (x.active) y = (fl & kNotSimple) ? w.E[x.g] : (x.seg == 0 ? 0 : w.Y[x.g - 1]);
    const bool on = x.active && y != kNoEntry;
    const uint64_t cnt = on ? (y < x.b ? count_marks(marks + x.s.word_off, y, x.b) : 0) + w.PRE[x.g] : 0;
    if (x.active) {
        w.CNT[x.g] = (uint32_t)cnt;
        w.E[x.g] = on ? y : kNoEntry;
    }
    const uint64_t tot = wave_sum(cnt);
    if (threadIdx.x == 0) w.TSUM[blockIdx.x] = tot;
}

__global__ __launch_bounds__(64) void k_rice_scan(const UnpackStream *st, const UnpStreamRef *rs, int32_t *status,
                                                 RiceWs w) {
    const UnpStreamRef ref = rs[blockIdx.x];
    const UnpackStream s = st[ref.si];
    if (s.n == 0 || ref.n_tiles == 0 || (w.flags[blockIdx.x] & (kSerial | kBadParam))) return;
    const int lane = threadIdx.x;
    uint64_t base = 0;
    for (uint32_t k0 = 0; k0 < ref.n_tiles; k0 += 64) {
        const uint32_t k = k0 + lane;
        const uint64_t v = k < ref.n_tiles ? w.TSUM[ref.first_tile + k] : 0;
        uint64_t inc = v;
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t u = __shfl_up(inc, d, 64);
            if (lane >= d) inc += u;
        }
        if (k < ref.n_tiles) w.TOFF[ref.first_tile + k] = base + inc - v;
        base += __shfl(inc, 63, 64);
    }
    if (lane == 0) status[ref.si] = base < s.n ? NTC_ERR_FORMAT : 0;  // fewer codes than values
}

__global__ __launch_bounds__(kRiceTileSegs) void k_rice_decode(const uint64_t *payload, const UnpackStream *st,
                                                              const UnpTile *tiles, uint64_t *vals, int32_t *status,
                                                              RiceWs w) {
    const RiceSeg x = rice_seg(st, tiles);
    if (w.flags[x.r] & (kSerial | kBadParam)) return;
    __shared__ uint64_t sw[kRiceWin];
    const uint64_t w0 = (uint64_t)tiles[blockIdx.x].tile * kRiceTileSegs * kRiceSegBits / 64;
    stage_words(sw, payload + x.s.word_off, x.s.nwords, w0, kRiceWin);
    const uint64_t cnt = x.active ? w.CNT[x.g] : 0;
    const int lane = threadIdx.x;
    uint64_t inc = cnt;
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t u = __shfl_up(inc, d, 64);
        if (lane >= d) inc += u;
    }
    const uint64_t off = w.TOFF[blockIdx.x] + inc - cnt;
    int err = 0;
    if (cnt && off < x.s.n) {
        WinBits bt{payload + x.s.word_off, x.s.nwords, sw, w0, kRiceWin};
        uint64_t p = w.E[x.g];
        for (uint64_t j = 0; j < cnt && off + j < x.s.n; j++) {
            const Code c = rice_at(bt, p, (uint32_t)x.s.param);
            if (!c.len) {
                err = NTC_ERR_FORMAT;
                break;
            }
            vals[x.s.val_off + off + j] = c.val;
            p += c.len;
        }
    }
    if (err) atomicOr(&status[tiles[blockIdx.x].si], err);
}

// Minimal-binary streams (s1, s4).  Their codes are l or l + 1 bits, mostly one of the two,
// and chains started at different offsets rarely meet (fixed-length codes never do), so a
// segment's codes are found through its transfer: for each of the L = l + 1 offsets e a code
// can start at past the segment's first bit, where that chain leaves the segment (the first
// code start past it, at most l bits on) and how many codes it holds.  Transfers compose, so
// the true entries come from a two-level walk:
//   k_mb_tab     a thread per (entry, segment) pair computes that transfer (segments of
//                kMbSegBits bits); lane e of a tile (kMbTileSegs segments) follows entry e
//                through the tile's segments in LDS -> the tile's own transfer;
//   k_mb_walk    a wave per stream follows the true entry from tile to tile (bit 0 enters
//                tile 0 at offset 0) -> each tile's entry and its codes' first value index;
//   k_mb_decode  a tile follows its entry through its segments in LDS, scans the segments'
//                code counts and decodes each segment's true codes into place.
// The work is L transfers of every bit, spread over all CUs (a tile per workgroup).
#ifndef NTC_MB_SEG_BITS
#define NTC_MB_SEG_BITS 256
#endif
constexpr int kMbSegBits = NTC_MB_SEG_BITS;  // bits per segment (>= 64 > l + 1; a multiple of 64)
constexpr int kMbTileSegs = 256;  // segments per tile (threads of k_mb_decode)
constexpr int kMbTabThreads = 1024;  // k_mb_tab: a thread per (entry, segment) pair
constexpr uint8_t kMbDead = 255;  // a chain that ran past the stream's end
constexpr int kMbWalkTiles = 128; // tiles per LDS chunk of k_mb_walk
constexpr uint32_t kMbWin = kMbTileSegs * kMbSegBits / 64 + 2;  // LDS words: the tile + the last code

struct MbParams {
    uint32_t l, L;
    uint64_t limit, nbits;
};
__device__ __forceinline__ MbParams mb_params(const UnpackStream &s) {
    MbParams q;
    q.l = 63u - (uint32_t)__builtin_clzll(s.param);
    q.L = q.l + 1;
    q.limit = (q.l == 63 ? 0ull : (2ull << q.l)) - s.param;
    q.nbits = s.nwords * 64;
    return q;
}

// transfer tables: X[(tile * 64 + e) * kMbTileSegs + seg] exit offsets, C[...] code counts
// (entry-major, so a tile's lanes store and load consecutive bytes); TX / TC the tiles' own
__global__ __launch_bounds__(kMbTabThreads) void k_mb_tab(const uint64_t *payload, const UnpackStream *st,
                                                         const UnpTile *tiles, uint8_t *X, uint16_t *C, uint8_t *TX,
                                                         uint32_t *TC) {
    const UnpTile tl = tiles[blockIdx.x];
    const UnpackStream s = st[tl.si];
    const MbParams q = mb_params(s);
    const int t = threadIdx.x;
    __shared__ uint8_t sX[64 * kMbTileSegs];
    __shared__ uint16_t sC[64 * kMbTileSegs];
    __shared__ uint64_t sw[kMbWin];
    const uint64_t seg0 = (uint64_t)tl.tile * kMbTileSegs;
    const uint64_t w0 = seg0 * kMbSegBits / 64;
    stage_words(sw, payload + s.word_off, s.nwords, w0, kMbWin);
    const uint64_t tbase = (uint64_t)blockIdx.x * 64 * kMbTileSegs;
    // a thread per (entry, segment) pair, consecutive threads on consecutive segments of one
    // entry (so the stores below are consecutive bytes): each chain covers one segment
    for (uint32_t idx = (uint32_t)t; idx < q.L * kMbTileSegs; idx += kMbTabThreads) {
        const uint32_t e = idx / kMbTileSegs, u = idx % kMbTileSegs;
        const uint64_t a = (seg0 + u) * kMbSegBits;
        if (a >= q.nbits) continue;
        const uint64_t b = a + kMbSegBits < q.nbits ? a + kMbSegBits : q.nbits;
        WinBits bt{payload + s.word_off, s.nwords, sw, w0, kMbWin};
        uint64_t pos = a + e;
        uint32_t cnt = 0;
        bool dead = false;
        while (pos < b) {
            const Code c = mb_at(bt, pos, q.l, q.limit);
            if (!c.len) {
                dead = true;
                break;
            }
            pos += c.len;
            cnt++;
        }
        const uint8_t x = dead ? kMbDead : (uint8_t)(pos - b);
        sX[idx] = x;
        sC[idx] = (uint16_t)cnt;
        X[tbase + idx] = x;
        C[tbase + idx] = (uint16_t)cnt;
    }
    __syncthreads();
    if ((uint32_t)t < q.L) {
        const uint64_t segs = (q.nbits + kMbSegBits - 1) / kMbSegBits;
        const uint32_t ns = (uint32_t)(segs - seg0 < kMbTileSegs ? segs - seg0 : kMbTileSegs);
        uint32_t ex = (uint32_t)t, cnt = 0;
        for (uint32_t u = 0; u < ns && ex != kMbDead; u++) {
            cnt += sC[ex * kMbTileSegs + u];
            ex = sX[ex * kMbTileSegs + u];
        }
        TX[(uint64_t)blockIdx.x * 64 + t] = (uint8_t)ex;
        TC[(uint64_t)blockIdx.x * 64 + t] = cnt;
    }
}

// a wave per minimal-binary stream: tile entries TE and first value indices TP; the stream's
// status (param 0 decodes no value; fewer codes than values)
__global__ __launch_bounds__(64) void k_mb_walk(const UnpackStream *st, const UnpStreamRef *mbs, const uint8_t *TX,
                                               const uint32_t *TC, uint8_t *TE, uint64_t *TP, int32_t *status) {
    const UnpStreamRef m = mbs[blockIdx.x];
    const UnpackStream s = st[m.si];
    const int t = threadIdx.x;
    if (s.param < 1 || s.n == 0) {
        if (t == 0) status[m.si] = s.n == 0 ? 0 : NTC_ERR_FORMAT;
        return;
    }
    __shared__ uint8_t sX[kMbWalkTiles * 64];
    __shared__ uint32_t sC[kMbWalkTiles * 64];
    uint32_t e = 0;
    uint64_t p = 0;
    for (uint32_t k0 = 0; k0 < m.n_tiles; k0 += kMbWalkTiles) {
        const uint32_t nk = m.n_tiles - k0 < (uint32_t)kMbWalkTiles ? m.n_tiles - k0 : (uint32_t)kMbWalkTiles;
        const uint64_t g0 = (uint64_t)m.first_tile + k0;
        for (uint32_t i = t; i < nk * 64; i += 64) {
            sX[i] = TX[g0 * 64 + i];
            sC[i] = TC[g0 * 64 + i];
        }
        __syncthreads();
        if (t == 0) {
            for (uint32_t k = 0; k < nk; k++) {
                TE[g0 + k] = (uint8_t)e;
                TP[g0 + k] = p;
                if (e == kMbDead) continue;
                p += sC[k * 64 + e];
                e = sX[k * 64 + e];
            }
        }
        __syncthreads();
        e = __shfl(e, 0, 64);
        p = __shfl(p, 0, 64);
    }
    if (t == 0) status[m.si] = p < s.n ? NTC_ERR_FORMAT : 0;  // fewer codes than values
}

__global__ __launch_bounds__(kMbTileSegs) void k_mb_decode(const uint64_t *payload, const UnpackStream *st,
                                                          const UnpTile *tiles, const uint8_t *X, const uint16_t *C,
                                                          const uint8_t *TE, const uint64_t *TP, uint64_t *vals,
                                                          int32_t *status) {
    const uint8_t e0 = TE[blockIdx.x];
    if (e0 == kMbDead) return;  // the stream's codes ended in an earlier tile
    const UnpTile tl = tiles[blockIdx.x];
    const UnpackStream s = st[tl.si];
    const MbParams q = mb_params(s);
    const int t = threadIdx.x;
    __shared__ uint8_t sX[64 * kMbTileSegs];
    __shared__ uint8_t sE[kMbTileSegs];
    __shared__ uint64_t sh[kMbTileSegs / 64];
    __shared__ uint64_t sw[kMbWin];
    __shared__ int s_err;
    const uint64_t tbase = (uint64_t)blockIdx.x * 64 * kMbTileSegs;
    for (uint32_t e = 0; e < q.L; e++) sX[e * kMbTileSegs + t] = X[tbase + (uint64_t)e * kMbTileSegs + t];
    if (t == 0) s_err = 0;
    __syncthreads();
    const uint64_t seg0 = (uint64_t)tl.tile * kMbTileSegs;
    const uint64_t w0 = seg0 * kMbSegBits / 64;
    stage_words(sw, payload + s.word_off, s.nwords, w0, kMbWin);
    const uint64_t segs = (q.nbits + kMbSegBits - 1) / kMbSegBits;
    const uint32_t ns = (uint32_t)(segs - seg0 < kMbTileSegs ? segs - seg0 : kMbTileSegs);
    if (t == 0) {
        uint32_t e = e0;
        for (uint32_t u = 0; u < kMbTileSegs; u++) {
            sE[u] = (uint8_t)(u < ns ? e : kMbDead);
            if (u < ns && e != kMbDead) e = sX[e * kMbTileSegs + u];
        }
    }
    __syncthreads();
    const uint32_t en = sE[t];
    const uint64_t cnt = en != kMbDead ? C[tbase + (uint64_t)en * kMbTileSegs + t] : 0;
    uint64_t tot;
    const uint64_t off = TP[blockIdx.x] + block_exscan<kMbTileSegs>(cnt, &tot, sh);
    if (cnt && off < s.n) {
        WinBits bt{payload + s.word_off, s.nwords, sw, w0, kMbWin};
        uint64_t p = (seg0 + t) * kMbSegBits + en;
        for (uint64_t j = 0; j < cnt && off + j < s.n; j++) {
            const Code c = mb_at(bt, p, q.l, q.limit);
            if (!c.len || c.bad) {
                s_err = NTC_ERR_FORMAT;
                break;
            }
            vals[s.val_off + off + j] = c.val;
            p += c.len;
        }
    }
    __syncthreads();
    if (t == 0 && s_err) atomicOr(&status[tl.si], (int)NTC_ERR_FORMAT);
}

// The zip runs in segments of kZipSeg records, one workgroup each, so a call's few blocks
// fill the GPU.  k_zip_count: per segment, its long records and short bases.
constexpr uint64_t kZipSeg = 4096;
__global__ __launch_bounds__(kZipThreads) void k_zip_count(const UnpackStream *st, const uint64_t *vals, uint32_t nseg,
                                                          uint64_t *segc) {
    const uint32_t b = blockIdx.x / nseg, g = blockIdx.x % nseg;
    const UnpackStream s3 = st[4 * b + 2];
    const uint64_t *fl = vals + s3.val_off;
    const uint64_t r0 = (uint64_t)g * kZipSeg, r1 = r0 + kZipSeg < s3.n ? r0 + kZipSeg : s3.n;
    uint64_t nl = 0, ns = 0;
    for (uint64_t r = r0 + threadIdx.x; r < r1; r += kZipThreads) {
        const uint64_t f = fl[r];
        nl += !(f & 2);
        ns += (f & 0xFC) >> 2;  // T counts every flag's bits 2..7 (decode.rs:114)
    }
    nl = wave_sum(nl);
    ns = wave_sum(ns);
    __shared__ unsigned long long s_l, s_s;
    if (threadIdx.x == 0) s_l = s_s = 0;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&s_l, (unsigned long long)nl);
        atomicAdd(&s_s, (unsigned long long)ns);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        segc[2 * (uint64_t)blockIdx.x] = s_l;
        segc[2 * (uint64_t)blockIdx.x + 1] = s_s;
    }
}

// k_zip_write: per segment, the records from the block's s1 / s2 / s3 / s4 values (its
// first long index and short base from the segments before it), the checks decode.rs
// makes, and the segment's reads and bases added to its block's out3 (zeroed by the host):
// out3[3 b] = reads (first flags), out3[3 b + 1] = bases, out3[3 b + 2] = status (ORed).
__global__ __launch_bounds__(kZipThreads) void k_zip_write(const UnpackStream *st, const uint64_t *vals,
                                                          const uint64_t *rec_off, uint64_t *recs,
                                                          const int32_t *status, uint32_t nseg, const uint64_t *segc,
                                                          unsigned long long *out3) {
    const uint32_t b = blockIdx.x / nseg, g = blockIdx.x % nseg;
    const UnpackStream s1 = st[4 * b], s2 = st[4 * b + 1], s3 = st[4 * b + 2], s4 = st[4 * b + 3];
    const uint64_t nrec = s3.n;
    const uint64_t r0 = (uint64_t)g * kZipSeg;
    if (r0 >= nrec && !(g == 0 && nrec == 0)) return;
    const uint64_t r1 = r0 + kZipSeg < nrec ? r0 + kZipSeg : nrec;
    const uint64_t *c1 = vals + s1.val_off, *c2 = vals + s2.val_off, *fl = vals + s3.val_off,
                   *bn = vals + s4.val_off;
    uint64_t *out = recs + rec_off[b];
    __shared__ uint64_t sh[kZipThreads / 64];
    __shared__ int s_err;
    __shared__ uint64_t s_li, s_sj, s_T;
    const int t = threadIdx.x;
    if (t == 0) {
        int err = status[4 * b] | status[4 * b + 1] | status[4 * b + 2] | status[4 * b + 3];
        if (!err && s1.n != s2.n) err = NTC_ERR_FORMAT;  // decode.rs: c1.len() != c2.len()
        uint64_t li = 0, sj = 0, T = 0;
        const uint64_t ns = (nrec + kZipSeg - 1) / kZipSeg;
        for (uint64_t q = 0; q < ns; q++) {
            const uint64_t l = segc[2 * ((uint64_t)b * nseg + q)], x = segc[2 * ((uint64_t)b * nseg + q) + 1];
            if (q < g) {
                li += l;
                sj += x;
            }
            T += x;
        }
        if (!err && T && s4.n != (T + 30) / 31) err = NTC_ERR_FORMAT;  // short-base chunks
        s_err = err;
        s_li = li;
        s_sj = sj;
        s_T = T;
    }
    __syncthreads();
    if (s_err) {
        if (t == 0) atomicOr(&out3[3 * b + 2], (unsigned long long)NTC_ERR_FORMAT);
        return;
    }
    const uint64_t T = s_T;
    uint64_t li = s_li, sj = s_sj, reads = 0, bases = 0;
    for (uint64_t q0 = r0; q0 < r1; q0 += (uint64_t)kZipThreads * kZipPer) {
        uint64_t f[kZipPer], nl = 0, ns = 0;
#pragma unroll
        for (int j = 0; j < kZipPer; j++) {
            const uint64_t r = q0 + (uint64_t)t * kZipPer + j;
            const bool in = r < r1;
            f[j] = in ? fl[r] : 0;
            nl += in && !(f[j] & 2);
            ns += in && (f[j] & 2) ? ((f[j] & 0xFF) >> 2) : 0;
        }
        uint64_t tl, ts;
        const uint64_t el = block_exscan<kZipThreads>(nl, &tl, sh);
        const uint64_t es = block_exscan<kZipThreads>(ns, &ts, sh);
        uint64_t i = li + el, jb = sj + es;
        int err = 0;
#pragma unroll
        for (int j = 0; j < kZipPer; j++) {
            const uint64_t r = q0 + (uint64_t)t * kZipPer + j;
            if (r >= r1) break;
            const uint32_t flag = (uint32_t)(f[j] & 0xFF);
            uint64_t w;
            if (!(flag & 2)) {
                if (i >= s1.n) {
                    err = NTC_ERR_FORMAT;
                    break;
                }
                w = (c1[i] & 0xFFFFFFFFull) | ((c2[i] & 0xFFFFFFull) << 32);
                bases += (c2[i] & 0xFFFFFFull);
                i++;
            } else {
                const uint32_t L = flag >> 2;
                if (jb + L > T) {
                    err = NTC_ERR_FORMAT;
                    break;
                }
                // bases jb .. jb + L - 1 of the concatenation: chunk q / 31, base q % 31
                w = 0;
                if (L <= 32) {  // from at most two chunks
                    const uint64_t c = jb / 31;
                    const uint32_t o = (uint32_t)(jb - 31 * c), t0 = 31 - o < L ? 31 - o : L;
                    if (t0) w = (bn[c] >> (2 * o)) & ((1ull << (2 * t0)) - 1);
                    if (L > t0) w |= (bn[c + 1] & ((1ull << (2 * (L - t0))) - 1)) << (2 * t0);
                } else {  // (longer than as_2bit takes; the host decoder's shifts)
                    for (uint32_t u = 0; u < L; u++) {
                        const uint64_t q = jb + u;
                        w |= ((bn[q / 31] >> (2 * (q % 31))) & 3ull) << ((2 * u) & 63);
                    }
                }
                w &= 0x00FFFFFFFFFFFFFFull;
                bases += L;
                jb += L;
            }
            reads += flag & 1u;
            out[r] = w | ((uint64_t)flag << 56);
        }
        if (err) atomicExch(&s_err, err);
        li += tl;
        sj += ts;
        __syncthreads();
        if (s_err) break;  // uniform: read after the barrier
    }
    const uint64_t rd = wave_sum(reads), bs = wave_sum(bases);
    if ((t & 63) == 0) {
        atomicAdd(&out3[3 * b], (unsigned long long)rd);
        atomicAdd(&out3[3 * b + 1], (unsigned long long)bs);
    }
    if (t == 0 && s_err) atomicOr(&out3[3 * b + 2], (unsigned long long)s_err);
}

}  // namespace

void unpack_plan(const UnpackStream *st, uint64_t n_blocks, UnpackPlan &plan) {
    plan = UnpackPlan{};
    for (uint64_t b = 0; b < n_blocks; b++)
        for (int i = 0; i < 4; i++) {
            const uint32_t si = (uint32_t)(4 * b + (uint64_t)i);
            const UnpackStream &s = st[si];
            const bool mb = i == 0 || i == 3;
            const uint64_t seg_bits = mb ? kMbSegBits : kRiceSegBits, per = mb ? kMbTileSegs : kRiceTileSegs;
            const uint64_t segs = (s.nwords * 64 + seg_bits - 1) / seg_bits;
            const bool run = s.n && (mb ? s.param >= 1 : s.param <= 63);
            const uint32_t nt = run ? (uint32_t)((segs + per - 1) / per) : 0;
            auto &tiles = mb ? plan.mb_tiles : plan.rice_tiles;
            auto &refs = mb ? plan.mb_streams : plan.rice_streams;
            for (uint32_t k = 0; k < nt; k++) tiles.push_back(UnpTile{si, k, (uint32_t)refs.size(), 0});
            refs.push_back(UnpStreamRef{si, (uint32_t)(tiles.size() - nt), nt, 0});
        }
}

// minimal binary: X (u8) + C (u16) per tile entry and segment, TX (u8) + TC (u32) per tile
// entry, TE + TP per tile; then the Rice tables
static uint64_t mb_ws_bytes(uint64_t n_tiles) { return (n_tiles * (64 * kMbTileSegs * 3 + 64 * 5 + 16) + 64) & ~63ull; }
uint64_t unpack_ws_bytes(const UnpackPlan &plan) {
    return mb_ws_bytes(plan.mb_tiles.size()) + rice_ws_bytes(plan.rice_tiles.size(), plan.rice_streams.size());
}

void launch_unpack(const UnpackDev &d, hipStream_t s) {
    if (!d.n_blocks) return;
    const uint32_t nseg = (uint32_t)((d.max_recs + kZipSeg - 1) / kZipSeg) + 1;
    // Rice streams
    const RiceWs rw = rice_ws((uint8_t *)d.ws + mb_ws_bytes(d.n_mb_tiles), d.n_rice_tiles, d.n_rice_streams);
    (void)hipMemsetAsync(rw.flags, 0, (uint64_t)d.n_rice_streams * 4, s);
    if (d.n_rice_tiles) {
        hipLaunchKernelGGL(k_rice_a, dim3(d.n_rice_tiles), dim3(kRiceTileSegs), 0, s, d.payload, d.st, d.rice_tiles,
                           d.marks, rw);
        hipLaunchKernelGGL(k_rice_b, dim3(d.n_rice_tiles), dim3(kRiceTileSegs), 0, s, d.payload, d.st, d.rice_tiles,
                           (const uint64_t *)d.marks, rw);
    }
    hipLaunchKernelGGL(k_rice_walk, dim3(d.n_rice_streams), dim3(64), 0, s, d.payload, d.st, d.rice_streams, d.vals,
                       d.status, rw);
    if (d.n_rice_tiles)
        hipLaunchKernelGGL(k_rice_count, dim3(d.n_rice_tiles), dim3(kRiceTileSegs), 0, s, d.st, d.rice_tiles,
                           (const uint64_t *)d.marks, rw);
    hipLaunchKernelGGL(k_rice_scan, dim3(d.n_rice_streams), dim3(64), 0, s, d.st, d.rice_streams, d.status, rw);
    if (d.n_rice_tiles)
        hipLaunchKernelGGL(k_rice_decode, dim3(d.n_rice_tiles), dim3(kRiceTileSegs), 0, s, d.payload, d.st,
                           d.rice_tiles, d.vals, d.status, rw);
    // minimal-binary streams: X, C, TC, TP, TX, TE
    const uint64_t nt = d.n_mb_tiles;
    uint8_t *X = (uint8_t *)d.ws;
    uint16_t *C = (uint16_t *)(X + nt * 64 * kMbTileSegs);
    uint32_t *TC = (uint32_t *)(C + nt * 64 * kMbTileSegs);
    uint64_t *TP = (uint64_t *)(TC + nt * 64);
    uint8_t *TX = (uint8_t *)(TP + nt);
    uint8_t *TE = TX + nt * 64;
    if (nt)
        hipLaunchKernelGGL(k_mb_tab, dim3(d.n_mb_tiles), dim3(kMbTabThreads), 0, s, d.payload, d.st, d.mb_tiles, X, C, TX,
                           TC);
    hipLaunchKernelGGL(k_mb_walk, dim3(d.n_mb_streams), dim3(64), 0, s, d.st, d.mb_streams, TX, TC, TE, TP, d.status);
    if (nt)
        hipLaunchKernelGGL(k_mb_decode, dim3(d.n_mb_tiles), dim3(kMbTileSegs), 0, s, d.payload, d.st, d.mb_tiles, X, C,
                           TE, TP, d.vals, d.status);
    (void)hipMemsetAsync(d.out3, 0, d.n_blocks * 3 * 8, s);
    hipLaunchKernelGGL(k_zip_count, dim3((uint32_t)(d.n_blocks * nseg)), dim3(kZipThreads), 0, s, d.st, d.vals, nseg,
                       d.segc);
    hipLaunchKernelGGL(k_zip_write, dim3((uint32_t)(d.n_blocks * nseg)), dim3(kZipThreads), 0, s, d.st, d.vals,
                       d.rec_off, d.recs, d.status, nseg, d.segc, (unsigned long long *)d.out3);
}

uint64_t unpack_seg_words(uint64_t n_blocks, uint64_t max_recs) {
    return 2 * n_blocks * ((max_recs + kZipSeg - 1) / kZipSeg + 1);
}

}  // namespace ntc
