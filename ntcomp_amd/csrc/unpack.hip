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
// binary: l or l + 1 bits), so its code boundaries are found in parallel the way a
// self-synchronising prefix code allows (k_unpack_streams, one workgroup per stream):
// Rice streams (s2, s3; k_unpack_streams):
//   A  every thread decodes its segment of the stream from the segment's first bit as if a
//      code started there, marking the code starts of its chain in a bitmap;
//   B  each thread goes on past its segment's end into the next segment until its chain
//      meets a position the next thread's chain marked: from there both chains agree.
//      Thread 0's chain is the true one (the stream starts with a code), so by induction
//      every segment's true codes are: the ones the previous thread decoded before the
//      meeting point, then the next thread's marked starts;
//   C  true codes per segment (a count + a popcount of the bitmap), block scan -> offsets;
//   D  each thread decodes its segment's true codes into place.
// A chain that never meets the next one within that segment (possible for pathological
// streams, never seen on ntcomp's) makes the workgroup decode its stream sequentially.
// Minimal-binary streams (s1, s4; k_unpack_mb) are l- or (l + 1)-bit codes, nearly all of one
// length, and such chains need not ever meet: there every segment's transfer is computed for
// each of the l + 1 offsets a code can start at, and one thread follows the true entries.
//
// k_zip_count + k_zip_write (a workgroup per 16,384 records of a block) zip the four value
// streams back into u64 records with two block scans (long records -> s1/s2 index, short
// records -> base offset; each segment starts from the counts of the ones before it), check
// what read_block_impl checks (stream sizes, flags past the streams), and sums the reads
// (first flags) and bases the FASTA writer needs.
//
// Bound: the payload is read ~3x (speculative, continuation, final decode) and the values
// once; about 1 B per record of payload at C91.
#include <hip/hip_runtime.h>

#include "../../include/ntcomp_gpu.h"
#include "kernels.h"

namespace ntc {

namespace {

constexpr int kUnpThreads = 1024;  // threads (segments) per stream
constexpr int kZipThreads = 256;   // threads per block in the zip
constexpr int kZipPer = 4;         // records per thread per zip tile

__device__ __forceinline__ uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

// The 64 stream bits from bit position pos (MSB first), zero past the stream's end.  The
// cursor keeps the two words under the last position: a thread's positions only grow, so a
// code costs a load only when it crosses into the next word.
struct Bits64 {
    const uint64_t *w;
    uint64_t nwords;
    uint64_t wi = ~0ull - 1, hi = 0, lo = 0;  // (not ~0: ~0 + 1 would look like "the next word" of word 0)
    __device__ __forceinline__ uint64_t load(uint64_t i) const { return i < nwords ? bswap64(w[i]) : 0; }
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

struct Code {
    uint64_t len;  // bits (0: no code here -- it runs past the end of the stream)
    uint64_t val;  // the value the reference's decoder returns (minimal binary: v - 1)
    bool bad;      // minimal binary v == 0 (decode.rs's check)
};

// Rice (param p): zeros up to a one, then p bits
__device__ __forceinline__ Code rice_at(Bits64 &bt, uint64_t pos, uint32_t p) {
    const uint64_t nbits = bt.nwords * 64;
    uint64_t q = 0, at = pos;
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
__device__ __forceinline__ Code mb_at(Bits64 &bt, uint64_t pos, uint32_t l, uint64_t limit) {
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

struct StreamCoder {
    const uint64_t *w;
    uint64_t nwords;
    bool rice;
    uint32_t p, l;
    uint64_t limit;
    Bits64 bt;
    __device__ Code at(uint64_t pos) { return rice ? rice_at(bt, pos, p) : mb_at(bt, pos, l, limit); }
};

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

// exclusive block scan (kUnpThreads or kZipThreads threads), through sh (>= threads / 64 words)
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

// Rice streams (s2, s3 of every block: workgroup 2 i + j takes stream 4 i + 1 + j)
__global__ __launch_bounds__(kUnpThreads) void k_unpack_streams(const uint64_t *payload, const UnpackStream *st,
                                                               uint64_t *marks, uint64_t *vals, int32_t *status) {
    const uint32_t si = 4 * (blockIdx.x >> 1) + 1 + (blockIdx.x & 1);
    const UnpackStream s = st[si];
    const int t = threadIdx.x;
    __shared__ uint64_t sh[kUnpThreads / 64];
    __shared__ uint64_t s_f[kUnpThreads + 1], s_y[kUnpThreads + 1], s_pre[kUnpThreads + 1];
    __shared__ int s_fail, s_err;
    const uint64_t nbits = s.nwords * 64;
    if (t == 0) {
        s_fail = 0;
        s_err = 0;
    }
    StreamCoder cd{payload + s.word_off, s.nwords, true, 0, 0, 0, Bits64{payload + s.word_off, s.nwords}};
    if (cd.rice) {
        if (s.param > 63) {
            if (t == 0) status[si] = NTC_ERR_FORMAT;
            return;
        }
        cd.p = (uint32_t)s.param;
    } else {
        if (s.param < 1) {  // minimal_binary_decode: param 0 decodes no value
            if (t == 0) status[si] = s.n == 0 ? 0 : NTC_ERR_FORMAT;
            return;
        }
        cd.l = 63u - (uint32_t)__builtin_clzll(s.param);
        cd.limit = (cd.l == 63 ? 0ull : (2ull << cd.l)) - s.param;
    }
    if (s.n == 0) {
        if (t == 0) status[si] = 0;
        return;
    }
    uint64_t *m = marks + s.word_off;
    // segments of S bits (a multiple of 64: each thread owns whole bitmap words)
    const uint64_t S = ((nbits + kUnpThreads - 1) / kUnpThreads + 63) & ~63ull;
    const uint64_t a = (uint64_t)t * S, b = a + S < nbits ? a + S : nbits;
    const bool active = a < nbits;
    // ---- A: speculative chain from the segment's first bit, starts marked -------------------
    uint64_t pos = a, own = 0;
    bool dead = false;
    if (active) {
        for (uint64_t i = a >> 6; i < (b + 63) >> 6; i++) m[i] = 0;
        uint64_t word = 0, wi = a >> 6;
        while (pos < b) {
            const Code c = cd.at(pos);
            if (!c.len) {
                dead = true;
                break;
            }
            if ((pos >> 6) != wi) {
                m[wi] = word;
                wi = pos >> 6;
                word = 0;
            }
            word |= 1ull << (pos & 63);
            own++;
            pos += c.len;
        }
        m[wi] = word;
    }
    __syncthreads();
    // ---- B: on into the next segment until the next thread's chain is met ---------------------
    // (thread t writes s_f / s_y / s_pre of segment t + 1: its true first start, the meeting
    // point and the codes before it)
    if (active && b < nbits) {
        const uint64_t nb = b + S < nbits ? b + S : nbits;
        uint64_t q = pos, pre = 0;
        bool met = false;
        if (!dead) {
            while (q < nb) {
                if (marked(m, q)) {
                    met = true;
                    break;
                }
                const Code c = cd.at(q);
                if (!c.len) break;
                q += c.len;
                pre++;
            }
        }
        // a chain that ran past the stream's end (dead) ends the stream's codes: the segments
        // after it hold none (fine when the first n codes all lie before it)
        if (dead) {
            s_f[t + 1] = nbits;
            s_y[t + 1] = nbits;
            s_pre[t + 1] = 0;
        } else if (met) {
            s_f[t + 1] = pos;
            s_y[t + 1] = q;
            s_pre[t + 1] = pre;
        } else if (q >= nb && pos < nb) {
            s_fail = 1;  // the chains did not meet within the next segment
        } else {
            // pos >= nb: a code longer than a segment; or the chain died in the next segment
            s_fail = 1;
        }
    }
    __syncthreads();
    if (s_fail) {  // sequential fallback: thread 0 walks the whole stream
        if (t == 0) {
            uint64_t p = 0;
            int err = 0;
            for (uint64_t i = 0; i < s.n; i++) {
                const Code c = cd.at(p);
                if (!c.len || c.bad) {
                    err = NTC_ERR_FORMAT;
                    break;
                }
                vals[s.val_off + i] = c.val;
                p += c.len;
            }
            status[si] = err;
        }
        return;
    }
    // ---- C: true codes per segment, offsets ----------------------------------------------------
    uint64_t cnt = 0, f = 0;
    if (active) {
        if (t == 0) {
            cnt = dead ? own : count_marks(m, 0, b);
            f = 0;
        } else {
            f = s_f[t];
            const uint64_t y = s_y[t];
            cnt = s_pre[t] + (y < b ? count_marks(m, y, b) : 0);
            // a dead chain of this thread: its marks after the meeting point run up to where it
            // died; the codes past that (the stream's tail padding) do not exist
        }
    }
    uint64_t tot;
    const uint64_t off = block_exscan<kUnpThreads>(cnt, &tot, sh);
    if (t == 0 && tot < s.n) s_err = NTC_ERR_FORMAT;  // fewer codes than values
    // ---- D: decode this segment's true codes into place ---------------------------------------
    if (active && off < s.n) {
        uint64_t p = f;
        for (uint64_t j = 0; j < cnt && off + j < s.n; j++) {
            const Code c = cd.at(p);
            if (!c.len || c.bad) {
                atomicExch(&s_err, (int)NTC_ERR_FORMAT);
                break;
            }
            vals[s.val_off + off + j] = c.val;
            p += c.len;
        }
    }
    __syncthreads();
    if (t == 0) status[si] = s_err;
}

// Minimal-binary streams (s1, s4: workgroup 2 i + j takes stream 4 i + 3 j).  Their codes are
// l or l + 1 bits, mostly one of the two, and chains started at different offsets rarely
// meet (fixed-length codes never do), so each segment's transfer is computed for every entry
// offset a code can start at: thread t decodes its segment from each e < l + 1 bits past its
// first bit and records where that chain leaves (the first code start past the segment, at
// most l bits on) and its codes; thread 0 then follows the true entry from segment to segment
// (one LDS lookup each), and each segment's true codes are decoded into place.
__global__ __launch_bounds__(kUnpThreads) void k_unpack_mb(const uint64_t *payload, const UnpackStream *st,
                                                          uint32_t *chainc, uint64_t *vals, int32_t *status) {
    const uint32_t si = 4 * (blockIdx.x >> 1) + ((blockIdx.x & 1) ? 3 : 0);
    const UnpackStream s = st[si];
    const int t = threadIdx.x;
    __shared__ uint8_t s_x[kUnpThreads * 64];  // exit offset past the segment per entry (255: dead)
    __shared__ uint8_t s_entry[kUnpThreads];
    __shared__ uint64_t sh[kUnpThreads / 64];
    __shared__ int s_err;
    if (s.param < 1) {  // minimal_binary_decode: param 0 decodes no value
        if (t == 0) status[si] = s.n == 0 ? 0 : NTC_ERR_FORMAT;
        return;
    }
    if (s.n == 0) {
        if (t == 0) status[si] = 0;
        return;
    }
    if (t == 0) s_err = 0;
    StreamCoder cd{payload + s.word_off, s.nwords, false, 0, 0, 0, Bits64{payload + s.word_off, s.nwords}};
    cd.l = 63u - (uint32_t)__builtin_clzll(s.param);
    cd.limit = (cd.l == 63 ? 0ull : (2ull << cd.l)) - s.param;
    const uint32_t L = cd.l + 1;  // entry offsets 0 .. l (codes are at most l + 1 bits)
    const uint64_t nbits = s.nwords * 64;
    uint64_t S = (nbits + kUnpThreads - 1) / kUnpThreads;
    if (S < 64) S = 64;
    const uint64_t a = (uint64_t)t * S, b = a + S < nbits ? a + S : nbits;
    const bool active = a < nbits;
    uint32_t *cc = chainc + (uint64_t)blockIdx.x * kUnpThreads * 64 + (uint64_t)t * 64;
    // ---- A: the segment's transfer for every entry offset --------------------------------------
    if (active) {
        for (uint32_t e = 0; e < L; e++) {
            uint64_t pos = a + e;
            uint32_t cnt = 0;
            bool dead = false;
            while (pos < b) {
                const Code c = cd.at(pos);
                if (!c.len) {
                    dead = true;
                    break;
                }
                pos += c.len;
                cnt++;
            }
            s_x[t * 64 + e] = dead ? 255 : (uint8_t)(pos - b);
            cc[e] = cnt;
        }
    }
    __syncthreads();
    // ---- B: the true entry of every segment (segment 0: the stream's first bit) ----------------
    if (t == 0) {
        uint32_t e = 0;
        for (int u = 0; u < kUnpThreads; u++) {
            if ((uint64_t)u * S >= nbits || e == 255) {
                s_entry[u] = 255;
                continue;
            }
            s_entry[u] = (uint8_t)e;
            e = s_x[u * 64 + e];
        }
    }
    __syncthreads();
    // ---- C + D: true codes per segment, offsets, decode into place ----------------------------
    const uint32_t en = s_entry[t];
    const uint64_t cnt = active && en != 255 ? cc[en] : 0;
    uint64_t tot;
    const uint64_t off = block_exscan<kUnpThreads>(cnt, &tot, sh);
    if (t == 0 && tot < s.n) s_err = NTC_ERR_FORMAT;  // fewer codes than values
    if (cnt && off < s.n) {
        uint64_t p = a + en;
        for (uint64_t j = 0; j < cnt && off + j < s.n; j++) {
            const Code c = cd.at(p);
            if (!c.len || c.bad) {
                atomicExch(&s_err, (int)NTC_ERR_FORMAT);
                break;
            }
            vals[s.val_off + off + j] = c.val;
            p += c.len;
        }
    }
    __syncthreads();
    if (t == 0) status[si] = s_err;
}

// The zip runs in segments of kZipSeg records, one workgroup each, so a call's few blocks
// fill the GPU.  k_zip_count: per segment, its long records and short bases.
constexpr uint64_t kZipSeg = 16384;
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
                for (uint32_t u = 0; u < L; u++) {
                    const uint64_t q = jb + u;
                    w |= ((bn[q / 31] >> (2 * (q % 31))) & 3ull) << (2 * u);
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

void launch_unpack(const uint64_t *payload, const UnpackStream *st, uint64_t n_blocks, uint64_t max_recs,
                   uint64_t *marks, uint32_t *chainc, uint64_t *vals, int32_t *stream_status, const uint64_t *rec_off,
                   uint64_t *recs, uint64_t *segc, uint64_t *out3, hipStream_t s) {
    if (!n_blocks) return;
    const uint32_t nseg = (uint32_t)((max_recs + kZipSeg - 1) / kZipSeg) + 1;
    hipLaunchKernelGGL(k_unpack_streams, dim3((uint32_t)(2 * n_blocks)), dim3(kUnpThreads), 0, s, payload, st, marks,
                       vals, stream_status);
    hipLaunchKernelGGL(k_unpack_mb, dim3((uint32_t)(2 * n_blocks)), dim3(kUnpThreads), 0, s, payload, st, chainc, vals,
                       stream_status);
    (void)hipMemsetAsync(out3, 0, n_blocks * 3 * 8, s);
    hipLaunchKernelGGL(k_zip_count, dim3((uint32_t)(n_blocks * nseg)), dim3(kZipThreads), 0, s, st, vals, nseg, segc);
    hipLaunchKernelGGL(k_zip_write, dim3((uint32_t)(n_blocks * nseg)), dim3(kZipThreads), 0, s, st, vals, rec_off, recs,
                       stream_status, nseg, segc, (unsigned long long *)out3);
}

uint64_t unpack_chain_words(uint64_t n_blocks) { return 2 * n_blocks * kUnpThreads * 64; }  // u32 words

uint64_t unpack_seg_words(uint64_t n_blocks, uint64_t max_recs) {
    return 2 * n_blocks * ((max_recs + kZipSeg - 1) / kZipSeg + 1);
}

}  // namespace ntc
