// GPU block packer: write_block_to (src/lib.rs:232-252) up to deflate, for every
// 65,536-read block of an encoded batch, straight from the records k_emit4 left in HBM.
//
//   split_encoded_dictionary   src/encode.rs:168-229   s1 colex, s2 length, s3 flag byte,
//                                                      s4 short bases in 31-base chunks
//   rice_encode                src/encode.rs:59-75     s2, s3
//   minimal_binary_encode      src/encode.rs:77-94     s1, s4 (v + 1, max = maxval + 2)
//   compress_block's bytes     src/encode.rs:107-109   words stored big-endian (the MSB-first
//                                                      bit stream of dsi-bitstream's BE writer)
//
// Workgroups of 1024 threads (16 waves), tiles of 4096 records (4 consecutive records per
// thread: two 16-byte loads per lane, coalesced); pass 1 one workgroup per block:
//
//   k_pack_stats  stream totals (long records, max colex, length / flag sums, short bases)
//                 and the s4 chunk values: a block scan gives every short record its base
//                 position, its 2-bit bases are OR-ed into an LDS chunk buffer, finished
//                 chunks go to a scratch array (8 B per chunk), the unfinished last chunk
//                 stays in LDS for the next tile.
//   (host)        Rice parameters with glibc's f64 log/exp (codec_params.h: the reference's
//                 f64 math; the device's libm may differ in the last ulp, and the parameter
//                 is a ceil), minimal-binary widths, per-block payload offsets from exact
//                 upper bounds, capacity check.
//   k_pack_seglen / k_pack_segscan   pass 2 runs in segments of 16,384 records (or s4
//                 chunks), each its own workgroup: their bits per stream, then each
//                 segment's first bit within its block's streams (and the streams' totals).
//   k_pack_write  per segment, per tile: code lengths, a 3-way block scan (s1, s2, s3) gives
//                 every code its bit position, codes are OR-ed into per-stream LDS word
//                 buffers (a unary run of zeros costs nothing: only the terminating one and
//                 the remainder are written), then complete words are stored once
//                 (big-endian), the partial last word carries into the next tile; a segment's
//                 first and last words, shared with the neighbouring segments, are OR-ed into
//                 the zeroed payload.  A tile whose bits do not fit its LDS buffer
//                 (pathological unary runs) ORs straight into the payload with global
//                 atomics.  s4 the same way over the chunk segments.
//
// Bound: HBM bytes -- reads 8 B per record twice + 8 B per s4 chunk, writes the payload
// (about 1 B per record at C91) and the chunks.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace ntc {

namespace {

constexpr int kPackThreads = 1024;
constexpr int kPackPer = 4;                                // records per thread per tile
constexpr int kPackTile = kPackThreads * kPackPer;         // 4096 records
constexpr int kChunkBufWords = kPackTile * 32 / 31 + 4;    // s4 chunks a tile can touch (<= 32 bases/record)
constexpr int kBuf1 = kPackTile * 33 / 64 + 4;             // s1: <= 33 bits per code
constexpr int kBuf2 = 2048;                                // s2: 131 k bits (~32 per code)
constexpr int kBuf3 = 1024;                                // s3: 65 k bits (~16 per code)
constexpr int kS4Per = 2;                                  // s4 chunks per thread per tile
constexpr int kS4Tile = kPackThreads * kS4Per;
static_assert(kS4Tile * 63 / 64 + 4 <= kBuf1, "s4 tile must fit the s1 buffer");

__device__ __forceinline__ uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

// First s4 chunk slot of block b whose records start at beg.  A block of n records holds at
// most 32 n short bases (from_2bit's limit; longer ones are flagged bad), i.e. ceil(32 n / 31)
// <= n + floor(n / 31) + 1 chunks, and chunk_base(end, b + 1) - chunk_base(beg, b) >=
// n + floor(n / 31) + 2, so neighbouring blocks never overlap (pack_chunk_words sizes it).
__device__ __forceinline__ uint64_t chunk_base(uint64_t beg, uint64_t b) { return beg + beg / 31 + 2 * b; }

// 3-way exclusive block scan of u64 values (kPackThreads threads); sh: 3 * 16 words
__device__ __forceinline__ void block_scan3(const uint64_t v[3], uint64_t ex[3], uint64_t tot[3], uint64_t *sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t inc[3] = {v[0], v[1], v[2]};
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const uint64_t t = __shfl_up(inc[k], d, 64);
            if (lane >= d) inc[k] += t;
        }
    }
    if (lane == 63)
        for (int k = 0; k < 3; k++) sh[wid * 3 + k] = inc[k];
    __syncthreads();
    uint64_t base[3] = {0, 0, 0}, all[3] = {0, 0, 0};
    for (int w = 0; w < kPackThreads / 64; w++)
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const uint64_t x = sh[w * 3 + k];
            base[k] += w < wid ? x : 0;
            all[k] += x;
        }
#pragma unroll
    for (int k = 0; k < 3; k++) {
        ex[k] = base[k] + inc[k] - v[k];
        tot[k] = all[k];
    }
    __syncthreads();
}

// block-wide max / sum helpers through sh (16 words)
__device__ __forceinline__ uint64_t wave_max(uint64_t x) {
    for (int d = 32; d; d >>= 1) {
        const uint64_t t = __shfl_xor(x, d, 64);
        x = t > x ? t : x;
    }
    return x;
}
__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
    for (int d = 32; d; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

// OR the nb (<= 64) low bits of v into a MSB-first word array at bit position at
__device__ __forceinline__ void or_bits_lds(uint64_t *w, uint64_t at, uint64_t v, int nb) {
    const uint64_t i = at >> 6;
    const int off = (int)(at & 63);
    if (off + nb <= 64) {
        atomicOr((unsigned long long *)&w[i], (unsigned long long)(v << (64 - off - nb)));
    } else {
        const int spill = off + nb - 64;  // 1..63
        atomicOr((unsigned long long *)&w[i], (unsigned long long)(v >> spill));
        atomicOr((unsigned long long *)&w[i + 1], (unsigned long long)(v << (64 - spill)));
    }
}
// same into the big-endian payload in HBM (fallback tiles)
__device__ __forceinline__ void or_bits_hbm(uint64_t *w, uint64_t at, uint64_t v, int nb) {
    const uint64_t i = at >> 6;
    const int off = (int)(at & 63);
    if (off + nb <= 64) {
        atomicOr((unsigned long long *)&w[i], (unsigned long long)bswap64(v << (64 - off - nb)));
    } else {
        const int spill = off + nb - 64;
        atomicOr((unsigned long long *)&w[i], (unsigned long long)bswap64(v >> spill));
        atomicOr((unsigned long long *)&w[i + 1], (unsigned long long)bswap64(v << (64 - spill)));
    }
}

__device__ __forceinline__ void load_tile(const uint64_t *recs, uint64_t i0, uint64_t end, uint64_t r[kPackPer]) {
#pragma unroll
    for (int j = 0; j < kPackPer; j++) {
        const uint64_t i = i0 + j;
        r[j] = i < end ? recs[i] : 0;
    }
}

// A fallback tile's partial last word lives in HBM (atomics): read it back as the carry
__device__ void flush_tile_hbm(uint64_t bit1, bool last, uint64_t *out, uint64_t *carry) {
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
        *carry = 0;
        if (!last && (bit1 & 63))
            *carry = bswap64(__hip_atomic_load((unsigned long long *)&out[bit1 >> 6], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT));
    }
    __syncthreads();
}

// Pass 1 in segments of kPackSegReads reads (a block's reads in order), each its own
// workgroup.  Segment sg of block b = sg / spb (spb = segments per block) covers reads
// [b * block_reads + (sg % spb) * kPackSegReads, ...) within the block; the last block's
// trailing segments may be empty.
constexpr uint64_t kPackSegReads = 4096;
struct SegRange {
    uint64_t b, r0, r1;
};
__device__ __forceinline__ SegRange seg_range(uint64_t sg, uint64_t spb, uint32_t block_reads, uint64_t n_reads) {
    SegRange g;
    g.b = sg / spb;
    const uint64_t bend = g.b * block_reads + block_reads < n_reads ? g.b * block_reads + block_reads : n_reads;
    g.r0 = g.b * block_reads + (sg % spb) * kPackSegReads;
    g.r1 = g.r0 + kPackSegReads < bend ? g.r0 + kPackSegReads : bend;
    if (g.r0 > g.r1) g.r0 = g.r1;
    return g;
}
// per-segment words of the scratch: n_long, max1, sum2, sum3, short bases, bad, first short base
constexpr int kSegStat = 8;

// 1a: a segment's stream totals
__global__ void __launch_bounds__(kPackThreads) k_pstat_seg(const uint64_t *recs, const uint64_t *roffs,
                                                            uint64_t n_reads, uint32_t block_reads, uint64_t spb,
                                                            uint64_t *seg) {
    const SegRange g = seg_range(blockIdx.x, spb, block_reads, n_reads);
    const uint64_t beg = roffs[g.r0], end = roffs[g.r1];
    uint64_t n_long = 0, max1 = 0, sum2 = 0, sum3 = 0, nb = 0, bad = 0;
    for (uint64_t i = beg + threadIdx.x; i < end; i += kPackThreads) {
        const uint64_t w = recs[i], flag = w >> 56;
        sum3 += flag;
        if ((flag & 2) == 0) {
            n_long++;
            const uint64_t c = w & 0xFFFFFFFFULL;
            max1 = c > max1 ? c : max1;
            sum2 += (w >> 32) & 0xFFFFFFULL;
        } else {
            const uint64_t len = flag >> 2;
            if (len > 32) bad = 1;  // from_2bit panics past 32 bases (encode.rs:220)
            else nb += len;
        }
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t red[6] = {wave_sum(n_long), wave_max(max1), wave_sum(sum2), wave_sum(sum3), wave_sum(nb), wave_max(bad)};
    __shared__ uint64_t rs[16][6];
    if (lane == 0)
        for (int k = 0; k < 6; k++) rs[wid][k] = red[k];
    __syncthreads();
    if (threadIdx.x < 6) {
        const int k = threadIdx.x;
        uint64_t t = 0;
        for (int w = 0; w < kPackThreads / 64; w++) t = (k == 1 || k == 5) ? (rs[w][k] > t ? rs[w][k] : t) : t + rs[w][k];
        seg[blockIdx.x * kSegStat + k] = t;
    }
}

// 1b: per block (one thread each), the segments combined and each segment's first short base
__global__ void __launch_bounds__(256) k_pstat_block(const uint64_t *roffs, uint64_t n_reads, uint32_t block_reads,
                                                     uint64_t n_blocks, uint64_t spb, uint64_t *seg,
                                                     PackStats *stats) {
    const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= n_blocks) return;
    const uint64_t r0 = b * block_reads, r1 = r0 + block_reads < n_reads ? r0 + block_reads : n_reads;
    PackStats S{};
    uint64_t T = 0;
    for (uint64_t j = b * spb; j < (b + 1) * spb; j++) {
        uint64_t *x = seg + j * kSegStat;
        S.n_long += x[0];
        S.max1 = x[1] > S.max1 ? x[1] : S.max1;
        S.sum2 += x[2];
        S.sum3 += x[3];
        S.bad |= x[5];
        x[6] = T;
        T += x[4];
    }
    S.rec_begin = roffs[r0];
    S.n_recs = roffs[r1] - roffs[r0];
    S.T = T;
    stats[b] = S;
}

// 1c: a segment's s4 chunks -- a block scan gives every short record its base position, its
// 2-bit bases are OR-ed into an LDS chunk buffer, finished chunks go out; the segment's first
// and last chunks, shared with the neighbouring segments, are OR-ed into the zeroed array
__global__ void __launch_bounds__(kPackThreads) k_pstat_chunks(const uint64_t *recs, const uint64_t *roffs,
                                                               uint64_t n_reads, uint32_t block_reads, uint64_t spb,
                                                               const uint64_t *seg, const PackStats *stats,
                                                               uint64_t *chunks) {
    __shared__ uint64_t cbuf[kChunkBufWords];
    __shared__ uint64_t sh[64];
    const uint64_t sg = blockIdx.x;
    const uint64_t nbs = seg[sg * kSegStat + 4];
    if (nbs == 0) return;  // no short base in this segment
    const SegRange g = seg_range(sg, spb, block_reads, n_reads);
    const uint64_t beg = roffs[g.r0], end = roffs[g.r1];
    uint64_t *ch = chunks + chunk_base(stats[g.b].rec_begin, g.b);  // block b's chunks
    uint64_t T = seg[sg * kSegStat + 6];                              // the segment's first short base
    const uint64_t first_c = T / 31, last_c = (T + nbs - 1) / 31;
    for (uint64_t i = threadIdx.x; i < kChunkBufWords; i += kPackThreads) cbuf[i] = 0;
    __syncthreads();
    for (uint64_t t0 = beg; t0 < end; t0 += kPackTile) {
        uint64_t r[kPackPer];
        load_tile(recs, t0 + threadIdx.x * kPackPer, end, r);
        uint64_t nb = 0;
#pragma unroll
        for (int j = 0; j < kPackPer; j++) {
            const uint64_t i = t0 + threadIdx.x * kPackPer + j, flag = r[j] >> 56;
            if (i < end && (flag & 2) && (flag >> 2) <= 32) nb += flag >> 2;
        }
        uint64_t v[3] = {nb, 0, 0}, ex[3], tot[3];
        block_scan3(v, ex, tot, sh);
        // chunk index of the tile's first base: T / 31; cbuf[0] already holds its bases
        const uint64_t c0 = T / 31;
        uint64_t pos = T + ex[0];
#pragma unroll
        for (int j = 0; j < kPackPer; j++) {
            const uint64_t i = t0 + threadIdx.x * kPackPer + j;
            const uint64_t w = r[j], flag = w >> 56;
            if (i >= end || (flag & 2) == 0 || (flag >> 2) > 32) continue;
            const int len = (int)(flag >> 2);
            if (!len) continue;
            uint64_t bits = w & 0x00FFFFFFFFFFFFFFULL;
            if (len < 28) bits &= (1ULL << (2 * len)) - 1;
            const uint64_t c = pos / 31 - c0;
            const int sh2 = (int)(pos % 31) * 2;  // 0..60
            atomicOr((unsigned long long *)&cbuf[c], (unsigned long long)((bits << sh2) & ((1ULL << 62) - 1)));
            if (sh2 && 2 * len > 62 - sh2)
                atomicOr((unsigned long long *)&cbuf[c + 1], (unsigned long long)(bits >> (62 - sh2)));
            pos += (uint64_t)len;
        }
        __syncthreads();
        const uint64_t T1 = T + tot[0];
        const bool last = t0 + kPackTile >= end;
        // finished chunks: [c0, T1 / 31), plus the partial last one at the end of the segment
        const uint64_t cend = last ? (T1 + 30) / 31 : T1 / 31;
        for (uint64_t c = c0 + threadIdx.x; c < cend; c += kPackThreads) {
            const uint64_t x = cbuf[c - c0];
            if (c == first_c || c == last_c) atomicOr((unsigned long long *)&ch[c], (unsigned long long)x);
            else ch[c] = x;
        }
        __syncthreads();
        // carry the unfinished chunk to slot 0, clear the rest
        const uint64_t keep = (!last && (T1 % 31)) ? cbuf[T1 / 31 - c0] : 0;
        __syncthreads();
        for (uint64_t i = threadIdx.x; i < kChunkBufWords; i += kPackThreads) cbuf[i] = i ? 0 : keep;
        __syncthreads();
        T = T1;
    }
}

// 1d: per block, the largest s4 chunk (after every segment's chunks are in)
__global__ void __launch_bounds__(kPackThreads) k_pstat_max4(const uint64_t *chunks, PackStats *stats) {
    const uint64_t b = blockIdx.x;
    const PackStats S = stats[b];
    const uint64_t *ch = chunks + chunk_base(S.rec_begin, b);
    const uint64_t nch = (S.T + 30) / 31;
    uint64_t m = 0;
    for (uint64_t c = threadIdx.x; c < nch; c += kPackThreads) m = ch[c] > m ? ch[c] : m;
    m = wave_max(m);
    __shared__ uint64_t rs[16];
    if ((threadIdx.x & 63) == 0) rs[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 0; w < kPackThreads / 64; w++) m = rs[w] > m ? rs[w] : m;
        stats[b].max4 = m;
    }
}

// code of one record in stream s1 / s2 / s3: value (the bits to OR) at bit offset skip
// from the code start, nb bits; len = whole code length
struct Code {
    uint64_t v;
    uint64_t skip;
    int nb;
    uint64_t len;
};

__device__ __forceinline__ Code mb_code(uint64_t x, int l, uint64_t lim) {  // minimal binary of x + 1
    const uint64_t v = x + 1;
    if (v < lim) return Code{v, 0, l, (uint64_t)l};
    return Code{v + lim, 0, l + 1, (uint64_t)l + 1};
}
__device__ __forceinline__ Code rice_code(uint64_t x, int p) {  // unary(x >> p) then p bits
    const uint64_t q = x >> p;
    const uint64_t v = (1ULL << p) | (x & ((1ULL << p) - 1));
    return Code{v, q, p + 1, q + 1 + (uint64_t)p};
}

// pass 2a: every segment's bits per stream (the code lengths k_pack_write will write)
__global__ void __launch_bounds__(kPackThreads) k_pack_seglen(const uint64_t *recs, const uint64_t *chunks,
                                                              const PackStats *stats, const PackParams *params,
                                                              const PackSeg *segs, uint64_t *seg_bits) {
    __shared__ uint64_t rs[16][3];
    const PackSeg g = segs[blockIdx.x];
    const PackParams P = params[g.block];
    uint64_t v[3] = {0, 0, 0};
    if (g.kind == 0) {
        for (uint64_t i = g.first + threadIdx.x; i < g.first + g.count; i += kPackThreads) {
            const uint64_t w = recs[i], flag = w >> 56;
            v[2] += rice_code(flag, P.p3).len;
            if ((flag & 2) == 0) {
                v[0] += mb_code(w & 0xFFFFFFFFULL, P.l1, P.lim1).len;
                v[1] += rice_code((w >> 32) & 0xFFFFFFULL, P.p2).len;
            }
        }
    } else {
        const uint64_t *ch = chunks + chunk_base(stats[g.block].rec_begin, g.block);
        for (uint64_t i = g.first + threadIdx.x; i < g.first + g.count; i += kPackThreads)
            v[0] += mb_code(ch[i], P.l4, P.lim4).len;
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int k = 0; k < 3; k++) v[k] = wave_sum(v[k]);
    if (lane == 0)
        for (int k = 0; k < 3; k++) rs[wid][k] = v[k];
    __syncthreads();
    if (threadIdx.x < 3) {
        uint64_t t = 0;
        for (int w = 0; w < kPackThreads / 64; w++) t += rs[w][threadIdx.x];
        seg_bits[3 * blockIdx.x + threadIdx.x] = t;
    }
}

// pass 2b: per block, each segment's first bit in each stream and the streams' totals
__global__ void __launch_bounds__(256) k_pack_segscan(const PackParams *params, const PackSeg *segs,
                                                      uint64_t n_blocks, const uint64_t *seg_bits,
                                                      uint64_t *seg_start, uint64_t *bits_out) {
    const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= n_blocks) return;
    const PackParams P = params[b];
    uint64_t pos[4] = {0, 0, 0, 0};
    if (!P.skip)
        for (uint32_t j = P.seg0; j < P.seg0 + P.nseg; j++) {
            if (segs[j].kind == 0) {
                for (int k = 0; k < 3; k++) {
                    seg_start[3 * j + k] = pos[k];
                    pos[k] += seg_bits[3 * j + k];
                }
            } else {
                seg_start[3 * j] = pos[3];
                pos[3] += seg_bits[3 * j];
            }
        }
    for (int k = 0; k < 4; k++) bits_out[b * 4 + k] = pos[k];
}

// Store the words [w0, wend) of a tile's LDS buffer (big-endian); the segment's first and last
// words may hold bits of the neighbouring segments' workgroups: OR-ed into the zeroed payload
__device__ __forceinline__ void store_words(const uint64_t *buf, uint64_t w0, uint64_t wend, uint64_t first_w,
                                            uint64_t last_w, uint64_t *out) {
    for (uint64_t i = w0 + threadIdx.x; i < wend; i += kPackThreads) {
        const uint64_t x = bswap64(buf[i - w0]);
        if (i == first_w || i == last_w) atomicOr((unsigned long long *)&out[i], (unsigned long long)x);
        else out[i] = x;
    }
}

// One stream's tile within a segment: codes already OR-ed into buf (buf[0] held the carry
// word of the previous tile); [bit0, bit1) is the tile's span in the stream.  Stores the
// complete words, keeps the partial last one in carry (or stores it too at the segment end).
__device__ void flush_seg_tile(uint64_t *buf, uint64_t bit0, uint64_t bit1, bool last, uint64_t first_w,
                               uint64_t last_w, uint64_t *out, uint64_t *carry) {
    const uint64_t w0 = bit0 >> 6;
    const uint64_t wend = last ? (bit1 + 63) >> 6 : bit1 >> 6;  // words to store: [w0, wend)
    store_words(buf, w0, wend, first_w, last_w, out);
    __syncthreads();
    if (threadIdx.x == 0) *carry = (!last && (bit1 & 63)) ? buf[(bit1 >> 6) - w0] : 0;
    __syncthreads();
}

// pass 2c: one workgroup per segment (a block's records in kPackSegRecs pieces, then its s4
// chunks in kPackSegChunks pieces), all in parallel: tiles of the segment in order, codes into
// LDS word buffers at the bit positions a block scan gives, complete words stored once.  (One
// workgroup per block walked all 60-odd tiles of a C91 block in order: 2.1 ms per 4-block call
// of the encode pipeline, where 64 workgroups now share it.)
__global__ void __launch_bounds__(kPackThreads) k_pack_write(const uint64_t *recs, const uint64_t *chunks,
                                                             const PackStats *stats, const PackParams *params,
                                                             const PackSeg *segs, const uint64_t *seg_bits,
                                                             const uint64_t *seg_start, uint64_t *payload) {
    __shared__ uint64_t buf1[kBuf1], buf2[kBuf2], buf3[kBuf3];
    __shared__ uint64_t sh[64];
    __shared__ uint64_t carry[4];
    const uint64_t sg = blockIdx.x;
    const PackSeg g = segs[sg];
    const PackParams P = params[g.block];
    if (threadIdx.x < 4) carry[threadIdx.x] = 0;
    __syncthreads();
    if (g.kind == 0) {
        uint64_t *out[3] = {payload + P.off[0], payload + P.off[1], payload + P.off[2]};
        uint64_t pos[3], first_w[3], last_w[3];  // the same in every thread
        for (int s = 0; s < 3; s++) {
            pos[s] = seg_start[3 * sg + s];
            const uint64_t e = pos[s] + seg_bits[3 * sg + s];
            first_w[s] = pos[s] >> 6;
            last_w[s] = e ? (e - 1) >> 6 : 0;
        }
        const uint64_t beg = g.first, end = g.first + g.count;
        for (uint64_t t0 = beg; t0 < end; t0 += kPackTile) {
            uint64_t r[kPackPer];
            load_tile(recs, t0 + threadIdx.x * kPackPer, end, r);
            uint64_t v[3] = {0, 0, 0};
#pragma unroll
            for (int j = 0; j < kPackPer; j++) {
                const uint64_t i = t0 + threadIdx.x * kPackPer + j;
                if (i >= end) continue;
                const uint64_t w = r[j], flag = w >> 56;
                v[2] += rice_code(flag, P.p3).len;
                if ((flag & 2) == 0) {
                    v[0] += mb_code(w & 0xFFFFFFFFULL, P.l1, P.lim1).len;
                    v[1] += rice_code((w >> 32) & 0xFFFFFFULL, P.p2).len;
                }
            }
            uint64_t ex[3], tot[3];
            block_scan3(v, ex, tot, sh);
            const bool last = t0 + kPackTile >= end;
            // spans in words of each stream's LDS buffer: fits?  (uniform across the workgroup)
            bool fit[3];
            for (int s = 0; s < 3; s++) {
                uint64_t *buf = s == 0 ? buf1 : s == 1 ? buf2 : buf3;
                const uint64_t cap = s == 0 ? kBuf1 : s == 1 ? kBuf2 : kBuf3;
                const uint64_t w0 = pos[s] >> 6, w1 = (pos[s] + tot[s] + 63) >> 6;
                fit[s] = w1 - w0 + 1 <= cap;
                if (fit[s]) {
                    for (uint64_t i = threadIdx.x; i < cap; i += kPackThreads) buf[i] = i ? 0 : carry[s];
                } else if (threadIdx.x == 0 && carry[s]) {
                    atomicOr((unsigned long long *)&out[s][w0], (unsigned long long)bswap64(carry[s]));
                }
            }
            __syncthreads();
            uint64_t at[3] = {pos[0] + ex[0], pos[1] + ex[1], pos[2] + ex[2]};
            const uint64_t base[3] = {(pos[0] >> 6) << 6, (pos[1] >> 6) << 6, (pos[2] >> 6) << 6};
#pragma unroll
            for (int j = 0; j < kPackPer; j++) {
                const uint64_t i = t0 + threadIdx.x * kPackPer + j;
                if (i >= end) continue;
                const uint64_t w = r[j], flag = w >> 56;
                Code c[3];
                c[2] = rice_code(flag, P.p3);
                const bool lng = (flag & 2) == 0;
                if (lng) {
                    c[0] = mb_code(w & 0xFFFFFFFFULL, P.l1, P.lim1);
                    c[1] = rice_code((w >> 32) & 0xFFFFFFULL, P.p2);
                }
                for (int s = lng ? 0 : 2; s < 3; s++) {
                    if (fit[s]) or_bits_lds(s == 0 ? buf1 : s == 1 ? buf2 : buf3, at[s] + c[s].skip - base[s], c[s].v,
                                            c[s].nb);
                    else or_bits_hbm(out[s], at[s] + c[s].skip, c[s].v, c[s].nb);
                    at[s] += c[s].len;
                }
            }
            __syncthreads();
            for (int s = 0; s < 3; s++) {
                if (fit[s])
                    flush_seg_tile(s == 0 ? buf1 : s == 1 ? buf2 : buf3, pos[s], pos[s] + tot[s], last, first_w[s],
                                   last_w[s], out[s], &carry[s]);
                else
                    flush_tile_hbm(pos[s] + tot[s], last, out[s], &carry[s]);
                pos[s] += tot[s];
            }
        }
        return;
    }
    // s4: minimal binary over the segment's chunks, 2 chunks per thread per tile, in buf1
    uint64_t *out4 = payload + P.off[3];
    const uint64_t *ch = chunks + chunk_base(stats[g.block].rec_begin, g.block);
    uint64_t p4 = seg_start[3 * sg];
    const uint64_t e4 = p4 + seg_bits[3 * sg], first_w = p4 >> 6, last_w = e4 ? (e4 - 1) >> 6 : 0;
    const uint64_t c0 = g.first, c1 = g.first + g.count;
    for (uint64_t t0 = c0; t0 < c1; t0 += kS4Tile) {
        uint64_t x[kS4Per];
        uint64_t v[3] = {0, 0, 0};
#pragma unroll
        for (int j = 0; j < kS4Per; j++) {
            const uint64_t i = t0 + threadIdx.x * kS4Per + j;
            x[j] = i < c1 ? ch[i] : 0;
            if (i < c1) v[0] += mb_code(x[j], P.l4, P.lim4).len;
        }
        uint64_t ex[3], tot[3];
        block_scan3(v, ex, tot, sh);
        const bool last = t0 + kS4Tile >= c1;
        for (uint64_t i = threadIdx.x; i < (uint64_t)kBuf1; i += kPackThreads) buf1[i] = i ? 0 : carry[3];
        __syncthreads();
        uint64_t at = p4 + ex[0];
        const uint64_t base = (p4 >> 6) << 6;
#pragma unroll
        for (int j = 0; j < kS4Per; j++) {
            const uint64_t i = t0 + threadIdx.x * kS4Per + j;
            if (i >= c1) continue;
            const Code c = mb_code(x[j], P.l4, P.lim4);
            or_bits_lds(buf1, at - base, c.v, c.nb);
            at += c.len;
        }
        __syncthreads();
        flush_seg_tile(buf1, p4, p4 + tot[0], last, first_w, last_w, out4, &carry[3]);
        p4 += tot[0];
    }
}

}  // namespace

uint64_t pack_stats_scratch_words(uint64_t n_blocks, uint32_t block_reads) {
    return n_blocks * ((block_reads + kPackSegReads - 1) / kPackSegReads) * kSegStat + 8;
}

void launch_pack_stats(const uint64_t *recs, const uint64_t *roffs, uint64_t n_reads, uint32_t block_reads,
                       uint64_t n_blocks, uint64_t *chunks, uint64_t chunk_words, uint64_t *scratch,
                       PackStats *stats, hipStream_t s) {
    if (!n_blocks) return;
    const uint64_t spb = (block_reads + kPackSegReads - 1) / kPackSegReads, n_segs = n_blocks * spb;
    (void)hipMemsetAsync(chunks, 0, chunk_words * 8, s);  // shared chunks are OR-ed in
    hipLaunchKernelGGL(k_pstat_seg, dim3((uint32_t)n_segs), dim3(kPackThreads), 0, s, recs, roffs, n_reads,
                       block_reads, spb, scratch);
    hipLaunchKernelGGL(k_pstat_block, dim3((uint32_t)((n_blocks + 255) / 256)), dim3(256), 0, s, roffs, n_reads,
                       block_reads, n_blocks, spb, scratch, stats);
    hipLaunchKernelGGL(k_pstat_chunks, dim3((uint32_t)n_segs), dim3(kPackThreads), 0, s, recs, roffs, n_reads,
                       block_reads, spb, (const uint64_t *)scratch, (const PackStats *)stats, chunks);
    hipLaunchKernelGGL(k_pstat_max4, dim3((uint32_t)n_blocks), dim3(kPackThreads), 0, s, (const uint64_t *)chunks,
                       stats);
}

void launch_pack_write(const uint64_t *recs, const uint64_t *chunks, const PackStats *stats,
                       const PackParams *params, uint64_t n_blocks, const PackSeg *segs, uint64_t n_segs,
                       uint64_t *seg_bits, uint64_t *seg_start, uint64_t *payload, uint64_t *bits_out,
                       hipStream_t s) {
    if (n_segs)
        hipLaunchKernelGGL(k_pack_seglen, dim3((uint32_t)n_segs), dim3(kPackThreads), 0, s, recs, chunks, stats,
                           params, segs, seg_bits);
    hipLaunchKernelGGL(k_pack_segscan, dim3((uint32_t)((n_blocks + 255) / 256)), dim3(256), 0, s, params, segs,
                       n_blocks, (const uint64_t *)seg_bits, seg_start, bits_out);
    if (n_segs)
        hipLaunchKernelGGL(k_pack_write, dim3((uint32_t)n_segs), dim3(kPackThreads), 0, s, recs, chunks, stats,
                           params, segs, (const uint64_t *)seg_bits, (const uint64_t *)seg_start, payload);
}

}  // namespace ntc
