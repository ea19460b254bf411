// SBWT subset matrix + LCS built on the GPU (ntc_build_index_device[_ex]): the same index
// as the host builder (sbwt_build.cpp, the stand-in for kbo::build, src/main.rs:111-134) --
// identical rows, C and LCS -- in passes whose device memory stays inside a budget, the
// counterpart of kbo's BuildOpts { mem_gb, temp_dir, dedup_batches } (src/cli.rs:56-61,
// src/main.rs:111-134).
//
// Keys.  A node is its characters read right to left (last character first), 2 bits each,
// MSB first in W = ceil(2k / 64) words, plus its count of real (non-$) characters: sorting
// by (words, count) is colex order with $ < A (sbwt_build.cpp's Node<W>).  A key's BUCKET is
// its first m characters (m = min(7, k - 1)): the node's last m, the most significant part of
// colex order, so nodes sorted bucket range by bucket range and concatenated are in global
// order.  Every pass below works on one contiguous range of buckets (a PARTITION) sized so
// that its keys fit the budget; partitions are independent, so their sorts never see more
// than 2^32 keys (the radix sort's uint32 permutation) whatever the input size.
//
//   plan      one pass over the sequence (streamed to the device in chunks when it does not
//             fit) counts the k-mer occurrences per bucket (LDS histograms): partitions of
//             at most `cap` occurrences;
//   k-mers    per partition, per sequence chunk: the windows whose forward or reverse-
//             complement key falls in the partition are appended to a device accumulator
//             (wave-aggregated atomics); an accumulator that fills is sorted and deduplicated
//             in place (kbo's dedup batches) and the chunk re-run; the sorted unique k-mers go
//             to the KEY STORE (host memory, or files under --temp-dir past the host budget);
//   sources   k-mer x has an in-neighbour iff x[0..k-1] is the (k-1)-suffix of a k-mer.  The
//             suffixes of partition Q are Q's own keys (masked); the x asking about them have
//             buckets c.(Q's buckets / 4), four contiguous ranges of the key store, streamed
//             in slices and answered by binary search; each x is answered by exactly one Q;
//   nodes     node partitions (k-mers + dummies $^(k-r) x[0..r] of sources + the root) planned
//             from the unique k-mers' and the dummies' bucket counts, each assembled, sorted
//             and deduplicated on the device, then kept in the NODE STORE;
//   LCS       per node partition, with the last node of the previous one as the carry;
//   labels    node u = x.c sets bit c of the first node of x's (k-1)-suffix group, found by
//             binary search over the group-first nodes of the partition holding x's bucket;
//             the u asking come from the node store's four ranges as above.  Rows are set in
//             a device slice per partition and OR-ed into the host rows (edge words shared).
// SoA layout on the device: word j of key i at keys[j * stride + i]; counts in a byte array.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kernels.h"
#include "ntc_internal.h"

namespace ntc {

namespace {

constexpr uint32_t kMaxBucketChars = 7;  // 16,384 buckets: a 64 KB LDS histogram of u32

__device__ __forceinline__ int dev_code(uint8_t b) {
    switch (b) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return -1;
    }
}

__host__ __device__ __forceinline__ uint32_t bucket_of(uint64_t w0, uint32_t m) {
    return m ? (uint32_t)(w0 >> (64 - 2 * m)) : 0u;
}

// mask keeping characters t < m of a W-word key
template <int W>
__device__ __forceinline__ uint64_t char_mask_w(uint32_t m, int j) {
    const int64_t c = (int64_t)m - 32 * j;
    return c >= 32 ? ~0ULL : c <= 0 ? 0ULL : ~0ULL << (64 - 2 * c);
}

template <int W>
__device__ __forceinline__ void load_key(const uint64_t *keys, uint64_t stride, uint64_t i, uint64_t (&w)[W]) {
#pragma unroll
    for (int j = 0; j < W; j++) w[j] = keys[(uint64_t)j * stride + i];
}

// characters shifted towards t = 0 by s (the first s dropped)
template <int W>
__device__ __forceinline__ void shl_chars(uint64_t (&w)[W], uint32_t s) {
    const uint32_t bits = 2 * s, ws = bits / 64, bs = bits % 64;
#pragma unroll
    for (int j = 0; j < W; j++) {
        const uint64_t hi = (j + (int)ws < W) ? w[j + ws] : 0;
        const uint64_t lo = (j + (int)ws + 1 < W) ? w[j + ws + 1] : 0;
        w[j] = bs ? ((hi << bs) | (lo >> (64 - bs))) : hi;
    }
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// ---- sequence chunks ------------------------------------------------------------------
// A chunk buffer holds sequence bytes [g0, g0 + len) (absolute positions of the caller's
// concatenation); windows ENDING at p in [p0, p1) are the chunk's, and g0 <= p0 - (k - 1)
// unless p0 is near the start.  cb[i]: 2-bit code | 4 (not ACGT) | 8 (a sequence starts
// here); ok[i] = 1 when the k-window ending at g0 + i is all ACGT inside one sequence.
__global__ __launch_bounds__(256) void k_codes(uint8_t *cb, uint64_t len) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= len) return;
    const int c = dev_code(cb[i]);
    cb[i] = c < 0 ? 4 : (uint8_t)c;
}
__global__ __launch_bounds__(256) void k_mark_starts(uint8_t *cb, const uint64_t *starts, uint64_t n, uint64_t g0) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) cb[starts[i] - g0] |= 8;
}
__global__ __launch_bounds__(256) void k_valid(const uint8_t *cb, uint64_t g0, uint64_t p0, uint64_t p1, uint32_t k,
                                               uint8_t *ok) {
    const uint64_t p = p0 + (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= p1) return;
    const uint64_t i = p - g0;
    uint8_t v = p + 1 >= g0 + k;  // the window lies inside the buffer
    for (uint32_t t = 0; v && t < k; t++) {
        const uint8_t x = cb[i - t];
        if ((x & 4) || (t + 1 < k && (x & 8))) v = 0;  // a start inside the window (not at its first base)
    }
    ok[i] = v;
}

__device__ __forceinline__ void kmer_buckets(const uint8_t *cb, uint64_t i, uint32_t k, uint32_t m, uint32_t &bf,
                                             uint32_t &bg) {
    bf = bg = 0;
    for (uint32_t t = 0; t < m; t++) {
        const uint32_t cf = t < k ? (cb[i - t] & 3) : 0;
        const uint32_t cg = t < k ? 3 - (cb[i - k + 1 + t] & 3) : 0;
        bf = (bf << 2) | cf;
        bg = (bg << 2) | cg;
    }
}

// occurrences per bucket of the chunk's windows (forward and, with revcomp, reverse complement)
__global__ __launch_bounds__(1024) void k_hist_kmers(const uint8_t *cb, const uint8_t *ok, uint64_t g0, uint64_t p0,
                                                     uint64_t p1, uint32_t k, uint32_t rc, uint32_t m,
                                                     unsigned long long *hist) {
    __shared__ uint32_t lh[1u << (2 * kMaxBucketChars)];
    const uint32_t nb = 1u << (2 * m);
    for (uint32_t b = threadIdx.x; b < nb; b += 1024) lh[b] = 0;
    __syncthreads();
    for (uint64_t p = p0 + (uint64_t)blockIdx.x * 1024 + threadIdx.x; p < p1; p += (uint64_t)gridDim.x * 1024) {
        const uint64_t i = p - g0;
        if (!ok[i]) continue;
        uint32_t bf, bg;
        kmer_buckets(cb, i, k, m, bf, bg);
        atomicAdd(&lh[bf], 1u);
        if (rc) atomicAdd(&lh[bg], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += 1024)
        if (lh[b]) atomicAdd(&hist[b], (unsigned long long)lh[b]);
}

// append n_mine keys of this lane after the wave's earlier lanes' (one atomic per wave);
// returns the lane's first slot
__device__ __forceinline__ uint64_t wave_append(uint32_t n_mine, unsigned long long *cnt) {
    uint32_t incl = n_mine;
    const uint32_t lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(incl, d, 64);
        if ((int)lane >= d) incl += t;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    unsigned long long base = 0;
    if (lane == 63 && total) base = atomicAdd(cnt, (unsigned long long)total);
    base = __shfl(base, 63, 64);
    return base + incl - n_mine;
}

// Block-level append: kEmitPer positions per thread (strided by the block, coalesced), the
// block's in-range keys counted first (a 2-bit mask per position kept in a register), one
// atomic per block of 4096 positions, then the keys built and stored.  (A wave-level atomic
// on the one counter serialised at ~170 M/s and bounded the pass.)
constexpr uint32_t kEmitPer = 16;
constexpr uint32_t kEmitTile = 256 * kEmitPer;

// exclusive block scan of one u32 per thread (256 threads); *total for the block
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t *sh, uint32_t &total) {
    const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(incl, d, 64);
        if ((int)lane >= d) incl += t;
    }
    if (lane == 63) sh[wid] = incl;
    __syncthreads();
    uint32_t base = 0;
    total = 0;
    for (uint32_t w = 0; w < 4; w++) {
        base += w < wid ? sh[w] : 0;
        total += sh[w];
    }
    __syncthreads();
    return base + incl - v;
}

template <int W>
__global__ __launch_bounds__(256) void k_emit_kmers(const uint8_t *cb, const uint8_t *ok, uint64_t g0, uint64_t p0,
                                                    uint64_t p1, uint32_t k, uint32_t rc, uint32_t m, uint32_t blo,
                                                    uint32_t bhi, uint64_t *acc, uint64_t stride,
                                                    unsigned long long *cnt) {
    __shared__ uint32_t sh[4];
    __shared__ unsigned long long sbase;
    const uint64_t t0 = p0 + (uint64_t)blockIdx.x * kEmitTile;
    uint32_t mask = 0, mine = 0;  // bits 2j, 2j + 1: forward / reverse complement of position j
#pragma unroll
    for (uint32_t j = 0; j < kEmitPer; j++) {
        const uint64_t p = t0 + threadIdx.x + 256 * j;
        if (p >= p1) continue;
        const uint64_t i = p - g0;
        if (!ok[i]) continue;
        uint32_t bf, bg;
        kmer_buckets(cb, i, k, m, bf, bg);
        const uint32_t inf = bf >= blo && bf < bhi, ing = rc && bg >= blo && bg < bhi;
        mask |= (inf | (ing << 1)) << (2 * j);
        mine += inf + ing;
    }
    uint32_t total;
    const uint32_t ex = block_excl_scan256(mine, sh, total);
    if (threadIdx.x == 0) sbase = total ? atomicAdd(cnt, (unsigned long long)total) : 0;
    __syncthreads();
    uint64_t slot = sbase + ex;
    while (mask) {
        const uint32_t j = (uint32_t)__builtin_ctz(mask) / 2;
        const uint32_t two = (mask >> (2 * j)) & 3u;
        mask &= ~(3u << (2 * j));
        const uint64_t i = t0 + threadIdx.x + 256 * j - g0;
        uint64_t f[W], g[W];
#pragma unroll
        for (int q = 0; q < W; q++) f[q] = g[q] = 0;
        for (uint32_t t = 0; t < k; t++) {
            // forward: character t is seq[p - t]; reverse complement: t is the complement of
            // seq[p - k + 1 + t]
            const uint64_t c = cb[i - t] & 3;
            const uint64_t r = 3 - (uint64_t)(cb[i - k + 1 + t] & 3);
            const uint32_t jj = t / 32, sft = 62 - 2 * (t % 32);
#pragma unroll
            for (int q = 0; q < W; q++)
                if (q == (int)jj) {
                    f[q] |= c << sft;
                    g[q] |= r << sft;
                }
        }
        if (two & 1) {
            if (slot < stride)
#pragma unroll
                for (int q = 0; q < W; q++) acc[(uint64_t)q * stride + slot] = f[q];
            slot++;
        }
        if (two & 2) {
            if (slot < stride)
#pragma unroll
                for (int q = 0; q < W; q++) acc[(uint64_t)q * stride + slot] = g[q];
            slot++;
        }
    }
}

// ---- sort / unique ----------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_iota(uint32_t *v, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}
__global__ __launch_bounds__(256) void k_gather_u64(const uint64_t *src, const uint32_t *perm, uint64_t n,
                                                    uint64_t *dst) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) dst[i] = src[perm[i]];
}
__global__ __launch_bounds__(256) void k_gather_u8(const uint8_t *src, const uint32_t *perm, uint64_t n,
                                                   uint8_t *dst) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) dst[i] = src[perm[i]];
}
// 1 where node i differs from node i - 1 (words or count)
template <int W>
__global__ __launch_bounds__(256) void k_uniq_flags(const uint64_t *keys, uint64_t stride, const uint8_t *len,
                                                    uint64_t n, uint32_t *flag) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t d = i == 0;
    if (i) {
#pragma unroll
        for (int j = 0; j < W; j++) d |= keys[(uint64_t)j * stride + i] != keys[(uint64_t)j * stride + i - 1];
        if (len) d |= len[i] != len[i - 1];
    }
    flag[i] = d;
}
template <int W>
__global__ __launch_bounds__(256) void k_compact(const uint64_t *keys, uint64_t stride, const uint8_t *len,
                                                 uint64_t n, const uint32_t *flag, const uint64_t *rank,
                                                 uint64_t ostride, uint64_t *okeys, uint8_t *olen) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n || !flag[i]) return;
    const uint64_t o = rank[i];
#pragma unroll
    for (int j = 0; j < W; j++) okeys[(uint64_t)j * ostride + o] = keys[(uint64_t)j * stride + i];
    if (len) olen[o] = len[i];
}

// keys per bucket of sorted keys (word 0)
__global__ __launch_bounds__(1024) void k_hist_keys(const uint64_t *w0, uint64_t n, uint32_t m,
                                                    unsigned long long *hist) {
    __shared__ uint32_t lh[1u << (2 * kMaxBucketChars)];
    const uint32_t nb = 1u << (2 * m);
    for (uint32_t b = threadIdx.x; b < nb; b += 1024) lh[b] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 1024)
        atomicAdd(&lh[bucket_of(w0[i], m)], 1u);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += 1024)
        if (lh[b]) atomicAdd(&hist[b], (unsigned long long)lh[b]);
}

// ---- sources ----------------------------------------------------------------------------
// x (candidate) asks whether x[0..k-1] is a (k-1)-suffix among the sorted k-mers K of the
// partition owning that suffix's bucket [qlo, qhi): flag 2 = source, 1 = has an in-neighbour,
// 0 = another partition answers it
template <int W>
__global__ __launch_bounds__(256) void k_src_check(const uint64_t *xk, uint64_t xstride, uint64_t nx,
                                                   const uint64_t *K, uint64_t nK, uint32_t k, uint32_t m,
                                                   uint32_t qlo, uint32_t qhi, uint32_t *flag) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nx) return;
    uint64_t key[W];
    load_key<W>(xk, xstride, i, key);
    shl_chars<W>(key, 1);
    const uint32_t qb = bucket_of(key[0], m);
    if (qb < qlo || qb >= qhi) {
        flag[i] = 0;
        return;
    }
    uint64_t lo = 0, hi = nK;  // first k-mer whose words are >= key
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        int cmp = 0;
#pragma unroll
        for (int j = 0; j < W; j++) {
            const uint64_t a = K[(uint64_t)j * nK + mid];
            if (cmp == 0 && a != key[j]) cmp = a < key[j] ? -1 : 1;
        }
        if (cmp < 0) lo = mid + 1;
        else hi = mid;
    }
    uint32_t found = lo < nK;
    if (found) {
#pragma unroll
        for (int j = 0; j < W; j++)
            if ((K[(uint64_t)j * nK + lo] & char_mask_w<W>(k - 1, j)) != key[j]) found = 0;
    }
    flag[i] = found ? 1 : 2;
}
template <int W>
__global__ __launch_bounds__(256) void k_src_compact(const uint64_t *xk, uint64_t xstride, uint64_t nx,
                                                     const uint32_t *flag, uint64_t *out, unsigned long long *cnt) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t mine = i < nx && flag[i] == 2;
    const uint64_t slot = wave_append(mine, cnt);
    if (!mine) return;
#pragma unroll
    for (int j = 0; j < W; j++) out[slot * W + j] = xk[(uint64_t)j * xstride + i];  // AoS
}

// ---- dummies ----------------------------------------------------------------------------
// dummy r (r = 1..k-1 real characters) of source x: $^(k-r) x[0..r]
template <int W>
__device__ __forceinline__ void dummy_key(const uint64_t (&x)[W], uint32_t k, uint32_t r, uint64_t (&d)[W]) {
#pragma unroll
    for (int j = 0; j < W; j++) d[j] = x[j];
    shl_chars<W>(d, k - r);
#pragma unroll
    for (int j = 0; j < W; j++) d[j] &= char_mask_w<W>(r, j);
}
template <int W>
__global__ __launch_bounds__(256) void k_hist_dummies(const uint64_t *src, uint64_t ns, uint32_t k, uint32_t m,
                                                      unsigned long long *hist) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= ns) return;
    uint64_t x[W], d[W];
#pragma unroll
    for (int j = 0; j < W; j++) x[j] = src[i * W + j];
    for (uint32_t r = 1; r < k; r++) {
        dummy_key<W>(x, k, r, d);
        atomicAdd(&hist[bucket_of(d[0], m)], 1ULL);
    }
}
template <int W>
__global__ __launch_bounds__(256) void k_emit_dummies(const uint64_t *src, uint64_t ns, uint32_t k, uint32_t m,
                                                      uint32_t blo, uint32_t bhi, uint64_t *acc, uint8_t *alen,
                                                      uint64_t stride, unsigned long long *cnt) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint64_t x[W], d[W];
    uint32_t mine = 0;
    if (i < ns) {
#pragma unroll
        for (int j = 0; j < W; j++) x[j] = src[i * W + j];
        for (uint32_t r = 1; r < k; r++) {
            dummy_key<W>(x, k, r, d);
            const uint32_t b = bucket_of(d[0], m);
            mine += b >= blo && b < bhi;
        }
    }
    uint64_t s = wave_append(mine, cnt);
    if (!mine) return;
    for (uint32_t r = 1; r < k; r++) {
        dummy_key<W>(x, k, r, d);
        const uint32_t b = bucket_of(d[0], m);
        if (b < blo || b >= bhi) continue;
        if (s < stride) {
#pragma unroll
            for (int j = 0; j < W; j++) acc[(uint64_t)j * stride + s] = d[j];
            alen[s] = (uint8_t)r;
        }
        s++;
    }
}

// ---- LCS, groups, labels ----------------------------------------------------------------
// nodes[0] is the previous partition's last node (has_prev) and nodes[1 + i] local node i;
// lcs[i] = longest common suffix of nodes i - 1 and i (global), capped at 255; gflag = first
// node of its (k-1)-suffix group
template <int W>
__global__ __launch_bounds__(256) void k_lcs(const uint64_t *keys, const uint8_t *len, uint64_t stride, uint64_t n,
                                             uint32_t has_prev, uint8_t *lcs, uint32_t *gflag, uint32_t k) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t l = 0;
    if (i || has_prev) {
        const uint64_t a = i, b = i + 1;  // buffer slots of node i - 1 and node i
        uint32_t common = 32 * W;
        bool done = false;
#pragma unroll
        for (int j = 0; j < W; j++) {
            const uint64_t d = keys[(uint64_t)j * stride + b] ^ keys[(uint64_t)j * stride + a];
            if (!done && d) {
                common = 32 * j + (uint32_t)__builtin_clzll(d) / 2;
                done = true;
            }
        }
        l = min(common, min((uint32_t)len[b], (uint32_t)len[a]));
        l = min(l, 255u);
    }
    lcs[i] = (uint8_t)l;
    gflag[i] = (i == 0 && !has_prev) || l < k - 1;
}
__global__ __launch_bounds__(256) void k_gfirst(const uint32_t *gflag, const uint64_t *rank, uint64_t n,
                                                uint32_t *gfirst) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n && gflag[i]) gfirst[rank[i]] = (uint32_t)i;
}
// compare (words & (k-1)-mask, min(count, k-1)) of group-first node g against (key, klen)
template <int W>
__device__ __forceinline__ int group_cmp(const uint64_t *keys, const uint8_t *len, uint64_t stride, uint64_t g,
                                         uint32_t k, const uint64_t (&key)[W], uint32_t klen) {
#pragma unroll
    for (int j = 0; j < W; j++) {
        const uint64_t a = keys[(uint64_t)j * stride + g] & char_mask_w<W>(k - 1, j);
        if (a != key[j]) return a < key[j] ? -1 : 1;
    }
    const uint32_t gl = min((uint32_t)len[g], k - 1);
    return gl == klen ? 0 : (gl < klen ? -1 : 1);
}
// candidate u = x.c (last character c, x its first count - 1 characters) whose group bucket
// lies in [qlo, qhi) labels the first node of the group equal to x with c: bit (gi + bit0) of
// the partition's row slice
template <int W>
__global__ __launch_bounds__(256) void k_labels(const uint64_t *uk, const uint8_t *ul, uint64_t ustride, uint64_t nu,
                                                const uint64_t *nodes, const uint8_t *nlen, uint64_t nstride,
                                                const uint32_t *gfirst, uint64_t G, uint32_t k, uint32_t m,
                                                uint32_t qlo, uint32_t qhi, unsigned long long *rows, uint64_t nw,
                                                uint64_t bit0, unsigned int *bad) {
    const uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= nu || ul[u] == 0) return;
    uint64_t key[W];
    load_key<W>(uk, ustride, u, key);
    const uint32_t c = (uint32_t)(key[0] >> 62);
    shl_chars<W>(key, 1);
    const uint32_t qb = bucket_of(key[0], m);
    if (qb < qlo || qb >= qhi) return;
    const uint32_t klen = (uint32_t)ul[u] - 1;
    uint64_t lo = 0, hi = G;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (group_cmp<W>(nodes, nlen, nstride, gfirst[mid], k, key, klen) < 0) lo = mid + 1;
        else hi = mid;
    }
    if (lo >= G || group_cmp<W>(nodes, nlen, nstride, gfirst[lo], k, key, klen) != 0) {
        atomicOr(bad, 1u);
        return;
    }
    const uint64_t b = (uint64_t)gfirst[lo] + bit0;
    atomicOr(rows + (uint64_t)c * nw + (b >> 6), 1ULL << (b & 63));
}

inline dim3 grid(uint64_t n) { return dim3((uint32_t)std::max<uint64_t>(1, (n + 255) / 256)); }

// ---- device memory ----------------------------------------------------------------------
// Device memory of one build.  Buffers of 1 MB and more are cached when released and
// handed out again to requests of up to their size (down to half of it): every pass
// allocates the same few large buffers, and fresh hipMalloc'd memory of tens of GB made a
// partition's sort up to 15x slower than the same sort in reused memory (3 Gbp build,
// NTC_BUILD_TRACE).  The cache is dropped whenever holding it would pass the budget.
struct Arena {
    std::vector<std::pair<void *, uint64_t>> ptrs, cache;
    uint64_t live = 0, cached = 0, peak = 0, budget = ~0ULL;
    static constexpr uint64_t kCacheMin = 1ULL << 20;
    ~Arena() {
        for (auto &p : ptrs) (void)hipFree(p.first);
        drop_cache();
    }
    void drop_cache() {
        for (auto &p : cache) (void)hipFree(p.first);
        cache.clear();
        cached = 0;
    }
    template <class T>
    T *get(uint64_t count) {
        void *p = nullptr;
        uint64_t bytes = std::max<uint64_t>(count * sizeof(T), 64);
        if (bytes >= kCacheMin) {
            bytes = (bytes + kCacheMin - 1) & ~(kCacheMin - 1);
            size_t best = cache.size();
            for (size_t i = 0; i < cache.size(); i++)
                if (cache[i].second >= bytes && cache[i].second <= 2 * bytes &&
                    (best == cache.size() || cache[i].second < cache[best].second))
                    best = i;
            if (best < cache.size()) {
                auto e = cache[best];
                cache.erase(cache.begin() + (long)best);
                cached -= e.second;
                ptrs.push_back(e);
                live += e.second;
                peak = std::max(peak, live + cached);
                return (T *)e.first;
            }
            if (live + cached + bytes > budget) drop_cache();
        }
        if (hipMalloc(&p, bytes) != hipSuccess) {
            (void)hipGetLastError();
            if (cache.empty()) return nullptr;
            drop_cache();
            if (hipMalloc(&p, bytes) != hipSuccess) {
                (void)hipGetLastError();
                return nullptr;
            }
        }
        ptrs.push_back({p, bytes});
        live += bytes;
        peak = std::max(peak, live + cached);
        return (T *)p;
    }
    void release(void *p) {
        if (!p) return;
        for (auto it = ptrs.begin(); it != ptrs.end(); ++it)
            if (it->first == p) {
                live -= it->second;
                if (it->second >= kCacheMin) {
                    cache.push_back(*it);
                    cached += it->second;
                } else {
                    (void)hipFree(p);
                }
                ptrs.erase(it);
                return;
            }
    }
};

#define BTRY(expr)                                                                   \
    do {                                                                             \
        hipError_t e_ = (expr);                                                      \
        if (e_ != hipSuccess) {                                                      \
            err = std::string("hip: ") + #expr + ": " + hipGetErrorString(e_);      \
            return false;                                                            \
        }                                                                            \
    } while (0)
#define BALLOC(var, T, count)                                                                         \
    T *var = A.get<T>(count);                                                                         \
    if (!var) {                                                                                       \
        err = "device allocation failed (" #var ", " + std::to_string((uint64_t)(count) * sizeof(T)) + \
              " bytes): lower the memory budget (-m) or free device memory";                          \
        return false;                                                                                 \
    }

// ---- host key stores ----------------------------------------------------------------------
// Sorted keys of consecutive bucket ranges, concatenated = globally sorted: SoA words (+
// counts) per partition, in host memory up to the host budget, past it in files under the
// temp dir (mapped; unlinked at once, so nothing is left behind).
class KeyStore {
  public:
    KeyStore(int W, bool with_len, uint32_t m, uint64_t host_budget, std::string dir, BuildStats *st)
        : W_(W), with_len_(with_len), budget_(host_budget), dir_(std::move(dir)), st_(st),
          bucket_cnt_((size_t)1 << (2 * m), 0) {}
    ~KeyStore() {
        for (auto &p : parts_)
            if (p.map) munmap(p.map, p.map_bytes);
    }
    uint64_t size() const { return total_; }

    // d_keys: SoA at stride n; d_hist: that partition's per-bucket counts (host)
    bool add(const uint64_t *d_keys, const uint8_t *d_len, uint64_t n, const std::vector<uint64_t> &hist,
             hipStream_t s, std::string &err) {
        Part p;
        p.base = total_;
        p.n = n;
        if (!place(p, n, err)) return false;
        if (n) {
            BTRY(hipMemcpyAsync((void *)p.wp, d_keys, (uint64_t)W_ * n * 8, hipMemcpyDeviceToHost, s));
            if (with_len_) BTRY(hipMemcpyAsync((void *)p.lp, d_len, n, hipMemcpyDeviceToHost, s));
            BTRY(hipStreamSynchronize(s));
        }
        for (size_t b = 0; b < hist.size(); b++) bucket_cnt_[b] += hist[b];
        total_ += n;
        parts_.push_back(std::move(p));
        return true;
    }
    // keep d_keys / d_len (allocated from the build's arena) as the partition itself: later
    // uploads are device-to-device copies, so a build that fits one pass never round-trips
    // its keys through the host
    void add_device(uint64_t *d_keys, uint8_t *d_len, uint64_t n, const std::vector<uint64_t> &hist) {
        Part p;
        p.base = total_;
        p.n = n;
        p.dw = d_keys;
        p.dl = d_len;
        for (size_t b = 0; b < hist.size(); b++) bucket_cnt_[b] += hist[b];
        total_ += n;
        parts_.push_back(std::move(p));
    }
    uint64_t device_bytes() const {
        uint64_t b = 0;
        for (const Part &p : parts_)
            if (p.dw) b += p.n * (8 * (uint64_t)W_ + (with_len_ ? 1 : 0));
        return b;
    }
    // device partitions -> host memory (or files past the host budget), device buffers freed
    template <class Ar>
    bool evict(Ar &A, hipStream_t s, std::string &err) {
        for (Part &p : parts_) {
            if (!p.dw) continue;
            Part h;
            if (!place(h, p.n, err)) return false;
            if (p.n) {
                BTRY(hipMemcpyAsync((void *)h.wp, p.dw, (uint64_t)W_ * p.n * 8, hipMemcpyDeviceToHost, s));
                if (with_len_) BTRY(hipMemcpyAsync((void *)h.lp, p.dl, p.n, hipMemcpyDeviceToHost, s));
                BTRY(hipStreamSynchronize(s));
            }
            A.release(p.dw);
            A.release(p.dl);
            h.base = p.base;
            h.n = p.n;
            p = std::move(h);
        }
        return true;
    }
    template <class Ar>
    void release_device(Ar &A) {
        for (Part &p : parts_) {
            A.release(p.dw);
            A.release(p.dl);
            p.dw = nullptr;
            p.dl = nullptr;
        }
    }
    void finalize() {
        bucket_begin_.assign(bucket_cnt_.size() + 1, 0);
        for (size_t b = 0; b < bucket_cnt_.size(); b++) bucket_begin_[b + 1] = bucket_begin_[b] + bucket_cnt_[b];
    }
    uint64_t bucket_begin(uint64_t b) const { return bucket_begin_[std::min<uint64_t>(b, bucket_cnt_.size())]; }
    const std::vector<uint64_t> &bucket_counts() const { return bucket_cnt_; }
    size_t n_parts() const { return parts_.size(); }
    uint64_t part_base(size_t i) const { return parts_[i].base; }
    uint64_t part_n(size_t i) const { return parts_[i].n; }

    // global keys [a, b) into a device SoA at stride (offset off), counts into d_len + off
    bool upload(uint64_t a, uint64_t b, uint64_t *d_keys, uint64_t stride, uint64_t off, uint8_t *d_len,
                hipStream_t s, std::string &err) const {
        for (const Part &p : parts_) {
            const uint64_t lo = std::max(a, p.base), hi = std::min(b, p.base + p.n);
            if (lo >= hi) continue;
            const uint64_t i0 = lo - p.base, cnt = hi - lo, o = off + (lo - a);
            const uint64_t *w = p.dw ? p.dw : p.wp;
            const uint8_t *l = p.dw ? p.dl : p.lp;
            const hipMemcpyKind kind = p.dw ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
            for (int j = 0; j < W_; j++)
                BTRY(hipMemcpyAsync(d_keys + (uint64_t)j * stride + o, w + (uint64_t)j * p.n + i0, cnt * 8, kind, s));
            if (with_len_ && d_len) BTRY(hipMemcpyAsync(d_len + o, l + i0, cnt, kind, s));
        }
        BTRY(hipStreamSynchronize(s));
        return true;
    }

  private:
    struct Part {
        uint64_t base = 0, n = 0;
        std::vector<uint64_t> w;
        std::vector<uint8_t> len;
        void *map = nullptr;
        size_t map_bytes = 0;
        const uint64_t *wp = nullptr;
        const uint8_t *lp = nullptr;
        uint64_t *dw = nullptr;  // a device-resident partition (add_device)
        uint8_t *dl = nullptr;
    };
    bool place(Part &p, uint64_t n, std::string &err) {
        const uint64_t bytes = n * (8 * (uint64_t)W_ + (with_len_ ? 1 : 0));
        uint64_t *w = nullptr;
        uint8_t *l = nullptr;
        if (budget_ && host_bytes_ + bytes > budget_ && bytes) {
            // spill: a file under the temp dir, mapped (its pages are the page cache's)
            std::string path = dir_ + "/ntcomp_build_" + std::to_string(getpid()) + "_" +
                               std::to_string((uint64_t)(uintptr_t)this) + "_" + std::to_string(files_++);
            const int fd = ::open(path.c_str(), O_RDWR | O_CREAT | O_EXCL, 0600);
            if (fd < 0) {
                err = "cannot create a partition file in " + dir_ + " (--temp-dir)";
                return false;
            }
            ::unlink(path.c_str());
            if (ftruncate(fd, (off_t)bytes) != 0) {
                ::close(fd);
                err = "cannot size a partition file in " + dir_ + " (disk full?)";
                return false;
            }
            void *mp = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            ::close(fd);
            if (mp == MAP_FAILED) {
                err = "cannot map a partition file in " + dir_;
                return false;
            }
            p.map = mp;
            p.map_bytes = bytes;
            w = (uint64_t *)mp;
            l = with_len_ ? (uint8_t *)(w + (uint64_t)W_ * n) : nullptr;
            if (st_) st_->spilled_bytes += bytes;
        } else {
            p.w.resize((uint64_t)W_ * n);
            if (with_len_) p.len.resize(n);
            w = p.w.data();
            l = with_len_ ? p.len.data() : nullptr;
            host_bytes_ += bytes;
        }
        p.wp = w;
        p.lp = l;
        return true;
    }
    int W_;
    bool with_len_;
    uint64_t budget_, host_bytes_ = 0, total_ = 0, files_ = 0;
    std::string dir_;
    BuildStats *st_;
    std::vector<uint64_t> bucket_cnt_, bucket_begin_;
    std::vector<Part> parts_;
};

// contiguous bucket ranges of at most cap (a single heavier bucket stands alone)
std::vector<std::pair<uint32_t, uint32_t>> plan_parts(const std::vector<uint64_t> &cnt, uint64_t cap) {
    std::vector<std::pair<uint32_t, uint32_t>> out;
    uint32_t lo = 0;
    uint64_t acc = 0;
    for (uint32_t b = 0; b < (uint32_t)cnt.size(); b++) {
        if (acc && acc + cnt[b] > cap) {
            out.push_back({lo, b});
            lo = b;
            acc = 0;
        }
        acc += cnt[b];
    }
    out.push_back({lo, (uint32_t)cnt.size()});
    return out;
}

// the four key-store ranges whose keys x have shl(x, 1) in buckets [qlo, qhi)
std::vector<std::pair<uint64_t, uint64_t>> asker_ranges(const KeyStore &st, uint32_t m, uint32_t qlo, uint32_t qhi) {
    std::vector<std::pair<uint64_t, uint64_t>> r;
    if (m == 0) {
        r.push_back({0, st.size()});
        return r;
    }
    const uint64_t q = 1ULL << (2 * (m - 1));
    for (uint64_t c = 0; c < 4; c++) {
        const uint64_t a = st.bucket_begin(c * q + (qlo >> 2)), b = st.bucket_begin(c * q + ((qhi - 1) >> 2) + 1);
        if (a < b) r.push_back({a, b});
    }
    return r;
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// NTC_BUILD_TRACE=1: per-step seconds on stderr (stream synchronised at each mark)
struct Tracer {
    bool on = std::getenv("NTC_BUILD_TRACE") != nullptr;
    double t = now_s();
    void mark(hipStream_t s, const char *what, uint64_t x = 0) {
        if (!on) return;
        (void)hipStreamSynchronize(s);
        const double n = now_s();
        std::fprintf(stderr, "[build] %-28s %8.3f s  %llu\n", what, n - t, (unsigned long long)x);
        t = n;
    }
};

template <int W>
struct Builder {
    hipStream_t s;
    uint32_t k, m;
    bool rc;
    std::string &err;
    Arena &A;
    BuildStats &st;
    uint64_t cap = 0;          // keys per partition pass
    uint64_t seq_chunk = 0;    // window-end positions per sequence chunk
    uint64_t host_budget = 0;
    std::string temp_dir;

    // exclusive scan of 0/1 flags -> ranks (rank[n] = total), synchronised total
    bool scan_flags(const uint32_t *flag, uint64_t n, uint64_t *rank, uint64_t &total) {
        BALLOC(tmp, uint64_t, scan_tmp_words(n) + 8);
        scan_excl_u32(flag, n, rank, tmp, s);
        BTRY(hipGetLastError());
        BTRY(hipMemcpyAsync(&total, rank + n, 8, hipMemcpyDeviceToHost, s));
        BTRY(hipStreamSynchronize(s));
        A.release(tmp);
        return true;
    }

    // sort n nodes (SoA keys at stride, optional counts) into new compact arrays (stride n);
    // LSD: counts, then words from the least significant (word W-1: only its top bits hold
    // characters).  n < 2^32: the permutation is 32-bit (partitions guarantee it).
    bool sort(const uint64_t *keys, uint64_t stride, const uint8_t *len, uint64_t n, uint64_t *&okeys,
              uint8_t *&olen) {
        const double t0 = now_s();
        struct Acc {
            double t0, &sum;
            ~Acc() { sum += now_s() - t0; }
        } acc_{t0, st.seconds_sort};
        if (n >= (1ULL << 32)) {
            err = "internal: a sort pass of 2^32 or more keys";
            return false;
        }
        BALLOC(perm, uint32_t, n);
        BALLOC(perm2, uint32_t, n);
        BALLOC(ka, uint64_t, n);
        BALLOC(kb, uint64_t, n);
        if (n) hipLaunchKernelGGL(k_iota, grid(n), dim3(256), 0, s, perm, n);
        size_t tb = 0, tb2 = 0;
        BTRY(rocprim::radix_sort_pairs(nullptr, tb, ka, kb, perm, perm2, n, 0, 64, s));
        BTRY(rocprim::radix_sort_pairs(nullptr, tb2, (uint8_t *)ka, (uint8_t *)kb, perm, perm2, n, 0, 8, s));
        BALLOC(tmp, uint8_t, std::max(tb, tb2));
        tb = std::max(tb, tb2);
        if (len && n) {
            hipLaunchKernelGGL(k_gather_u8, grid(n), dim3(256), 0, s, len, perm, n, (uint8_t *)ka);
            BTRY(rocprim::radix_sort_pairs(tmp, tb, (uint8_t *)ka, (uint8_t *)kb, perm, perm2, n, 0, 8, s));
            std::swap(perm, perm2);
        }
        for (int j = W - 1; j >= 0 && n; j--) {
            // the whole word: a begin_bit above 0 (word W-1 holds characters only in its top
            // bits) gave unsorted output for k >= 3 on this rocPRIM
            hipLaunchKernelGGL(k_gather_u64, grid(n), dim3(256), 0, s, keys + (uint64_t)j * stride, perm, n, ka);
            BTRY(rocprim::radix_sort_pairs(tmp, tb, ka, kb, perm, perm2, n, 0, 64, s));
            std::swap(perm, perm2);
        }
        A.release(tmp);
        A.release(ka);
        A.release(kb);
        A.release(perm2);
        BALLOC(ok, uint64_t, (uint64_t)W * n);
        uint8_t *ol = nullptr;
        if (len) {
            ol = A.get<uint8_t>(n);
            if (!ol) {
                err = "device allocation failed (counts): lower the memory budget (-m)";
                return false;
            }
        }
        for (int j = 0; j < W && n; j++)
            hipLaunchKernelGGL(k_gather_u64, grid(n), dim3(256), 0, s, keys + (uint64_t)j * stride, perm, n,
                               ok + (uint64_t)j * n);
        if (len && n) hipLaunchKernelGGL(k_gather_u8, grid(n), dim3(256), 0, s, len, perm, n, ol);
        BTRY(hipGetLastError());
        BTRY(hipStreamSynchronize(s));
        A.release(perm);
        okeys = ok;
        olen = ol;
        return true;
    }

    // drop repeated nodes (sorted input at stride n).  out == nullptr: into new compact
    // arrays (stride m); else into out / olen at ostride (m <= ostride)
    bool unique(const uint64_t *keys, const uint8_t *len, uint64_t n, uint64_t *&out, uint8_t *&olen,
                uint64_t ostride, uint64_t &m) {
        BALLOC(flag, uint32_t, n + 1);
        BALLOC(rank, uint64_t, n + 1);
        if (n) hipLaunchKernelGGL(k_uniq_flags<W>, grid(n), dim3(256), 0, s, keys, n, len, n, flag);
        if (!scan_flags(flag, n, rank, m)) return false;
        if (!out) {
            ostride = m;
            out = A.get<uint64_t>((uint64_t)W * m);
            olen = len ? A.get<uint8_t>(m) : nullptr;
            if (!out || (len && !olen)) {
                err = "device allocation failed (unique keys): lower the memory budget (-m)";
                return false;
            }
        }
        if (n)
            hipLaunchKernelGGL(k_compact<W>, grid(n), dim3(256), 0, s, keys, n, len, n, flag, rank, ostride, out,
                               len ? olen : nullptr);
        BTRY(hipGetLastError());
        BTRY(hipStreamSynchronize(s));
        A.release(flag);
        A.release(rank);
        return true;
    }

    // sorted unique keys of an accumulator's first n (stride acc_stride) -> new compact
    // arrays; the accumulator is released after the sort
    bool sort_unique_release(uint64_t *acc, uint64_t acc_stride, uint8_t *alen, uint64_t n, uint64_t *&out,
                             uint8_t *&olen, uint64_t &m) {
        uint64_t *sk;
        uint8_t *sl;
        if (!sort(acc, acc_stride, alen, n, sk, sl)) return false;
        A.release(acc);
        A.release(alen);
        out = nullptr;
        olen = nullptr;
        if (!unique(sk, sl, n, out, olen, 0, m)) return false;
        A.release(sk);
        A.release(sl);
        return true;
    }

    // sort + dedup the accumulator's first n keys in place (stride cap), m <- distinct count
    bool compact_acc(uint64_t *acc, uint8_t *alen, uint64_t n, uint64_t &m) {
        uint64_t *sk;
        uint8_t *sl;
        if (!sort(acc, cap, alen, n, sk, sl)) return false;
        uint64_t *o = acc;
        uint8_t *ol = alen;
        if (!unique(sk, sl, n, o, ol, cap, m)) return false;
        A.release(sk);
        A.release(sl);
        st.compactions++;
        return true;
    }

    // per-bucket counts of sorted compact keys (word 0 at w0)
    bool key_hist(const uint64_t *w0, uint64_t n, std::vector<uint64_t> &h) {
        const uint64_t nb = 1ULL << (2 * m);
        BALLOC(d, unsigned long long, nb);
        BTRY(hipMemsetAsync(d, 0, nb * 8, s));
        if (n)
            hipLaunchKernelGGL(k_hist_keys, dim3((uint32_t)std::min<uint64_t>(1024, (n + 1023) / 1024)), dim3(1024),
                               0, s, w0, n, m, d);
        h.assign(nb, 0);
        BTRY(hipMemcpyAsync(h.data(), d, nb * 8, hipMemcpyDeviceToHost, s));
        BTRY(hipStreamSynchronize(s));
        A.release(d);
        return true;
    }

    // ---- sequence chunks ------------------------------------------------------------------
    struct Seq {
        const uint8_t *h;        // caller's bytes (absolute positions)
        const uint64_t *offs;    // n_seqs + 1
        uint64_t n_seqs, P0, P1; // window ends live in [P0, P1)
    };
    struct Chunk {
        uint8_t *cb = nullptr, *ok = nullptr;
        uint64_t g0 = 0, p0 = 0, p1 = 0;
    };
    Chunk resident;  // the whole sequence when it fits one chunk

    bool load_chunk(const Seq &q, uint64_t p0, uint64_t p1, Chunk &c) {
        const uint64_t g0 = p0 >= q.P0 + (k - 1) ? p0 - (k - 1) : q.P0;
        const uint64_t len = p1 - g0;
        c.g0 = g0;
        c.p0 = p0;
        c.p1 = p1;
        BALLOC(cb, uint8_t, len);
        BALLOC(okb, uint8_t, len);
        c.cb = cb;
        c.ok = okb;
        BTRY(hipMemcpyAsync(cb, q.h + g0, len, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_codes, grid(len), dim3(256), 0, s, cb, len);
        // sequence starts inside the buffer
        const uint64_t *sb = std::lower_bound(q.offs, q.offs + q.n_seqs, g0);
        const uint64_t *se = std::lower_bound(q.offs, q.offs + q.n_seqs, g0 + len);
        const uint64_t ns = (uint64_t)(se - sb);
        if (ns) {
            BALLOC(starts, uint64_t, ns);
            BTRY(hipMemcpyAsync(starts, sb, ns * 8, hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(k_mark_starts, grid(ns), dim3(256), 0, s, cb, starts, ns, g0);
            BTRY(hipStreamSynchronize(s));
            A.release(starts);
        }
        BTRY(hipMemsetAsync(okb, 0, len, s));
        hipLaunchKernelGGL(k_valid, grid(p1 - p0), dim3(256), 0, s, cb, g0, p0, p1, k, okb);
        BTRY(hipGetLastError());
        BTRY(hipStreamSynchronize(s));
        st.seq_uploads++;
        return true;
    }
    void drop_chunk(Chunk &c) {
        if (c.cb == resident.cb) return;
        A.release(c.cb);
        A.release(c.ok);
        c.cb = c.ok = nullptr;
    }
    // f(chunk) for every sequence chunk (the resident one when the sequence fits)
    template <class F>
    bool for_chunks(const Seq &q, F f) {
        if (resident.cb) return f(resident);
        for (uint64_t p0 = q.P0; p0 < q.P1; p0 += seq_chunk) {
            Chunk c;
            if (!load_chunk(q, p0, std::min(q.P1, p0 + seq_chunk), c)) return false;
            const bool ok = f(c);
            drop_chunk(c);
            if (!ok) return false;
        }
        return true;
    }

    // k-mers of bucket range [blo, bhi) from window ends [p0, p1) of chunk c appended to acc
    // (n keys so far).  When the accumulator fills, its keys are sorted and deduplicated in
    // place and the range runs again (keys it already appended are deduplicated later), in
    // halves when the range's keys would not fit next to the distinct ones.
    bool emit_range(const Chunk &c, uint64_t p0, uint64_t p1, uint32_t blo, uint32_t bhi, uint64_t *acc,
                    unsigned long long *d_cnt, uint64_t &n) {
        if (p0 >= p1) return true;
        const uint64_t n_before = n;
        BTRY(hipMemcpyAsync(d_cnt, &n, 8, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_emit_kmers<W>, dim3((uint32_t)((p1 - p0 + kEmitTile - 1) / kEmitTile)), dim3(256), 0, s,
                           c.cb, c.ok, c.g0, p0, p1, k,
                           (uint32_t)rc, m, blo, bhi, acc, cap, d_cnt);
        BTRY(hipGetLastError());
        uint64_t got = 0;
        BTRY(hipMemcpyAsync(&got, d_cnt, 8, hipMemcpyDeviceToHost, s));
        BTRY(hipStreamSynchronize(s));
        if (got <= cap) {
            n = got;
            return true;
        }
        if (!compact_acc(acc, nullptr, cap, n)) return false;
        if (n > cap - cap / 4) {
            err = "more distinct k-mers in one bucket range than a pass holds (" + std::to_string(n) +
                  "): raise the memory budget (-m)";
            return false;
        }
        const uint64_t fresh = got - n_before;  // this range's keys
        if (n + fresh <= cap || p1 - p0 == 1) return emit_range(c, p0, p1, blo, bhi, acc, d_cnt, n);
        const uint64_t mid = p0 + (p1 - p0) / 2;
        return emit_range(c, p0, mid, blo, bhi, acc, d_cnt, n) && emit_range(c, mid, p1, blo, bhi, acc, d_cnt, n);
    }

    bool run(const uint8_t *h_seq, const uint64_t *h_offs, uint64_t n_seqs, const BuildOpts &o, HostIndex &out) {
        const double t0 = now_s();
        Tracer tr;
        Seq q{h_seq, h_offs, n_seqs, n_seqs ? h_offs[0] : 0, n_seqs ? h_offs[n_seqs] : 0};
        const uint64_t T = q.P1 - q.P0;
        const uint64_t nb = 1ULL << (2 * m);
        // ---- budget ------------------------------------------------------------------------
        uint64_t budget = o.device_budget;
        if (!budget) {
            size_t fr = 0, tot = 0;
            BTRY(hipMemGetInfo(&fr, &tot));
            budget = (uint64_t)((double)fr * 0.85);
        }
        // a pass: the accumulator (8W B per key) and the sort (permutations, key buffers,
        // rocPRIM's double buffers, the sorted copy): ~16W + 48 B per key
        const uint64_t per_key = 16 * (uint64_t)W + 48;
        const uint64_t seq_bytes = std::min<uint64_t>(budget / 4, 2 * T + 64);  // cb + ok per position
        seq_chunk = std::max<uint64_t>(1, seq_bytes / 2);
        cap = (budget - std::min(budget, seq_bytes)) / per_key;
        if (cap < 1024) {
            err = "memory budget too small for a build pass (" + std::to_string(budget) + " bytes)";
            return false;
        }
        // >= 1024 keys: a source's k - 1 <= 254 dummies fit a quarter of a pass
        if (o.max_partition_keys) cap = std::min<uint64_t>(cap, std::max<uint64_t>(1024, o.max_partition_keys));
        // and <= 2^30: rocPRIM's radix sort of 3 G pairs took 4x longer per key than of 0.7 G
        // (3 Gbp build: 6.0 against 0.7 s of sorting), so big budgets make more passes
        cap = std::min<uint64_t>(cap, 1ULL << 30);
        host_budget = o.host_budget;
        temp_dir = o.temp_dir;
        A.budget = budget;
        st.device_budget = budget;
        st.pass_keys = cap;

        // ---- 1. plan: occurrences per bucket ---------------------------------------------------
        BALLOC(d_hist, unsigned long long, nb);
        BTRY(hipMemsetAsync(d_hist, 0, nb * 8, s));
        if (T >= k) {
            if (T <= seq_chunk) {
                if (!load_chunk(q, q.P0, q.P1, resident)) return false;
            }
            const bool ok = for_chunks(q, [&](const Chunk &c) {
                const uint64_t np = c.p1 - c.p0;
                hipLaunchKernelGGL(k_hist_kmers, dim3((uint32_t)std::min<uint64_t>(2048, (np + 1023) / 1024)),
                                   dim3(1024), 0, s, c.cb, c.ok, c.g0, c.p0, c.p1, k, (uint32_t)rc, m, d_hist);
                return hipGetLastError() == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
            });
            if (!ok) {
                if (err.empty()) err = "hip: k-mer histogram failed";
                return false;
            }
        }
        std::vector<uint64_t> occ(nb);
        BTRY(hipMemcpyAsync(occ.data(), d_hist, nb * 8, hipMemcpyDeviceToHost, s));
        BTRY(hipStreamSynchronize(s));
        st.seconds_plan = now_s() - t0;
        tr.mark(s, "plan (seq + histogram)", T);
        A.release(d_hist);
        for (uint64_t x : occ) st.occurrences += x;
        const auto kparts = plan_parts(occ, cap);
        st.kmer_partitions = (uint32_t)kparts.size();

        // ---- 2. k-mers per partition -> key store ------------------------------------------------
        KeyStore kstore(W, false, m, host_budget, temp_dir, &st);
        {
            BALLOC(d_cnt, unsigned long long, 1);
            for (const auto &pr : kparts) {
                uint64_t want = 0;
                for (uint32_t b = pr.first; b < pr.second; b++) want += occ[b];
                std::vector<uint64_t> h;
                if (!want) {
                    h.assign(nb, 0);
                    if (!kstore.add(nullptr, nullptr, 0, h, s, err)) return false;
                    continue;
                }
                const uint64_t acc_keys = std::min<uint64_t>(cap, want);
                const uint64_t save_cap = cap;
                cap = acc_keys;  // the accumulator's stride
                BALLOC(acc, uint64_t, (uint64_t)W * cap);
                uint64_t n = 0;
                const bool ok = for_chunks(q, [&](const Chunk &c) {
                    return emit_range(c, c.p0, c.p1, pr.first, pr.second, acc, d_cnt, n);
                });
                if (!ok) return false;
                uint64_t *u;
                uint8_t *ul;
                uint64_t mu = 0;
                tr.mark(s, "kmers: emit", n);
                if (!sort_unique_release(acc, cap, nullptr, n, u, ul, mu)) return false;
                tr.mark(s, "kmers: sort+unique", mu);
                cap = save_cap;
                if (!key_hist(u, mu, h)) return false;
                if (kparts.size() == 1) {
                    kstore.add_device(u, nullptr, mu, h);  // one pass: the k-mers stay in HBM
                } else {
                    if (!kstore.add(u, nullptr, mu, h, s, err)) return false;
                    A.release(u);
                }
                st.kmers += mu;
                tr.mark(s, "kmers: hist+store", mu);
            }
            A.release(d_cnt);
        }
        kstore.finalize();
        if (resident.cb) {
            A.release(resident.cb);
            A.release(resident.ok);
            resident = Chunk{};
        }
        const double t1 = now_s();
        st.seconds_kmers = t1 - t0;

        // ---- 3. sources -------------------------------------------------------------------
        std::vector<uint64_t> sources;  // AoS, W words each
        if (kstore.size()) {
            BALLOC(d_cnt, unsigned long long, 1);
            for (size_t pi = 0; pi < kstore.n_parts(); pi++) {
                const uint64_t nK = kstore.part_n(pi);
                if (!nK) continue;
                const uint32_t qlo = kparts[pi].first, qhi = kparts[pi].second;
                BALLOC(K, uint64_t, (uint64_t)W * nK);
                if (!kstore.upload(kstore.part_base(pi), kstore.part_base(pi) + nK, K, nK, 0, nullptr, s, err))
                    return false;
                const uint64_t slice = std::max<uint64_t>(1024, std::min<uint64_t>(cap, 1ULL << 26));
                BALLOC(xk, uint64_t, (uint64_t)W * slice);
                BALLOC(flag, uint32_t, slice);
                BALLOC(so, uint64_t, (uint64_t)W * slice);
                for (const auto &r : asker_ranges(kstore, m, qlo, qhi))
                    for (uint64_t a = r.first; a < r.second; a += slice) {
                        const uint64_t b = std::min(r.second, a + slice), nx = b - a;
                        if (!kstore.upload(a, b, xk, slice, 0, nullptr, s, err)) return false;
                        hipLaunchKernelGGL(k_src_check<W>, grid(nx), dim3(256), 0, s, xk, slice, nx, K, nK, k, m, qlo,
                                           qhi, flag);
                        BTRY(hipMemsetAsync(d_cnt, 0, 8, s));
                        hipLaunchKernelGGL(k_src_compact<W>, grid(nx), dim3(256), 0, s, xk, slice, nx, flag, so,
                                           d_cnt);
                        BTRY(hipGetLastError());
                        uint64_t ns = 0;
                        BTRY(hipMemcpyAsync(&ns, d_cnt, 8, hipMemcpyDeviceToHost, s));
                        BTRY(hipStreamSynchronize(s));
                        if (ns) {
                            const size_t at = sources.size();
                            sources.resize(at + ns * W);
                            BTRY(hipMemcpyAsync(sources.data() + at, so, ns * W * 8, hipMemcpyDeviceToHost, s));
                            BTRY(hipStreamSynchronize(s));
                        }
                    }
                A.release(xk);
                A.release(flag);
                A.release(so);
                A.release(K);
            }
            A.release(d_cnt);
        }
        const uint64_t nsrc = sources.size() / W;
        st.sources = nsrc;
        tr.mark(s, "sources", nsrc);
        const double t2 = now_s();
        st.seconds_sources = t2 - t1;

        // ---- 4. node partitions: k-mers + dummies + root --------------------------------------
        uint64_t *d_src = nullptr;
        std::vector<uint64_t> ncnt = kstore.bucket_counts();
        ncnt[0] += 1;  // the root ($^k: all-zero words)
        if (nsrc) {
            d_src = A.get<uint64_t>(nsrc * W);
            if (!d_src) {
                err = "device allocation failed (sources): lower the memory budget (-m)";
                return false;
            }
            BTRY(hipMemcpyAsync(d_src, sources.data(), nsrc * W * 8, hipMemcpyHostToDevice, s));
            BALLOC(dh, unsigned long long, nb);
            BTRY(hipMemsetAsync(dh, 0, nb * 8, s));
            hipLaunchKernelGGL(k_hist_dummies<W>, grid(nsrc), dim3(256), 0, s, d_src, nsrc, k, m, dh);
            std::vector<uint64_t> dcnt(nb);
            BTRY(hipMemcpyAsync(dcnt.data(), dh, nb * 8, hipMemcpyDeviceToHost, s));
            BTRY(hipStreamSynchronize(s));
            A.release(dh);
            for (uint64_t b = 0; b < nb; b++) ncnt[b] += dcnt[b];
        }
        std::vector<uint64_t>().swap(sources);
        const auto nparts = plan_parts(ncnt, cap);
        st.node_partitions = (uint32_t)nparts.size();
        {
            uint64_t most = 0;
            for (const auto &pr : nparts) {
                uint64_t w = 0;
                for (uint32_t b = pr.first; b < pr.second; b++) w += ncnt[b];
                most = std::max(most, std::min(w, cap));
            }
            if (kstore.device_bytes() && A.live + per_key * most > budget && !kstore.evict(A, s, err)) return false;
        }
        KeyStore nstore(W, true, m, host_budget, temp_dir, &st);
        {
            BALLOC(d_cnt, unsigned long long, 1);
            for (const auto &pr : nparts) {
                uint64_t want = 0;
                for (uint32_t b = pr.first; b < pr.second; b++) want += ncnt[b];
                const uint64_t ka = kstore.bucket_begin(pr.first), kb = kstore.bucket_begin(pr.second);
                const uint64_t save_cap = cap;
                cap = std::max<uint64_t>(std::min<uint64_t>(save_cap, want), kb - ka + 1);
                if (cap > 0xFFFFFFFFULL - 1024) {
                    err = "more than 2^32 k-mers in one bucket";
                    return false;
                }
                BALLOC(acc, uint64_t, (uint64_t)W * cap);
                BALLOC(alen, uint8_t, cap);
                uint64_t n = 0;
                if (kb > ka) {
                    if (!kstore.upload(ka, kb, acc, cap, 0, nullptr, s, err)) return false;
                    BTRY(hipMemsetAsync(alen, (int)k, kb - ka, s));
                    n = kb - ka;
                }
                if (pr.first == 0) {  // the root
                    for (int j = 0; j < W; j++) BTRY(hipMemsetAsync(acc + (uint64_t)j * cap + n, 0, 8, s));
                    BTRY(hipMemsetAsync(alen + n, 0, 1, s));
                    n++;
                }
                // dummies of this bucket range, in source slices; a full accumulator is
                // compacted and the slice re-run
                // (an accumulator sized for every candidate never fills: one launch)
                const uint64_t sslice = want <= cap ? std::max<uint64_t>(1, nsrc)
                                                        : std::max<uint64_t>(1, cap / (4 * (uint64_t)k));
                for (uint64_t a = 0; a < nsrc; a += sslice) {
                    const uint64_t ns = std::min(nsrc, a + sslice) - a;
                    for (int attempt = 0;; attempt++) {
                        BTRY(hipMemcpyAsync(d_cnt, &n, 8, hipMemcpyHostToDevice, s));
                        hipLaunchKernelGGL(k_emit_dummies<W>, grid(ns), dim3(256), 0, s, d_src + a * W, ns, k, m,
                                           pr.first, pr.second, acc, alen, cap, d_cnt);
                        BTRY(hipGetLastError());
                        uint64_t got = 0;
                        BTRY(hipMemcpyAsync(&got, d_cnt, 8, hipMemcpyDeviceToHost, s));
                        BTRY(hipStreamSynchronize(s));
                        if (got <= cap) {
                            n = got;
                            break;
                        }
                        if (!compact_acc(acc, alen, cap, n)) return false;
                        if (attempt >= 2 || n > cap - cap / 4) {
                            err = "more distinct dummy nodes in one bucket range than a pass holds: raise the "
                                  "memory budget (-m)";
                            return false;
                        }
                    }
                }
                uint64_t *u;
                uint8_t *ul;
                uint64_t mu = 0;
                tr.mark(s, "nodes: assemble", n);
                if (!sort_unique_release(acc, cap, alen, n, u, ul, mu)) return false;
                tr.mark(s, "nodes: sort+unique", mu);
                cap = save_cap;
                std::vector<uint64_t> h;
                if (!key_hist(u, mu, h)) return false;
                if (nparts.size() == 1 && A.live + (8 * (uint64_t)W + 40) * mu <= budget) {
                    nstore.add_device(u, ul, mu, h);  // one pass: the nodes stay in HBM
                } else {
                    if (!nstore.add(u, ul, mu, h, s, err)) return false;
                    A.release(u);
                    A.release(ul);
                }
            }
            A.release(d_cnt);
        }
        A.release(d_src);
        kstore.release_device(A);  // the k-mers are no longer needed
        nstore.finalize();
        const uint64_t n = nstore.size();
        st.nodes = n;
        if (n >= (1ULL << 32)) {
            err = "index too large for 32-bit colex ranks (" + std::to_string(n) + " nodes)";
            return false;
        }
        // the k-mer store is no longer needed
        tr.mark(s, "nodes: stored", n);
        const double t3 = now_s();
        st.seconds_nodes = t3 - t2;

        // ---- 5. LCS, groups, labels per node partition -------------------------------------
        const uint64_t nw = (n + 63) / 64;
        out.n = n;
        out.k = k;
        out.lcs.assign(n, 0);
        for (int c = 0; c < 4; c++) out.rows[c].assign(nw, 0);
        {
            BALLOC(bad, unsigned int, 1);
            BTRY(hipMemsetAsync(bad, 0, 4, s));
            for (size_t pi = 0; pi < nstore.n_parts(); pi++) {
                const uint64_t base = nstore.part_base(pi), nj = nstore.part_n(pi);
                if (!nj) continue;
                const uint32_t qlo = nparts[pi].first, qhi = nparts[pi].second;
                const uint64_t S = nj + 1;  // slot 0: the previous partition's last node
                BALLOC(nk, uint64_t, (uint64_t)W * S);
                BALLOC(nl, uint8_t, S);
                const uint32_t has_prev = base > 0;
                if (!nstore.upload(base - has_prev, base + nj, nk, S, 1 - has_prev, nl, s, err)) return false;
                BALLOC(lcs, uint8_t, nj);
                BALLOC(gflag, uint32_t, nj + 1);
                BALLOC(grank, uint64_t, nj + 1);
                hipLaunchKernelGGL(k_lcs<W>, grid(nj), dim3(256), 0, s, nk, nl, S, nj, has_prev, lcs, gflag, k);
                uint64_t G = 0;
                if (!scan_flags(gflag, nj, grank, G)) return false;
                BALLOC(gfirst, uint32_t, G);
                hipLaunchKernelGGL(k_gfirst, grid(nj), dim3(256), 0, s, gflag, grank, nj, gfirst);
                tr.mark(s, "labels: lcs+groups", G);
                BTRY(hipMemcpyAsync(out.lcs.data() + base, lcs, nj, hipMemcpyDeviceToHost, s));
                tr.mark(s, "labels: lcs d2h", nj);
                A.release(gflag);
                A.release(grank);
                A.release(lcs);
                // row slice: words [w0, w1) of every row
                const uint64_t w0 = base / 64, w1 = (base + nj + 63) / 64, sw = w1 - w0;
                BALLOC(rows, unsigned long long, 4 * sw);
                BTRY(hipMemsetAsync(rows, 0, 4 * sw * 8, s));
                const uint64_t slice = std::max<uint64_t>(1024, std::min<uint64_t>(cap, 1ULL << 26));
                BALLOC(uk, uint64_t, (uint64_t)W * slice);
                BALLOC(ul, uint8_t, slice);
                for (const auto &r : asker_ranges(nstore, m, qlo, qhi))
                    for (uint64_t a = r.first; a < r.second; a += slice) {
                        const uint64_t b = std::min(r.second, a + slice), nu = b - a;
                        if (!nstore.upload(a, b, uk, slice, 0, ul, s, err)) return false;
                        hipLaunchKernelGGL(k_labels<W>, grid(nu), dim3(256), 0, s, uk, ul, slice, nu, nk + 1, nl + 1,
                                           S, gfirst, G, k, m, qlo, qhi, rows, sw, base - 64 * w0, bad);
                        BTRY(hipGetLastError());
                        BTRY(hipStreamSynchronize(s));
                    }
                tr.mark(s, "labels: kernels", nj);
                std::vector<uint64_t> hr(4 * sw);
                BTRY(hipMemcpyAsync(hr.data(), rows, 4 * sw * 8, hipMemcpyDeviceToHost, s));
                BTRY(hipStreamSynchronize(s));
                for (int c = 0; c < 4; c++)
                    for (uint64_t w = 0; w < sw; w++) out.rows[c][w0 + w] |= hr[c * sw + w];
                for (void *p : {(void *)uk, (void *)ul, (void *)rows, (void *)gfirst, (void *)nk, (void *)nl})
                    A.release(p);
                tr.mark(s, "labels: rows d2h+or", sw);
            }
            unsigned int hbad = 0;
            BTRY(hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, s));
            BTRY(hipStreamSynchronize(s));
            if (hbad) {
                err = "internal: node without a predecessor group";
                return false;
            }
        }
        uint64_t before = 1;
        for (int c = 0; c < 4; c++) {
            out.C[c] = before;
            for (uint64_t w = 0; w < nw; w++) before += (uint64_t)__builtin_popcountll(out.rows[c][w]);
        }
        if (before != n) {
            err = "internal: labels do not cover every non-root node (" + std::to_string(before - 1) + " labels, " +
                  std::to_string(n) + " nodes, " + std::to_string(st.kmers) + " k-mers, " + std::to_string(nsrc) +
                  " sources)";
            return false;
        }
        st.seconds_labels = now_s() - t3;
        st.peak_device_bytes = A.peak;
        return true;
    }
};

template <int W>
bool build_w(hipStream_t s, const uint8_t *seqs, const uint64_t *offs, uint64_t n_seqs, uint32_t k, bool revcomp,
             const BuildOpts &o, HostIndex &out, BuildStats &st, std::string &err) {
    Arena A;
    const uint32_t m = k >= 2 ? std::min<uint32_t>(kMaxBucketChars, k - 1) : 0;
    Builder<W> b{s, k, m, revcomp, err, A, st};
    return b.run(seqs, offs, n_seqs, o, out);
}

}  // namespace

bool build_index_device(hipStream_t s, const uint8_t *seqs, const uint64_t *offs, uint64_t n_seqs, uint32_t k,
                        bool revcomp, const BuildOpts &o, HostIndex &out, BuildStats &st, std::string &err) {
    if (k < 1 || k > 255) {
        err = "k must be in [1, 255]";
        return false;
    }
    st = BuildStats{};
    const double t0 = now_s();
    bool ok;
    switch ((2 * k + 63) / 64) {
    case 1: ok = build_w<1>(s, seqs, offs, n_seqs, k, revcomp, o, out, st, err); break;
    case 2: ok = build_w<2>(s, seqs, offs, n_seqs, k, revcomp, o, out, st, err); break;
    case 3: ok = build_w<3>(s, seqs, offs, n_seqs, k, revcomp, o, out, st, err); break;
    case 4: ok = build_w<4>(s, seqs, offs, n_seqs, k, revcomp, o, out, st, err); break;
    case 5: ok = build_w<5>(s, seqs, offs, n_seqs, k, revcomp, o, out, st, err); break;
    case 6: ok = build_w<6>(s, seqs, offs, n_seqs, k, revcomp, o, out, st, err); break;
    case 7: ok = build_w<7>(s, seqs, offs, n_seqs, k, revcomp, o, out, st, err); break;
    default: ok = build_w<8>(s, seqs, offs, n_seqs, k, revcomp, o, out, st, err); break;
    }
    st.seconds = now_s() - t0;
    return ok;
}

}  // namespace ntc
