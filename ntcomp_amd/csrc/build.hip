// SBWT subset matrix + LCS built on the GPU (ntc_build_index_device): the same index as the
// host builder (sbwt_build.cpp, the stand-in for kbo::build, src/main.rs:111-134) --
// identical rows, C and LCS -- with every pass over the k-mers in HBM:
//
//   k-mers   one thread per sequence position: the k-window ending there, if all ACGT and
//            inside one sequence, becomes its forward and reverse-complement node keys
//            (characters read right to left, 2 bits each, MSB first, W = ceil(2k/64)
//            words: sorting by the words is colex order, sbwt_build.cpp's Node<W>);
//   sort     LSD over the words (plus the real-character count for dummies) with rocPRIM's
//            radix sort of (word, node) pairs, the least significant word first; duplicates
//            dropped by a flag scan;
//   sources  k-mers with no in-neighbour: binary search of the (k-1)-prefix among the
//            (k-1)-suffixes; their k-1 dummy nodes $^(k-r) x[0..r] (r = 1..k-1) and the root
//            are appended and everything sorted again;
//   LCS      adjacent nodes, first differing character (clz of the XOR);
//   labels   node u = x.c sets bit c of the first node of the (k-1)-suffix group equal to x,
//            found by binary search over the group-first nodes.
// SoA layout: word j of node i at keys[j * n + i]; counts (real characters) in a byte array.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "kernels.h"
#include "ntc_internal.h"

namespace ntc {

namespace {

__device__ __forceinline__ int dev_code(uint8_t b) {
    switch (b) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return -1;
    }
}

// mask keeping characters t < m of a W-word key
template <int W>
__device__ __forceinline__ uint64_t char_mask_w(uint32_t m, int j) {
    const int64_t c = (int64_t)m - 32 * j;
    return c >= 32 ? ~0ULL : c <= 0 ? 0ULL : ~0ULL << (64 - 2 * c);
}

template <int W>
__device__ __forceinline__ void load_key(const uint64_t *keys, uint64_t n, uint64_t i, uint64_t (&w)[W]) {
#pragma unroll
    for (int j = 0; j < W; j++) w[j] = keys[(uint64_t)j * n + i];
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

// sequence holding position p (offs sorted, n_seqs >= 1)
__device__ __forceinline__ uint64_t seq_of(const uint64_t *offs, uint64_t n_seqs, uint64_t p) {
    uint64_t lo = 0, hi = n_seqs;  // offs[lo] <= p < offs[hi]
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) / 2;
        if (offs[mid] <= p) lo = mid;
        else hi = mid;
    }
    return lo;
}

// 1 when the k-window ending at p is all ACGT inside one sequence
__global__ __launch_bounds__(256) void k_kmer_flags(const uint8_t *seq, const uint64_t *offs, uint64_t n_seqs,
                                                    uint64_t T, uint32_t k, uint32_t *flag) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= T) return;
    const uint64_t s0 = offs[seq_of(offs, n_seqs, p)];
    uint32_t ok = p + 1 >= s0 + k;
    for (uint32_t i = 0; ok && i < k; i++) ok = dev_code(seq[p - i]) >= 0;
    flag[p] = ok;
}

template <int W>
__global__ __launch_bounds__(256) void k_kmer_emit(const uint8_t *seq, uint64_t T, uint32_t k, bool revcomp,
                                                   const uint32_t *flag, const uint64_t *rank, uint64_t *keys,
                                                   uint64_t n) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= T || !flag[p]) return;
    uint64_t f[W], g[W];
#pragma unroll
    for (int j = 0; j < W; j++) f[j] = g[j] = 0;
    for (uint32_t i = 0; i < k; i++) {
        // forward: character t = i is seq[p - i]; reverse complement: t = i is the
        // complement of seq[p - k + 1 + i]
        const uint64_t c = (uint64_t)dev_code(seq[p - i]);
        const uint64_t r = 3 - (uint64_t)dev_code(seq[p - k + 1 + i]);
        const uint32_t j = i / 32, sh = 62 - 2 * (i % 32);
#pragma unroll
        for (int q = 0; q < W; q++)
            if (q == (int)j) {
                f[q] |= c << sh;
                g[q] |= r << sh;
            }
    }
    const uint64_t o = rank[p] * (revcomp ? 2 : 1);
#pragma unroll
    for (int j = 0; j < W; j++) {
        keys[(uint64_t)j * n + o] = f[j];
        if (revcomp) keys[(uint64_t)j * n + o + 1] = g[j];
    }
}

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
__global__ __launch_bounds__(256) void k_uniq_flags(const uint64_t *keys, const uint8_t *len, uint64_t n,
                                                    uint32_t *flag) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t d = i == 0;
    if (i) {
#pragma unroll
        for (int j = 0; j < W; j++) d |= keys[(uint64_t)j * n + i] != keys[(uint64_t)j * n + i - 1];
        if (len) d |= len[i] != len[i - 1];
    }
    flag[i] = d;
}

template <int W>
__global__ __launch_bounds__(256) void k_compact(const uint64_t *keys, const uint8_t *len, uint64_t n,
                                                 const uint32_t *flag, const uint64_t *rank, uint64_t m,
                                                 uint64_t *okeys, uint8_t *olen) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n || !flag[i]) return;
    const uint64_t o = rank[i];
#pragma unroll
    for (int j = 0; j < W; j++) okeys[(uint64_t)j * m + o] = keys[(uint64_t)j * n + i];
    if (len) olen[o] = len[i];
}

// k-mers (sorted, unique, all k characters) without an in-neighbour: no k-mer y with
// y[1..k] = x[0..k-1], i.e. no node whose first k - 1 characters (t < k - 1) are x's
// characters t = 1..k-1 (sbwt_build.cpp step 3)
template <int W>
__global__ __launch_bounds__(256) void k_sources(const uint64_t *keys, uint64_t n, uint32_t k, uint32_t *src) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint64_t key[W];
    load_key<W>(keys, n, i, key);
    shl_chars<W>(key, 1);
    // first node whose words are >= key (key's count 0 is below every k-mer's)
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        int cmp = 0;
#pragma unroll
        for (int j = 0; j < W; j++) {
            const uint64_t a = keys[(uint64_t)j * n + mid];
            if (cmp == 0 && a != key[j]) cmp = a < key[j] ? -1 : 1;
        }
        if (cmp < 0) lo = mid + 1;
        else hi = mid;
    }
    uint32_t found = lo < n;
    if (found) {
#pragma unroll
        for (int j = 0; j < W; j++)
            if ((keys[(uint64_t)j * n + lo] & char_mask_w<W>(k - 1, j)) != key[j]) found = 0;
    }
    src[i] = !found;
}

// dummies of source x: $^(k-r) x[0..r] for r = 1..k-1 (r real characters), then the root
template <int W>
__global__ __launch_bounds__(256) void k_dummies(const uint64_t *keys, uint64_t n, uint32_t k, const uint32_t *src,
                                                 const uint64_t *rank, uint64_t *okeys, uint8_t *olen, uint64_t m,
                                                 uint64_t base) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n || !src[i]) return;
    uint64_t x[W];
    load_key<W>(keys, n, i, x);
    const uint64_t o0 = base + rank[i] * (k - 1);
    for (uint32_t r = 1; r < k; r++) {
        uint64_t d[W];
#pragma unroll
        for (int j = 0; j < W; j++) d[j] = x[j];
        shl_chars<W>(d, k - r);
#pragma unroll
        for (int j = 0; j < W; j++) okeys[(uint64_t)j * m + o0 + r - 1] = d[j] & char_mask_w<W>(r, j);
        olen[o0 + r - 1] = (uint8_t)r;
    }
}

// lcs[i]: longest common suffix of nodes i - 1 and i (characters), capped at 255
template <int W>
__global__ __launch_bounds__(256) void k_lcs(const uint64_t *keys, const uint8_t *len, uint64_t n, uint8_t *lcs,
                                             uint32_t *gflag, uint32_t k) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t l = 0;
    if (i) {
        uint32_t common = 32 * W;
        bool done = false;
#pragma unroll
        for (int j = 0; j < W; j++) {
            const uint64_t d = keys[(uint64_t)j * n + i] ^ keys[(uint64_t)j * n + i - 1];
            if (!done && d) {
                common = 32 * j + (uint32_t)__builtin_clzll(d) / 2;
                done = true;
            }
        }
        l = min(common, min((uint32_t)len[i], (uint32_t)len[i - 1]));
        l = min(l, 255u);
    }
    lcs[i] = (uint8_t)l;
    gflag[i] = i == 0 || l < k - 1;  // first node of its (k-1)-suffix group
}

// compare (words & (k-1)-mask, min(count, k-1)) of group-first node g against (key, klen)
template <int W>
__device__ __forceinline__ int group_cmp(const uint64_t *keys, const uint8_t *len, uint64_t n, uint64_t g,
                                         uint32_t k, const uint64_t (&key)[W], uint32_t klen) {
#pragma unroll
    for (int j = 0; j < W; j++) {
        const uint64_t a = keys[(uint64_t)j * n + g] & char_mask_w<W>(k - 1, j);
        if (a != key[j]) return a < key[j] ? -1 : 1;
    }
    const uint32_t gl = min((uint32_t)len[g], k - 1);
    return gl == klen ? 0 : (gl < klen ? -1 : 1);
}

// node u = x.c (u's last character c, x its first count - 1 characters) labels the first
// node of the (k-1)-suffix group equal to x with c (sbwt_build.cpp step 5)
template <int W>
__global__ __launch_bounds__(256) void k_labels(const uint64_t *keys, const uint8_t *len, uint64_t n, uint32_t k,
                                                const uint32_t *gfirst, uint64_t G, unsigned long long *rows,
                                                uint64_t nw, unsigned int *bad) {
    const uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= n || len[u] == 0) return;
    uint64_t key[W];
    load_key<W>(keys, n, u, key);
    const uint32_t c = (uint32_t)(key[0] >> 62);
    shl_chars<W>(key, 1);
    const uint32_t klen = (uint32_t)len[u] - 1;
    uint64_t lo = 0, hi = G;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (group_cmp<W>(keys, len, n, gfirst[mid], k, key, klen) < 0) lo = mid + 1;
        else hi = mid;
    }
    if (lo >= G || group_cmp<W>(keys, len, n, gfirst[lo], k, key, klen) != 0) {
        atomicOr(bad, 1u);
        return;
    }
    const uint64_t gi = gfirst[lo];
    atomicOr(rows + (uint64_t)c * nw + (gi >> 6), 1ULL << (gi & 63));
}

__global__ __launch_bounds__(256) void k_gfirst(const uint32_t *gflag, const uint64_t *rank, uint64_t n,
                                                uint32_t *gfirst) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n && gflag[i]) gfirst[rank[i]] = (uint32_t)i;
}

inline dim3 grid(uint64_t n) { return dim3((uint32_t)((n + 255) / 256)); }

// device buffers of one build, freed together
struct Arena {
    std::vector<void *> ptrs;
    std::string *err;
    ~Arena() {
        for (void *p : ptrs) (void)hipFree(p);
    }
    template <class T>
    T *get(uint64_t count) {
        void *p = nullptr;
        if (hipMalloc(&p, std::max<uint64_t>(count * sizeof(T), 64)) != hipSuccess) return nullptr;
        ptrs.push_back(p);
        return (T *)p;
    }
    void release(void *p) {
        auto it = std::find(ptrs.begin(), ptrs.end(), p);
        if (it != ptrs.end()) {
            (void)hipFree(p);
            ptrs.erase(it);
        }
    }
};

#define BTRY(expr)                                                                   \
    do {                                                                             \
        hipError_t e_ = (expr);                                                      \
        if (e_ != hipSuccess) {                                                      \
            err = std::string(#expr) + ": " + hipGetErrorString(e_);                 \
            return false;                                                            \
        }                                                                            \
    } while (0)
#define BALLOC(var, T, count)                                                        \
    T *var = A.get<T>(count);                                                        \
    if (!var) {                                                                      \
        err = "device allocation failed (" #var ")";                                 \
        return false;                                                                \
    }

template <int W>
struct Builder {
    hipStream_t s;
    uint32_t k;
    std::string &err;
    Arena &A;

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

    // sort n nodes (SoA keys, optional counts) into new arrays; LSD: counts, then words
    // from the least significant (word W-1: only its top bits hold characters)
    bool sort(const uint64_t *keys, const uint8_t *len, uint64_t n, uint64_t *&okeys, uint8_t *&olen) {
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
            hipLaunchKernelGGL(k_gather_u64, grid(n), dim3(256), 0, s, keys + (uint64_t)j * n, perm, n, ka);
            BTRY(rocprim::radix_sort_pairs(tmp, tb, ka, kb, perm, perm2, n, 0, 64, s));
            std::swap(perm, perm2);
        }
        BALLOC(ok, uint64_t, (uint64_t)W * n);
        uint8_t *ol = nullptr;
        if (len) {
            ol = A.get<uint8_t>(n);
            if (!ol) {
                err = "device allocation failed (counts)";
                return false;
            }
        }
        for (int j = 0; j < W && n; j++)
            hipLaunchKernelGGL(k_gather_u64, grid(n), dim3(256), 0, s, keys + (uint64_t)j * n, perm, n,
                               ok + (uint64_t)j * n);
        if (len && n) hipLaunchKernelGGL(k_gather_u8, grid(n), dim3(256), 0, s, len, perm, n, ol);
        BTRY(hipGetLastError());
        BTRY(hipStreamSynchronize(s));
        for (void *p : {(void *)perm, (void *)perm2, (void *)ka, (void *)kb, (void *)tmp}) A.release(p);
        okeys = ok;
        olen = ol;
        return true;
    }

    // drop repeated nodes (sorted input)
    bool unique(const uint64_t *keys, const uint8_t *len, uint64_t n, uint64_t *&okeys, uint8_t *&olen,
                uint64_t &m) {
        BALLOC(flag, uint32_t, n + 1);
        BALLOC(rank, uint64_t, n + 1);
        if (n) hipLaunchKernelGGL(k_uniq_flags<W>, grid(n), dim3(256), 0, s, keys, len, n, flag);
        if (!scan_flags(flag, n, rank, m)) return false;
        BALLOC(ok, uint64_t, (uint64_t)W * m);
        uint8_t *ol = nullptr;
        if (len) {
            ol = A.get<uint8_t>(m);
            if (!ol) {
                err = "device allocation failed (counts)";
                return false;
            }
        }
        if (n) hipLaunchKernelGGL(k_compact<W>, grid(n), dim3(256), 0, s, keys, len, n, flag, rank, m, ok, ol);
        BTRY(hipGetLastError());
        BTRY(hipStreamSynchronize(s));
        A.release(flag);
        A.release(rank);
        okeys = ok;
        olen = ol;
        return true;
    }

    bool run(const uint8_t *h_seq, const uint64_t *h_offs, uint64_t n_seqs, bool revcomp, HostIndex &out) {
        const uint64_t o0 = n_seqs ? h_offs[0] : 0, T = n_seqs ? h_offs[n_seqs] - o0 : 0;
        // ---- 1. k-mers -----------------------------------------------------------------
        uint64_t nk = 0;
        uint64_t *K = nullptr;
        if (T >= k) {
            BALLOC(seq, uint8_t, T);
            BALLOC(offs, uint64_t, n_seqs + 1);
            std::vector<uint64_t> ho(n_seqs + 1);
            for (uint64_t i = 0; i <= n_seqs; i++) ho[i] = h_offs[i] - o0;
            BTRY(hipMemcpyAsync(seq, h_seq + o0, T, hipMemcpyHostToDevice, s));
            BTRY(hipMemcpyAsync(offs, ho.data(), (n_seqs + 1) * 8, hipMemcpyHostToDevice, s));
            BALLOC(flag, uint32_t, T + 1);
            BALLOC(rank, uint64_t, T + 1);
            hipLaunchKernelGGL(k_kmer_flags, grid(T), dim3(256), 0, s, seq, offs, n_seqs, T, k, flag);
            uint64_t nv = 0;
            if (!scan_flags(flag, T, rank, nv)) return false;
            nk = nv * (revcomp ? 2 : 1);
            if (nk) {
                BALLOC(keys, uint64_t, (uint64_t)W * nk);
                hipLaunchKernelGGL(k_kmer_emit<W>, grid(T), dim3(256), 0, s, seq, T, k, revcomp, flag, rank, keys, nk);
                BTRY(hipGetLastError());
                BTRY(hipStreamSynchronize(s));
                for (void *p : {(void *)seq, (void *)offs, (void *)flag, (void *)rank}) A.release(p);
                uint64_t *sk;
                uint8_t *sl;
                if (!sort(keys, nullptr, nk, sk, sl)) return false;
                A.release(keys);
                if (!unique(sk, nullptr, nk, K, sl, nk)) return false;
                A.release(sk);
            }
        }
        // ---- 2. sources, dummies, root; all nodes sorted ----------------------------------
        uint64_t nsrc = 0;
        BALLOC(src, uint32_t, nk + 1);
        BALLOC(srank, uint64_t, nk + 1);
        if (nk) hipLaunchKernelGGL(k_sources<W>, grid(nk), dim3(256), 0, s, K, nk, k, src);
        if (!scan_flags(src, nk, srank, nsrc)) return false;
        const uint64_t m = nk + 1 + nsrc * (k - 1);
        BALLOC(allk, uint64_t, (uint64_t)W * m);
        BALLOC(alll, uint8_t, m);
        for (int j = 0; j < W; j++) {
            if (nk) BTRY(hipMemcpyAsync(allk + (uint64_t)j * m, K + (uint64_t)j * nk, nk * 8, hipMemcpyDeviceToDevice, s));
            BTRY(hipMemsetAsync(allk + (uint64_t)j * m + nk, 0, 8, s));  // the root
        }
        BTRY(hipMemsetAsync(alll, (int)k, nk, s));
        BTRY(hipMemsetAsync(alll + nk, 0, 1, s));
        if (nsrc) hipLaunchKernelGGL(k_dummies<W>, grid(nk), dim3(256), 0, s, K, nk, k, src, srank, allk, alll, m, nk + 1);
        BTRY(hipGetLastError());
        BTRY(hipStreamSynchronize(s));
        for (void *p : {(void *)src, (void *)srank}) A.release(p);
        if (K) A.release(K);
        uint64_t *sk, *nodes;
        uint8_t *sl, *nlen;
        if (!sort(allk, alll, m, sk, sl)) return false;
        A.release(allk);
        A.release(alll);
        uint64_t n = 0;
        if (!unique(sk, sl, m, nodes, nlen, n)) return false;
        A.release(sk);
        A.release(sl);
        if (n >= (1ULL << 32)) {
            err = "index too large for 32-bit colex ranks";
            return false;
        }
        // ---- 3. LCS, groups, labels -------------------------------------------------------
        const uint64_t nw = (n + 63) / 64;
        BALLOC(lcs, uint8_t, n);
        BALLOC(gflag, uint32_t, n + 1);
        BALLOC(grank, uint64_t, n + 1);
        hipLaunchKernelGGL(k_lcs<W>, grid(n), dim3(256), 0, s, nodes, nlen, n, lcs, gflag, k);
        uint64_t G = 0;
        if (!scan_flags(gflag, n, grank, G)) return false;
        BALLOC(gfirst, uint32_t, G);
        hipLaunchKernelGGL(k_gfirst, grid(n), dim3(256), 0, s, gflag, grank, n, gfirst);
        BALLOC(rows, unsigned long long, 4 * nw);
        BALLOC(bad, unsigned int, 1);
        BTRY(hipMemsetAsync(rows, 0, 4 * nw * 8, s));
        BTRY(hipMemsetAsync(bad, 0, 4, s));
        hipLaunchKernelGGL(k_labels<W>, grid(n), dim3(256), 0, s, nodes, nlen, n, k, gfirst, G, rows, nw, bad);
        BTRY(hipGetLastError());
        out.n = n;
        out.k = k;
        out.lcs.resize(n);
        for (int c = 0; c < 4; c++) out.rows[c].resize(nw);
        unsigned int hbad = 0;
        BTRY(hipMemcpyAsync(out.lcs.data(), lcs, n, hipMemcpyDeviceToHost, s));
        for (int c = 0; c < 4; c++)
            BTRY(hipMemcpyAsync(out.rows[c].data(), rows + (uint64_t)c * nw, nw * 8, hipMemcpyDeviceToHost, s));
        BTRY(hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, s));
        BTRY(hipStreamSynchronize(s));
        if (hbad) {
            err = "internal: node without a predecessor group";
            return false;
        }
        uint64_t before = 1;
        for (int c = 0; c < 4; c++) {
            out.C[c] = before;
            for (uint64_t w = 0; w < nw; w++) before += (uint64_t)__builtin_popcountll(out.rows[c][w]);
        }
        if (before != n) {
            err = "internal: labels do not cover every non-root node (" + std::to_string(before - 1) + " labels, " +
                  std::to_string(n) + " nodes, " + std::to_string(nk) + " k-mers, " + std::to_string(nsrc) +
                  " sources, " + std::to_string(G) + " groups)";
            return false;
        }
        return true;
    }
};

template <int W>
bool build_w(hipStream_t s, const uint8_t *seqs, const uint64_t *offs, uint64_t n_seqs, uint32_t k, bool revcomp,
             HostIndex &out, std::string &err) {
    Arena A;
    A.err = &err;
    Builder<W> b{s, k, err, A};
    return b.run(seqs, offs, n_seqs, revcomp, out);
}

}  // namespace

bool build_index_device(hipStream_t s, const uint8_t *seqs, const uint64_t *offs, uint64_t n_seqs, uint32_t k,
                        bool revcomp, HostIndex &out, std::string &err) {
    if (k < 1 || k > 255) {
        err = "k must be in [1, 255]";
        return false;
    }
    switch ((2 * k + 63) / 64) {
    case 1: return build_w<1>(s, seqs, offs, n_seqs, k, revcomp, out, err);
    case 2: return build_w<2>(s, seqs, offs, n_seqs, k, revcomp, out, err);
    case 3: return build_w<3>(s, seqs, offs, n_seqs, k, revcomp, out, err);
    case 4: return build_w<4>(s, seqs, offs, n_seqs, k, revcomp, out, err);
    case 5: return build_w<5>(s, seqs, offs, n_seqs, k, revcomp, out, err);
    case 6: return build_w<6>(s, seqs, offs, n_seqs, k, revcomp, out, err);
    case 7: return build_w<7>(s, seqs, offs, n_seqs, k, revcomp, out, err);
    default: return build_w<8>(s, seqs, offs, n_seqs, k, revcomp, out, err);
    }
}

}  // namespace ntc
