// Plain FASTQ parsed on the GPU: the encode pipeline's ingest (DESIGN.md "End-to-end").
// The host hands over the raw text of n whole 4-line records (pipeline.cpp cuts batches
// at record boundaries) and the device does what fastx.cpp parse_fq_range does per record
// -- '@' header, sequence line, '+' line, a quality line as long as the sequence (one '\r'
// stripped from each, as needletail strips CRLF), normalize(iupac = true) of the sequence
// (fastx.cpp norm_table, needletail 0.6) -- and leaves bases + read offsets in HBM for the
// encoder, so only the text crosses PCIe and no host thread touches a base.
//
//   k_fq_count  newlines per 16 KiB tile (256 threads x 64 bytes, SWAR byte compare)
//   (scan)      exclusive scan of the tile counts -> each tile's first line number
//   k_fq_lines  the position of every newline, in order (block scan within the tile)
//   k_fq_recs   one wave per record: the structure checks on lane 0, and the bases the
//               sequence line keeps (wave ballot of norm_table != 0)
//   (scan)      exclusive scan of the kept counts -> read offsets
//   k_fq_norm   one wave per record: normalised bases, compacted with a ballot prefix
//
// Blank lines (which parse_fq_range skips between records, and which make a record's line
// numbers depend on everything before it) are not handled here: the text must hold exactly
// 4 n lines (the last may lack its newline), and the pipeline parses a batch holding a
// line that starts with '\n' or '\r' on the host instead (pipeline.cpp fq_scan_piece).
// HBM traffic per byte of text: 3 reads (count, lines, and the sequence line twice more
// for recs / norm) + 4 B per line for the newline table; all of it is < 2 % of an encode
// call's bytes.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace ntc {

namespace {

constexpr uint32_t kFqThreads = 256, kFqBytes = 64, kFqTile = kFqThreads * kFqBytes;

// fastx.cpp init_norm: A C G T N - kept; a c g t u U n -> upper case / T / N; . ~ -> -;
// IUPAC B D H V R Y S W K M kept (lower case upper-cased); whitespace dropped (0); else N
__device__ __forceinline__ uint8_t norm_of(uint32_t c) {
    switch (c) {
    case 'A': case 'C': case 'G': case 'T': case 'N': case '-':
    case 'B': case 'D': case 'H': case 'V': case 'R': case 'Y': case 'S': case 'W': case 'K': case 'M':
        return (uint8_t)c;
    case 'a': case 'c': case 'g': case 't': case 'n':
    case 'b': case 'd': case 'h': case 'v': case 'r': case 'y': case 's': case 'w': case 'k': case 'm':
        return (uint8_t)(c - 'a' + 'A');
    case 'u': case 'U': return 'T';
    case '.': case '~': return '-';
    case ' ': case '\t': case '\r': case '\n': return 0;
    default: return 'N';
    }
}

// bit 8 j + 7 set where byte j of w is '\n' (exact: no borrow between bytes)
__device__ __forceinline__ uint64_t nl_bits(uint64_t w) {
    const uint64_t x = w ^ 0x0A0A0A0A0A0A0A0Aull;
    const uint64_t t = ((x & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | x;
    return ~t & 0x8080808080808080ull;
}

// the thread's 64 bytes as 8 words (bytes past n read as 0, which is not '\n')
__device__ __forceinline__ void load64(const uint8_t *raw, uint64_t n, uint64_t at, uint64_t w[8]) {
    if (at + kFqBytes <= n) {
        const uint4 *p = (const uint4 *)(raw + at);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint4 v = p[j];
            w[2 * j] = (uint64_t)v.x | (uint64_t)v.y << 32;
            w[2 * j + 1] = (uint64_t)v.z | (uint64_t)v.w << 32;
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = 0;
    for (uint64_t i = at; i < n && i < at + kFqBytes; i++) w[(i - at) >> 3] |= (uint64_t)raw[i] << (8 * ((i - at) & 7));
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// exclusive scan over the block's 256 threads (and the block total)
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t &total) {
    __shared__ uint32_t wsum[kFqThreads / 64];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o);
        if (lane >= (uint32_t)o) inc += t;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t off = 0;
    total = 0;
    for (uint32_t w = 0; w < kFqThreads / 64; w++) {
        if (w < wave) off += wsum[w];
        total += wsum[w];
    }
    return off + inc - v;
}

__global__ __launch_bounds__(kFqThreads) void k_fq_count(const uint8_t *raw, uint64_t n, uint32_t *cnt) {
    uint64_t w[8];
    load64(raw, n, (uint64_t)blockIdx.x * kFqTile + threadIdx.x * kFqBytes, w);
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) c += (uint32_t)__popcll(nl_bits(w[j]));
    __shared__ uint32_t part[kFqThreads / 64];
    c = wave_sum(c);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

__global__ __launch_bounds__(kFqThreads) void k_fq_lines(const uint8_t *raw, uint64_t n, const uint64_t *tile_base,
                                                        uint32_t *nl, uint64_t nl_cap) {
    const uint64_t at = (uint64_t)blockIdx.x * kFqTile + threadIdx.x * kFqBytes;
    uint64_t w[8];
    load64(raw, n, at, w);
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) c += (uint32_t)__popcll(nl_bits(w[j]));
    uint32_t total;
    uint64_t pos = tile_base[blockIdx.x] + block_excl(c, total);
#pragma unroll
    for (int j = 0; j < 8; j++) {
        for (uint64_t m = nl_bits(w[j]); m; m &= m - 1, pos++)
            if (pos < nl_cap) nl[pos] = (uint32_t)(at + 8 * j + (__builtin_ctzll(m) >> 3));
    }
}

struct FqLines {  // the four lines of record r
    uint64_t h0, s0, s1, q0, q1;
};
__device__ __forceinline__ FqLines fq_lines(const uint32_t *nl, uint64_t n_nl, uint64_t n_raw, uint64_t r) {
    const uint64_t L = 4 * r;
    FqLines f;
    f.h0 = r ? (uint64_t)nl[L - 1] + 1 : 0;
    f.s0 = (uint64_t)nl[L] + 1;
    f.s1 = nl[L + 1];
    f.q0 = (uint64_t)nl[L + 2] + 1;
    f.q1 = L + 3 < n_nl ? (uint64_t)nl[L + 3] : n_raw;
    return f;
}

__device__ __forceinline__ void fq_fail(unsigned long long *status, uint64_t r) {
    atomicMin(status, (unsigned long long)(r << 8 | kErrFormat));
}

// n_nl = the scan total; the text is n whole records: 4 n newlines with the last at the
// end, or 4 n - 1 and a last line without one
__global__ __launch_bounds__(kFqThreads) void k_fq_recs(const uint8_t *raw, uint64_t n_raw, const uint32_t *nl,
                                                       const uint64_t *n_nl_p, uint64_t n, uint32_t *kept,
                                                       unsigned long long *status) {
    __shared__ uint8_t tab[256];
    tab[threadIdx.x] = norm_of(threadIdx.x);
    __syncthreads();
    const uint64_t n_nl = *n_nl_p;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t waves = (uint64_t)gridDim.x * (kFqThreads / 64);
    if (n_nl + 1 < 4 * n || n_nl > 4 * n || (n_nl == 4 * n && n && (n_raw == 0 || raw[n_raw - 1] != '\n'))) {
        if (blockIdx.x == 0 && threadIdx.x == 0) fq_fail(status, n_nl / 4 < n ? n_nl / 4 : (n ? n - 1 : 0));
        return;
    }
    for (uint64_t r = (uint64_t)blockIdx.x * (kFqThreads / 64) + (threadIdx.x >> 6); r < n; r += waves) {
        const FqLines f = fq_lines(nl, n_nl, n_raw, r);
        if (lane == 0) {
            const uint64_t ls = f.s1 - f.s0 - (f.s1 > f.s0 && raw[f.s1 - 1] == '\r');
            const uint64_t lq = f.q1 - f.q0 - (f.q1 > f.q0 && raw[f.q1 - 1] == '\r');
            if (raw[f.h0] != '@' || raw[f.s1 + 1] != '+' || ls != lq) fq_fail(status, r);
        }
        uint32_t k = 0;
        for (uint64_t b = 0; b < f.s1 - f.s0; b += 64) {
            const uint64_t i = f.s0 + b + lane;
            const bool keep = i < f.s1 && tab[raw[i]] != 0;
            k += (uint32_t)__popcll(__ballot(keep));
        }
        if (lane == 0) kept[r] = k;
    }
}

__global__ __launch_bounds__(kFqThreads) void k_fq_norm(const uint8_t *raw, uint64_t n_raw, const uint32_t *nl,
                                                       const uint64_t *n_nl_p, uint64_t n, const uint64_t *offs,
                                                       const unsigned long long *status, uint8_t *out) {
    __shared__ uint8_t tab[256];
    tab[threadIdx.x] = norm_of(threadIdx.x);
    __syncthreads();
    if (*status != ~0ull) return;  // the text failed a check: nothing is written
    const uint64_t n_nl = *n_nl_p;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t below = lane ? ~0ull >> (64 - lane) : 0;
    const uint64_t waves = (uint64_t)gridDim.x * (kFqThreads / 64);
    for (uint64_t r = (uint64_t)blockIdx.x * (kFqThreads / 64) + (threadIdx.x >> 6); r < n; r += waves) {
        const FqLines f = fq_lines(nl, n_nl, n_raw, r);
        uint64_t o = offs[r];
        for (uint64_t b = 0; b < f.s1 - f.s0; b += 64) {
            const uint64_t i = f.s0 + b + lane;
            const uint8_t v = i < f.s1 ? tab[raw[i]] : 0;
            const uint64_t m = __ballot(v != 0);
            if (v) out[o + (uint64_t)__popcll(m & below)] = v;
            o += (uint64_t)__popcll(m);
        }
    }
}

}  // namespace

uint64_t fastq_tiles(uint64_t n_raw) { return (n_raw + kFqTile - 1) / kFqTile; }

void launch_fastq_parse(const FastqArgs &a, hipStream_t s) {
    const uint64_t tiles = fastq_tiles(a.n_raw);
    if (tiles == 0) {
        (void)hipMemsetAsync(a.tile_base, 0, 8, s);
    } else {
        hipLaunchKernelGGL(k_fq_count, dim3((uint32_t)tiles), dim3(kFqThreads), 0, s, a.raw, a.n_raw, a.tile_cnt);
        scan_excl_u32(a.tile_cnt, tiles, a.tile_base, a.tmp, s);
        hipLaunchKernelGGL(k_fq_lines, dim3((uint32_t)tiles), dim3(kFqThreads), 0, s, a.raw, a.n_raw,
                           (const uint64_t *)a.tile_base, a.nl, 4 * a.n_reads);
    }
    if (a.n_reads == 0) {
        (void)hipMemsetAsync(a.offs, 0, 8, s);
        return;
    }
    const uint64_t blocks = std::min<uint64_t>((a.n_reads + 3) / 4, 65536);
    hipLaunchKernelGGL(k_fq_recs, dim3((uint32_t)blocks), dim3(kFqThreads), 0, s, a.raw, a.n_raw,
                       (const uint32_t *)a.nl, (const uint64_t *)(a.tile_base + tiles), a.n_reads, a.kept, a.status);
    scan_excl_u32(a.kept, a.n_reads, a.offs, a.tmp, s);
    hipLaunchKernelGGL(k_fq_norm, dim3((uint32_t)blocks), dim3(kFqThreads), 0, s, a.raw, a.n_raw,
                       (const uint32_t *)a.nl, (const uint64_t *)(a.tile_base + tiles), a.n_reads,
                       (const uint64_t *)a.offs, (const unsigned long long *)a.status, a.bases);
}

}  // namespace ntc
