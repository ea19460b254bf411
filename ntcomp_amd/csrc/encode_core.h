// Per-read lane logic of the encode and decode kernels.  Written once as
// __host__ __device__ code: the HIP kernels in kernels.hip call these functions, one
// GPU lane per read, and the test-only host emulation (tests/emu/) compiles the very
// same functions for the CPU so the kernel's algorithm can be checked against the
// oracle on a machine without a GPU.  The product library never runs them on the host.
//
// Reference semantics restated here (file:line into /root/reference):
//   ms_step      StreamingIndex::matching_statistics [ext sbwt 0.3.11], lib.rs:172-173
//   encode_lane  encode_sequence lib.rs:163-230 fused with encode_dictionary
//                encode.rs:129-166; left_extend_kmer lib.rs:94-128 restated as an O(1)
//                per-step test
//   decode_read  decode_sequence lib.rs:254-318; access_kmer + left_extend_kmer2
//                lib.rs:130-161 restated as one inverse-SBWT walk (Appendix A.5)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#define NTC_HD __host__ __device__ __forceinline__
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
#ifndef NTC_NT
#define NTC_NT 17  // streaming (nontemporal) hints, bit mask: 1 table entries, 16 entry stores,
                   // 2 exact presence bits, 4 path stream, 8 query words, 32 pair / window words
                   // (k_ms4), 64 fork block entries, 128 rank words (k_ms4), 256 colex_at and
                   // pos_of_node (k_ms4)
#endif

// Line tracing for the test-only emulator (tests/emu, -DNTC_TRACE): every index load
// reports (kind, address) so per-read cache-line footprints can be counted on the CPU.
#if defined(NTC_TRACE) && !defined(__HIP_DEVICE_COMPILE__)
void ntc_touch(int kind, const void *p);
#define NTC_TOUCH(kind, p) ntc_touch(kind, (const void *)(p))
#else
#define NTC_TOUCH(kind, p) ((void)0)
#endif
enum { kTrRank, kTrLcs, kTrUniq, kTrTabU, kTrTabLo, kTrBits, kTrFilt, kTrColex, kTrPon, kTrPst, kTrQ, kTrE,
       kTrPuniq, kTrEw, kTrKinds };

namespace ntc {

#if defined(NTC_STATS) && !defined(__HIP_DEVICE_COMPILE__)
extern uint64_t ntc_stats[16];  // host emulation only: unit counts by kind
#define NTC_STAT(i) (ntc_stats[i]++)
inline void ntc_stat_add(int i, uint64_t v) { ntc_stats[i] += v; }
#else
#define NTC_STAT(i) ((void)0)
NTC_HD void ntc_stat_add(int, uint64_t) {}
#endif

// Rank words: row c of the subset matrix as one 8-byte word per 32 positions, x = C[c] +
// (ones of row c before the word), y = the 32 row bits.  extend = two 8-byte loads + two
// popcounts (DESIGN.md "Data layout in HBM").  Rows live in 4 separate arrays of rwords.

// Inverse-walk jump table: the kWalkSpan = 112 characters met by walking 112 steps
// backwards from node j, in text order t0..t111 (t111 = node j's own last character), and
// the node reached.  One 32-byte entry (one 128 B line) replaces 112 dependent select()s of
// access_kmer: a long record of up to 112 bases (every long record of a 150 bp read at
// k = 91 with errors) is ONE random line, where 48-character entries took 1.1 per record.
struct alignas(32) WalkEntry {
    uint64_t w0;     // t80..t111 (character t80 + i in bits 2i..2i+1)
    uint64_t w1;     // t48..t79
    uint64_t w2;     // t16..t47
    uint32_t older;  // t0..t15
    uint32_t jump;   // the node kWalkSpan steps back
};
constexpr uint32_t kWalkSpan = 112;
// 16-byte doubling steps the table is built from at upload (k_walk_*, build_walk_host):
// chars = the last 32 characters of the step (text order), older = the 16 before them
struct alignas(16) WalkStep {
    uint64_t chars;
    uint32_t jump;
    uint32_t older;
};
// 112-step entry of node j from its 48-step entry x, the 48-step entry y at x's jump and the
// 16-step entry z at y's jump
NTC_HD WalkEntry walk_compose(const WalkStep &x, const WalkStep &y, const WalkStep &z) {
    WalkEntry e;
    e.w0 = x.chars;                                            // t80..t111
    e.w1 = (y.chars >> 32) | ((uint64_t)x.older << 32);        // t48..t63 | t64..t79
    e.w2 = (uint64_t)y.older | ((y.chars & 0xFFFFFFFFull) << 32);  // t16..t31 | t32..t47
    e.older = (uint32_t)z.chars;                               // t0..t15
    e.jump = z.jump;
    return e;
}

// Two-character rank chunks: per 32 SBWT positions (block b, positions 32b ... 32b + 31)
// and first character c1, one 64-byte chunk (two per 128-byte line):
//   base      = C[c1] + rank_c1(32b)           (where the block's c1-successors start, L0)
//   bits      = row c1's 32 bits of the block
//   pbase[c2] = C[c2] + rank_c2(L0), pbits[c2] = row c2's 32 bits at L0 ... L0 + 31
// so ext(ext([l, r), c1), c2) -- two MS steps -- costs the chunks of l's and r's blocks
// (one line when they share a block) instead of two dependent rank-word lines.  At most 32
// positions of a block carry c1, so l1 - L0 <= 32 stays inside pbits.
struct alignas(64) Rank2Chunk {
    uint32_t base;
    uint32_t bits;
    uint32_t pbase[4];
    uint32_t pbits[4];
    uint32_t pad[6];
};
static_assert(sizeof(Rank2Chunk) == 64, "rank2 chunk");
NTC_HD uint64_t rank2_blocks(uint64_t n) { return (n >> 5) + 2; }  // every block of 32 positions up to n

struct DevIndex {
    const uint2 *rank;      // [4][rwords] rank words
    const uint8_t *lcs;     // [n]
    const uint32_t *uniq;   // bit z: node z's (k-1)-suffix group is {z}
    const WalkEntry *walk;  // [n]
    uint32_t rwords;        // n / 32 + 2
    uint32_t n;
    uint32_t k;
    uint32_t t_jump;        // first contraction probe below d-1 (see ms_step)
    uint32_t C[5];          // C[4] = n
    // path walk (encode v2): a path cover of the de Bruijn graph, see derived.cpp
    uint32_t has_paths;
    const uint4 *pstream;         // path text in 32-char groups: {chars (2-bit, u64), end bits, 0}
    const uint32_t *colex_at;     // node | uniq << 31 at each k-mer start, 0xFFFFFFFF elsewhere
    const uint32_t *pos_of_node;  // text position of each real node's k-mer, or 0xFFFFFFFF
    const uint64_t *puniq;        // bit j: that node's (k-1)-suffix group is a singleton
    const uint2 *tab;             // suffix table, levels 1..tab_u (see tab_make)
    const uint32_t *tab_bits;     // bit key of level tab_u: that U-mer is present (long)
    const uint32_t *filt_bits;    // presence bits of level filt_f = U - 2 (L2-resident), or null
    uint32_t filt_f;              // 0: no filter
    const uint16_t *pair_w;       // pair word of each (U-1)-mer (see pair_word), or null
    uint32_t path_len;            // path text length (has_paths): path positions are < path_len
    uint32_t tab_pos;             // 1: top-level singleton entries carry the path position
    uint32_t tab_u;               // U: longest tabulated length (1 <= U <= min(k, kTabMaxU))
    uint32_t absent;              // bit c: no node ends with character c
    const Rank2Chunk *rank2;      // [4][rank2_blocks(n)] two-character rank chunks, or null
    uint32_t joint;               // 1: encode with joint path runs (k_ms4<true>, MsLaneT)
    const uint32_t *win_w;        // window words of each (U-3)-mer (see win_word), or null
    uint32_t forks;               // 1: colex_at holds fork blocks after each path end (fork_block)
};

// Fork blocks (k >= kForkBlockMinK, derived.cpp build_paths, kernels.hip k_path_forks).  A
// path's last node at position t - 1 is followed by k free colex_at slots; the 16 from
// fork_block(t) (16-byte aligned, so each entry is one load inside one line) hold, per
// character c, the entry {y, the 32 path characters from y's k-mer end (2 bits each), their
// k-mer end bits} of the node y = v[1..k]c's path position (y = 0xFFFFFFFF: none).  A run
// that stops at the path end hops to y with one load, and the entry's characters are the
// first 32 positions of the run from y (MsLaneT::step, the run block).
constexpr uint32_t kForkBlockMinK = 19;
NTC_HD uint64_t fork_block(uint64_t t) { return (t + 3) & ~3ull; }
// 32 path characters from text position T and the k-mer end bits there (pstream groups)
NTC_HD void path_text32(const uint4 *pstream, uint64_t T, uint64_t &chars, uint32_t &ends) {
    const uint4 g0 = pstream[T >> 5], g1 = pstream[(T >> 5) + 1];
    const uint32_t sh = (uint32_t)(T & 31);
    const uint64_t c0 = (uint64_t)g0.x | ((uint64_t)g0.y << 32), c1 = (uint64_t)g1.x | ((uint64_t)g1.y << 32);
    chars = sh ? ((c0 >> (2 * sh)) | (c1 << (64 - 2 * sh))) : c0;
    ends = sh ? ((g0.z >> sh) | (g1.z << (32 - sh))) : g0.z;
}

// per-read status codes (values of ntc_status)
enum : int {
    kErrInvalidBase = 2,
    kErrEmptyRead = 3,
    kErrLength = 4,
    kErrCapacity = 5,
    kErrFormat = 8,
    kErrRefPanic = 11,  // an input on which the reference panics (NTC_ERR_REFERENCE_PANIC)
};

NTC_HD int base_code(uint8_t b) {
    // A=0 C=1 G=2 T=3 (bitnuc as_2bit order), anything else -1
    switch (b) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    default: return -1;
    }
}

NTC_HD uint8_t base_char(uint32_t c) { return (uint8_t)(0x54474341u >> (8 * (c & 3))); }

NTC_HD uint32_t clz32(uint32_t x) { return x ? (uint32_t)__builtin_clz(x) : 32u; }

NTC_HD uint2 mk2(uint32_t x, uint32_t y) {
    uint2 v;
    v.x = x;
    v.y = y;
    return v;
}
NTC_HD uint2 load2(const uint2 *p) {
#ifdef __HIP_DEVICE_COMPILE__
    return *p;
#else
    return mk2(p->x, p->y);
#endif
}
template <int kBit, typename T>
NTC_HD T ld_hint(const T *p) {
#ifdef __HIP_DEVICE_COMPILE__
    if constexpr ((NTC_NT & kBit) != 0) return __builtin_nontemporal_load(p);
#endif
    return *p;
}
template <int kBit>
NTC_HD uint4 ld4(const uint4 *p) {
#ifdef __HIP_DEVICE_COMPILE__
    if constexpr ((NTC_NT & kBit) != 0) {
        const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t *>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    }
#endif
    return *p;
}
// a load with no reuse (suffix-table entries: 2.9 GB, random): streaming hint, so that it
// does not push the L2-resident filter bitmap out
NTC_HD uint2 load2_stream(const uint2 *p) {
#if defined(__HIP_DEVICE_COMPILE__) && (NTC_NT & 1)
    const uint64_t v = __builtin_nontemporal_load(reinterpret_cast<const uint64_t *>(p));
    return mk2((uint32_t)v, (uint32_t)(v >> 32));
#else
    return load2(p);
#endif
}
template <int kBit>
NTC_HD uint2 load2h(const uint2 *p) {  // load2 with the NTC_NT hint kBit
#ifdef __HIP_DEVICE_COMPILE__
    if constexpr ((NTC_NT & kBit) != 0) {
        const uint64_t v = __builtin_nontemporal_load(reinterpret_cast<const uint64_t *>(p));
        return mk2((uint32_t)v, (uint32_t)(v >> 32));
    }
#endif
    return load2(p);
}
NTC_HD uint32_t rank_word(uint2 w, uint32_t x) {  // C[c] + rank_c(x) from x's word
    return w.x + (uint32_t)__builtin_popcount(w.y & ((1u << (x & 31)) - 1u));
}

// extend_right(I, c) = [C[c] + rank_c(l), C[c] + rank_c(r))
NTC_HD void extend(const DevIndex &ix, int c, uint32_t l, uint32_t r, uint32_t &nl, uint32_t &nr) {
    const uint2 *row = ix.rank + (uint64_t)c * ix.rwords;
    NTC_TOUCH(kTrRank, row + (l >> 5));
    NTC_TOUCH(kTrRank, row + (r >> 5));
    const uint2 a = load2h<128>(row + (l >> 5)), b = load2h<128>(row + (r >> 5));
    nl = rank_word(a, l);
    nr = rank_word(b, r);
}

// 32 bits of row c starting at position x, from the rank words
NTC_HD uint32_t row_bits32(const DevIndex &ix, int c, uint64_t x) {
    const uint2 *row = ix.rank + (uint64_t)c * ix.rwords;
    const uint32_t sh = (uint32_t)(x & 31);
    const uint32_t a = row[x >> 5].y;
    return sh ? (a >> sh) | (row[(x >> 5) + 1].y << (32 - sh)) : a;
}
// chunk (block b, c1) of the two-character rank table (built at upload: k_rank2 / build_rank2_host)
NTC_HD Rank2Chunk rank2_make(const DevIndex &ix, uint64_t b, int c1) {
    Rank2Chunk e{};
    const uint64_t x0 = 32 * b;
    const uint64_t x = x0 <= ix.n ? x0 : ix.n;  // blocks past the end: empty
    e.base = rank_word(ix.rank[(uint64_t)c1 * ix.rwords + (x >> 5)], (uint32_t)x);
    e.bits = x0 <= ix.n ? ix.rank[(uint64_t)c1 * ix.rwords + (x0 >> 5)].y : 0u;
    const uint64_t L0 = e.base <= ix.n ? e.base : ix.n;
    for (int c2 = 0; c2 < 4; c2++) {
        e.pbase[c2] = rank_word(ix.rank[(uint64_t)c2 * ix.rwords + (L0 >> 5)], (uint32_t)L0);
        e.pbits[c2] = row_bits32(ix, c2, L0);
    }
    return e;
}
// ext by c1 then c2 from [l, r): (l1, r1) after c1 and (l2, r2) after c2 (empty = failure)
NTC_HD void extend2(const DevIndex &ix, int c1, int c2, uint32_t l, uint32_t r, uint32_t &l1, uint32_t &r1,
                    uint32_t &l2, uint32_t &r2) {
    // c1-major: chunks of neighbouring blocks share 128-byte lines
    const Rank2Chunk *T = ix.rank2 + (uint64_t)c1 * rank2_blocks(ix.n);
    const Rank2Chunk *A = T + (l >> 5), *B = T + (r >> 5);
    NTC_TOUCH(kTrRank, A);
    NTC_TOUCH(kTrRank, B);
    const uint32_t abase = A->base, abits = A->bits, apb = A->pbase[c2], apbits = A->pbits[c2];
    const uint32_t bbase = B->base, bbits = B->bits, bpb = B->pbase[c2], bpbits = B->pbits[c2];
    const uint32_t ol = (uint32_t)__builtin_popcount(abits & ((1u << (l & 31)) - 1u));
    const uint32_t orr = (uint32_t)__builtin_popcount(bbits & ((1u << (r & 31)) - 1u));
    l1 = abase + ol;
    r1 = bbase + orr;
    l2 = apb + (uint32_t)__builtin_popcountll((uint64_t)apbits & ((1ull << ol) - 1ull));
    r2 = bpb + (uint32_t)__builtin_popcountll((uint64_t)bpbits & ((1ull << orr) - 1ull));
}

// contract_left(I, t) [ext sbwt]: widen I to all nodes sharing the last t characters.
NTC_HD void widen(const DevIndex &ix, uint32_t &l, uint32_t &r, uint32_t t) {
    while (l > 0 && (NTC_TOUCH(kTrLcs, ix.lcs + l), ix.lcs[l]) >= t) l--;
    while (r < ix.n && (NTC_TOUCH(kTrLcs, ix.lcs + r), ix.lcs[r]) >= t) r++;
}

// One character of k-bounded matching statistics.  State (d, [l, r)) = length and colex
// interval of the longest suffix (<= k) of the query prefix that is a suffix of a node.
// The reference contracts one level at a time: while extend fails, t = d-1, d-2, ...
// It stops at t* = max{t < d : extend(I_t, c) != empty}.  For t <= k-1 that predicate
// is "suffix_t . c is a substring of the k-spectrum", monotone in t, so t* can be found
// by probing: d-1 first (the non-group-first d = k case), then t_jump (~log4 n + 2, below
// which random matches live), then binary search above t_jump or linear descent below
// it.  Same (d, I) as the reference for every input (tests: golden + oracle parity).
NTC_HD void ms_step(const DevIndex &ix, int c, uint32_t &d, uint32_t &l, uint32_t &r) {
    uint32_t nl, nr;
    extend(ix, c, l, r, nl, nr);
    if (nl < nr) {
        l = nl;
        r = nr;
        d = d + 1 < ix.k ? d + 1 : ix.k;
        return;
    }
    if (d == 0) return;
    uint32_t hi = d - 1;
    uint32_t l1 = l, r1 = r;
    widen(ix, l1, r1, hi);
    extend(ix, c, l1, r1, nl, nr);
    if (nl < nr) {
        l = nl;
        r = nr;
        d = hi + 1;
        return;
    }
    uint32_t cl = l1, cr = r1;  // I_hi, extension known to fail at hi
    const uint32_t tj = ix.t_jump;
    if (hi > tj + 1) {
        uint32_t l2 = l1, r2 = r1;
        widen(ix, l2, r2, tj);
        extend(ix, c, l2, r2, nl, nr);
        if (nl < nr) {
            uint32_t lo = tj, bl = nl, br = nr;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                uint32_t lm = l1, rm = r1;
                widen(ix, lm, rm, mid);
                uint32_t ml, mr;
                extend(ix, c, lm, rm, ml, mr);
                if (ml < mr) {
                    lo = mid;
                    bl = ml;
                    br = mr;
                } else {
                    hi = mid;
                }
            }
            l = bl;
            r = br;
            d = lo + 1;
            return;
        }
        hi = tj;
        cl = l2;
        cr = r2;
    }
    while (hi > 0) {
        const uint32_t t = hi - 1;
        widen(ix, cl, cr, t);
        extend(ix, c, cl, cr, nl, nr);
        if (nl < nr) {
            l = nl;
            r = nr;
            d = t + 1;
            return;
        }
        hi = t;
    }
    l = cl;  // contracted to the empty suffix: [0, n)
    r = cr;
    d = 0;
}

// This lane's slice of the per-tile scratch: element p of a read lives at [p * 64].
struct LaneScratch {
    uint8_t *D;   // MS length per position
    uint32_t *S;  // colex start per position
    uint32_t *F;  // bit p%32 of F[(p/32)*64]: d == k and the k-mer's group is a singleton
    uint64_t *R;  // records, rightmost first
};

// consecutive set flags at positions p, p-1, ... (at most cap)
NTC_HD uint32_t run_from(const uint32_t *F, uint32_t p, uint32_t cap, uint32_t stride = 64) {
    int64_t w = p >> 5;
    const uint32_t b = p & 31;
    uint32_t x = F[w * stride];
    const uint32_t z = clz32((~x) << (31 - b));
    if (z <= b) return z < cap ? z : cap;
    uint32_t cnt = b + 1;
    for (w = w - 1; w >= 0 && cnt < cap; w--) {
        x = F[w * stride];
        if (x == 0xFFFFFFFFu) {
            cnt += 32;
            continue;
        }
        cnt += clz32(~x);
        break;
    }
    return cnt < cap ? cnt : cap;
}

// encode_sequence + encode_dictionary for one read.  Returns #records (>= 1) or -status.
NTC_HD int encode_lane(const DevIndex &ix, const uint8_t *q, uint32_t len, uint32_t rows,
                       LaneScratch s) {
    if (len == 0) return -kErrEmptyRead;
    if (len > rows) return -kErrCapacity;
    const uint32_t k = ix.k;
    uint32_t d = 0, l = 0, r = ix.n, fw = 0;
    // ---- matching statistics, left to right ---------------------------------------
    for (uint32_t p = 0; p < len; p++) {
        const int c = base_code(q[p]);
        if (c < 0) return -kErrInvalidBase;
        ms_step(ix, c, d, l, r);
        if (d == 0) return -kErrInvalidBase;  // lib.rs:207 would never terminate
        s.D[(uint64_t)p * 64] = (uint8_t)d;
        s.S[(uint64_t)p * 64] = l;
        uint32_t f = 0;
        if (d == k) f = (ix.uniq[l >> 5] >> (l & 31)) & 1u;
        fw |= f << (p & 31);
        if ((p & 31) == 31 || p + 1 == len) {
            s.F[(uint64_t)(p >> 5) * 64] = fw;
            fw = 0;
        }
    }
    // ---- greedy right-to-left parse, lib.rs:175-218 -------------------------------
    uint32_t i = len;
    int nrec = 0;
    while (i > 0) {
        const uint32_t di = s.D[(uint64_t)(i - 1) * 64];
        const uint32_t st = s.S[(uint64_t)(i - 1) * 64];
        const uint32_t segend = i;
        uint32_t seglen;
        if (di == k && i > k + 1) {
            // left_extend_kmer: step e succeeds iff the k-mer ending at i-2-e is indexed
            // and its (k-1)-suffix group is a singleton (Appendix A.3), e < i-k-1
            const uint32_t ext = run_from(s.F, i - 2, i - k - 1);
            const uint32_t L = k + ext;
            uint32_t m = L, p = i;
            for (;;) {  // jump loop lib.rs:193-203
                const uint32_t dp = s.D[(uint64_t)(p - 1) * 64];
                if (dp < m) {
                    if (dp >= p) return -kErrFormat;  // unreachable for a valid index
                    m -= dp;
                    p -= dp;
                } else {
                    break;
                }
            }
            seglen = L - (m - 1);
            i = p;
        } else {
            seglen = di;
            if (i > di) i -= di - 1;
            else i = 0;
        }
        if (seglen >= (1u << 24)) return -kErrLength;  // lib.rs:226
        // encode_dictionary record word (encode.rs:144-158)
        const uint64_t first = nrec == 0 ? 1u : 0u;
        uint64_t w;
        if (seglen > 11) {
            w = (uint64_t)st | ((uint64_t)(seglen & 0xFFFFFFu) << 32) | (first << 56);
        } else {
            // encode.rs:151-152 slices kmer[(k - len)..k]: len > k (only for k <= 10) panics
            if (seglen > k) return -kErrRefPanic;
            // bitnuc::as_2bit of the segment == the query bases it covers
            uint64_t bits = 0;
            for (uint32_t j = 0; j < seglen; j++)
                bits |= (uint64_t)base_code(q[segend - seglen + j]) << (2 * j);
            w = bits | ((uint64_t)((first + 2) | (seglen << 2)) << 56);
        }
        s.R[(uint64_t)nrec * 64] = w;
        nrec++;
        if (i > 0) i -= 1;
        else break;
    }
    return nrec;
}

// ======================================================================================
// Suffix table (encode v5).  d_p, the matching statistic at query position p, is BY
// DEFINITION the length of the longest suffix (<= k) of q[0..p] that is a suffix of some
// node (make_golden.py; StreamingIndex::matching_statistics, lib.rs:172-173), so it only
// depends on q[p-U+1..p] whenever that U-mer is absent.  For every u-mer (u <= U) the
// table holds either its colex interval [x, y) (the u-mer is a node suffix: "long") or,
// when it is absent, y = kTabShort | m and x = S, where m is the length of its longest
// present suffix and S the interval start of that suffix ("short").  Level u holds 4^u
// entries at tab_base(u); key = the u 2-bit codes, first character in the low bits.
// ======================================================================================
constexpr uint32_t kTabShort = 0xFFFFFF00u;  // y >= kTabShort: absent, m = y & 0xFF
constexpr uint32_t kTabPos = 0x80000000u;    // top level, tab_pos: y = kTabPos | path position
                                             // of the single node x (interval [x, x + 1))
constexpr uint32_t kTabMaxU = 15;            // 4^15 entries x 8 B (8.6 GB) at the top level (tab_u option)
constexpr uint32_t kTabDefaultMaxU = 14;     // default cap, one deeper past kTabMaxDensity (default_tab_u)
constexpr double kTabMaxDensity = 0.25;      // distinct U-mers / 4^U

NTC_HD uint64_t tab_base(uint32_t u) { return ((1ULL << (2 * u)) - 4) / 3; }
NTC_HD bool tab_long(uint2 e) { return e.y < kTabShort; }
NTC_HD uint64_t tab_bits_words(uint32_t U) { return U >= 3 ? (1ULL << (2 * U)) / 32 : 1; }
constexpr uint32_t kFiltGap = 2;   // filter level F = U - kFiltGap
constexpr uint32_t kFiltMinU = 12; // below this the level-U bitmap is small enough alone
// auto mode: no filter above 60 % presence (measured: C91's filter at 45 % saves 28 % of
// k_ms4; S91's at 72 % passes ~ 0.72^3 of the positions and costs 5 %)
constexpr int64_t kFiltMaxDensityPpm = 600000;
// joint path runs (MsLaneT<true>) by default when the path cover averages fewer nodes per path
constexpr uint64_t kJointAutoNodesPerPath = 4096;
// interval of a present top-level entry (+ path position of a single node, or ~0)
NTC_HD void tab_interval(const DevIndex &ix, uint2 te, uint32_t &l, uint32_t &r, uint32_t &j) {
    l = te.x;
    if (ix.tab_pos && (te.y & kTabPos)) {
        r = l + 1;
        j = te.y & ~kTabPos;
    } else {
        r = te.y;
        j = 0xFFFFFFFFu;
    }
}

// Pair word of the (U-1)-mer M (by key), from level U of the suffix table:
//   bit a      the U-mer a.M is present (long),
//   bit 4 + c  the U-mer M.c is present,
//   bit 8 + a  the U-mer a.M is present and its interval is a single node,
//   bit 12 + c the U-mer M.c is present and its interval is a single node.
// For M = the (U-1)-mer ending at y, a = the character before M and c = the one after it,
// one word says whether the U-mers ending at y AND y + 1 are present (one cache line per
// SCAN pair test instead of two bitmap lines).  4^(U-1) x 2 bytes.
NTC_HD uint64_t pair_words_count(uint32_t U) { return 1ULL << (2 * (U - 1)); }
NTC_HD bool tab_single(uint2 e) {  // a long entry whose interval is one node
    return tab_long(e) && ((e.y & kTabPos) ? true : e.y == e.x + 1);
}
NTC_HD uint32_t pair_word(const uint2 *top, uint32_t U, uint64_t M) {
    uint32_t w = 0;
    for (uint32_t a = 0; a < 4; a++) {
        const uint2 e = top[a | (M << 2)];
        w |= ((uint32_t)tab_long(e) << a) | ((uint32_t)tab_single(e) << (8 + a));
    }
    for (uint32_t c = 0; c < 4; c++) {
        const uint2 e = top[M | ((uint64_t)c << (2 * (U - 1)))];
        w |= ((uint32_t)tab_long(e) << (4 + c)) | ((uint32_t)tab_single(e) << (12 + c));
    }
    return w;
}

// Window word of the (U-3)-mer K, 8 x 32 bits: bit 64 j + ctx (j = 0..3) says whether the
// U-mer  (3 - j characters) . K . (j characters)  is present, ctx = the 3 - j characters
// before K in the low bits, the j after K above them (2 bits each, first character lowest,
// as key_at packs them).  For K ending at e in a read, one 32-byte entry answers "is the
// U-mer ending at e + j present" for j = 0..3 -- four SCAN positions per cache line, where a
// pair word answers two.  4^(U-3) x 32 bytes (134 MB at U = 14), built from the level-U
// presence bitmap.
NTC_HD uint64_t win_words_count(uint32_t U) { return 1ULL << (2 * (U - 3)); }
NTC_HD uint32_t win_ctx(uint64_t ukey, uint32_t U, uint32_t j) {  // context of the U-mer ending at e + j
    return (uint32_t)(ukey & ((1ULL << (2 * (3 - j))) - 1)) | (uint32_t)((ukey >> (2 * (U - j))) << (2 * (3 - j)));
}
NTC_HD uint32_t win_word(const uint32_t *bits, uint32_t U, uint64_t K, uint32_t i) {  // 32-bit word i of K's entry
    uint32_t w = 0;
    for (uint32_t b = 0; b < 32; b++) {
        const uint32_t j = (32 * i + b) >> 6, ctx = (32 * i + b) & 63u;
        const uint32_t lo = 2 * (3 - j);
        const uint64_t key = (uint64_t)(ctx & ((1u << lo) - 1u)) | (K << lo) | ((uint64_t)(ctx >> lo) << (2 * (U - j)));
        w |= ((bits[key >> 5] >> (key & 31)) & 1u) << b;
    }
    return w;
}

// presence bits of one level: bit key of word key / 32
NTC_HD uint32_t tab_bits_word(const uint2 *top, uint64_t w) {
    uint32_t b = 0;
    for (uint32_t i = 0; i < 32; i++) b |= (uint32_t)tab_long(top[32 * w + i]) << i;
    return b;
}

// entry of u-mer `key` from level u-1 (`prev`; unused for u = 1): the u-mer is present
// iff its (u-1)-prefix is and extends by its last character; else it inherits the
// longest present suffix of its (u-1)-suffix.
NTC_HD uint2 tab_make(const DevIndex &ix, uint32_t u, uint64_t key, const uint2 *prev, bool with_pos = false) {
    const int c = (int)((key >> (2 * (u - 1))) & 3u);
    if (u == 1) {
        const uint32_t a = ix.C[c], b = ix.C[c + 1];
        return a < b ? mk2(a, b) : mk2(0u, kTabShort);
    }
    const uint64_t m1 = (1ULL << (2 * (u - 1))) - 1;
    const uint2 pre = prev[key & m1];
    if (tab_long(pre)) {
        uint32_t nl, nr;
        extend(ix, c, pre.x, pre.y, nl, nr);
        if (nl < nr) {
            if (with_pos && nr == nl + 1 && ix.pos_of_node[nl] != 0xFFFFFFFFu)
                return mk2(nl, kTabPos | ix.pos_of_node[nl]);
            return mk2(nl, nr);
        }
    }
    const uint2 suf = prev[key >> 2];
    return tab_long(suf) ? mk2(suf.x, kTabShort | (u - 1)) : suf;
}

// ======================================================================================
// shared by the flattened encoders
// ======================================================================================
struct BaseReader {
    const uint8_t *q;
    uint64_t blk;
    uint32_t w0, w1, w2, w3;
    NTC_HD explicit BaseReader(const uint8_t *qq) : q(qq), blk(~0ULL), w0(0), w1(0), w2(0), w3(0) {}
    NTC_HD uint32_t get(uint32_t p) {
        const uint64_t a = (uint64_t)(uintptr_t)(q + p);
        if ((a >> 4) != blk) {
            blk = a >> 4;
#ifdef __HIP_DEVICE_COMPILE__
            const uint4 v = *reinterpret_cast<const uint4 *>((uintptr_t)(blk << 4));
            w0 = v.x; w1 = v.y; w2 = v.z; w3 = v.w;
#else
            const uint32_t *v = reinterpret_cast<const uint32_t *>((uintptr_t)(blk << 4));
            w0 = v[0]; w1 = v[1]; w2 = v[2]; w3 = v[3];
#endif
        }
        const uint32_t b = (uint32_t)(a & 15);
        const uint32_t w = (b & 8) ? ((b & 4) ? w3 : w2) : ((b & 4) ? w1 : w0);
        return (w >> ((b & 3) * 8)) & 0xFFu;
    }
};

enum : uint32_t { kModeScan = 0, kModeExt = 1, kModeP1 = 2, kModeBs = 3, kModeBrk = 4, kModeFirst = 5, kModeEnter = 6,
                  kModeBrkLong = 7, kModeExtFail = 8 };
#ifndef NTC_EXT_EAGER
#define NTC_EXT_EAGER 0  // 1: every EXT also loads p's table entry (HBM line) in case the extension fails
#endif
constexpr uint32_t kScanW = 16;      // presence probes per SCAN unit (U + kScanW - 1 <= 32)
#ifndef NTC_SCAN_MODE
#define NTC_SCAN_MODE 0  // 2: SCAN loads the first candidate pair's table entry directly
#endif
constexpr uint32_t kScanExact = 4;   // filter candidates tested exactly per SCAN
#ifndef NTC_BRK_PAIR
#define NTC_BRK_PAIR 1  // run break: long/short from the pair word, not the table entry
#endif
#ifndef NTC_BRK_MERGE
#define NTC_BRK_MERGE 1  // run break check issued with the SCAN after it
#endif
#ifndef NTC_GUESS
#define NTC_GUESS 1  // SCAN after a run break guesses the node along the same path
#endif
#ifndef NTC_GUESS_SLACK
#define NTC_GUESS_SLACK 2  // guess only for x - ge in [U, U + slack] (a lone substitution: x = ge + U)
#endif
#ifndef NTC_BRK_IN_WIN
#define NTC_BRK_IN_WIN 1  // the SCAN after a run break starts at the break position (window words test it)
#endif
#ifndef NTC_BRK_LATE
// 1 (k_ms4 without joint runs): a run break's pair word goes out with the SCAN's pair words,
// only when the break position passes the filter (55 % of breaks at C91 do not: the F-mer
// ending there holds the sequencing error); 0: with the SCAN's filter loads, always
#define NTC_BRK_LATE 1
#endif
#ifndef NTC_START_WINDOW
#define NTC_START_WINDOW 1  // MsLaneT::start loads the read-start query window (see start)
#endif
#ifndef NTC_FIRST_PAIR
// 1: the read start also loads the pair word of position U (is it long?) beside U - 1's
// table entry.  0: a long U - 1 enters the walk directly and the extension at U decides
// (U is short after a long U - 1 only for an error at U or a chance U-mer, ~1 % of reads,
// which then pay the EXT and its failure's table entry instead of one pair-word line per read)
#define NTC_FIRST_PAIR 0
#endif
#ifndef NTC_CHAIN
// A wave runs the blocks of MsLane::step in program order for all its lanes (a wave
// iteration holds ~7.6 distinct modes on C91, so nearly every block runs anyway): a lane
// whose run breaks goes on into the break / SCAN blocks below within the same call instead
// of waiting for the next iteration
#define NTC_CHAIN 1
#endif
#ifndef NTC_PAIR_TESTS
#define NTC_PAIR_TESTS 4  // pair words loaded per SCAN
#endif
#ifndef NTC_WIN_ENTRIES
#define NTC_WIN_ENTRIES 2  // window-word entries per SCAN (4 positions each, one 32-bit load per position)
#endif
#ifndef NTC_PAIR_STRIDE
#define NTC_PAIR_STRIDE 2  // SCAN pair words at non-overlapping positions (or window words): 1 in the joint-run build, 2 always, 0 never
#endif
#ifndef NTC_SEEK_BS
#define NTC_SEEK_BS 1  // EntryView::seek: binary search instead of a forward scan
#endif
constexpr uint32_t kJointPending = 0xFFFFFFFEu;  // joint run wanted, path positions not loaded yet

// ======================================================================================
// Matching statistics as RUN-LENGTH entries.  Positions whose U-mer is absent ("short")
// are not walked at all: the suffix table gives their (d, S).  A position whose U-mer is
// present ("long") right after a short one has d = U exactly (d_p <= d_{p-1} + 1) and S =
// the U-mer's interval start, so it is table-determined too.  A lane only walks the SBWT
// inside stretches of >= 2 consecutive long positions, starting from the first one's
// table interval: one extension per position, or a path RUN once the interval is a single
// node (the next m positions follow the path while the query equals the path text; m is
// found 32 bases at a time by XOR-ing 2-bit words, see derived.cpp "path cover").  When an
// extension fails at a long position, the contraction target t* = max{t < d : ext(I_t, c)}
// is >= U-1 (the U-mer ending there is present), so only the probes above U-1 remain
// (t = d-1, then binary search between U-1 and d-1, each a widen + extend).
// Entries cover exactly the walked positions; the parse reads the rest from the table.
// ======================================================================================
// Characters (<= 64) from path text position T (its three 32-char groups g0..g2) that equal
// the query words qa, qb and end a node's k-mer; with pre > 0 (verifying a guessed node) only
// the k-mer after the first pre characters must be a node
NTC_HD uint32_t path_lim(const uint4 &g0, const uint4 &g1, const uint4 &g2, uint32_t sh, uint64_t qa, uint64_t qb,
                         uint32_t pre) {
    const uint64_t c0 = (uint64_t)g0.x | ((uint64_t)g0.y << 32);
    const uint64_t c1 = (uint64_t)g1.x | ((uint64_t)g1.y << 32);
    const uint64_t c2 = (uint64_t)g2.x | ((uint64_t)g2.y << 32);
    const uint64_t pa = sh ? ((c0 >> (2 * sh)) | (c1 << (64 - 2 * sh))) : c0;
    const uint64_t pb = sh ? ((c1 >> (2 * sh)) | (c2 << (64 - 2 * sh))) : c1;
    uint32_t va = sh ? ((g0.z >> sh) | (g1.z << (32 - sh))) : g0.z;
    if (pre) va |= (1u << (pre - 1)) - 1u;  // of the verified k-mers only node j's must exist
    const uint32_t vb = sh ? ((g1.z >> sh) | (g2.z << (32 - sh))) : g1.z;
    const uint64_t xa = qa ^ pa, xb = qb ^ pb;
    uint32_t la = xa ? (uint32_t)(__builtin_ctzll(xa) >> 1) : 32u;
    const uint32_t ia = ~va ? (uint32_t)__builtin_ctz(~va) : 32u;
    if (ia < la) la = ia;
    // second half computed unconditionally: its loads issue with the first half's
    uint32_t lb = xb ? (uint32_t)(__builtin_ctzll(xb) >> 1) : 32u;
    const uint32_t ib = ~vb ? (uint32_t)__builtin_ctz(~vb) : 32u;
    if (ib < lb) lb = ib;
    return la == 32 ? 32 + lb : la;
}

// path_lim, and in end whether the k-mer end bit at the stop is clear (a path end) when the
// stop is inside the 64 positions
NTC_HD uint32_t path_lim_end(const uint4 &g0, const uint4 &g1, const uint4 &g2, uint32_t sh, uint64_t qa, uint64_t qb,
                             bool &end) {
    const uint64_t c0 = (uint64_t)g0.x | ((uint64_t)g0.y << 32);
    const uint64_t c1 = (uint64_t)g1.x | ((uint64_t)g1.y << 32);
    const uint64_t c2 = (uint64_t)g2.x | ((uint64_t)g2.y << 32);
    const uint64_t pa = sh ? ((c0 >> (2 * sh)) | (c1 << (64 - 2 * sh))) : c0;
    const uint64_t pb = sh ? ((c1 >> (2 * sh)) | (c2 << (64 - 2 * sh))) : c1;
    const uint32_t va = sh ? ((g0.z >> sh) | (g1.z << (32 - sh))) : g0.z;
    const uint32_t vb = sh ? ((g1.z >> sh) | (g2.z << (32 - sh))) : g1.z;
    const uint64_t xa = qa ^ pa, xb = qb ^ pb;
    uint32_t la = xa ? (uint32_t)(__builtin_ctzll(xa) >> 1) : 32u;
    const uint32_t ia = ~va ? (uint32_t)__builtin_ctz(~va) : 32u;
    if (ia < la) la = ia;
    uint32_t lb = xb ? (uint32_t)(__builtin_ctzll(xb) >> 1) : 32u;
    const uint32_t ib = ~vb ? (uint32_t)__builtin_ctz(~vb) : 32u;
    if (ib < lb) lb = ib;
    end = la < 32 ? la == ia : lb < 32 && lb == ib;
    return la == 32 ? 32 + lb : la;
}

struct Entry {       // 16 bytes, one uint4 store
    uint32_t p;      // first position
    uint32_t v;      // SBWT entry: colex start S; run entry: path position of node at p
    uint32_t m;      // positions covered (1 for an SBWT entry)
    uint32_t dk;     // d at p | run << 31
};
constexpr uint32_t kRunTag = 0x80000000u;

// w[0], w[1] with one 16-byte load (w 8-byte aligned: global loads need dword alignment only)
typedef uint64_t u64x2_a8 __attribute__((ext_vector_type(2), aligned(8)));
NTC_HD void load_w2(const uint64_t *w, uint64_t &a, uint64_t &b) {
#ifdef __HIP_DEVICE_COMPILE__
    const u64x2_a8 v = *reinterpret_cast<const u64x2_a8 *>(w);
    a = v.x;
    b = v.y;
#else
    a = w[0];
    b = w[1];
#endif
}
// 32 two-bit characters starting at character offset off (the packed query arrays carry
// padding words past their end, so w[i + 1] is always readable)
NTC_HD uint64_t window2(const uint64_t *w, uint64_t off) {
    const uint64_t i = off >> 5;
    const uint32_t sh = (uint32_t)(off & 31) * 2;
    uint64_t a, b;
    load_w2(w + i, a, b);
    return sh ? ((a >> sh) | (b << (64 - sh))) : a;
}
// 64 bits starting at bit offset off of a bitvector
NTC_HD uint64_t window1(const uint64_t *w, uint32_t off) {
    const uint32_t i = off >> 6, sh = off & 63;
    const uint64_t a = w[i];
    return sh ? ((a >> sh) | (w[i + 1] << (64 - sh))) : a;
}
NTC_HD uint32_t ctz64(uint64_t x) { return x ? (uint32_t)__builtin_ctzll(x) : 64u; }
NTC_HD uint32_t uniq_bit(const DevIndex &ix, uint32_t v) {
    NTC_TOUCH(kTrUniq, ix.uniq + (v >> 5));
    return (ix.uniq[v >> 5] >> (v & 31)) & 1u;
}

// (d, S) of a position not covered by an entry, from the suffix table: u = min(x+1, U)
// characters ending at x; long => d = u (x < U-1: the whole prefix; else the predecessor
// is short, so d = U), short => d = m.
NTC_HD void tab_ds(const DevIndex &ix, const uint64_t *Q, uint64_t qo, uint32_t x, uint32_t &d, uint32_t &s) {
    const uint32_t u = x + 1 < ix.tab_u ? x + 1 : ix.tab_u;
    const uint64_t key = window2(Q, qo + x + 1 - u) & ((1ULL << (2 * u)) - 1);
    NTC_TOUCH(u == ix.tab_u ? kTrTabU : kTrTabLo, ix.tab + tab_base(u) + key);
    const uint2 e = ix.tab[tab_base(u) + key];
    d = tab_long(e) ? u : (e.y & 0xFFu);
    s = e.x;
}

// consecutive set bits at positions a, a-1, ... (at most maxn) of bitvector w.
// NTC_ONES_PAIR=1 loads the word holding a and the one below it together, so that a run
// crossing into the lower word (C31: up to ~100 positions of d = k per record) costs one
// round trip instead of two dependent ones; A/B on one box (round 6, 3 runs each): C31
// 309.7-311.7 Gbases/s with it, 309.9-310.4 without -- the parse's time is not there, so
// it stays off.
#ifndef NTC_ONES_PAIR
#define NTC_ONES_PAIR 0
#endif
NTC_HD uint32_t ones_down(const uint64_t *w, uint32_t a, uint32_t maxn) {
    uint32_t cnt = 0;
    int64_t pos = a;
#if NTC_ONES_PAIR
    {
        const uint32_t wi = (uint32_t)(pos >> 6), b = (uint32_t)(pos & 63);
        NTC_TOUCH(kTrPuniq, w + wi);
        const uint64_t hiw = w[wi], low = w[wi > 0 ? wi - 1 : 0];  // both issued before either is used
        const uint64_t x = ~hiw << (63 - b);
        const uint32_t z = x ? (uint32_t)__builtin_clzll(x) : 64u;
        if (z <= b || wi == 0 || maxn <= b + 1) return (z <= b ? z : b + 1) < maxn ? (z <= b ? z : b + 1) : maxn;
        NTC_TOUCH(kTrPuniq, w + wi - 1);
        cnt = b + 1;
        const uint64_t y = ~low;
        const uint32_t z2 = y ? (uint32_t)__builtin_clzll(y) : 64u;
        if (z2 < 64) { cnt += z2; return cnt < maxn ? cnt : maxn; }
        cnt += 64;
        pos -= b + 1 + 64;
        if (pos < 0) return cnt < maxn ? cnt : maxn;
    }
#endif
    while (cnt < maxn) {
        const uint32_t wi = (uint32_t)(pos >> 6), b = (uint32_t)(pos & 63);
        NTC_TOUCH(kTrPuniq, w + wi);
        const uint64_t x = ~w[wi] << (63 - b);  // bit b -> bit 63
        const uint32_t z = x ? (uint32_t)__builtin_clzll(x) : 64u;
        if (z <= b) { cnt += z; break; }
        cnt += b + 1;
        pos -= b + 1;
        if (pos < 0) break;
    }
    return cnt < maxn ? cnt : maxn;
}

NTC_HD Entry load_entry(const Entry *E, int32_t i) {
    NTC_TOUCH(kTrE, E + i);
#ifdef __HIP_DEVICE_COMPILE__
    const uint4 v = *reinterpret_cast<const uint4 *>(E + i);
    return Entry{v.x, v.y, v.z, v.w};
#else
    return E[i];
#endif
}

// Entry j of a read: j < kEntSlot in the dense slots Ed[j * es] (the kernels keep each read's
// first entries together, Ed = base + read id * kEntSlot, es = 1: k_ms4 writes them as one
// 64-byte group when the read ends, MsLane::finish, and the parse finds a read's first
// entries in one line); the next S in the read's secondary slots, E[j] (E = the read's
// S-entry slot - kEntSlot); any later ones in the overflow pool, E2[j] (E2 = the read's
// reservation - kEntSlot - S, MsLaneT::reserve).  Ed = E with S = kNoLimit is the plain
// contiguous layout.  Every slot is sized by need: S per read from the index kind, the pool
// from what earlier calls used (grown and re-run when a call runs out, capi.cpp).
constexpr uint32_t kEntSlot = 4;
constexpr uint32_t kNoLimit = 0xFFFFFFFFu;
NTC_HD const Entry *ent_ptr(const Entry *E, const Entry *Ed, uint64_t es, uint32_t j, const Entry *E2 = nullptr,
                            uint32_t S = kNoLimit) {
    return j < kEntSlot ? Ed + (uint64_t)j * es : (j - kEntSlot < S ? E + j : E2 + j);
}

// Right-to-left reader of one read's entries (+ suffix table for uncovered positions).
struct EntryView {
    const Entry *E;
    const Entry *Ed;  // dense slots (see ent_ptr)
    const Entry *E2;  // overflow reservation (see ent_ptr)
    uint32_t S;
    uint64_t es;
    const DevIndex *ix;
    const uint64_t *Q;
    uint64_t qo;
    uint32_t k;
    int32_t e;  // cursor (-1: the read has no entries); moves left only
    Entry cur;  // E[e]
    // the dense group in registers (k_parse4 loads it in one round trip; dc = held): entries
    // 0..3 then cost no dependent load in the seeks and run scans
    Entry c0{0, 0, 0, 0}, c1{0, 0, 0, 0}, c2{0, 0, 0, 0}, c3{0, 0, 0, 0};
    bool dc = false;
    NTC_HD EntryView(const Entry *E_, const DevIndex *ix_, const uint64_t *Q_, uint64_t qo_, uint32_t k_, int32_t e_,
                     const Entry *Ed_ = nullptr, uint64_t es_ = 1, const Entry *pre = nullptr,
                     const Entry *E2_ = nullptr, uint32_t S_ = kNoLimit)
        : E(E_), Ed(Ed_ ? Ed_ : E_), E2(E2_), S(S_), es(Ed_ ? es_ : 1), ix(ix_), Q(Q_), qo(qo_), k(k_), e(e_),
          cur{0, 0, 0, 0} {
        if (pre) {
            c0 = pre[0];
            c1 = pre[1];
            c2 = pre[2];
            c3 = pre[3];
            dc = true;
        }
        if (e >= 0) cur = at(e);
    }
    NTC_HD Entry at(int32_t i) const {
        if (dc && i < (int32_t)kEntSlot) {  // field by field: a select of whole structs goes through scratch
            uint32_t p = c0.p, v = c0.v, m = c0.m, dk = c0.dk;
            p = i == 1 ? c1.p : p; v = i == 1 ? c1.v : v; m = i == 1 ? c1.m : m; dk = i == 1 ? c1.dk : dk;
            p = i == 2 ? c2.p : p; v = i == 2 ? c2.v : v; m = i == 2 ? c2.m : m; dk = i == 2 ? c2.dk : dk;
            p = i == 3 ? c3.p : p; v = i == 3 ? c3.v : v; m = i == 3 ? c3.m : m; dk = i == 3 ? c3.dk : dk;
            return Entry{p, v, m, dk};
        }
        return load_entry(ent_ptr(E, Ed, es, (uint32_t)i, E2, S), 0);
    }
    NTC_HD void seek(uint32_t x) {  // last entry with p <= x, or entry 0
        if (e <= 0 || cur.p <= x) return;
        // every entry covers >= 1 position, so entry e - (p - x) starts at or before x
        int32_t g = e - (int32_t)(cur.p - x);
        if (g < 0) g = 0;
#if NTC_SEEK_BS
        // binary search in [g, e): run entries cover many positions each (joint runs on
        // strain collections), so the bound g is often far below the answer and a forward
        // scan from it is a long chain of dependent loads
        int32_t hi = e;
        Entry eg{0, 0, 0, 0};
        bool have = false;

        while (hi - g > 1) {
            const int32_t mid = (g + hi) >> 1;
            const Entry em = at(mid);
            if (em.p <= x) {
                g = mid;
                eg = em;
                have = true;
            } else {
                hi = mid;
            }
        }
        if (!have) eg = at(g);
#else
        Entry eg = at(g);
        while (g + 1 < e) {
            const Entry nx = at(g + 1);
            if (nx.p > x) break;
            g++;
            eg = nx;
        }
#endif
        e = g;
        cur = eg;
    }
    NTC_HD bool covered(uint32_t x) {
        seek(x);
        return e >= 0 && cur.p <= x && x < cur.p + cur.m;
    }
    NTC_HD uint32_t dval(const Entry &en, uint32_t x) const {
        const uint32_t d0 = en.dk & 0xFFu;
        const uint32_t d = d0 + (x - en.p);
        return (en.dk & kRunTag) ? (d < k ? d : k) : d0;
    }
    NTC_HD uint32_t sval(const Entry &en, uint32_t x) const {
        if (en.dk & kRunTag) NTC_TOUCH(kTrColex, ix->colex_at + en.v + (x - en.p));
        return (en.dk & kRunTag) ? (ix->colex_at[en.v + (x - en.p)] & 0x7FFFFFFFu) : en.v;
    }
    NTC_HD uint32_t D(uint32_t x) {
        if (covered(x)) return dval(cur, x);
        uint32_t d, s;
        tab_ds(*ix, Q, qo, x, d, s);
        return d;
    }
    // d at x, and S at x when S is needed for a record (d > 11 or d = k)
    NTC_HD void DS(uint32_t x, uint32_t &d, uint32_t &s) {
        if (covered(x)) {
            d = dval(cur, x);
            s = (d > 11 || d == k) ? sval(cur, x) : 0u;
        } else {
            tab_ds(*ix, Q, qo, x, d, s);
        }
    }
    // consecutive positions x, x-1, ... with d = k and a singleton (k-1)-suffix group
    // (left_extend_kmer's per-step test)
    NTC_HD uint32_t run_from(uint32_t x, uint32_t cap) const {
        int32_t c = e;
        uint32_t cnt = 0;
        int64_t pos = x;
        Entry en = cur;
        while (cnt < cap && pos >= 0) {
            while (c > 0 && en.p > (uint32_t)pos) en = at(--c);
            if (!(c >= 0 && en.p <= (uint32_t)pos && (uint32_t)pos < en.p + en.m)) {
                // uncovered: d = min(pos + 1, U), = k only for U = k and a long position
                if (ix->tab_u != k || (uint32_t)pos + 1 < k) break;
                uint32_t d, s;
                tab_ds(*ix, Q, qo, (uint32_t)pos, d, s);
                if (d != k || !uniq_bit(*ix, s)) break;
                cnt++;
                pos--;
                continue;
            }
            const uint32_t d0 = en.dk & 0xFFu;
            if (!(en.dk & kRunTag)) {
                if (d0 != k || !uniq_bit(*ix, en.v)) break;
                cnt++;
                pos--;
                continue;
            }
            const uint32_t tx = (uint32_t)pos - en.p;
            const uint32_t tk = d0 >= k ? 0u : k - d0;  // first t with d = k
            if (tx < tk) break;
            const uint32_t want = tx - tk + 1;
            const uint32_t got = ones_down(ix->puniq, en.v + tx, want);
            cnt += got;
            if (got < want || tk > 0) break;
            pos = (int64_t)en.p - 1;
        }
        return cnt < cap ? cnt : cap;
    }
};

// ======================================================================================
// encode pipeline:
//   k_pack   : reads -> 2-bit words in "position space" (character x of the batch at
//              bits 2(x%32) of word x/32); validates bases.
//   k_ms     : persistent waves; each lane runs MsLane units (one per loop iteration) and,
//              when its read is done, takes the next read from a wave-local pool refilled
//              by one atomicAdd per 64 reads (a read with many errors does not hold 63
//              finished lanes hostage).
//   k_parse  : one lane per read: right-to-left parse over the entries -> records.
// Entries and records live in position space (read r at [P_r, P_r + len_r)).
// ======================================================================================
NTC_HD int pack_read(const uint8_t *q, uint32_t len, uint64_t *Q, uint32_t absent) {
    if (len == 0) return -kErrEmptyRead;
    BaseReader br(q);
    uint64_t acc = 0;
    for (uint32_t p = 0; p < len; p++) {
        const int c = base_code((uint8_t)br.get(p));
        if (c < 0 || ((absent >> c) & 1u)) return -kErrInvalidBase;
        acc |= (uint64_t)c << (2 * (p & 31));
        if ((p & 31) == 31) {
            Q[p >> 5] = acc;
            acc = 0;
        }
    }
    if (len & 31) Q[len >> 5] = acc;
    return 0;
}

// 2-bit code of an ASCII base: ((b >> 1) ^ (b >> 2)) & 3 maps A,C,G,T to 0,1,2,3
NTC_HD uint32_t fast_code(uint32_t b) { return ((b >> 1) ^ (b >> 2)) & 3u; }
NTC_HD bool is_acgt(uint32_t b) { return b == 'A' || b == 'C' || b == 'G' || b == 'T'; }


NTC_HD void store_entry(Entry *E, uint64_t i, uint32_t p, uint32_t v, uint32_t m, uint32_t dk) {
    NTC_TOUCH(kTrEw, E + i);
#if defined(__HIP_DEVICE_COMPILE__) && (NTC_NT & 16)
    u32x4_t x = {p, v, m, dk};
    __builtin_nontemporal_store(x, reinterpret_cast<u32x4_t *>(E + i));
#elif defined(__HIP_DEVICE_COMPILE__)
    *reinterpret_cast<uint4 *>(E + i) = make_uint4(p, v, m, dk);
#else
    E[i] = Entry{p, v, m, dk};
#endif
}

// The batch's packed query stream and entry slots: the same for every lane, so they are
// passed to each call (scalar registers) rather than held per lane.
struct MsBufs {
    const uint64_t *Q;
    Entry *Es;    // secondary slots: spilled entry s < S of read rid at Es[rid * S + s] (S % 4 == 0)
    Entry *Ed;    // dense entry slots (ent_ptr): entry j < kEntSlot of read rid at Ed[rid * ds + j * es]
    uint64_t es;
    uint4 *stage = nullptr;  // k_ms4: the block's LDS write-combining slots (MsLane::put_entry)
    uint64_t ds = 1;
    uint32_t S = kNoLimit;   // secondary slots per read (kNoLimit: Es holds all of a read's spill)
    Entry *Ep = nullptr;     // overflow pool: reservations of 4-entry groups (MsLaneT::reserve)
    uint64_t pcap = 0;       // pool entries
    unsigned long long *pcnt = nullptr;  // pool entries reserved (zeroed per call)
    uint32_t *obase = nullptr;           // each overflowing read's reservation start
    unsigned long long *status = nullptr;
    uint2 *bs = nullptr;  // k_ms4 with joint runs: each lane's binary-search best interval in LDS
};
// The call ran out of an overflow pool: status 0 (below every read's (read << 8 | code)), the
// parse and emit skip, and the host grows the pool to the reserved total and runs it again.
constexpr unsigned long long kStatusRegrow = 0;
// the host emulator's lane (tests/emu): its slot of the staging array, as threadIdx.x in k_ms4
inline uint32_t ntc_host_lane = 0;
NTC_HD uint32_t stage_lane() {
#ifdef __HIP_DEVICE_COMPILE__
    return threadIdx.x;
#else
    return ntc_host_lane;
#endif
}
#ifndef NTC_ECOMB
#define NTC_ECOMB 1  // combine a read's spilled entries into 64-byte groups in LDS before storing
#endif
constexpr uint32_t kStageSlots = 4;  // 64 B: one write request instead of four 16 B partial ones
// k_ms4 keeps a read's entry 0 in LDS too and stores it when the read is done, with the read's
// entry count in bits 8..30 of its dk (d is 8 bits, bit 31 the run tag): the separate 4-byte
// count store per read (a partial write request of its own) is needed only for counts
// >= kNeInE0 (read_entry_count)
constexpr uint32_t kNeInE0 = 0x7FFFFFu;
NTC_HD uint32_t entry0_count(const Entry &e0) { return (e0.dk >> 8) & kNeInE0; }

// NTC_QCACHE: the non-joint run loop keeps its query words as two aligned pairs across chunks
// (MsLaneT::qA0..qB1).  It takes k_ms4 to 72 VGPRs, so the non-joint build runs at 7 waves
// (NTC_MS_WAVES): A/B on one box, 3 runs each, C91 k_ms4 2.70-2.72 -> 2.60-2.64 ms, step
// 4.31-4.33 -> 4.26-4.27 ms (351.6-351.9 against 346.5-347.9 Gbases/s); 7 waves without the
// cache 2.67-2.68 ms, 4.34-4.37 ms (profiles/round6/ab_qcache/).  The joint build has no room.
#ifndef NTC_QCACHE
#define NTC_QCACHE 1
#endif
// kJoint: joint path runs over multi-node intervals (note_single); k_ms4 is built both ways
// and the upload picks one (ctx option "joint"), since the code costs C91 ~1 % of k_ms4
template <bool kJoint>
struct MsLaneT {
    uint64_t qo;        // this read starts at character qo of Q; its entries at E + qo
    uint32_t rid;       // read id (dense entry slots; a call holds < 2^32 reads)
    uint64_t qw;        // query characters [qb, qb + 32) of this read, cached
    uint32_t qb;
    uint32_t len, p, d, l, r, j, ne, mode, hi, lo, l1, r1, bl, bR;
    uint32_t gj, ge;    // last run break: at position ge, node before it at path position gj (ge = 0: none)
    // (the read's overflow reservation is read back from b.obase[rid], which reserve() writes:
    // a register for it, live across the whole loop, cost the joint build its 7th wave)
    uint32_t vfy;       // the next run first verifies the vfy characters ending at node j
    // Joint run (note_single): path position of the interval's last node, else 0xFFFFFFFF.
    // It lives in l1, which only the binary-search probes use (written before read in
    // kModeBs); a separate field costs k_ms4 a wave of occupancy (72 VGPRs is the 7-wave limit).
    NTC_HD uint32_t &jy() { return l1; }
    bool try_run;
#if NTC_QCACHE
    // (non-joint build) the run loop's query words as two aligned pairs, pair qpa (words
    // 2 qpa, 2 qpa + 1) and pair qpa + 1: the next 64-character chunk of a run needs at most
    // one new pair, so the loop loads 16 aligned bytes instead of 24 at each chunk and none
    // when the run stopped inside the chunk before.  Q does not change during a launch, so a
    // pair held from an earlier read stays valid.
    uint64_t qA0 = 0, qA1 = 0, qB0 = 0, qB1 = 0;
    uint32_t qpa = 0xFFFFFFFFu;
#endif

    // Q (NTC_START_WINDOW): the read-start window is loaded here, so that its round trip
    // overlaps the other lanes' run loads instead of adding one to the read-start block
    NTC_HD void start(const DevIndex &ix, uint64_t qo_, uint32_t len_, uint64_t rid_ = 0, const uint64_t *Q = nullptr) {
        qo = qo_;
        rid = (uint32_t)rid_;
        len = len_;
        qw = 0;
        qb = 0xFFFFFFFFu;
        if (NTC_START_WINDOW && Q && len_ >= ix.tab_u + 1) {
            qb = 0;
            NTC_TOUCH(kTrQ, Q + (qo_ >> 5));
            NTC_TOUCH(kTrQ, Q + (qo_ >> 5) + 1);
            qw = window2(Q, qo_);
        }
        p = 0; d = 0; l = 0; r = ix.n; j = 0xFFFFFFFFu; ne = 0;
        mode = kModeFirst; lo = r1 = bl = bR = 0;
        hi = kScanW;  // SCAN width cap (hi is free while scanning)
        gj = ge = vfy = 0;
        jy() = 0xFFFFFFFFu;
        try_run = false;
    }
    NTC_HD void window(const MsBufs &b, uint32_t from) {
        const uint64_t *Q = b.Q;
        qb = from;
        NTC_TOUCH(kTrQ, Q + ((qo + from) >> 5));
        NTC_TOUCH(kTrQ, Q + ((qo + from) >> 5) + 1);
        qw = window2(Q, qo + from);
    }
    // the binary search's best interval ext(I_lo, c): in LDS in the joint build on the device
    // (two registers live across the loop cost it the 7th wave), else in bl / bR
    NTC_HD void put_best(const MsBufs &b, uint32_t x, uint32_t y) {
#ifdef __HIP_DEVICE_COMPILE__
        if constexpr (kJoint) {
            b.bs[stage_lane()] = make_uint2(x, y);
            return;
        }
#endif
        (void)b;
        bl = x;
        bR = y;
    }
    NTC_HD uint2 best(const MsBufs &b) const {
#ifdef __HIP_DEVICE_COMPILE__
        if constexpr (kJoint) return b.bs[stage_lane()];
#endif
        (void)b;
        return make_uint2(bl, bR);
    }
    NTC_HD bool covers(uint32_t x0, uint32_t x1) const { return qb != 0xFFFFFFFFu && x0 >= qb && x1 < qb + 32; }
    NTC_HD uint64_t key_at(uint32_t x, uint32_t U) const {  // U-mer ending at x (cached window)
        return (qw >> (2 * (x + 1 - U - qb))) & ((1ULL << (2 * U)) - 1);
    }
    // Spilled entry s (entry kEntSlot + s): secondary slot s < S, else the overflow
    // reservation (null when the pool ran out: the call is re-run, nothing is read back).
    NTC_HD Entry *spill_at(const MsBufs &b, uint32_t s) const {
        if (s < b.S) return b.Es + (uint64_t)rid * b.S + s;
        const uint32_t ob = b.obase[rid];  // written by reserve() (this lane, earlier)
        return ob == kNoLimit ? nullptr : b.Ep + ob + (s - b.S);
    }
    // First overflow entry, at position p_: the read has at most len - p_ entries from here
    // (each starts at its own position), reserved in 4-entry groups so that the 64-byte
    // write groups stay aligned.
    NTC_HD void reserve(const MsBufs &b, uint32_t p_) {
        const uint64_t need = (uint64_t)((len - p_ + 3u) & ~3u);
#ifdef __HIP_DEVICE_COMPILE__
        const uint64_t at = atomicAdd(b.pcnt, (unsigned long long)need);
#else
        const uint64_t at = *b.pcnt;
        *b.pcnt += need;
#endif
        if (at + need <= b.pcap) {
            b.obase[rid] = (uint32_t)at;
        } else {
            b.obase[rid] = kNoLimit;
#ifdef __HIP_DEVICE_COMPILE__
            atomicMin(b.status, kStatusRegrow);
#else
            *b.status = kStatusRegrow;
#endif
        }
    }
    NTC_HD void put_entry(const MsBufs &b, uint32_t p_, uint32_t v, uint32_t m, uint32_t dk) {
        if (ne >= kEntSlot && ne - kEntSlot == b.S) reserve(b, p_);
#if NTC_ECOMB
        // Spilled entries of one read are consecutive 16 B slots, written one per lane
        // iteration; stored one by one, each became its own 32 B partial write request past
        // L2 (S91: 60 per read, 38 % of k_ms4's requests).  They are collected per aligned
        // 64-byte group in LDS and stored together, so L2 sends one 64 B request.  The dense
        // slots of a read are one 64-byte group too (k_ms4 lays them out read-major,
        // Ed[rid * kEntSlot + j]): staged until the read ends, or until its first spilled
        // entry, when entries 1..3 go out and entry 0 moves to slot kStageSlots to wait for
        // the count (finish).
        static_assert(kEntSlot == kStageSlots, "dense slots and staging groups share the LDS slots");
        const uint32_t t = stage_lane();
        if (ne < kEntSlot) {
            b.stage[ne * 256 + t] = make_uint4(p_, v, m, dk);
            ne++;
            return;
        }
        if (ne == kEntSlot) {
            Entry *dst = b.Ed + (uint64_t)rid * b.ds;
#pragma unroll
            for (uint32_t i = 1; i < kEntSlot; i++) {
                const uint4 x = b.stage[i * 256 + t];
                store_entry(dst, (uint64_t)i * b.es, x.x, x.y, x.z, x.w);
            }
            b.stage[kStageSlots * 256 + t] = b.stage[t];
        }
        const uint32_t s = ne - kEntSlot;
        b.stage[(s & (kStageSlots - 1)) * 256 + t] = make_uint4(p_, v, m, dk);
        ne++;
        if ((s & (kStageSlots - 1)) == kStageSlots - 1) flush_stage(b);
        return;
#endif
        Entry *dst = ne < kEntSlot ? b.Ed + (uint64_t)rid * b.ds : spill_at(b, ne - kEntSlot);
        if (dst) store_entry(dst, ne < kEntSlot ? (uint64_t)ne * b.es : 0, p_, v, m, dk);
        ne++;
    }
    // the staged entries of the group holding entry ne - 1 (at the end of a group or of the
    // read); groups start at spilled entry 0, S and the reservation start, all multiples of 4
    NTC_HD void flush_stage(const MsBufs &b) {
#if NTC_ECOMB
        if (ne <= kEntSlot) return;
        const uint32_t last = ne - 1 - kEntSlot, g = last & ~(kStageSlots - 1);
        Entry *dst = spill_at(b, g);
        if (!dst) return;
        const uint32_t t = stage_lane();
#pragma unroll
        for (uint32_t i = 0; i < kStageSlots; i++) {
            if (g + i <= last) {
                const uint4 x = b.stage[i * 256 + t];
                store_entry(dst, i, x.x, x.y, x.z, x.w);
            }
        }
#else
        (void)b;
#endif
    }
    // the read is done: staged entries out, entry 0 with the count; true when the count does
    // not fit entry 0 and goes to the count array instead
    NTC_HD bool finish(const MsBufs &b) {
#if NTC_ECOMB
        const uint32_t t = stage_lane();
        const uint32_t c = ne < kNeInE0 ? ne : kNeInE0;
        Entry *dst = b.Ed + (uint64_t)rid * b.ds;
        if (ne > kEntSlot) {
            flush_stage(b);
            const uint4 x = b.stage[kStageSlots * 256 + t];
            store_entry(dst, 0, x.x, x.y, x.z, (x.w & ~(kNeInE0 << 8)) | (c << 8));
        } else {  // the dense group: entry 0 (with the count, also for ne = 0) .. ne - 1
            const uint4 x = ne ? b.stage[t] : make_uint4(0, 0, 0, 0);
            store_entry(dst, 0, x.x, x.y, x.z, (x.w & ~(kNeInE0 << 8)) | (c << 8));
#pragma unroll
            for (uint32_t i = 1; i < kEntSlot; i++)
                if (i < ne) {
                    const uint4 y = b.stage[i * 256 + t];
                    store_entry(dst, (uint64_t)i * b.es, y.x, y.y, y.z, y.w);
                }
        }
        return c == kNeInE0;
#else
        (void)b;
        return true;
#endif
    }
    // after a commit: look for the path position of a single-node interval.  A multi-node
    // interval [l, r) (d < k: strains sharing the read's suffix) starts a JOINT run when both
    // its first and its last node lie on paths: while both paths go on with the query's next
    // character c, both nodes have edge c and ext([l, r), c) = [succ(l), succ(r - 1) + 1)
    // (successors keep colex order; the first and last nodes with edge c bound the
    // extension), so the interval start follows l's path and d climbs by one per position --
    // the entries are ordinary run entries on l's path
    NTC_HD void note_single(const DevIndex &ix) {
        j = 0xFFFFFFFFu;
        jy() = 0xFFFFFFFFu;
        if (ix.has_paths && r == l + 1 && d >= ix.t_jump) {
            NTC_TOUCH(kTrPon, ix.pos_of_node + l);
            j = ld_hint<256>(ix.pos_of_node + l);
            try_run = j != 0xFFFFFFFFu;
        }
        else if (kJoint && ix.has_paths && r > l + 1 && d >= ix.t_jump && d + 1 < ix.k) {
            jy() = kJointPending;  // both path positions are looked up by the run block (step)
            try_run = true;
        }
    }
    NTC_HD int commit(const DevIndex &ix, const MsBufs &b, uint32_t nl, uint32_t nr, uint32_t nd) {
        l = nl; r = nr; d = nd;
        put_entry(b, p, l, 1u, d);
        p++;
        mode = kModeExt;
        note_single(ix);
        return p >= len ? 1 : 0;
    }
    // position p is short with table value m: d_{p+i} <= m + i, so p+1 .. p+U-1-m are
    // short too.  A lone error at p leaves the pair (p + U, p + U + 1): the next SCAN
    // needs m + 2 positions to reach it.
    NTC_HD void skip_short(const MsBufs &b, uint2 te, uint32_t U) {
        const uint32_t m = te.y & 0xFFu;
        p += U - m;
        mode = kModeScan;
        hi = m + 2 < kScanW ? m + 2 : kScanW;
    }
    // x and x + 1 are long, x's predecessor short: walk from x (d = U, table interval)
    NTC_HD int enter_pair(const DevIndex &ix, const MsBufs &b, uint32_t x, uint2 te) {
        uint32_t jj;
        tab_interval(ix, te, l, r, jj);
        d = ix.tab_u;
        p = x + 1;
        mode = kModeExt;
        if (ix.tab_pos) {  // the table already holds the path position (d = U >= t_jump)
            jy() = 0xFFFFFFFFu;
            j = jj;
            try_run = jj != 0xFFFFFFFFu;
        } else {
            note_single(ix);
        }
        return 0;
    }
    // one unit of work: 1 = read finished, 0 = continue, < 0 = error
    NTC_HD int step(const DevIndex &ix, const MsBufs &b) {
        const uint32_t k = ix.k, U = ix.tab_u;
        const uint64_t *Q = b.Q;
        if (p >= len) return 1;
        if (kJoint && try_run && jy() == kJointPending) {
            NTC_TOUCH(kTrPon, ix.pos_of_node + l);
            NTC_TOUCH(kTrPon, ix.pos_of_node + r - 1);
            j = ld_hint<256>(ix.pos_of_node + l);
            jy() = ld_hint<256>(ix.pos_of_node + r - 1);
            if (j == 0xFFFFFFFFu || jy() == 0xFFFFFFFFu) {
                jy() = 0xFFFFFFFFu;
                try_run = false;  // on with the extension at p
            }
        }
        if (try_run) {
            try_run = false;
            uint32_t pre = vfy & 0xFFu, m = 0;
            // (joint-run build) hop pending: the run before stopped inside its window at p - 1
            // with the read going on, its entry written; j (and jy() for a joint run) is the path
            // position of the last node it covered on each side, vfy >> 8 = 4 + the read's
            // character c at p (see the stop below)
            uint32_t hopc = kJoint ? vfy >> 8 : 0u;
            bool nohop = false;
            vfy = 0;
            for (;;) {
                // 64 path characters after node j's k-mer (from pre characters before its end
                // when verifying a guessed node), and whether the k-mer ending at each of them
                // is a node, from three interleaved 32-char groups
                const uint64_t T = (uint64_t)j + k + m - pre;
                NTC_TOUCH(kTrPst, ix.pstream + (T >> 5));
                NTC_TOUCH(kTrPst, ix.pstream + (T >> 5) + 2);
                NTC_TOUCH(kTrQ, Q + ((qo + p + m - pre) >> 5));
                NTC_TOUCH(kTrQ, Q + ((qo + p + m - pre) >> 5) + 2);
                const uint4 g0 = ld4<4>(ix.pstream + (T >> 5)), g1 = ld4<4>(ix.pstream + (T >> 5) + 1),
                            g2 = ld4<4>(ix.pstream + (T >> 5) + 2);
                // a hop loads the fork block entry of c with the path text: one round trip
                uint4 ex = make_uint4(0, 0, 0, 0);
                if (kJoint && (hopc & 8u)) {
                    NTC_TOUCH(kTrColex, ix.colex_at + fork_block((uint64_t)j + 1) + 4 * (hopc & 3u));
                    ex = ld4<64>(reinterpret_cast<const uint4 *>(ix.colex_at + fork_block((uint64_t)j + 1)) + (hopc & 3u));
                }
                const uint32_t sh = (uint32_t)(T & 31);
                const uint64_t c0 = (uint64_t)g0.x | ((uint64_t)g0.y << 32);
                const uint64_t c1 = (uint64_t)g1.x | ((uint64_t)g1.y << 32);
                const uint64_t c2 = (uint64_t)g2.x | ((uint64_t)g2.y << 32);
                uint64_t pa = sh ? ((c0 >> (2 * sh)) | (c1 << (64 - 2 * sh))) : c0;
                uint64_t pb = sh ? ((c1 >> (2 * sh)) | (c2 << (64 - 2 * sh))) : c1;
                uint32_t va = sh ? ((g0.z >> sh) | (g1.z << (32 - sh))) : g0.z;
                if (pre) va |= (1u << (pre - 1)) - 1u;  // of the verified k-mers only node j's must exist
                uint32_t vb = sh ? ((g1.z >> sh) | (g2.z << (32 - sh))) : g1.z;
                // hop, x side: the path's next node when the path goes on with c (mid-path: a
                // node's only successor), the fork block's node and characters at a path end
                // (k-mer end bit clear), else none
                uint32_t nx = j + 1, cap = 64;
                if (kJoint && hopc) {
                    NTC_STAT(0);
                    if (!(va & 1u)) {
                        NTC_STAT(1);
                        nx = ex.x;
                        pa = (uint64_t)ex.y | ((uint64_t)ex.z << 32);
                        va = ex.w;
                        pb = 0;
                        vb = 0;
                        cap = 32;
                    } else if ((uint32_t)(pa & 3u) != (hopc & 3u)) {
                        nx = 0xFFFFFFFFu;
                    }
                }
                const uint64_t q = qo + p + m - pre;
                const uint64_t qi = q >> 5;
                const uint32_t qs = (uint32_t)(q & 31) * 2;
                uint64_t w0, w1, w2;
#if NTC_QCACHE
                if constexpr (!kJoint) {
                    const uint32_t a2 = (uint32_t)(qi >> 1);  // words qi .. qi + 2 lie in pairs a2, a2 + 1
                    const bool hit = a2 == qpa, slide = qpa != 0xFFFFFFFFu && a2 == qpa + 1;
                    uint64_t L0 = slide ? qB0 : qA0, L1 = slide ? qB1 : qA1, H0 = qB0, H1 = qB1;
                    if (!hit && !slide) load_w2(Q + 2 * (uint64_t)a2, L0, L1);
                    if (!hit) load_w2(Q + 2 * (uint64_t)a2 + 2, H0, H1);
                    qpa = a2;
                    qA0 = L0;
                    qA1 = L1;
                    qB0 = H0;
                    qB1 = H1;
                    const bool odd = qi & 1;
                    w0 = odd ? L1 : L0;
                    w1 = odd ? H0 : L1;
                    w2 = odd ? H1 : H0;
                } else
#endif
                {
                    load_w2(Q + qi, w0, w1);
                    w2 = Q[qi + 2];
                }
                const uint64_t qa = qs ? ((w0 >> qs) | (w1 << (64 - qs))) : w0;
                const uint64_t qb2 = qs ? ((w1 >> qs) | (w2 << (64 - qs))) : w1;
                const uint64_t xa = qa ^ pa, xb = qb2 ^ pb;
                uint32_t la = xa ? ctz64(xa) >> 1 : 32u;
                const uint32_t ia = ~va ? (uint32_t)__builtin_ctz(~va) : 32u;
                if (ia < la) la = ia;
                // second half computed unconditionally: its loads issue with the first half's
                uint32_t lb = xb ? ctz64(xb) >> 1 : 32u;
                const uint32_t ib = ~vb ? (uint32_t)__builtin_ctz(~vb) : 32u;
                if (ib < lb) lb = ib;
                uint32_t lim = la == 32 ? 32 + lb : la;
                const uint32_t lx = lim;
                const bool xend = la < 32 ? la == ia : lb < 32 && lb == ib;  // x's stop (at lx) is a path end
                uint32_t ny = nx, ly = 64;
                bool yend = false;  // the y side's stop (at ly) is a path end
                if (kJoint && jy() != 0xFFFFFFFFu) {  // joint run: the interval's last node follows its path too
#if defined(__HIP_DEVICE_COMPILE__)
                    __asm__ volatile("" ::: "memory");  // after lim: the loads below must not overlap the x path's
#endif
                    const uint64_t Ty = (uint64_t)jy() + k + m;
                    NTC_TOUCH(kTrPst, ix.pstream + (Ty >> 5));
                    NTC_TOUCH(kTrPst, ix.pstream + (Ty >> 5) + 2);
                    const uint4 h0 = ld4<4>(ix.pstream + (Ty >> 5)), h1 = ld4<4>(ix.pstream + (Ty >> 5) + 1),
                                h2 = ld4<4>(ix.pstream + (Ty >> 5) + 2);
                    uint4 ey = make_uint4(0, 0, 0, 0);
                    if (hopc & 16u) {
                        NTC_TOUCH(kTrColex, ix.colex_at + fork_block((uint64_t)jy() + 1) + 4 * (hopc & 3u));
                        ey = ld4<64>(reinterpret_cast<const uint4 *>(ix.colex_at + fork_block((uint64_t)jy() + 1)) +
                                    (hopc & 3u));
                    }
                    const uint32_t shy = (uint32_t)(Ty & 31);
                    ny = jy() + 1;
                    if (hopc) NTC_STAT(2);
                    if (hopc && !((h0.z >> shy) & 1u)) {  // hop, y side at its path end
                        NTC_STAT(3);
                        ny = ey.x;
                        const uint64_t x = qa ^ ((uint64_t)ey.y | ((uint64_t)ey.z << 32));
                        ly = x ? ctz64(x) >> 1 : 32u;
                        const uint32_t iv = ~ey.w ? (uint32_t)__builtin_ctz(~ey.w) : 32u;
                        yend = iv <= ly;
                        if (iv < ly) ly = iv;
                        cap = 32;
                    } else {
                        if (hopc && ((shy < 16 ? h0.x >> (2 * shy) : h0.y >> (2 * (shy - 16))) & 3u) != (hopc & 3u))
                            ny = 0xFFFFFFFFu;
                        ly = path_lim_end(h0, h1, h2, shy, qa, qb2, yend);
                    }
                    if (ly < lim) lim = ly;
                }
                if (kJoint && hopc) {
                    // the extension of the interval is the interval of the sides' next nodes (the
                    // first and last node of an interval with edge c extend to the first and last
                    // node of the extension) at depth d + 1: a single node (or both sides at one
                    // node) or, below k - 1, a joint interval, under the conditions note_single
                    // applies.  The run goes on from there as a new run entry (the same (d, S) per
                    // position as the SBWT entry + run of the path through colex_at, EXT and
                    // pos_of_node it replaces).  (A next node at path position 0 would make
                    // j = nx - 1 the "none" value: left to EXT.)
                    hopc = 0;
                    const bool joint = jy() != 0xFFFFFFFFu, single = !joint || ny == nx;
                    const uint32_t d1 = d + 1 < k ? d + 1 : k;
                    if (nx == 0xFFFFFFFFu || nx == 0 || ny == 0xFFFFFFFFu || ny == 0 || d1 < ix.t_jump ||
                        (!single && d1 + 1 >= k)) {
                        NTC_STAT(4);
                        nohop = true;
                        break;
                    }
                    NTC_STAT(cap == 32 ? (lim < 32 ? 5 : 6) : 7);
                    j = nx - 1;
                    if (joint) jy() = single ? 0xFFFFFFFFu : ny - 1;
                }
                if (len + pre - p - m < lim) lim = len + pre - p - m;
                if (lim < pre) {  // the guessed node is not the U-mer's: take it from the table
                    mode = kModeEnter;
#if NTC_CHAIN
                    break;  // m = 0: on to the Enter block below, in this same call
#else
                    return 0;
#endif
                }
                m += lim - pre;
                pre = 0;
                if (lim < cap) {  // (cap 32: a fork block's characters, the run going on past them)
                    if constexpr (kJoint) {
                        // the run stopped inside its window with the read going on: its entry
                        // now, the hop across the path end (or to both sides' next nodes) with
                        // the next call's run.  Hops chained in one call hold the whole wave on
                        // this lane's dependent loads (round 3, A/B, S91 k_ms4: 12.3 ms before,
                        // 16.3 ms with every hop chained, 12.4 with one, 12.0 with none)
                        // A hop needs each side at a path end or going on with the read's
                        // character c (else: a mismatch, mostly a sequencing error, on with EXT
                        // or the break now) and the depth note_single asks for
                        // (a side whose own stop lies past lim goes on with c)
                        const uint32_t c = (uint32_t)((lim < 32 ? qa >> (2 * lim) : qb2 >> (2 * (lim - 32))) & 3u);
                        const uint32_t d1 = d + m + 1 < k ? d + m + 1 : k;
                        if (ix.forks && m > 0 && p + m < len && (lx > lim || xend) && (ly > lim || yend) &&
                            d1 >= ix.t_jump && (jy() == 0xFFFFFFFFu || d1 + 1 < k)) {
                            put_entry(b, p, j + 1, m, (d + 1 < k ? d + 1 : k) | kRunTag);
                            p += m;
                            d = d + m < k ? d + m : k;
                            j += m;
                            if (jy() != 0xFFFFFFFFu) jy() += m;
                            vfy = (4u + c + (lx > lim ? 0u : 8u) + (ly > lim ? 0u : 16u)) << 8;
                            try_run = true;
                            return 0;
                        }
                    }
                    break;
                }
            }
            if (kJoint && jy() != 0xFFFFFFFFu) {
                // joint run over a multi-node interval [l, r) (its first and last nodes followed
                // along their paths): the interval at p + m - 1 is [node at j + m, node at jy + m
                // + 1) and the extension at p + m goes on from it (see note_path); no hop after
                // a run (nohop): its entry is written, the interval at p - 1 the same way
                if (m > 0) {
                    put_entry(b, p, j + 1, m, (d + 1 < k ? d + 1 : k) | kRunTag);
                    p += m;
                    d = d + m < k ? d + m : k;
                    if (p >= len) { jy() = 0xFFFFFFFFu; return 1; }
                }
                if (m > 0 || nohop) {
                    NTC_TOUCH(kTrColex, ix.colex_at + j + m);
                    NTC_TOUCH(kTrColex, ix.colex_at + jy() + m);
                    l = ld_hint<256>(ix.colex_at + j + m) & 0x7FFFFFFFu;
                    r = (ld_hint<256>(ix.colex_at + jy() + m) & 0x7FFFFFFFu) + 1;
#if defined(NTC_STATS) && !defined(__HIP_DEVICE_COMPILE__)
                    if (p < len) {  // (emulator census) the stop's first/last node: edge of the read's character?
                        const int c = (int)((Q[(qo + p) >> 5] >> (2 * ((qo + p) & 31))) & 3u);
                        const bool el = (ix.rank[(uint64_t)c * ix.rwords + (l >> 5)].y >> (l & 31)) & 1u;
                        const bool er = (ix.rank[(uint64_t)c * ix.rwords + ((r - 1) >> 5)].y >> ((r - 1) & 31)) & 1u;
                        NTC_STAT(el && er ? 8 : (el || er ? 9 : 10));
                    }
#endif
                }
                jy() = 0xFFFFFFFFu;
                m = 0;  // on into the EXT block below, in this same call
                nohop = false;
            }
            if (m > 0 || nohop) {
                if (m > 0) {
                    put_entry(b, p, j + 1, m, (d + 1 < k ? d + 1 : k) | kRunTag);
                    p += m;
                    j += m;
                    d = d + m < k ? d + m : k;
                    if (p >= len) return 1;
                }
                gj = j;
                ge = p;
#if defined(NTC_STATS) && !defined(__HIP_DEVICE_COMPILE__)
                {  // (emulator census) the node before the break: edge of the read's character?
                    const uint32_t v = ix.colex_at[j] & 0x7FFFFFFFu;
                    const int c = (int)((Q[(qo + p) >> 5] >> (2 * ((qo + p) & 31))) & 3u);
                    NTC_STAT(((ix.rank[(uint64_t)c * ix.rwords + (v >> 5)].y >> (v & 31)) & 1u) ? 11 : 12);
                }
#endif
                // the run broke at p (mostly a sequencing error): table first
                window(b, p + 1 - U);
                mode = kModeBrk;
#if !NTC_CHAIN
                return 0;
#endif
            }
        }
        if (mode == kModeFirst) {
            // read start: positions < U - 1 are short by length; error-free starts have the
            // pair (U - 1, U), so test it directly with U - 1's full entry
            mode = kModeScan;
            if (len >= U + 1) {
                if (!covers(0, U)) window(b, 0);
                NTC_TOUCH(kTrTabU, ix.tab + tab_base(U) + key_at(U - 1, U));
                const uint2 te = load2_stream(ix.tab + tab_base(U) + key_at(U - 1, U));
                uint32_t b2 = 1u;
                if (!NTC_FIRST_PAIR) {
                    // U decided by the extension at U (a failure loads U's entry then)
                } else if (ix.pair_w) {
                    // U is long iff bit 4 + q[U] of the pair word of the (U-1)-mer ending at U - 1
                    // (the 32 MB level-U bitmap then stays out of the Infinity Cache entirely)
                    const uint64_t M = key_at(U - 1, U - 1);
                    NTC_TOUCH(kTrBits, ix.pair_w + M);
                    b2 = (ld_hint<32>(ix.pair_w + M) >> (4 + ((uint32_t)(qw >> (2 * U)) & 3u))) & 1u;
                } else {
                    const uint64_t k2 = key_at(U, U);
                    NTC_TOUCH(kTrBits, ix.tab_bits + (k2 >> 5));
                    b2 = (ix.tab_bits[k2 >> 5] >> (k2 & 31)) & 1u;
                }
                if (!tab_long(te)) {
                    p = U - 1 + U - (te.y & 0xFFu);  // d_{U-1+i} <= m + i
                    if (p >= len || !NTC_CHAIN) return p >= len ? 1 : 0;
                } else if (!b2) {
                    p = U + 1;  // U is short
                    if (p >= len || !NTC_CHAIN) return p >= len ? 1 : 0;
                } else {
                    return enter_pair(ix, b, U - 1, te);
                }
                // (NTC_CHAIN) on into the SCAN block below, in this same call
            }
        }
        // SCAN pair words at non-overlapping positions / window words (see the SCAN block)
        constexpr bool kStrideScan = NTC_PAIR_STRIDE == 2 || (NTC_PAIR_STRIDE == 1 && kJoint);
        bool brk0 = false;  // the SCAN starts at a run break position p, whose long/short it tests
#if NTC_BRK_MERGE
        // The run broke at p.  p is short after almost every break, so p's long/short test
        // (its pair word, and the node before p for a long p) is issued together with the
        // SCAN of p + 1, ...; a long p abandons that SCAN for EXT at p.  One round trip.
        // (The stride SCAN keeps the break word with its first loads.)
        uint32_t bpw = 0, bc = 0;
        bool brk = false;  // (brk0: see below)
        constexpr bool kBrkLate = NTC_BRK_LATE && !kStrideScan;
        if (mode == kModeBrk && ix.pair_w && p + 2 < len) {
            if (!covers(p + 1 - U, p + 2)) window(b, p + 1 - U);
            bc = (uint32_t)(qw >> (2 * (p - qb))) & 3u;
            // Window words answer p itself: the SCAN starts AT p (its first position tells
            // whether p is long) and no break word is loaded -- one random line less per break.
            const bool in_win = NTC_BRK_IN_WIN && kStrideScan && ix.win_w != nullptr;
            if (!kBrkLate && !in_win) {
                const uint64_t M = key_at(p - 1, U - 1);
                NTC_TOUCH(kTrBits, ix.pair_w + M);
                bpw = ld_hint<32>(ix.pair_w + M);
            }
            brk = !in_win;
            brk0 = in_win;
            if (!in_win) p += 1;  // a short p: m <= U - 1 skips nothing beyond p itself
            mode = kModeScan;
            hi = U + 1 + in_win < kScanW ? U + 1 + in_win : kScanW;
        }
#endif
        if (mode == kModeScan) {
            // find the first pair of consecutive long positions at or after p (position
            // p - 1 is short, or p = 0); positions < U - 1 are short by length
            if (p < U - 1) p = U - 1;
            if (p + 1 >= len) { p = len; return 1; }
            if (!covers(p + 1 - U, p + 1)) window(b, p + 1 - U);
            uint32_t W = qb + 32 - p;
            if (W > hi) W = hi;
            if (W > len - p) W = len - p;
            hi = kScanW;
            // a present U-mer has its three F-mers (F = U - 2, at offsets 0, 1, 2) present:
            // test them in the small level-F bitmap first; the F-mer ending at y is shared
            // by the U-mers ending at y, y + 1 and y + 2, so W + 2 filter bits cover W positions
            uint32_t cand = (1u << W) - 1u;
            uint32_t bpass = 1u;  // (late break word) the break position p - 1 passes the filter
            if (ix.filt_f) {
                const uint32_t F = ix.filt_f;
                uint32_t fm = 0;  // bit i: F-mer ending at p - 2 + i is present
                // every load unconditional and issued before the first use: one L2 round
                // trip, not W + 2 dependent ones
                // F-mer of slot i = characters p - U + 1 + i ... p - 2 + i: bits 2i.. of v.
                // Slots past W + 2 repeat slot 0's word (an L1 hit, no extra L2 request).
                const uint64_t v = qw >> (2 * (p + 1 - U - qb));
                const uint32_t fmask = (1u << (2 * F)) - 1u;
                const uint32_t f0 = (uint32_t)v & fmask;
                uint32_t fw[kScanW + kFiltGap];
#pragma unroll
                for (uint32_t i = 0; i < kScanW + kFiltGap; i++) {
                    const uint32_t fk = i < W + kFiltGap ? (uint32_t)(v >> (2 * i)) & fmask : f0;
                    if (i < W + kFiltGap) NTC_TOUCH(kTrFilt, ix.filt_bits + (fk >> 5));
                    fw[i] = ix.filt_bits[fk >> 5];
                }
#pragma unroll
                for (uint32_t i = 0; i < kScanW + kFiltGap; i++)
                    fm |= ((fw[i] >> ((uint32_t)(v >> (2 * i)) & 31u)) & 1u) << i;
                fm &= (1u << (W + kFiltGap)) - 1u;
                cand &= fm & (fm >> 1) & (fm >> kFiltGap);  // all three F-mers of the U-mer
                bpass = (fm & 3u) == 3u;  // the F-mers ending at p - 2 and p - 1
            }
#if NTC_BRK_MERGE
            // (the stride SCAN tests the break word after issuing its own loads, below: one round trip)
            if (!kBrkLate && !kStrideScan && brk && ((bpw >> (4 + bc)) & 1u)) {  // the break position is long: EXT there
                p -= 1;
                mode = kModeBrkLong;
                return 0;
            }
#endif
            if (ix.pair_w) {
                // Pair word of the (U-1)-mer ending at y: whether y AND y + 1 are long.
                //  * stride (genome collections, the k_ms4 build with joint runs): words go to
                //    non-overlapping positions -- the smallest position not yet known among those
                //    in a candidate pair (both pass the filter; with the filter off, every
                //    position), then the next unknown one, ...  A run of candidates costs one word
                //    per TWO positions, and a long pair straddling two words is read off both
                //    (S91: 20.5 -> 12.9 pair-word lines per read, emulator trace).
                //  * otherwise one word per candidate pair, the first NTC_PAIR_TESTS pairs (C91:
                //    candidates are sparse after the filter, and the lighter code keeps k_ms4 at
                //    7 waves).
                // Every load is issued before the first use.  A slot without a word repeats the
                // first one's (the same line, no further request past L2); with no candidate at
                // all every slot reads word 0, one line all lanes share.
                constexpr bool kStride = kStrideScan;
                const uint32_t cp = cand & (cand >> 1);  // candidate pair starts (<= W - 2)
                uint32_t slot[NTC_PAIR_TESTS], pbv[NTC_PAIR_TESTS];
                uint32_t hit = 0, single = 0, open = 0, keep = cand;
                if constexpr (kStride) {
                  if (ix.win_w) {
                    // window words: entry t (key: the (U-3)-mer ending at p + 4t) answers the
                    // four positions p + 4t .. p + 4t + 3; two entries, eight positions, two
                    // lines (stride pair words: four).  One 32-bit load per position, all
                    // issued before the first use (the loads of one entry share its line).
                    constexpr uint32_t kWin = NTC_WIN_ENTRIES;
                    uint32_t wv[4 * kWin];
#pragma unroll
                    for (uint32_t i = 0; i < 4 * kWin; i++) {
                        const uint32_t t = i >> 2, jj = i & 3u;
                        const uint64_t K = key_at(4 * t < W ? p + 4 * t : p, U - 3);  // past W: entry 0's line again
                        const uint32_t bi = i < W ? 64 * jj + win_ctx(key_at(p + i, U), U, jj) : 0u;
                        if (i < W && jj == 0) NTC_TOUCH(kTrBits, ix.win_w + K * 8);
                        wv[i] = ld_hint<32>(ix.win_w + K * 8 + (bi >> 5));
                    }
                    uint32_t longm = 0;
#pragma unroll
                    for (uint32_t i = 0; i < 4 * kWin; i++) {
                        const uint32_t jj = i & 3u;
                        const uint32_t bi = i < W ? 64 * jj + win_ctx(key_at(p + i, U), U, jj) : 0u;
                        longm |= ((wv[i] >> (bi & 31u)) & 1u) << i;
                    }
                    const uint32_t lim = W < 4 * kWin ? W : 4 * kWin;
                    const uint32_t known = (1u << lim) - 1u;
                    longm &= cand & known;  // a position failing the filter is short
                    if (brk0 && (longm & 1u)) {  // the break position p is long: EXT there
                        mode = kModeBrkLong;
                        return 0;
                    }
                    const uint32_t kshort = (known & ~longm) | (~cand & ((1u << W) - 1u));
                    hit = longm & (longm >> 1);
                    open = cp & ~kshort & ~(kshort >> 1) & ~(known & (known >> 1));
                    keep = cand & ~kshort;
                  } else {
                    uint32_t todo = cp | (cp << 1), starts = 0;
                    const uint32_t first = cp ? (uint32_t)__builtin_ctz(cp) : 0u;
#pragma unroll
                    for (uint32_t t = 0; t < NTC_PAIR_TESTS; t++) {
                        const uint32_t sx = todo ? (uint32_t)__builtin_ctz(todo) : 32u;
                        const bool real = sx + 2 <= W;  // y + 1 inside the window
                        slot[t] = real ? sx : first;
                        starts |= real ? 1u << sx : 0u;
                        todo &= real ? ~(3u << sx) : 0u;
                    }
                    const uint64_t M0 = cp ? key_at(p + first, U - 1) : 0u;
#pragma unroll
                    for (uint32_t t = 0; t < NTC_PAIR_TESTS; t++) {
                        const uint64_t M = ((starts >> slot[t]) & 1u) ? key_at(p + slot[t], U - 1) : M0;
                        if ((starts >> slot[t]) & 1u) NTC_TOUCH(kTrBits, ix.pair_w + M);
                        pbv[t] = ld_hint<32>(ix.pair_w + M);
                    }
                    uint32_t longm = 0, known = 0;
#pragma unroll
                    for (uint32_t t = 0; t < NTC_PAIR_TESTS; t++) {
                        const uint32_t y = p + slot[t];
                        const uint32_t real = (starts >> slot[t]) & 1u;
                        const uint32_t a = (uint32_t)(qw >> (2 * (y + 1 - U - qb))) & 3u;
                        const uint32_t c = (uint32_t)(qw >> (2 * (y + 1 - qb))) & 3u;
                        const uint32_t w = real ? pbv[t] : 0u;
                        longm |= (((w >> a) & 1u) << slot[t]) | (((w >> (4 + c)) & 1u) << (slot[t] + 1));
                        single |= (((w >> (8 + a)) & 1u) << slot[t]) | (((w >> (12 + c)) & 1u) << (slot[t] + 1));
                        known |= (real * 3u) << slot[t];
                    }
                    hit = longm & (longm >> 1);
                    // undecided candidate pairs: neither position known short, not both known
                    const uint32_t kshort = known & ~longm;
                    open = cp & ~kshort & ~(kshort >> 1) & ~(known & (known >> 1));
                    keep = cand & ~kshort;
                  }
                } else {
                    uint32_t untested = cp;
#pragma unroll
                    for (uint32_t t = 0; t < NTC_PAIR_TESTS; t++) untested &= untested - 1;
                    const uint32_t tested = cp ^ untested;
                    uint32_t rem = tested;
                    const uint32_t first = tested ? (uint32_t)__builtin_ctz(tested) : 0u;
                    const uint64_t M0 = tested ? key_at(p + first, U - 1) : 0u;
#pragma unroll
                    for (uint32_t t = 0; t < NTC_PAIR_TESTS; t++) {
                        slot[t] = rem ? (uint32_t)__builtin_ctz(rem) : first;
                        const uint64_t M = rem ? key_at(p + slot[t], U - 1) : M0;
                        rem &= rem - 1;
                        if ((tested >> slot[t]) & 1u) NTC_TOUCH(kTrBits, ix.pair_w + M);
                        pbv[t] = ld_hint<32>(ix.pair_w + M);
                    }
#if NTC_BRK_MERGE
                    if (kBrkLate && brk) {
                        // the break position p - 1 can be long only if it passes the filter: its
                        // pair word (of the (U-1)-mer ending at p - 2, inside the window the break
                        // set) goes out with the SCAN's pair words, in their round trip, and only
                        // then (else slot 0's line again, no further request)
                        const uint64_t Mb = bpass ? key_at(p - 2, U - 1) : M0;
                        if (bpass) NTC_TOUCH(kTrBits, ix.pair_w + Mb);
                        bpw = ld_hint<32>(ix.pair_w + Mb);
                    }
#endif
#pragma unroll
                    for (uint32_t t = 0; t < NTC_PAIR_TESTS; t++) {
                        const uint32_t y = p + slot[t];
                        const uint32_t a = (uint32_t)(qw >> (2 * (y + 1 - U - qb))) & 3u;
                        const uint32_t c = (uint32_t)(qw >> (2 * (y + 1 - qb))) & 3u;
                        hit |= ((pbv[t] >> a) & (pbv[t] >> (4 + c)) & 1u) << slot[t];
                        single |= ((pbv[t] >> (8 + a)) & 1u) << slot[t];
                    }
                    hit &= tested;
                    open = untested;  // resume at the first untested candidate pair
                }
#if NTC_BRK_MERGE
                if ((kStrideScan || (kBrkLate && bpass)) && brk && ((bpw >> (4 + bc)) & 1u)) {  // the break position is long: EXT there
                    p -= 1;
                    mode = kModeBrkLong;
                    return 0;
                }
#endif
                if (hit) {
                    const uint32_t xi = (uint32_t)__builtin_ctz(hit);
                    const uint32_t x = p + xi;  // x, x + 1 long, x - 1 short
#if NTC_GUESS
                    // x's U-mer is one node.  After a run break at ge (mostly a substitution),
                    // the read most likely goes on along the same path: guess that node at
                    // path position gj + (x + 1 - ge) and let the run verify it (its U
                    // characters and that it is a node) instead of fetching x's table entry.
                    // Exact either way: a single-node interval holding a node whose k-mer
                    // ends with the U-mer is that node.
                    const uint32_t jg = gj + (x + 1 - ge);
                    if (((single >> xi) & 1u) && ix.tab_pos && ge != 0 && x - ge - U <= NTC_GUESS_SLACK &&
                        x >= ge + U && jg < ix.path_len) {
                        j = jg;
                        jy() = 0xFFFFFFFFu;
                        d = U;
                        p = x + 1;
                        vfy = U;
                        try_run = true;
                        mode = kModeBrk;  // a run of length 0 leaves p = x + 1, long: its break check
                        ge = 0;
                        return 0;
                    }
#endif
                    NTC_TOUCH(kTrTabU, ix.tab + tab_base(U) + key_at(x, U));
                    return enter_pair(ix, b, x, load2_stream(ix.tab + tab_base(U) + key_at(x, U)));
                }
                if (open) {
                    p += (uint32_t)__builtin_ctz(open);
                    return 0;
                }
                if (p + W >= len) { p = len; return 1; }
                p += W - ((keep >> (W - 1)) & 1u);  // a possibly long last position may start a pair
                return 0;
            }
#if NTC_SCAN_MODE == 2
            if (ix.filt_f) {
                // first candidate PAIR (x, x + 1 both pass the filter): its table entry is
                // needed anyway when x is long, so load it in place of x's exact bit
                const uint32_t cp = cand & (cand >> 1);
                if (cp == 0) {
                    if (p + W >= len) { p = len; return 1; }
                    p += W - ((cand >> (W - 1)) & 1u);  // a passing last position may start a pair
                    return 0;
                }
                const uint32_t x = p + (uint32_t)__builtin_ctz(cp);
                const uint64_t k1 = key_at(x + 1, U);
                NTC_TOUCH(kTrTabU, ix.tab + tab_base(U) + key_at(x, U));
                NTC_TOUCH(kTrBits, ix.tab_bits + (k1 >> 5));
                const uint2 te = load2_stream(ix.tab + tab_base(U) + key_at(x, U));
                const uint32_t b1 = (ld_hint<2>(ix.tab_bits + (k1 >> 5)) >> (k1 & 31)) & 1u;
                if (!tab_long(te)) {  // x short: d_{x+i} <= m + i
                    p = x;
                    skip_short(b, te, U);
                    return p >= len ? 1 : 0;
                }
                if (!b1) {  // x long, x + 1 short
                    p = x + 2;
                    return p >= len ? 1 : 0;
                }
                return enter_pair(ix, b, x, te);
            }
#endif
#if NTC_SCAN_MODE == 1
            if (ix.filt_f) {
                // exact bits only for the first two candidate PAIRS (x, x + 1 both pass)
                const uint32_t cp = cand & (cand >> 1);
                if (cp == 0) {
                    if (p + W >= len) { p = len; return 1; }
                    p += W - ((cand >> (W - 1)) & 1u);  // a passing last position may start a pair
                    return 0;
                }
                const uint32_t x0 = (uint32_t)__builtin_ctz(cp);
                const uint32_t rest = cp & (cp - 1);
                const uint32_t x1 = rest ? (uint32_t)__builtin_ctz(rest) : x0;
                const uint32_t starts = (1u << x0) | (1u << x1);
                const uint32_t tested = (3u << x0) | (3u << x1);
                uint32_t longm = 0;
#pragma unroll
                for (uint32_t i = 0; i < kScanW; i++)
                    if ((tested >> i) & 1u) {
                        const uint64_t key = key_at(p + i, U);
                        NTC_TOUCH(kTrBits, ix.tab_bits + (key >> 5));
                        longm |= ((ld_hint<2>(ix.tab_bits + (key >> 5)) >> (key & 31)) & 1u) << i;
                    }
                const uint32_t pairs = longm & (longm >> 1) & starts;
                if (pairs == 0) {
                    const uint32_t more = rest & (rest - 1);  // untested candidate pairs
                    if (more == 0) {
                        if (p + W >= len) { p = len; return 1; }
                        p += W - ((cand >> (W - 1)) & 1u);
                        return 0;
                    }
                    p += x1 + 1;
                    return p >= len ? 1 : 0;
                }
                const uint32_t x = p + (uint32_t)__builtin_ctz(pairs);
                NTC_TOUCH(kTrTabU, ix.tab + tab_base(U) + key_at(x, U));
                return enter_pair(ix, b, x, load2_stream(ix.tab + tab_base(U) + key_at(x, U)));
            }
#endif
            // exact test of the first kScanExact candidates only: the pair is almost always
            // among them, and positions past the last one tested are left to the next SCAN
            uint32_t tested = cand, span = W;
#pragma unroll
            for (uint32_t t = 0; t < kScanExact; t++) tested &= tested - 1;  // drop the first few
            if (tested) {
                span = (uint32_t)__builtin_ctz(tested);  // first untested candidate
                tested = cand & ((1u << span) - 1u);
            } else {
                tested = cand;
            }
            uint32_t longm = 0;
#pragma unroll
            for (uint32_t i = 0; i < kScanW; i++)
                if ((tested >> i) & 1u) {
                    const uint64_t key = key_at(p + i, U);
                    NTC_TOUCH(kTrBits, ix.tab_bits + (key >> 5));
                    longm |= ((ld_hint<2>(ix.tab_bits + (key >> 5)) >> (key & 31)) & 1u) << i;
                }
            const uint32_t pairs = longm & (longm >> 1);
            if (pairs == 0) {
                if (p + span >= len) { p = len; return 1; }
                p += span - ((longm >> (span - 1)) & 1u);  // keep a long last position
                return 0;
            }
            const uint32_t x = p + (uint32_t)__builtin_ctz(pairs);  // long, short predecessor
            NTC_TOUCH(kTrTabU, ix.tab + tab_base(U) + key_at(x, U));
            return enter_pair(ix, b, x, load2_stream(ix.tab + tab_base(U) + key_at(x, U)));
        }
        if (!covers(p + 1 - U, p)) window(b, p + 1 - U);
        if (mode == kModeBrkLong) {  // the run broke at a long p: extend from the node before p
            NTC_TOUCH(kTrColex, ix.colex_at + j);
            l = ld_hint<256>(ix.colex_at + j) & 0x7FFFFFFFu;
            r = l + 1;
            mode = kModeExt;
#if !NTC_CHAIN
            return 0;
#endif
        }
        if (mode == kModeEnter) {  // guessed node rejected: x = p - 1 from the table
            if (!covers(p - U, p - 1)) window(b, p - U);
            NTC_TOUCH(kTrTabU, ix.tab + tab_base(U) + key_at(p - 1, U));
            return enter_pair(ix, b, p - 1, load2_stream(ix.tab + tab_base(U) + key_at(p - 1, U)));
        }
        if (mode == kModeBrk) {
#if NTC_BRK_PAIR
            if (ix.pair_w) {
                // is p long?  One pair word (Infinity Cache) instead of p's table entry (HBM):
                // bit 4 + q[p] of the (U-1)-mer ending at p - 1.  A short p's m is not known
                // here; m <= U - 1 skips nothing beyond p itself.
                const uint64_t M = key_at(p - 1, U - 1);
                const uint32_t c = (uint32_t)(qw >> (2 * (p - qb))) & 3u;
                NTC_TOUCH(kTrBits, ix.pair_w + M);
                NTC_TOUCH(kTrColex, ix.colex_at + j);
                const uint32_t pw = ld_hint<32>(ix.pair_w + M);
                const uint32_t v = ld_hint<256>(ix.colex_at + j) & 0x7FFFFFFFu;  // node before p, for a long p
                if (!((pw >> (4 + c)) & 1u)) {
                    p += 1;
                    mode = kModeScan;
                    hi = U + 1 < kScanW ? U + 1 : kScanW;
                    return p >= len ? 1 : 0;
                }
                l = v;
                r = v + 1;
                mode = kModeExt;
                return 0;
            }
#endif
            NTC_TOUCH(kTrTabU, ix.tab + tab_base(U) + key_at(p, U));
            const uint2 te = load2_stream(ix.tab + tab_base(U) + key_at(p, U));
            NTC_TOUCH(kTrColex, ix.colex_at + j);
            const uint32_t v = ld_hint<256>(ix.colex_at + j) & 0x7FFFFFFFu;  // node before p, for a long p
            if (!tab_long(te)) {
                skip_short(b, te, U);
                return p >= len ? 1 : 0;
            }
            l = v;
            r = v + 1;
            mode = kModeExt;
            return 0;
        }
        const int c = (int)((qw >> (2 * (p - qb))) & 3u);
        if (mode == kModeExt && ix.rank2 && p + 1 < len && p + 1 < qb + 32) {
            // two positions from one line (Rank2Chunk): the usual case inside a climb from
            // d = U to k over a multi-node interval (strain collections)
            const int c2 = (int)((qw >> (2 * (p + 1 - qb))) & 3u);
            uint32_t l1, r1, l2, r2;
            extend2(ix, c, c2, l, r, l1, r1, l2, r2);
            if (l1 < r1) {
                const uint32_t d1 = d + 1 < k ? d + 1 : k;
                put_entry(b, p, l1, 1u, d1);
                p++;
                if (l2 < r2) return commit(ix, b, l2, r2, d1 + 1 < k ? d1 + 1 : k);
                l = l1; r = r1; d = d1;
                mode = kModeExtFail;  // the second extension failed: position p (was p + 1)
                return 0;
            }
            mode = kModeExtFail;  // the first failed: failure handling at p
            return 0;
        }
        if (mode == kModeExt || mode == kModeExtFail) {
            uint2 te;
            if (NTC_EXT_EAGER || mode == kModeExtFail) {
                // p's table entry, wanted only when the extension fails
                NTC_TOUCH(kTrTabU, ix.tab + tab_base(U) + key_at(p, U));
                te = load2_stream(ix.tab + tab_base(U) + key_at(p, U));
            }
            if (mode == kModeExt) {
                uint32_t nl, nr;
                extend(ix, c, l, r, nl, nr);
                if (nl < nr) return commit(ix, b, nl, nr, d + 1 < k ? d + 1 : k);
                if (!NTC_EXT_EAGER) {  // one more round trip for the entry, only on a failure
                    mode = kModeExtFail;
                    return 0;
                }
            }
            if (!tab_long(te)) {  // p is short: table-determined, scan on
                skip_short(b, te, U);
                return p >= len ? 1 : 0;
            }
            uint32_t tl, tr, tj;
            tab_interval(ix, te, tl, tr, tj);
            if (d == U) return commit(ix, b, tl, tr, U);  // t* = U - 1
            lo = U - 1;  // ext(I_{U-1}, c) = the U-mer's interval
            put_best(b, tl, tr);
            hi = d - 1;
            mode = kModeP1;
            return 0;
        }
        // kModeP1: probe t = d - 1 from I_d; kModeBs: t = mid from I_hi (l1, r1)
        const bool p1 = mode == kModeP1;
        const uint32_t t = p1 ? hi : (lo + hi) >> 1;
        uint32_t ql = p1 ? l : l1, qr = p1 ? r : r1;
        widen(ix, ql, qr, t);
        uint32_t el, er;
        extend(ix, c, ql, qr, el, er);
        if (el < er) {
            if (p1) return commit(ix, b, el, er, t + 1);
            lo = t;
            put_best(b, el, er);
        } else {
            hi = t; l1 = ql; r1 = qr;
        }
        if (hi - lo <= 1) {
            const uint2 bb = best(b);
            return commit(ix, b, bb.x, bb.y, lo + 1);
        }
        mode = kModeBs;
        return 0;
    }
};
using MsLane = MsLaneT<true>;

// (d, S) of every position of one read (diagnostics: ntc_debug_matching_statistics)
NTC_HD void read_ms(const DevIndex &ix, const uint64_t *Q, uint64_t qo, const Entry *E, uint32_t ne,
                    uint32_t len, uint32_t *d_out, uint32_t *s_out, const Entry *Ed = nullptr, uint64_t es = 1,
                    const Entry *E2 = nullptr, uint32_t S = kNoLimit) {
    EntryView ev(E, &ix, Q, qo, ix.k, -1, Ed, es, nullptr, E2, S);
    uint32_t x = 0;
    for (uint32_t i = 0; i <= ne && x < len; i++) {
        const Entry en = i < ne ? ev.at((int32_t)i) : Entry{0, 0, 0, 0};
        const uint32_t until = i < ne ? en.p : len;
        for (; x < until && x < len; x++) tab_ds(ix, Q, qo, x, d_out[x], s_out[x]);
        if (i == ne) break;
        for (uint32_t t = 0; t < en.m && x < len; t++, x++) {
            d_out[x] = ev.dval(en, x);
            s_out[x] = ev.sval(en, x);
        }
    }
}

constexpr uint32_t kRecSlot = 8;  // records per read in the dense slot; more spill

// Records past kRecSlot (k_parse4): a reservation in a pool sized by need, like the entries'
// (MsLaneT::reserve); the host re-runs a call that ran out of it.
struct RecPool {
    uint64_t *pool;
    uint64_t cap;
    unsigned long long *cnt;
    uint32_t *rbase;  // each overflowing read's reservation start
    unsigned long long *status;
    uint64_t rid;
};

// greedy right-to-left parse over the entries, lib.rs:175-218 (+ encode.rs:144-158).
// Record j goes to slot[j * sstride] (j < kRecSlot) or spill[j] (rp: spill is reserved at
// record kRecSlot, null when the pool ran out).  The kernel interleaves the reads' slots
// (sstride = reads in the batch): the loop runs in lock step over a wave's lanes, so the
// lanes' j-th records are one coalesced store.
NTC_HD int parse_read(const DevIndex &ix, const uint64_t *Q, uint64_t qo, const Entry *E, uint32_t ne,
                      uint32_t len, uint64_t *slot, uint64_t *spill, uint64_t sstride = 1,
                      const Entry *Ed = nullptr, uint64_t es = 1, const Entry *pre = nullptr,
                      const Entry *E2 = nullptr, uint32_t S = kNoLimit, const RecPool *rp = nullptr) {
    const uint32_t k = ix.k;
    EntryView ev(E, &ix, Q, qo, k, (int32_t)ne - 1, Ed, es, pre, E2, S);
    uint32_t i = len;
    int nrec = 0;
    while (i > 0) {
        const uint32_t x = i - 1;
        uint32_t di, st;
        ev.DS(x, di, st);
        const uint32_t segend = i;
        uint32_t seglen;
        if (di == k && i > k + 1) {
            const uint32_t ext = ev.run_from(i - 2, i - k - 1);
            const uint32_t L = k + ext;
            uint32_t m = L, pp = i;
            for (;;) {  // jump loop lib.rs:193-203
                const uint32_t dp = ev.D(pp - 1);
                if (dp < m) {
                    if (dp >= pp || dp == 0) return -kErrFormat;
                    m -= dp;
                    pp -= dp;
                } else {
                    break;
                }
            }
            seglen = L - (m - 1);
            i = pp;
        } else {
            if (di == 0) return -kErrFormat;
            seglen = di;
            if (i > di) i -= di - 1;
            else i = 0;
        }
        if (seglen >= (1u << 24)) return -kErrLength;
        const uint64_t first = nrec == 0 ? 1u : 0u;
        uint64_t w;
        if (seglen > 11) {
            w = (uint64_t)st | ((uint64_t)(seglen & 0xFFFFFFu) << 32) | (first << 56);
        } else {
            if (seglen > k) return -kErrRefPanic;  // encode.rs:151-152: kmer[(k - len)..k] underflows
            NTC_TOUCH(kTrQ, Q + ((qo + segend - seglen) >> 5));
            const uint64_t bits = window2(Q, qo + segend - seglen);
            w = (bits & ((1ULL << (2 * seglen)) - 1)) | ((uint64_t)((first + 2) | (seglen << 2)) << 56);
        }
        if (nrec < (int)kRecSlot) {
            slot[(uint64_t)nrec * sstride] = w;
        } else {
            if (rp && nrec == (int)kRecSlot) {
                // this record and at most one per position left of i (each starts one further left)
                const uint64_t need = 1 + (uint64_t)i;
#ifdef __HIP_DEVICE_COMPILE__
                const uint64_t at = atomicAdd(rp->cnt, (unsigned long long)need);
#else
                const uint64_t at = *rp->cnt;
                *rp->cnt += need;
#endif
                if (at + need <= rp->cap) {
                    rp->rbase[rp->rid] = (uint32_t)at;
                    spill = rp->pool + at - kRecSlot;
                } else {
                    spill = nullptr;
#ifdef __HIP_DEVICE_COMPILE__
                    atomicMin(rp->status, kStatusRegrow);
#else
                    *rp->status = kStatusRegrow;
#endif
                }
            }
            if (spill) spill[nrec] = w;
        }
        nrec++;
        if (i > 0) i -= 1;
        else break;
    }
    return nrec;
}

// ASCII of n <= 32 two-bit codes (code t at bits 2t) to out[0..n): aligned 4-byte stores
// (four codes -> "ACGT" bytes with one byte permute), single bytes at the ends
NTC_HD void store_codes(uint8_t *out, uint64_t codes, uint32_t n) {
    uint32_t i = 0;
    while (i < n && (((uintptr_t)(out + i)) & 3u)) {
        out[i] = base_char((uint32_t)(codes >> (2 * i)));
        i++;
    }
    for (; i + 4 <= n; i += 4) {
        const uint32_t x = (uint32_t)(codes >> (2 * i)) & 0xFFu;
        const uint32_t spread = (x & 3u) | ((x & 0xCu) << 6) | ((x & 0x30u) << 12) | ((x & 0xC0u) << 18);
#ifdef __HIP_DEVICE_COMPILE__
        *reinterpret_cast<uint32_t *>(out + i) = __builtin_amdgcn_perm(0u, 0x54474341u, spread);
#else
        for (uint32_t b = 0; b < 4; b++) out[i + b] = base_char(spread >> (8 * b));
#endif
    }
    for (; i < n; i++) out[i] = base_char((uint32_t)(codes >> (2 * i)));
}

// Block-staged decode output (k_dec_rec): the records of one block OR their 2-bit codes into
// a word buffer (LDS) covering output characters [32 w_lo, 32 (w_lo + words)), with a mask of
// the characters written; then every staged word goes out as ASCII exactly once (whole words
// with two 16-byte stores, words shared with other blocks byte by byte: records never share
// a byte).  No global atomics, no 2-bit round trip through HBM.
constexpr uint32_t kDecStageWords = 2048;  // 64 K characters per block of 512 records (error-free
                                           // 150 bp reads: 2 records per read, 38 K characters)
struct StageWriter {
    uint64_t *bits;  // word t: codes of characters 32 (w_lo + t) ... + 31
    uint32_t *mask;  // bit i of word t: character 32 (w_lo + t) + i is staged
    uint64_t w_lo;
    NTC_HD void put_part(uint64_t word, uint64_t b, uint32_t m) {
        const uint64_t t = word - w_lo;
#ifdef __HIP_DEVICE_COMPILE__
        atomicOr(reinterpret_cast<unsigned long long *>(bits + t), (unsigned long long)b);
        atomicOr(mask + t, m);
#else
        bits[t] |= b;
        mask[t] |= m;
#endif
    }
    // n <= 32 codes (code t at bits 2t) for characters [g, g + n)
    NTC_HD void put(uint64_t g, uint64_t codes, uint32_t n) {
        if (n == 0) return;
        if (n < 32) codes &= (1ULL << (2 * n)) - 1;
        const uint64_t w0 = g >> 5, w1 = (g + n - 1) >> 5;
        const uint32_t sh = (uint32_t)(g & 31);
        const uint32_t cm = n < 32 ? (1u << n) - 1u : 0xFFFFFFFFu;
        if (w1 != w0) put_part(w1, codes >> (64 - 2 * sh), cm >> (32 - sh));  // crossing: sh > 0
        put_part(w0, codes << (2 * sh), cm << sh);
    }
};

// ASCII of staged word wg (global word index) to out: the masked characters only
NTC_HD void stage_store_word(uint8_t *out, uint64_t wg, uint64_t bits, uint32_t mask) {
    if (!mask) return;
    uint8_t *o = out + 32 * wg;
    if (mask == 0xFFFFFFFFu) {
#ifdef __HIP_DEVICE_COMPILE__
        if ((((uintptr_t)o) & 15) == 0) {
            uint32_t v[8];
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const uint32_t x = (uint32_t)(bits >> (8 * q)) & 0xFFu;
                const uint32_t spread = (x & 3u) | ((x & 0xCu) << 6) | ((x & 0x30u) << 12) | ((x & 0xC0u) << 18);
                v[q] = __builtin_amdgcn_perm(0u, 0x54474341u, spread);
            }
            reinterpret_cast<uint4 *>(o)[0] = make_uint4(v[0], v[1], v[2], v[3]);
            reinterpret_cast<uint4 *>(o)[1] = make_uint4(v[4], v[5], v[6], v[7]);
            return;
        }
#endif
        store_codes(o, bits, 32);
        return;
    }
    for (uint32_t i = 0; i < 32; i++)
        if ((mask >> i) & 1u) o[i] = base_char((uint32_t)(bits >> (2 * i)));
}

// The L characters of the L-step inverse walk from node j, to output characters
// [g0, g0 + L) of a code writer (StageWriter); false on a malformed record.
// the characters of one walk entry for output characters ending at g0 + end (newest first)
template <class Writer>
NTC_HD void walk_put(uint32_t &end, uint64_t g0, Writer &cw, const WalkEntry &e) {
    const uint64_t piece[4] = {e.w0, e.w1, e.w2, (uint64_t)e.older};
    const uint32_t width[4] = {32, 32, 32, 16};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t t = end < width[i] ? end : width[i];
        if (t) cw.put(g0 + end - t, piece[i] >> (2 * (width[i] - t)), t);
        end -= t;
    }
}

NTC_HD WalkEntry walk_at(const DevIndex &ix, uint32_t cur) {
#ifdef __HIP_DEVICE_COMPILE__
    const uint4 a = reinterpret_cast<const uint4 *>(ix.walk + cur)[0];
    const uint4 b = reinterpret_cast<const uint4 *>(ix.walk + cur)[1];
    WalkEntry e;
    e.w0 = (uint64_t)a.x | ((uint64_t)a.y << 32);
    e.w1 = (uint64_t)a.z | ((uint64_t)a.w << 32);
    e.w2 = (uint64_t)b.x | ((uint64_t)b.y << 32);
    e.older = b.z;
    e.jump = b.w;
    return e;
#else
    return ix.walk[cur];
#endif
}

// The L characters of the L-step inverse walk from node j, to output characters
// [g0, g0 + L) of a code writer (StageWriter); false on a malformed record.
template <class Writer>
NTC_HD bool walk_record_codes(const DevIndex &ix, uint32_t j, uint32_t L, uint64_t g0, Writer &cw) {
    uint32_t end = L, cur = j;
    while (end > 0) {
        if (cur >= ix.n) return false;
        const WalkEntry e = walk_at(ix, cur);
        walk_put(end, g0, cw, e);
        cur = e.jump;
    }
    return true;
}

// ASCII straight to memory (a Writer for walk_put)
struct DirectWriter {
    uint8_t *out;  // output character 0
    NTC_HD void put(uint64_t g, uint64_t codes, uint32_t n) { store_codes(out + g, codes, n); }
};

// Writes the L characters of the L-step inverse walk from node j into out[0..L).
NTC_HD bool walk_record(const DevIndex &ix, uint32_t j, uint32_t L, uint8_t *out) {
    DirectWriter dw{out};
    return walk_record_codes(ix, j, L, 0, dw);
}

// decode_sequence for one read: its records [rb, re) were emitted rightmost first, so
// they are consumed last to first (lib.rs:266) and the segments concatenated.
NTC_HD int decode_read(const DevIndex &ix, const uint64_t *recs, uint64_t rb, uint64_t re,
                       uint8_t *out, uint64_t cap) {
    uint64_t pos = 0;
    for (uint64_t r = re; r-- > rb;) {
        const uint64_t w = recs[r];
        const uint32_t flag = (uint32_t)(w >> 56);
        if (flag & 2) {
            const uint32_t len = flag >> 2;
            if (pos + len > cap) return -kErrFormat;
            for (uint32_t j = 0; j < len; j++) out[pos + j] = base_char((uint32_t)(w >> (2 * j)));
            pos += len;
        } else {
            const uint32_t colex = (uint32_t)w;
            const uint32_t L = (uint32_t)(w >> 32) & 0xFFFFFFu;
            if (pos + L > cap) return -kErrFormat;
            if (!walk_record(ix, colex, L, out + pos)) return -kErrFormat;
            pos += L;
        }
    }
    return 0;
}

}  // namespace ntc
