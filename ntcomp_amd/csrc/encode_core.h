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

namespace ntc {

constexpr uint32_t kRankBlock = 448;  // positions per 64-byte rank line (7 x u64)

// One row's rank line: the row's ones before the line + 448 bits of the row.  A rank is
// ONE 64-byte load plus popcounts.  Lines of the 4 rows live in 4 separate arrays.
struct alignas(64) RankLine {
    uint32_t count;
    uint32_t pad;
    uint64_t w[7];
};

// Inverse-walk jump table: the 32 characters met by walking 32 steps backwards from node
// j (text order, character t in bits 2t..2t+1) and the node reached.  Replaces 32
// dependent select()s of access_kmer by one 16-byte load.
struct alignas(16) WalkEntry {
    uint64_t chars;
    uint32_t jump;
    uint32_t pad;
};

struct DevIndex {
    const RankLine *lines;  // [4][nlines]
    const uint8_t *lcs;     // [n]
    const uint32_t *uniq;   // bit z: node z's (k-1)-suffix group is {z}
    const WalkEntry *walk;  // [n]
    uint32_t nlines;
    uint32_t n;
    uint32_t k;
    uint32_t t_jump;        // first contraction probe below d-1 (see ms_step)
    uint32_t C[5];          // C[4] = n
};

// per-read status codes (values of ntc_status)
enum : int {
    kErrInvalidBase = 2,
    kErrEmptyRead = 3,
    kErrLength = 4,
    kErrCapacity = 5,
    kErrFormat = 8,
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

struct LineRegs {
    uint32_t count;
    uint64_t w[7];
};

NTC_HD void load_line(const RankLine *L, LineRegs &o) {
#ifdef __HIP_DEVICE_COMPILE__
    const uint4 *p = reinterpret_cast<const uint4 *>(L);
    uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    o.count = a.x;
    o.w[0] = (uint64_t)a.z | ((uint64_t)a.w << 32);
    o.w[1] = (uint64_t)b.x | ((uint64_t)b.y << 32);
    o.w[2] = (uint64_t)b.z | ((uint64_t)b.w << 32);
    o.w[3] = (uint64_t)c.x | ((uint64_t)c.y << 32);
    o.w[4] = (uint64_t)c.z | ((uint64_t)c.w << 32);
    o.w[5] = (uint64_t)d.x | ((uint64_t)d.y << 32);
    o.w[6] = (uint64_t)d.z | ((uint64_t)d.w << 32);
#else
    o.count = L->count;
    for (int j = 0; j < 7; j++) o.w[j] = L->w[j];
#endif
}

// ones in the line's positions [0, off), off < 448
NTC_HD uint32_t rank_in(const LineRegs &L, uint32_t off) {
    const uint32_t wi = off >> 6, bi = off & 63;
    uint32_t s = L.count;
#pragma unroll
    for (uint32_t j = 0; j < 7; j++) {
        uint64_t m = (j < wi) ? ~0ULL : ((j == wi) ? ((1ULL << bi) - 1) : 0ULL);
        s += (uint32_t)__builtin_popcountll(L.w[j] & m);
    }
    return s;
}

// extend_right(I, c) = [C[c] + rank_c(l), C[c] + rank_c(r))
NTC_HD void extend(const DevIndex &ix, int c, uint32_t l, uint32_t r, uint32_t &nl, uint32_t &nr) {
    const RankLine *rows = ix.lines + (uint64_t)c * ix.nlines;
    const uint32_t li = l / kRankBlock, ri = r / kRankBlock;
    LineRegs A;
    load_line(rows + li, A);
    const uint32_t rl = rank_in(A, l - li * kRankBlock);
    uint32_t rr;
    if (ri == li) {
        rr = rank_in(A, r - li * kRankBlock);
    } else {
        LineRegs B;
        load_line(rows + ri, B);
        rr = rank_in(B, r - ri * kRankBlock);
    }
    nl = ix.C[c] + rl;
    nr = ix.C[c] + rr;
}

// contract_left(I, t) [ext sbwt]: widen I to all nodes sharing the last t characters.
NTC_HD void widen(const DevIndex &ix, uint32_t &l, uint32_t &r, uint32_t t) {
    while (l > 0 && ix.lcs[l] >= t) l--;
    while (r < ix.n && ix.lcs[r] >= t) r++;
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
NTC_HD uint32_t run_from(const uint32_t *F, uint32_t p, uint32_t cap) {
    int64_t w = p >> 5;
    const uint32_t b = p & 31;
    uint32_t x = F[w * 64];
    const uint32_t z = clz32((~x) << (31 - b));
    if (z <= b) return z < cap ? z : cap;
    uint32_t cnt = b + 1;
    for (w = w - 1; w >= 0 && cnt < cap; w--) {
        x = F[w * 64];
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

// Writes the L characters of the L-step inverse walk from node j into out[0..L).
NTC_HD bool walk_record(const DevIndex &ix, uint32_t j, uint32_t L, uint8_t *out) {
    uint32_t end = L, cur = j;
    while (end > 0) {
        if (cur >= ix.n) return false;
#ifdef __HIP_DEVICE_COMPILE__
        const uint4 e4 = *reinterpret_cast<const uint4 *>(ix.walk + cur);
        const uint64_t chars = (uint64_t)e4.x | ((uint64_t)e4.y << 32);
        const uint32_t jump = e4.z;
#else
        const uint64_t chars = ix.walk[cur].chars;
        const uint32_t jump = ix.walk[cur].jump;
#endif
        const uint32_t take = end < 32 ? end : 32;
        const uint32_t sh = 32 - take;
        for (uint32_t u = 0; u < take; u++)
            out[end - take + u] = base_char((uint32_t)(chars >> (2 * (sh + u))));
        end -= take;
        cur = jump;
    }
    return true;
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
