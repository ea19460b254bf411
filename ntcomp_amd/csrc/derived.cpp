// Host construction of the device-side index layout (DESIGN.md "Data layout in HBM").
#include "derived.h"

#include <algorithm>
#include <cmath>
#include <string>
#include <thread>

namespace ntc {

bool build_derived(const HostIndex &ix, Derived &out, std::string &err, int threads) {
    (void)threads;
    const uint64_t n = ix.n;
    const uint32_t k = ix.k;
    if (n == 0 || n >= (1ULL << 32) - 1) {
        err = "index must have 1 <= n < 2^32 - 1 nodes";
        return false;
    }
    if (k < 1 || k > 255) {
        err = "k must be in [1, 255]";
        return false;
    }
    const uint64_t nw = (n + 63) / 64;
    for (int c = 0; c < 4; c++)
        if (ix.rows[c].size() < nw) {
            err = "subset-matrix row shorter than ceil(n/64) words";
            return false;
        }
    if (ix.lcs.size() < n) {
        err = "LCS array shorter than n";
        return false;
    }
    // rank lines: 448 positions = 7 words, so line li holds row words [7li, 7li+7)
    const uint64_t nlines = n / kRankBlock + 1;
    out.nlines = (uint32_t)nlines;
    out.lines.assign(4 * nlines, RankLine{});
    uint64_t ones[4] = {0, 0, 0, 0};
    for (int c = 0; c < 4; c++) {
        const uint64_t *row = ix.rows[c].data();
        uint64_t cnt = 0;
        for (uint64_t li = 0; li < nlines; li++) {
            RankLine &L = out.lines[c * nlines + li];
            L.count = (uint32_t)cnt;
            L.pad = 0;
            for (int j = 0; j < 7; j++) {
                uint64_t wi = li * 7 + j;
                uint64_t w = wi < nw ? row[wi] : 0;
                if (wi == nw - 1 && (n & 63)) w &= (1ULL << (n & 63)) - 1;
                L.w[j] = w;
                cnt += (uint64_t)__builtin_popcountll(w);
            }
        }
        ones[c] = cnt;
    }
    // C array must agree with the rows: C[c] = 1 + #labels < c, and n = 1 + #labels
    uint64_t acc = 1;
    for (int c = 0; c < 4; c++) {
        if (ix.C[c] != acc) {
            err = "C array inconsistent with the subset matrix";
            return false;
        }
        out.C[c] = (uint32_t)acc;
        acc += ones[c];
    }
    if (acc != n) {
        err = "label count != n - 1 (not an SBWT: every non-root node needs one in-edge)";
        return false;
    }
    out.C[4] = (uint32_t)n;
    for (uint64_t i = 0; i < n; i++)
        if (ix.lcs[i] >= k && i > 0) {
            err = "LCS value >= k";
            return false;
        }
    // unique-predecessor bits: group of node z by (k-1)-suffix is {z}
    out.uniq.assign(n / 32 + 2, 0);
    for (uint64_t z = 0; z < n; z++) {
        bool u = (k >= 2) && ix.lcs[z] < k - 1 && (z + 1 == n || ix.lcs[z + 1] < k - 1);
        if (z == 0) u = false;  // the root is never a k-mer
        if (u) out.uniq[z >> 5] |= 1u << (z & 31);
    }
    // inverse walk: node C[c] + r is reached from the r-th set of row c (= select)
    out.pred.assign(n, 0);
    out.code.assign(n, 0);
    for (int c = 0; c < 4; c++) {
        const uint64_t *row = ix.rows[c].data();
        uint64_t r = 0;
        for (uint64_t wi = 0; wi < nw; wi++) {
            uint64_t w = row[wi];
            if (wi == nw - 1 && (n & 63)) w &= (1ULL << (n & 63)) - 1;
            while (w) {
                uint64_t pos = wi * 64 + (uint64_t)__builtin_ctzll(w);
                out.pred[out.C[c] + r] = (uint32_t)pos;
                out.code[out.C[c] + r] = (uint8_t)c;
                r++;
                w &= w - 1;
            }
        }
    }
    // galloping probe: random (t+1)-mers stop matching around log4(n)
    double l4 = std::log((double)n) / std::log(4.0);
    uint32_t tj = (uint32_t)std::ceil(l4) + 2;
    out.t_jump = std::max<uint32_t>(1, tj);
    return true;
}

void build_walk_host(const Derived &dv, uint64_t n, std::vector<WalkEntry> &walk) {
    std::vector<WalkEntry> a(n), b(n);
    for (uint64_t j = 0; j < n; j++) {
        a[j].chars = dv.code[j];
        a[j].jump = dv.pred[j];
        a[j].pad = 0;
    }
    for (uint32_t m = 1; m < 32; m *= 2) {
        for (uint64_t j = 0; j < n; j++) {
            const WalkEntry &x = a[j];
            const WalkEntry &y = a[x.jump];
            b[j].chars = y.chars | (x.chars << (2 * m));
            b[j].jump = y.jump;
            b[j].pad = 0;
        }
        a.swap(b);
    }
    walk.swap(a);
}

DevIndex host_dev_index(const HostIndex &ix, const Derived &dv, const std::vector<WalkEntry> &walk) {
    DevIndex d{};
    d.lines = dv.lines.data();
    d.lcs = ix.lcs.data();
    d.uniq = dv.uniq.data();
    d.walk = walk.data();
    d.nlines = dv.nlines;
    d.n = (uint32_t)ix.n;
    d.k = ix.k;
    d.t_jump = dv.t_jump;
    for (int c = 0; c < 5; c++) d.C[c] = dv.C[c];
    return d;
}

}  // namespace ntc
