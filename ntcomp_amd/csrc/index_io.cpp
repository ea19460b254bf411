// <prefix>.sbwt / <prefix>.lcs -- the counterpart of kbo::index::serialize_sbwt
// (src/main.rs:138) and kbo::index::load_sbwt (src/main.rs:149, :190).  Like the reference,
// encode and decode both want the two files side by side (README.md:44).  Two layouts:
//
// kIndexOwn (`--index-format own`): this library's own, all integers little-endian:
//   .sbwt: "NTCSBWT1" u64 version=1, u64 n, u64 k, u64 C[4], u64 nwords, 4 x nwords u64
//   .lcs : "NTCLCS01" u64 n, n bytes
//
// kIndexSbwtRs (the default since round 5, as the reference always writes this layout,
// main.rs:138): a RESTATEMENT of sbwt 0.3.11 / kbo 0.5.1 serialisation [ext, recalled --
// PARITY UNPINNED: neither crate nor any reference-written index exists offline, so this
// layout is written from memory of the published crates and may differ from theirs].
// Built on simple-sds conventions (every integer a little-endian u64 word):
//   Vec<u64>   = u64 len, len words           RawVector = u64 len_bits, Vec<u64>
//   IntVector  = u64 len, u64 width, RawVector  (width-bit fields packed LSB-first)
//   Option<T>  = u64 size in words (0 = None), then the words
//   BitVector  = u64 ones, RawVector, Option<rank>, Option<select>, Option<select_zero>
//   .sbwt = u64 L, "plain-matrix" (the variant id, L bytes), then SbwtIndex<SubsetMatrix>:
//           4 BitVectors (rows A, C, G, T; n bits each), Vec<u64> C (4 entries),
//           u64 n_sets (= n), u64 k, prefix lookup table (sbwt's PrefixLookupTable, -p /
//           --prefix-precalc, src/cli.rs:46): u64 prefix_len p, u64 4^p, then per p-mer
//           (first character most significant) its colex interval as u64 start, u64 end
//           ([0, 0) when absent; p = 0: the single range [0, n))
//   .lcs  = IntVector of n entries, width = bits of k
// The reference builds its index with build_select = true (main.rs:118-119): sbwt's
// SubsetMatrix rows carry rank support (always: the search needs it) and select support
// (access_kmer, which the reference's decode calls, lib.rs:258, 286, 291), no select_zero.
// So each row is written with Some(rank), Some(select), None, as restated from simple-sds
// 0.3 [ext, recalled, unpinned]:
//   RankSupport   = Vec<(u64, u64)>: per 512-bit superblock (ones before it, the cumulative
//                   ones before each of its words 1..7 as 9-bit fields, word j at bit 9 (j-1))
//   SelectSupport = Vec<(u64, u64)> samples, IntVector long, IntVector short: the ones in
//                   superblocks of 4096; per superblock (position of its first one, offset):
//                   a superblock spanning more than 2^16 bits is "long" and lists every one's
//                   position in long (width = bits of the vector length, offset into long);
//                   else short holds, per block of 64 ones, the block's first one relative to
//                   the superblock's first (16 bits, offset into short).
// Read tolerantly: Options are skipped by their size, Some or None, so files with or without
// the supports load.  load_index detects the layout from the first 8 bytes.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "ntc_internal.h"

namespace ntc {

namespace {
struct File {
    FILE *f = nullptr;
    explicit File(const std::string &p, const char *mode) { f = std::fopen(p.c_str(), mode); }
    ~File() {
        if (f) std::fclose(f);
    }
};
bool wr(FILE *f, const void *p, size_t n) { return std::fwrite(p, 1, n, f) == n; }
bool rd(FILE *f, void *p, size_t n) { return std::fread(p, 1, n, f) == n; }
}  // namespace

bool save_index(const HostIndex &ix, const std::string &prefix, std::string &err) {
    const uint64_t nw = (ix.n + 63) / 64;
    {
        File f(prefix + ".sbwt", "wb");
        if (!f.f) { err = "cannot open " + prefix + ".sbwt for writing"; return false; }
        uint64_t hdr[1 + 1 + 1 + 4 + 1] = {1, ix.n, ix.k, ix.C[0], ix.C[1], ix.C[2], ix.C[3], nw};
        bool ok = wr(f.f, "NTCSBWT1", 8) && wr(f.f, hdr, sizeof(hdr));
        for (int c = 0; c < 4 && ok; c++) ok = wr(f.f, ix.rows[c].data(), nw * 8);
        if (!ok) { err = "write failed: " + prefix + ".sbwt"; return false; }
    }
    {
        File f(prefix + ".lcs", "wb");
        if (!f.f) { err = "cannot open " + prefix + ".lcs for writing"; return false; }
        uint64_t n = ix.n;
        if (!(wr(f.f, "NTCLCS01", 8) && wr(f.f, &n, 8) && wr(f.f, ix.lcs.data(), ix.n))) {
            err = "write failed: " + prefix + ".lcs";
            return false;
        }
    }
    return true;
}

namespace {
// ---- sbwt-rs / simple-sds layout (kIndexSbwtRs, see the header) -----------------------
const char kVariantId[] = "plain-matrix";

bool wr64(FILE *f, uint64_t v) { return wr(f, &v, 8); }
bool rd64(FILE *f, uint64_t &v) { return rd(f, &v, 8); }
bool wr_raw(FILE *f, const uint64_t *w, uint64_t bits) {  // RawVector
    const uint64_t nw = (bits + 63) / 64;
    return wr64(f, bits) && wr64(f, nw) && (nw == 0 || wr(f, w, nw * 8));
}
bool rd_raw(FILE *f, std::vector<uint64_t> &w, uint64_t &bits) {
    uint64_t nw = 0;
    if (!rd64(f, bits) || !rd64(f, nw) || nw != (bits + 63) / 64 || nw > (1ULL << 40)) return false;
    w.assign(nw, 0);
    return nw == 0 || rd(f, w.data(), nw * 8);
}
bool skip_option(FILE *f) {
    uint64_t sz = 0;
    return rd64(f, sz) && (sz == 0 || std::fseek(f, (long)(sz * 8), SEEK_CUR) == 0);
}

// simple-sds IntVector body: len, width, RawVector of the packed fields
void int_vector(const std::vector<uint64_t> &v, uint64_t width, std::vector<uint64_t> &out) {
    std::vector<uint64_t> packed((v.size() * width + 63) / 64, 0);
    for (uint64_t i = 0; i < v.size(); i++) {
        const uint64_t bit = i * width, x = width == 64 ? v[i] : v[i] & ((1ULL << width) - 1);
        packed[bit >> 6] |= x << (bit & 63);
        if ((bit & 63) + width > 64) packed[(bit >> 6) + 1] |= x >> (64 - (bit & 63));
    }
    out.push_back(v.size());
    out.push_back(width);
    out.push_back(v.size() * width);
    out.push_back(packed.size());
    out.insert(out.end(), packed.begin(), packed.end());
}

// RankSupport words (see the header) of an n-bit row
std::vector<uint64_t> rank_support(const uint64_t *w, uint64_t n) {
    const uint64_t nw = (n + 63) / 64, sb = (nw + 7) / 8;
    std::vector<uint64_t> out{sb};
    uint64_t before = 0;
    for (uint64_t s = 0; s < sb; s++) {
        uint64_t rel = 0, in = 0;
        for (uint64_t j = 0; j < 8 && 8 * s + j < nw; j++) {
            if (j) rel |= in << (9 * (j - 1));
            in += (uint64_t)__builtin_popcountll(w[8 * s + j]);
        }
        out.push_back(before);
        out.push_back(rel);
        before += in;
    }
    return out;
}

// SelectSupport words (see the header) of an n-bit row
std::vector<uint64_t> select_support(const uint64_t *w, uint64_t n) {
    constexpr uint64_t kSuper = 4096, kLongBits = 1ULL << 16, kBlock = 64;
    std::vector<uint64_t> ones;
    const uint64_t nw = (n + 63) / 64;
    for (uint64_t i = 0; i < nw; i++)
        for (uint64_t x = w[i]; x; x &= x - 1) ones.push_back(64 * i + (uint64_t)__builtin_ctzll(x));
    uint64_t width = 1;
    while (width < 64 && (1ULL << width) < n) width++;
    std::vector<uint64_t> samples, lng, shrt;
    for (uint64_t a = 0; a < ones.size(); a += kSuper) {
        const uint64_t b = std::min<uint64_t>(ones.size(), a + kSuper);
        if (ones[b - 1] - ones[a] + 1 > kLongBits) {
            samples.push_back(ones[a]);
            samples.push_back(lng.size());
            lng.insert(lng.end(), ones.begin() + (long)a, ones.begin() + (long)b);
        } else {
            samples.push_back(ones[a]);
            samples.push_back(shrt.size());
            for (uint64_t i = a; i < b; i += kBlock) shrt.push_back(ones[i] - ones[a]);
        }
    }
    std::vector<uint64_t> out{samples.size() / 2};
    out.insert(out.end(), samples.begin(), samples.end());
    int_vector(lng, width, out);
    int_vector(shrt, 16, out);
    return out;
}

bool wr_option(FILE *f, const std::vector<uint64_t> &body) {  // Some(T): size in words, then T
    return wr64(f, body.size()) && wr(f, body.data(), body.size() * 8);
}

bool save_sbwt_rs(const HostIndex &ix, const std::string &prefix, std::string &err) {
    {
        File f(prefix + ".sbwt", "wb");
        if (!f.f) { err = "cannot open " + prefix + ".sbwt for writing"; return false; }
        const uint64_t L = sizeof(kVariantId) - 1;
        bool ok = wr64(f.f, L) && wr(f.f, kVariantId, L);
        for (int c = 0; c < 4 && ok; c++) {
            uint64_t ones = 0;
            for (uint64_t x : ix.rows[c]) ones += (uint64_t)__builtin_popcountll(x);
            // Some(rank), Some(select), None(select_zero): build_select = true (main.rs:119)
            ok = wr64(f.f, ones) && wr_raw(f.f, ix.rows[c].data(), ix.n) &&
                 wr_option(f.f, rank_support(ix.rows[c].data(), ix.n)) &&
                 wr_option(f.f, select_support(ix.rows[c].data(), ix.n)) && wr64(f.f, 0);
        }
        ok = ok && wr64(f.f, 4);
        for (int c = 0; c < 4 && ok; c++) ok = wr64(f.f, ix.C[c]);
        ok = ok && wr64(f.f, ix.n) && wr64(f.f, ix.k);
        if (ix.prefix_len && ix.prefix_ranges.size() == 2 * (1ULL << (2 * ix.prefix_len))) {
            ok = ok && wr64(f.f, ix.prefix_len) && wr64(f.f, ix.prefix_ranges.size() / 2) &&
                 wr(f.f, ix.prefix_ranges.data(), ix.prefix_ranges.size() * 8);
        } else {
            ok = ok && wr64(f.f, 0) && wr64(f.f, 1) && wr64(f.f, 0) && wr64(f.f, ix.n);
        }
        if (!ok) { err = "write failed: " + prefix + ".sbwt"; return false; }
    }
    {
        File f(prefix + ".lcs", "wb");
        if (!f.f) { err = "cannot open " + prefix + ".lcs for writing"; return false; }
        uint64_t width = 1;
        while ((1ULL << width) <= ix.k) width++;
        std::vector<uint64_t> packed((ix.n * width + 63) / 64, 0);
        for (uint64_t i = 0; i < ix.n; i++) {
            const uint64_t bit = i * width, v = ix.lcs[i];
            packed[bit >> 6] |= v << (bit & 63);
            if ((bit & 63) + width > 64) packed[(bit >> 6) + 1] |= v >> (64 - (bit & 63));
        }
        if (!(wr64(f.f, ix.n) && wr64(f.f, width) && wr_raw(f.f, packed.data(), ix.n * width))) {
            err = "write failed: " + prefix + ".lcs";
            return false;
        }
    }
    return true;
}

bool load_sbwt_rs(const std::string &prefix, HostIndex &ix, std::string &err) {
    {
        File f(prefix + ".sbwt", "rb");
        if (!f.f) { err = "cannot open " + prefix + ".sbwt"; return false; }
        uint64_t L = 0;
        char id[64] = {0};
        if (!rd64(f.f, L) || L >= sizeof(id) || !rd(f.f, id, L) || std::strcmp(id, kVariantId) != 0) {
            err = prefix + ".sbwt: not a plain-matrix SBWT";
            return false;
        }
        uint64_t n = ~0ULL;
        for (int c = 0; c < 4; c++) {
            uint64_t ones = 0, bits = 0;
            if (!rd64(f.f, ones) || !rd_raw(f.f, ix.rows[c], bits) || !skip_option(f.f) || !skip_option(f.f) ||
                !skip_option(f.f)) {
                err = prefix + ".sbwt: truncated subset matrix";
                return false;
            }
            if (n != ~0ULL && bits != n) { err = prefix + ".sbwt: rows of different lengths"; return false; }
            n = bits;
        }
        uint64_t nc = 0, n_sets = 0, k = 0;
        if (!rd64(f.f, nc) || nc < 4 || nc > 8) { err = prefix + ".sbwt: bad C array"; return false; }
        for (uint64_t c = 0; c < nc; c++) {
            uint64_t v = 0;
            if (!rd64(f.f, v)) { err = prefix + ".sbwt: truncated C array"; return false; }
            if (c < 4) ix.C[c] = v;
        }
        if (!rd64(f.f, n_sets) || !rd64(f.f, k) || n_sets != n || k < 1 || k > 255) {
            err = prefix + ".sbwt: inconsistent header";
            return false;
        }
        ix.n = n;
        ix.k = (uint32_t)k;
        // the prefix lookup table (absent in files written before round 4)
        uint64_t p = 0, nr = 0;
        ix.prefix_len = 0;
        ix.prefix_ranges.clear();
        if (rd64(f.f, p) && rd64(f.f, nr) && p >= 1 && p <= 12 && nr == (1ULL << (2 * p))) {
            ix.prefix_ranges.resize(2 * nr);
            if (!rd(f.f, ix.prefix_ranges.data(), 16 * nr)) {
                err = prefix + ".sbwt: truncated prefix lookup table";
                return false;
            }
            ix.prefix_len = (uint32_t)p;
        }
    }
    {
        File f(prefix + ".lcs", "rb");
        if (!f.f) { err = "cannot open " + prefix + ".lcs"; return false; }
        uint64_t len = 0, width = 0, bits = 0;
        std::vector<uint64_t> packed;
        if (!rd64(f.f, len) || !rd64(f.f, width) || len != ix.n || width < 1 || width > 8 ||
            !rd_raw(f.f, packed, bits) || bits != len * width) {
            err = prefix + ".lcs: missing, foreign or not matching " + prefix + ".sbwt";
            return false;
        }
        ix.lcs.assign(len, 0);
        const uint64_t mask = (1ULL << width) - 1;
        for (uint64_t i = 0; i < len; i++) {
            const uint64_t bit = i * width;
            uint64_t v = packed[bit >> 6] >> (bit & 63);
            if ((bit & 63) + width > 64) v |= packed[(bit >> 6) + 1] << (64 - (bit & 63));
            ix.lcs[i] = (uint8_t)(v & mask);
        }
    }
    return true;
}
}  // namespace

// sbwt's search from [0, n) per character (extend_right: [C[c] + rank_c(l), C[c] + rank_c(r))),
// level by level: the p-mer X.c has index 4 idx(X) + c
void prefix_table(const HostIndex &ix, uint32_t p, std::vector<uint64_t> &ranges) {
    const uint64_t nw = (ix.n + 63) / 64;
    std::vector<uint64_t> cum[4];  // ones before every 8th word
    for (int c = 0; c < 4; c++) {
        cum[c].assign(nw / 8 + 2, 0);
        uint64_t acc = 0;
        for (uint64_t w = 0; w < nw; w++) {
            if (w % 8 == 0) cum[c][w / 8] = acc;
            acc += (uint64_t)__builtin_popcountll(ix.rows[c][w]);
        }
        cum[c][nw / 8 + 1] = acc;
        if (nw % 8 == 0) cum[c][nw / 8] = acc;
    }
    auto rank = [&](int c, uint64_t i) {  // ones of row c in [0, i)
        const uint64_t w = i / 64;
        uint64_t r = cum[c][w / 8];
        for (uint64_t x = w / 8 * 8; x < w; x++) r += (uint64_t)__builtin_popcountll(ix.rows[c][x]);
        if (i % 64) r += (uint64_t)__builtin_popcountll(ix.rows[c][w] & ((1ULL << (i % 64)) - 1));
        return r;
    };
    std::vector<uint64_t> cur = {0, ix.n}, nxt;
    for (uint32_t d = 1; d <= p; d++) {
        nxt.assign(cur.size() * 4, 0);
        for (uint64_t x = 0; x < cur.size() / 2; x++) {
            const uint64_t l = cur[2 * x], r = cur[2 * x + 1];
            for (int c = 0; c < 4; c++) {
                uint64_t a = 0, b = 0;
                if (l < r) {
                    a = ix.C[c] + rank(c, l);
                    b = ix.C[c] + rank(c, r);
                }
                if (a >= b) a = b = 0;
                nxt[2 * (4 * x + c)] = a;
                nxt[2 * (4 * x + c) + 1] = b;
            }
        }
        cur.swap(nxt);
    }
    ranges.swap(cur);
}

bool save_index_as(const HostIndex &ix, const std::string &prefix, int layout, std::string &err) {
    if (layout == kIndexSbwtRs) return save_sbwt_rs(ix, prefix, err);
    return save_index(ix, prefix, err);
}

bool load_index(const std::string &prefix, HostIndex &ix, std::string &err) {
    bool own = true;
    {  // layout detection: the own magic, else the sbwt-rs variant id
        File f(prefix + ".sbwt", "rb");
        if (!f.f) { err = "cannot open " + prefix + ".sbwt"; return false; }
        char magic[8];
        own = !(rd(f.f, magic, 8) && std::memcmp(magic, "NTCSBWT1", 8) != 0);
    }
    if (!own) return load_sbwt_rs(prefix, ix, err);
    {
        File f(prefix + ".sbwt", "rb");
        if (!f.f) { err = "cannot open " + prefix + ".sbwt"; return false; }
        char magic[8];
        uint64_t hdr[8];
        if (!rd(f.f, magic, 8) || std::memcmp(magic, "NTCSBWT1", 8) != 0 || !rd(f.f, hdr, sizeof(hdr)) ||
            hdr[0] != 1) {
            err = prefix + ".sbwt: not an ntcomp-mi355x index (or an unsupported version)";
            return false;
        }
        ix.n = hdr[1];
        ix.k = (uint32_t)hdr[2];
        for (int c = 0; c < 4; c++) ix.C[c] = hdr[3 + c];
        uint64_t nw = hdr[7];
        if (nw != (ix.n + 63) / 64 || ix.k < 1 || ix.k > 255) {
            err = prefix + ".sbwt: inconsistent header";
            return false;
        }
        for (int c = 0; c < 4; c++) {
            ix.rows[c].assign(nw, 0);
            if (!rd(f.f, ix.rows[c].data(), nw * 8)) { err = prefix + ".sbwt: truncated"; return false; }
        }
    }
    {
        File f(prefix + ".lcs", "rb");
        if (!f.f) { err = "cannot open " + prefix + ".lcs"; return false; }
        char magic[8];
        uint64_t n = 0;
        if (!rd(f.f, magic, 8) || std::memcmp(magic, "NTCLCS01", 8) != 0 || !rd(f.f, &n, 8) || n != ix.n) {
            err = prefix + ".lcs: missing, foreign or not matching " + prefix + ".sbwt";
            return false;
        }
        ix.lcs.assign(n, 0);
        if (!rd(f.f, ix.lcs.data(), n)) { err = prefix + ".lcs: truncated"; return false; }
    }
    return true;
}

}  // namespace ntc
