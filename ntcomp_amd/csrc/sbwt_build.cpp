// SBWT subset-matrix + LCS construction: the index producer that stands in for
// kbo::build (src/main.rs:111-134, tests/fasta_data.rs:56-63; kbo 0.5.1 -> sbwt 0.3.11
// [ext], Cargo.lock:740-743, 1358-1361) with add_revcomp = true.
//
// Definition (published SBWT, Alanko et al.):
//   nodes  = k-spectrum (k-mers of every maximal ACGT run, plus reverse complements)
//            + for every k-mer x with no in-neighbour: $^(k-i) x[0..i], i = 0..k-1
//            (i = 0 is the root $^k, always present),
//   order  = colexicographic, '$' < A < C < G < T,
//   label  = {c : v[1..k]c is a node}, stored on the colex-first node of each
//            (k-1)-suffix group only,
//   C[c]   = 1 + #labels with a character < c,
//   lcs[i] = longest common suffix of nodes i-1 and i, lcs[0] = 0.
//
// Representation: a node is its characters read right-to-left (last character first),
// 2 bits each, packed MSB-first into W = ceil(2k/64) words, plus its number of real
// (non-$) characters.  Sorting by (words, len) is exactly colex order with '$' < A
// because padding is 0 and a shorter real part means a '$' comes next.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "ntc_internal.h"

namespace ntc {

namespace {

template <int W>
struct Node {
    uint64_t w[W];
    uint32_t len;
};

template <int W>
inline bool node_less(const Node<W> &a, const Node<W> &b) {
    for (int j = 0; j < W; j++)
        if (a.w[j] != b.w[j]) return a.w[j] < b.w[j];
    return a.len < b.len;
}
template <int W>
inline bool node_eq(const Node<W> &a, const Node<W> &b) {
    for (int j = 0; j < W; j++)
        if (a.w[j] != b.w[j]) return false;
    return a.len == b.len;
}

inline int code_of(uint8_t b) {
    switch (b) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return -1;
    }
}

// mask keeping characters t < m
template <int W>
inline void char_mask(uint32_t m, uint64_t (&mask)[W]) {
    for (int j = 0; j < W; j++) {
        int64_t c = (int64_t)m - 32 * j;
        if (c >= 32) mask[j] = ~0ULL;
        else if (c <= 0) mask[j] = 0;
        else mask[j] = ~0ULL << (64 - 2 * c);
    }
}

template <int W>
inline void shl_bits(uint64_t (&w)[W], uint32_t bits) {  // towards lower t (drop t=0..)
    uint32_t ws = bits / 64, bs = bits % 64;
    for (int j = 0; j < W; j++) {
        uint64_t hi = (j + (int)ws < W) ? w[j + ws] : 0;
        uint64_t lo = (j + (int)ws + 1 < W) ? w[j + ws + 1] : 0;
        w[j] = bs ? ((hi << bs) | (lo >> (64 - bs))) : hi;
    }
}

template <class T, class Cmp>
void psort(T *a, size_t n, int threads, Cmp cmp) {
    if (threads <= 1 || n < 200000) {
        std::sort(a, a + n, cmp);
        return;
    }
    size_t mid = n / 2;
    std::thread t([&] { psort(a, mid, threads / 2, cmp); });
    psort(a + mid, n - mid, threads - threads / 2, cmp);
    t.join();
    std::inplace_merge(a, a + mid, a + n, cmp);
}

template <class F>
void parallel_for(size_t n, int threads, F f) {
    if (threads <= 1 || n < 10000) {
        f(0, n);
        return;
    }
    std::vector<std::thread> ts;
    size_t chunk = (n + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        size_t a = t * chunk, b = std::min(n, a + chunk);
        if (a >= b) break;
        ts.emplace_back([=] { f(a, b); });
    }
    for (auto &t : ts) t.join();
}

template <int W>
void build_w(const uint8_t *seqs, const uint64_t *offs, uint64_t nseqs, uint32_t k, bool revcomp,
             int threads, HostIndex &out) {
    uint64_t kmask[W], km1mask[W];
    char_mask<W>(k, kmask);
    char_mask<W>(k - 1, km1mask);

    // ---- 1. maximal ACGT runs ----------------------------------------------------
    struct Run { uint64_t a, b; };
    std::vector<Run> runs;
    uint64_t total_kmers = 0;
    for (uint64_t s = 0; s < nseqs; s++) {
        uint64_t p = offs[s], e = offs[s + 1];
        while (p < e) {
            while (p < e && code_of(seqs[p]) < 0) p++;
            uint64_t a = p;
            while (p < e && code_of(seqs[p]) >= 0) p++;
            if (p - a >= k) {
                // split very long runs so threads share the work (overlap k-1)
                const uint64_t piece = 1 << 20;
                for (uint64_t x = a; x + k <= p; x += piece) {
                    uint64_t y = std::min(p, x + piece + k - 1);
                    runs.push_back({x, y});
                    total_kmers += y - x - k + 1;
                }
            }
        }
    }
    // ---- 2. k-spectrum (+ reverse complements) -------------------------------------
    std::vector<Node<W>> K(total_kmers * (revcomp ? 2 : 1));
    std::vector<uint64_t> run_base(runs.size() + 1, 0);
    for (size_t r = 0; r < runs.size(); r++)
        run_base[r + 1] = run_base[r] + (runs[r].b - runs[r].a - k + 1) * (revcomp ? 2 : 1);
    parallel_for(runs.size(), threads, [&](size_t ra, size_t rb) {
        for (size_t r = ra; r < rb; r++) {
            Node<W> f{}, g{};
            f.len = g.len = k;
            uint64_t o = run_base[r];
            uint32_t have = 0;
            for (uint64_t p = runs[r].a; p < runs[r].b; p++) {
                uint64_t c = (uint64_t)code_of(seqs[p]);
                // forward, reversed packing: new char becomes t = 0
                for (int j = W - 1; j > 0; j--) f.w[j] = (f.w[j] >> 2) | (f.w[j - 1] << 62);
                f.w[0] = (f.w[0] >> 2) | (c << 62);
                for (int j = 0; j < W; j++) f.w[j] &= kmask[j];
                // reverse complement: complement in forward order, new char at t = k-1
                for (int j = 0; j < W - 1; j++) g.w[j] = (g.w[j] << 2) | (g.w[j + 1] >> 62);
                g.w[W - 1] <<= 2;
                uint32_t t = k - 1;
                g.w[t / 32] |= (3 - c) << (62 - 2 * (t % 32));
                for (int j = 0; j < W; j++) g.w[j] &= kmask[j];
                if (++have >= k) {
                    K[o++] = f;
                    if (revcomp) K[o++] = g;
                }
            }
        }
    });
    psort(K.data(), K.size(), threads, node_less<W>);
    K.erase(std::unique(K.begin(), K.end(), node_eq<W>), K.end());

    // ---- 3. sources (no in-neighbour) and their dummies -----------------------------
    std::vector<uint8_t> is_source(K.size(), 0);
    parallel_for(K.size(), threads, [&](size_t a, size_t b) {
        for (size_t i = a; i < b; i++) {
            Node<W> key{};
            for (int j = 0; j < W; j++) key.w[j] = K[i].w[j];
            shl_bits<W>(key.w, 2);  // x[0..k-1] as a (k-1)-suffix
            key.len = 0;
            auto it = std::lower_bound(K.begin(), K.end(), key, node_less<W>);
            bool found = false;
            if (it != K.end()) {
                found = true;
                for (int j = 0; j < W; j++)
                    if ((it->w[j] & km1mask[j]) != key.w[j]) { found = false; break; }
            }
            is_source[i] = !found;
        }
    });
    std::vector<Node<W>> nodes;
    nodes.reserve(K.size() + 1024);
    Node<W> root{};
    root.len = 0;
    nodes.push_back(root);
    for (size_t i = 0; i < K.size(); i++) {
        if (!is_source[i]) continue;
        for (uint32_t r = 1; r < k; r++) {  // r real characters: $^(k-r) x[0..r]
            Node<W> d{};
            for (int j = 0; j < W; j++) d.w[j] = K[i].w[j];
            shl_bits<W>(d.w, 2 * (k - r));
            uint64_t m[W];
            char_mask<W>(r, m);
            for (int j = 0; j < W; j++) d.w[j] &= m[j];
            d.len = r;
            nodes.push_back(d);
        }
    }
    psort(nodes.data(), nodes.size(), threads, node_less<W>);
    nodes.erase(std::unique(nodes.begin(), nodes.end(), node_eq<W>), nodes.end());
    // merge the (sorted) dummies with the (sorted) k-spectrum
    std::vector<Node<W>> all(nodes.size() + K.size());
    std::merge(nodes.begin(), nodes.end(), K.begin(), K.end(), all.begin(), node_less<W>);
    std::vector<Node<W>>().swap(nodes);
    std::vector<Node<W>>().swap(K);

    const uint64_t n = all.size();
    if (n >= (1ULL << 32)) throw std::runtime_error("index too large for 32-bit colex ranks");
    out.n = n;
    out.k = k;
    out.lcs.assign(n, 0);
    const uint64_t nw = (n + 63) / 64;
    for (int c = 0; c < 4; c++) out.rows[c].assign(nw, 0);

    // ---- 4. LCS ----------------------------------------------------------------------
    parallel_for(n, threads, [&](size_t a, size_t b) {
        for (size_t i = std::max<size_t>(a, 1); i < b; i++) {
            const Node<W> &x = all[i - 1], &y = all[i];
            uint32_t common = 32 * W;
            for (int j = 0; j < W; j++) {
                uint64_t d = x.w[j] ^ y.w[j];
                if (d) { common = 32 * j + (uint32_t)__builtin_clzll(d) / 2; break; }
            }
            uint32_t l = std::min(common, std::min(x.len, y.len));
            out.lcs[i] = (uint8_t)std::min<uint32_t>(l, 255);
        }
    });

    // ---- 5. labels: merge nodes-ending-with-c against (k-1)-suffix groups -------------
    // group-first nodes in order, with their (k-1)-suffix key
    std::vector<uint32_t> gfirst;
    gfirst.reserve(n / 2);
    for (uint64_t i = 0; i < n; i++)
        if (i == 0 || out.lcs[i] < k - 1) gfirst.push_back((uint32_t)i);
    auto gkey = [&](uint32_t gi, Node<W> &key) {
        const Node<W> &v = all[gi];
        for (int j = 0; j < W; j++) key.w[j] = v.w[j] & km1mask[j];
        key.len = std::min(v.len, k - 1);
    };
    uint64_t first_of[5];
    {
        // nodes ending with c: len >= 1 and top two bits == c; contiguous
        uint64_t i = 1;
        for (int c = 0; c < 4; c++) {
            first_of[c] = i;
            while (i < n && (all[i].w[0] >> 62) == (uint64_t)c) i++;
        }
        first_of[4] = i;
        if (i != n) throw std::runtime_error("internal: node order");
    }
    std::atomic<bool> bad{false};
    std::vector<std::thread> ts;
    for (int c = 0; c < 4; c++) {
        ts.emplace_back([&, c] {
            size_t g = 0;
            Node<W> gk{}, uk{};
            if (!gfirst.empty()) gkey(gfirst[0], gk);
            for (uint64_t u = first_of[c]; u < first_of[c + 1]; u++) {
                for (int j = 0; j < W; j++) uk.w[j] = all[u].w[j];
                shl_bits<W>(uk.w, 2);
                uk.len = all[u].len - 1;
                while (g < gfirst.size() && node_less<W>(gk, uk)) {
                    g++;
                    if (g < gfirst.size()) gkey(gfirst[g], gk);
                }
                if (g >= gfirst.size() || !node_eq<W>(gk, uk)) { bad = true; return; }
                uint64_t gi = gfirst[g];
                out.rows[c][gi >> 6] |= 1ULL << (gi & 63);  // rows[c] is owned by this thread
            }
        });
    }
    for (auto &t : ts) t.join();
    if (bad) throw std::runtime_error("internal: node without a predecessor group");
    for (int c = 0; c < 4; c++) {
        uint64_t before = 1;
        for (int cc = 0; cc < c; cc++)
            for (uint64_t w = 0; w < nw; w++) before += (uint64_t)__builtin_popcountll(out.rows[cc][w]);
        out.C[c] = before;
        if (before != first_of[c]) throw std::runtime_error("internal: C array mismatch");
    }
}

}  // namespace

void build_index(const uint8_t *seqs, const uint64_t *offs, uint64_t nseqs, uint32_t k,
                 bool revcomp, int threads, HostIndex &out) {
    if (k < 1 || k > 255) throw std::invalid_argument("k must be in [1, 255]");
    if (threads <= 0) threads = std::max(1u, std::thread::hardware_concurrency());
    int W = (int)((2 * k + 63) / 64);
    switch (W) {
    case 1: build_w<1>(seqs, offs, nseqs, k, revcomp, threads, out); break;
    case 2: build_w<2>(seqs, offs, nseqs, k, revcomp, threads, out); break;
    case 3: build_w<3>(seqs, offs, nseqs, k, revcomp, threads, out); break;
    case 4: build_w<4>(seqs, offs, nseqs, k, revcomp, threads, out); break;
    case 5: build_w<5>(seqs, offs, nseqs, k, revcomp, threads, out); break;
    case 6: build_w<6>(seqs, offs, nseqs, k, revcomp, threads, out); break;
    case 7: build_w<7>(seqs, offs, nseqs, k, revcomp, threads, out); break;
    default: build_w<8>(seqs, offs, nseqs, k, revcomp, threads, out); break;
    }
}

}  // namespace ntc
