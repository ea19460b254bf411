// Host construction of the device-side index layout (DESIGN.md "Data layout in HBM").
#include "derived.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>
#include <thread>

namespace ntc {

bool build_derived(const HostIndex &ix, Derived &out, std::string &err, bool host_paths) {
    const uint64_t n = ix.n;
    const uint32_t k = ix.k;
    if (n == 0 || n >= (uint64_t)kTabShort) {
        err = "index must have 1 <= n < 2^32 - 256 nodes";
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
    // C array must agree with the rows: C[c] = 1 + #labels < c, and n = 1 + #labels
    uint64_t ones[4] = {0, 0, 0, 0};
    for (int c = 0; c < 4; c++)
        for (uint64_t wi = 0; wi < nw; wi++) {
            uint64_t w = ix.rows[c][wi];
            if (wi == nw - 1 && (n & 63)) w &= (1ULL << (n & 63)) - 1;
            ones[c] += (uint64_t)__builtin_popcountll(w);
        }
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
    // rank words: 32 positions each, x = C[c] + ones before the word
    const uint64_t rw = n / 32 + 2;
    out.rwords = (uint32_t)rw;
    out.rank.assign(4 * rw, mk2(0, 0));
    for (int c = 0; c < 4; c++) {
        uint64_t cnt = out.C[c];
        for (uint64_t i = 0; i < rw; i++) {
            const uint64_t wi = i >> 1;
            uint64_t w = wi < nw ? ix.rows[c][wi] : 0;
            if (wi == nw - 1 && (n & 63)) w &= (1ULL << (n & 63)) - 1;
            const uint32_t bits = (uint32_t)(w >> (32 * (i & 1)));
            out.rank[c * rw + i] = mk2((uint32_t)cnt, bits);
            cnt += (uint64_t)__builtin_popcount(bits);
        }
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
    if (host_paths) build_paths(ix, out);
    out.absent = 0;
    for (int c = 0; c < 4; c++)
        if (out.C[c + 1] == out.C[c]) out.absent |= 1u << c;
    return true;
}

uint32_t default_tab_u(uint64_t n, uint32_t k, const uint8_t *lcs) {
    // random (t+1)-mers stop matching around log4(n): at U = ceil(log4 n) + 2 few absent
    // U-mers are present by chance, so few table-long positions need the SBWT
    const double l4 = std::log((double)std::max<uint64_t>(n, 2)) / std::log(4.0);
    uint32_t u = (uint32_t)std::ceil(l4) + 2;
    u = std::min<uint32_t>(u, kTabDefaultMaxU);
    u = std::max<uint32_t>(1u, std::min<uint32_t>(u, k));
    // What matters is how many distinct U-mers the index holds, not n: a collection of
    // strains (S91: 70 M nodes) shares most of them, one large genome does not.  Nodes with
    // a common U-suffix are adjacent in colex order, so the distinct U-suffixes are the
    // nodes whose LCS with their predecessor is < U.  Past kTabMaxDensity of all 4^U, a
    // random U-mer is present too often (SCAN finds false pairs, walks start on chance
    // matches): go one level deeper (a 100 Mbp genome, 200 M nodes: 53 % at U = 14, encode
    // 87 -> 132 Gbases/s at U = 15; S91 has 9 % and is slower at U = 15).
    if (lcs && u == kTabDefaultMaxU && u < std::min<uint32_t>(k, kTabMaxU)) {
        uint64_t groups = 0;
        for (uint64_t i = 0; i < n; i++) groups += lcs[i] < u;
        if ((double)groups > kTabMaxDensity * (double)(1ULL << (2 * u))) u++;
    }
    return u;
}

// presence bits of level u of a host table
static void level_bits(const std::vector<uint2> &tab, uint32_t u, std::vector<uint32_t> &bits) {
    bits.assign(tab_bits_words(u), 0);
    const uint2 *lv = tab.data() + tab_base(u);
    const uint64_t cnt = 1ULL << (2 * u);
    if (cnt >= 32) {
        for (uint64_t w = 0; w < cnt / 32; w++) bits[w] = tab_bits_word(lv, w);
    } else {
        for (uint64_t key = 0; key < cnt; key++) bits[0] |= (uint32_t)tab_long(lv[key]) << key;
    }
}

uint32_t filter_level(uint32_t U) { return U >= kFiltMinU ? U - kFiltGap : 0; }

void build_tab_host(const DevIndex &d, uint32_t U, std::vector<uint2> &tab, std::vector<uint32_t> &bits,
                    std::vector<uint32_t> &fbits) {
    tab.assign(tab_base(U + 1), mk2(0, 0));
    for (uint32_t u = 1; u <= U; u++) {
        uint2 *cur = tab.data() + tab_base(u);
        const uint2 *prev = u > 1 ? tab.data() + tab_base(u - 1) : nullptr;
        const uint64_t cnt = 1ULL << (2 * u);
        for (uint64_t key = 0; key < cnt; key++) cur[key] = tab_make(d, u, key, prev, d.tab_pos && u == U);
    }
    level_bits(tab, U, bits);
    fbits.clear();
    if (filter_level(U)) level_bits(tab, filter_level(U), fbits);
}

namespace {
inline uint32_t host_rank(const Derived &dv, int c, uint64_t i) {  // rank_c(i), without C[c]
    return rank_word(dv.rank[(uint64_t)c * dv.rwords + (i >> 5)], (uint32_t)i) - dv.C[c];
}
inline uint32_t labels_of(const Derived &dv, uint64_t g) {  // 4-bit label set of node g
    uint32_t m = 0;
    for (int c = 0; c < 4; c++) m |= ((dv.rank[(uint64_t)c * dv.rwords + (g >> 5)].y >> (g & 31)) & 1u) << c;
    return m;
}
}  // namespace

std::vector<uint8_t> dummy_nodes(const HostIndex &ix, const Derived &dv) {
    // dummies: BFS from the root through labels, depth < k
    const uint64_t n = ix.n;
    const uint32_t k = ix.k;
    std::vector<uint8_t> dummy(n, 0);
    std::vector<std::pair<uint32_t, uint32_t>> q;
    q.push_back({0, 0});
    dummy[0] = 1;
    for (size_t h = 0; h < q.size(); h++) {
        auto [v, dep] = q[h];
        if (dep + 1 >= k) continue;
        uint32_t m = labels_of(dv, v);
        for (int c = 0; c < 4; c++)
            if (m >> c & 1) {
                uint32_t z = dv.C[c] + host_rank(dv, c, v);
                if (!dummy[z]) {
                    dummy[z] = 1;
                    q.push_back({z, dep + 1});
                }
            }
    }
    return dummy;
}

uint32_t path_succ(const HostIndex &ix, const Derived &dv, const std::vector<uint8_t> &dummy, uint64_t z) {
    const uint64_t n = ix.n;
    const uint32_t k = ix.k;
    if (dummy[z]) return kNoNode;
    const bool head = k < 2 || ix.lcs[z] < k - 1;
    const bool alone = k < 2 || z + 1 == n || ix.lcs[z + 1] < k - 1;
    const uint32_t m = labels_of(dv, z);
    if (!head || !alone || m == 0 || (m & (m - 1))) return kNoNode;
    const int c = __builtin_ctz(m);
    const uint32_t y = dv.C[c] + host_rank(dv, c, z);
    return dummy[y] ? kNoNode : y;
}

// w[c] = path position of the node v[1..k]c, or kNoNode: the labels sit on the first node
// of v's (k-1)-suffix group (the SBWT's extension of v by c at depth k goes through it)
void fork_words(const HostIndex &ix, const Derived &dv, const std::vector<uint8_t> &dummy, uint32_t v, uint32_t *w) {
    uint64_t h = v;
    while (h > 0 && ix.lcs[h] >= ix.k - 1) h--;
    const uint32_t m = labels_of(dv, h);
    for (int c = 0; c < 4; c++) {
        w[c] = kNoNode;
        if (!((m >> c) & 1u)) continue;
        const uint32_t y = dv.C[c] + host_rank(dv, c, h);
        if (!dummy[y]) w[c] = dv.pos_of_node[y];
    }
}

bool path_link_on() {
    const char *e = std::getenv("NTC_PATH_LINK");
    return !(e && std::atoi(e) == 0);
}

// Unitig linking: a unitig's last node t whose successors y (each the first node of its own
// unitig) branch is joined to one of them, and so is a unitig's first node with several
// predecessors: t -> y is added when y is t's preferred successor AND t is y's preferred
// predecessor, preference going to the SHORTER unitig (then the smaller node).  In a
// collection of strains the unitigs through the sites every strain shares are short -- some
// strain branches off at almost every position -- while a strain's own variant spans one
// long, unbranched unitig (k nodes per SNP), so linking short unitigs strings the shared
// sequence into long paths and leaves the rare variants as their own paths.  A read then
// follows one path through the sites its strain shares with the others instead of hopping
// at every branch (L31: 18.7 fork hops per read with unitigs only).  Any edge of the graph is
// a valid path edge: the kernels stop a run wherever the read leaves the path and take the
// SBWT's own extension there (encode_core.h), so only speed depends on the choice.  The
// device builds the same cover (kernels.hip k_link_*).
void link_unitigs(const HostIndex &ix, const Derived &dv, const std::vector<uint8_t> &dummy,
                  std::vector<uint32_t> &nxt, std::vector<uint32_t> &prv) {
    const uint64_t n = ix.n;
    const uint32_t k = ix.k;
    std::vector<uint32_t> ulen(n, 0);  // nodes of the unitig each real node lies on (0: a cycle)
    for (uint64_t z = 1; z < n; z++) {
        if (dummy[z] || prv[z] != kNoNode) continue;
        uint32_t c = 0;
        for (uint32_t y = (uint32_t)z; y != kNoNode; y = nxt[y]) c++;
        for (uint32_t y = (uint32_t)z; y != kNoNode; y = nxt[y]) ulen[y] = c;
    }
    std::vector<uint64_t> best_pred(n, UINT64_MAX);
    std::vector<uint32_t> want(n, kNoNode);
    for (uint64_t t = 1; t < n; t++) {
        if (dummy[t] || !ulen[t] || nxt[t] != kNoNode) continue;
        uint64_t h = t;  // the (k-1)-suffix group's first node holds the labels
        while (h > 0 && ix.lcs[h] >= k - 1) h--;
        const uint32_t m = labels_of(dv, h);
        uint64_t best = UINT64_MAX;
        const uint64_t mine = (uint64_t)ulen[t] << 32 | t;
        for (int c = 0; c < 4; c++) {
            if (!((m >> c) & 1u)) continue;
            const uint32_t y = dv.C[c] + host_rank(dv, c, h);
            if (dummy[y] || prv[y] != kNoNode || !ulen[y]) continue;
            best = std::min(best, (uint64_t)ulen[y] << 32 | y);
            best_pred[y] = std::min(best_pred[y], mine);
        }
        if (best != UINT64_MAX) want[t] = (uint32_t)best;
    }
    for (uint64_t t = 1; t < n; t++) {
        const uint32_t y = want[t];
        if (y != kNoNode && best_pred[y] == ((uint64_t)ulen[t] << 32 | t)) {
            nxt[t] = y;
            prv[y] = (uint32_t)t;
        }
    }
}

// Path cover = the unitigs of the de Bruijn graph on real k-mers: edge z -> y when z is
// alone in its (k-1)-suffix group, has exactly one successor y, and neither is a dummy
// (y then has z as its only predecessor).  Paths start at real nodes without an in-edge;
// a cycle starts at its smallest node.  Paths are laid out by start node, ascending.
// The device builds the same cover in parallel (kernels.hip "path cover"); only speed
// depends on it -- the kernel uses a path step only when it provably equals the SBWT step
// (encode_core.h).
void build_paths(const HostIndex &ix, Derived &dv) {
    const uint64_t n = ix.n;
    const uint32_t k = ix.k;
    dv.has_paths = false;
    if (n >= (1ULL << 31) || k < 1) return;
    const std::vector<uint8_t> dummy = dummy_nodes(ix, dv);
    std::vector<uint32_t> nxt(n), prv(n, kNoNode);
    for (uint64_t z = 0; z < n; z++) {
        nxt[z] = path_succ(ix, dv, dummy, z);
        if (nxt[z] != kNoNode) prv[nxt[z]] = (uint32_t)z;
    }
    if (path_link_on()) link_unitigs(ix, dv, dummy, nxt, prv);
    std::vector<uint8_t> start(n, 0), seen(n, 0);
    for (uint64_t z = 1; z < n; z++)
        if (!dummy[z] && prv[z] == kNoNode) {
            start[z] = 1;
            for (uint32_t y = (uint32_t)z; y != kNoNode; y = nxt[y]) seen[y] = 1;
        }
    for (uint64_t z = 1; z < n; z++)  // what is left lies on cycles: cut each at its minimum
        if (!dummy[z] && !seen[z]) {
            start[z] = 1;
            for (uint32_t y = (uint32_t)z; !seen[y]; y = nxt[y]) seen[y] = 1;
        }
    std::vector<uint64_t> path_start;
    std::vector<uint32_t> order;
    order.reserve(n);
    for (uint64_t z = 1; z < n; z++) {
        if (!start[z]) continue;
        path_start.push_back(order.size());
        order.push_back((uint32_t)z);
        for (uint32_t y = nxt[z]; y != kNoNode && !start[y]; y = nxt[y]) order.push_back(y);
    }
    path_start.push_back(order.size());
    const uint64_t np = path_start.size() - 1;
    // text layout: per path k chars of its first k-mer, one char per further node, then
    // one pad position; colex_at is valid exactly at the k-mer start of each path node
    uint64_t tlen = 0;
    for (uint64_t p = 0; p < np; p++) tlen += (path_start[p + 1] - path_start[p]) + k;
    if (tlen + 64 >= (1ULL << 31)) return;
    dv.colex_at.assign(tlen + 8, kNoNode);
    dv.pos_of_node.assign(n, kNoNode);
    // groups read up to k + 64 characters past a node's position
    dv.pstream.assign((tlen + k) / 32 + 8, uint4{0, 0, 0, 0});
    dv.puniq.assign(tlen / 64 + 4, 0);
    auto put = [&](uint64_t t, uint32_t c) {
        uint4 &g = dv.pstream[t >> 5];
        const uint32_t o = (uint32_t)(t & 31);
        if (o < 16) g.x |= (c & 3u) << (2 * o);
        else g.y |= (c & 3u) << (2 * (o - 16));
    };
    uint64_t b = 0;
    std::vector<uint8_t> first(k);
    for (uint64_t p = 0; p < np; p++) {
        const uint64_t a = path_start[p], e = path_start[p + 1];
        // characters of the first k-mer: walk back k-1 predecessors
        uint32_t z = order[a];
        for (int64_t t = (int64_t)k - 1; t >= 0; t--) {
            first[t] = dv.code[z];
            z = dv.pred[z];
        }
        for (uint32_t t = 0; t < k; t++) put(b + t, first[t]);
        for (uint64_t i = a; i < e; i++) {
            const uint32_t node = order[i];
            const uint64_t pos = b + (i - a);
            if (i > a) put(pos + k - 1, dv.code[node]);
            const uint32_t u = (dv.uniq[node >> 5] >> (node & 31)) & 1u;
            dv.colex_at[pos] = node | (u << 31);
            dv.pos_of_node[node] = (uint32_t)pos;
            const uint64_t end = pos + k - 1;  // the node's k-mer ends at text position end
            dv.pstream[end >> 5].z |= 1u << (end & 31);
            if (u) dv.puniq[pos >> 6] |= 1ULL << (pos & 63);
        }
        b += (e - a) + k;  // last node at b+(e-a)-1; positions up to b+(e-a)+k-1 hold no node
    }
    // Fork blocks (encode_core.h fork_block, k >= kForkBlockMinK): in the k free positions
    // after a path's last node v, per character c the path position of the node v[1..k]c
    // (from the labels of v's (k-1)-suffix group head) and the 32 path characters from its
    // k-mer end.  k_ms4's joint-run build follows a run across the path end with one load
    // (MsLaneT::hop) instead of colex_at + extension + pos_of_node + the path text.
    if (k >= kForkBlockMinK) {
        b = 0;
        for (uint64_t p = 0; p < np; p++) {
            const uint64_t a = path_start[p], e = path_start[p + 1];
            const uint64_t pos = b + (e - a) - 1;
            uint32_t w[4];
            fork_words(ix, dv, dummy, order[e - 1], w);
            uint32_t *blk = dv.colex_at.data() + fork_block(pos + 1);
            for (int c = 0; c < 4; c++) {
                uint64_t chars = 0;
                uint32_t ends = 0;
                if (w[c] != kNoNode) path_text32(dv.pstream.data(), (uint64_t)w[c] + k - 1, chars, ends);
                blk[4 * c] = w[c];
                blk[4 * c + 1] = (uint32_t)chars;
                blk[4 * c + 2] = (uint32_t)(chars >> 32);
                blk[4 * c + 3] = ends;
            }
            b += (e - a) + k;
        }
    }
    dv.tlen = tlen;
    dv.n_paths = np;
    dv.has_paths = true;
}

void build_walk_host(const Derived &dv, uint64_t n, std::vector<WalkEntry> &walk) {
    std::vector<WalkStep> a(n), b(n);
    for (uint64_t j = 0; j < n; j++) {
        a[j].chars = dv.code[j];
        a[j].jump = dv.pred[j];
        a[j].older = 0;
    }
    for (uint32_t m = 1; m < 32; m *= 2) {
        for (uint64_t j = 0; j < n; j++) {
            const WalkStep &x = a[j];
            const WalkStep &y = a[x.jump];
            b[j].chars = y.chars | (x.chars << (2 * m));
            b[j].jump = y.jump;
            b[j].older = 0;
        }
        a.swap(b);
    }
    // a = 32-step entries, b = 16-step: extend a to 48 steps, then compose 48 + 48 + 16
    for (uint64_t j = 0; j < n; j++) {
        const WalkStep &y = b[a[j].jump];
        a[j].older = (uint32_t)y.chars;
        a[j].jump = y.jump;
    }
    walk.resize(n);
    for (uint64_t j = 0; j < n; j++) {
        const WalkStep &x = a[j], &y = a[x.jump];
        walk[j] = walk_compose(x, y, b[y.jump]);
    }
}

void build_rank2_host(const DevIndex &d, std::vector<Rank2Chunk> &out) {
    const uint64_t lines = rank2_blocks(d.n);
    out.resize(lines * 4);
    for (uint64_t i = 0; i < lines * 4; i++) out[i] = rank2_make(d, i % lines, (int)(i / lines));  // c1-major
}

DevIndex host_dev_index(const HostIndex &ix, const Derived &dv, const std::vector<WalkEntry> &walk) {
    DevIndex d{};
    d.rank = dv.rank.data();
    d.lcs = ix.lcs.data();
    d.uniq = dv.uniq.data();
    d.walk = walk.data();
    d.rwords = dv.rwords;
    d.n = (uint32_t)ix.n;
    d.k = ix.k;
    d.t_jump = dv.t_jump;
    for (int c = 0; c < 5; c++) d.C[c] = dv.C[c];
    d.has_paths = dv.has_paths ? 1u : 0u;
    d.path_len = dv.has_paths ? (uint32_t)(dv.colex_at.size() - 8) : 0u;
    d.pstream = dv.pstream.empty() ? nullptr : dv.pstream.data();
    d.colex_at = dv.colex_at.empty() ? nullptr : dv.colex_at.data();
    d.pos_of_node = dv.pos_of_node.empty() ? nullptr : dv.pos_of_node.data();
    d.puniq = dv.puniq.empty() ? nullptr : dv.puniq.data();
    d.forks = dv.has_paths && ix.k >= kForkBlockMinK ? 1u : 0u;
    d.absent = dv.absent;
    d.tab = nullptr;  // see build_tab_host
    d.tab_u = 0;
    return d;
}

}  // namespace ntc
