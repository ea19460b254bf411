// Device-layout structures derived from a HostIndex at upload time (host part).
#pragma once
#include <cstdint>
#include <vector>

#include "encode_core.h"
#include "ntc_internal.h"

namespace ntc {

struct Derived {
    uint32_t rwords = 0;
    std::vector<uint2> rank;      // [4][rwords] rank words (encode_core.h)
    std::vector<uint32_t> uniq;   // ceil(n/32) (+1) words
    std::vector<uint32_t> pred;   // inverse-walk predecessor (select), pred[0] = 0
    std::vector<uint8_t> code;    // last character of each node (root: 0)
    uint32_t C[5] = {0, 0, 0, 0, 0};
    uint32_t t_jump = 1;
    // path cover of the de Bruijn graph (DESIGN.md "Path walk"): every real k-mer node
    // sits at one position of a path text; consecutive positions are graph edges.
    bool has_paths = false;
    uint64_t tlen = 0;               // path text length (characters)
    std::vector<uint4> pstream;      // per 32 text chars: {chars lo, chars hi, end bits, 0}
    std::vector<uint32_t> colex_at;  // per text position: node | uniq << 31, or kNoNode
    std::vector<uint32_t> pos_of_node;  // per node: text position of its k-mer, or kNoNode
    std::vector<uint64_t> puniq;        // bit j: colex_at[j]'s group is a singleton
    uint64_t n_paths = 0;
    uint32_t absent = 0;                // bit c: C[c+1] == C[c] (no node ends with c)
};

constexpr uint32_t kNoNode = 0xFFFFFFFFu;

// Builds the path cover on the host (fills has_paths, tlen, pstream, colex_at,
// pos_of_node, puniq); test emulation -- the upload builds the same cover on the device.
void build_paths(const HostIndex &ix, Derived &dv);
// the path cover links unitigs across branches (derived.cpp link_unitigs) unless
// NTC_PATH_LINK=0; the upload's default for ctx option "path_link"
bool path_link_on();
// FNV-1a over the path-cover arrays (pstream, colex_at, pos_of_node, puniq) at the sizes
// build_paths gives them: lets a test compare the device-built cover with the host one.
inline uint64_t path_cover_hash(const uint4 *pstream, const uint32_t *colex_at, const uint32_t *pos_of_node,
                                const uint64_t *puniq, uint64_t n, uint32_t k, uint64_t tlen) {
    uint64_t h = 1469598103934665603ULL;
    auto mix = [&](const void *p, uint64_t bytes) {
        const uint8_t *b = (const uint8_t *)p;
        for (uint64_t i = 0; i < bytes; i++) h = (h ^ b[i]) * 1099511628211ULL;
    };
    mix(pstream, ((tlen + k) / 32 + 8) * 16);
    mix(colex_at, (tlen + 8) * 4);
    mix(pos_of_node, n * 4);
    mix(puniq, (tlen / 64 + 4) * 8);
    return h;
}
// dummy[z] = 1 when node z's k-mer contains '$' (BFS from the root, depth < k).
std::vector<uint8_t> dummy_nodes(const HostIndex &ix, const Derived &dv);
// Suffix-table depth U for an index of n nodes (encode_core.h "Suffix table").
uint32_t default_tab_u(uint64_t n, uint32_t k, const uint8_t *lcs = nullptr);
// Host build of the suffix table levels 1..U (test emulation; the GPU builds it on device).
// (bits: presence of level U; fbits: presence of the filter level, or empty).
void build_tab_host(const DevIndex &d, uint32_t U, std::vector<uint2> &tab, std::vector<uint32_t> &bits,
                    std::vector<uint32_t> &fbits);
// Level of the SCAN pre-filter bitmap for depth U (0 = none).
uint32_t filter_level(uint32_t U);

// Validates the index and fills rank lines, unique-predecessor bits, pred and code; with
// host_paths also the path cover (test emulation; the upload builds it on the device).
bool build_derived(const HostIndex &ix, Derived &out, std::string &err, bool host_paths);
// Host doubling of the walk table (the GPU builds the same table on device).
void build_walk_host(const Derived &dv, uint64_t n, std::vector<WalkEntry> &walk);
// two-character rank lines of d (Rank2Chunk, encode_core.h): host build for the emulation
void build_rank2_host(const DevIndex &d, std::vector<Rank2Chunk> &out);
// DevIndex over host arrays (test emulation only).
DevIndex host_dev_index(const HostIndex &ix, const Derived &dv, const std::vector<WalkEntry> &walk);

}  // namespace ntc
