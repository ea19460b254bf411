// TEST-ONLY host emulation of the encode/decode kernels: runs the exact lane functions
// of ntcomp_amd/csrc/encode_core.h (the ones k_encode / k_dec_walk call on the GPU) on
// the CPU, one read at a time, with the kernels' [tile][position][lane] scratch layout.
// It lets the -m "not gpu" suite check the kernel ALGORITHM against the oracle on a
// machine without a GPU.  It is not part of libntcomp_gpu.so and no product path loads it.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ntcomp_gpu.h"
#include "../../ntcomp_amd/csrc/derived.h"

using namespace ntc;

#ifdef NTC_TRACE
// Per-read footprint counters (trace build only): requests and distinct 128-byte lines by
// kind, for the MS phase (0) and the parse phase (1).
#include <unordered_set>
namespace {
int g_phase = -1;
std::unordered_set<uint64_t> g_lines[2][kTrKinds];
uint64_t g_req[2][kTrKinds], g_ltot[2][kTrKinds], g_reads;
uint64_t g_over[kTrKinds];  // parse lines the MS phase of the same reads touched too
// per lane step (one k_ms4 wave iteration): lines distinct within the step.  Between two
// iterations of one lane an XCD's L2 (4 MB) sees ~14 K other lanes' lines, so a line a read
// touches again in a later iteration is fetched again: the step count is the fetch estimate.
std::unordered_set<uint64_t> g_step_lines;
uint64_t g_step_ltot[kTrKinds];
void trace_phase(int ph) { g_phase = ph; }
void trace_step() { g_step_lines.clear(); }
uint64_t g_group = 0, g_in_group = 0;  // NTC_TRACE_GROUP=G: distinct lines per G consecutive reads
void trace_read_done() {
    if (g_group == 0) {
        const char *e = getenv("NTC_TRACE_GROUP");
        g_group = e && atoi(e) > 0 ? (uint64_t)atoi(e) : 1;
    }
    g_reads++;
    g_phase = -1;
    if (++g_in_group < g_group) return;
    g_in_group = 0;
    for (int b = 0; b < kTrKinds; b++)
        for (uint64_t x : g_lines[1][b]) g_over[b] += g_lines[0][b].count(x);
    for (int a = 0; a < 2; a++)
        for (int b = 0; b < kTrKinds; b++) {
            g_ltot[a][b] += g_lines[a][b].size();
            g_lines[a][b].clear();
        }
}
}  // namespace
void ntc_touch(int kind, const void *p) {
    if (g_phase < 0) return;
    g_req[g_phase][kind]++;
    g_lines[g_phase][kind].insert((uint64_t)(uintptr_t)p >> 7);
    if (g_phase == 0 && g_step_lines.insert(((uint64_t)(uintptr_t)p >> 7) * kTrKinds + kind).second) g_step_ltot[kind]++;
}
extern "C" void emu_trace_steps(uint64_t *out) {  // [K]: MS lines distinct per step, summed; cleared
    for (int b = 0; b < kTrKinds; b++) out[b] = g_step_ltot[b];
    memset(g_step_ltot, 0, sizeof g_step_ltot);
}
extern "C" void emu_trace_report(uint64_t *out) {  // [reads, req[2][K], lines[2][K]]
    out[0] = g_reads;
    for (int a = 0; a < 2; a++)
        for (int b = 0; b < kTrKinds; b++) {
            out[1 + a * kTrKinds + b] = g_req[a][b];
            out[1 + 2 * kTrKinds + a * kTrKinds + b] = g_ltot[a][b];
        }
    memset(g_req, 0, sizeof g_req);
    memset(g_ltot, 0, sizeof g_ltot);
    g_reads = 0;
}
#if defined(NTC_STATS) && !defined(__HIP_DEVICE_COMPILE__)
uint64_t ntc::ntc_stats[16];
extern "C" void emu_stats(uint64_t *out) {  // [16]: NTC_STAT counters (encode_core.h), then cleared
    for (int i = 0; i < 16; i++) out[i] = ntc_stats[i];
    memset(ntc_stats, 0, sizeof ntc_stats);
}
#endif
extern "C" void emu_trace_overlap(uint64_t *out) {  // [K]: parse lines also touched by the MS phase
    for (int b = 0; b < kTrKinds; b++) out[b] = g_over[b];
    memset(g_over, 0, sizeof g_over);
}
#else
namespace {
inline void trace_phase(int) {}
inline void trace_read_done() {}
inline void trace_step() {}
}  // namespace
#endif

namespace {
bool load(const ntc_index_view *v, HostIndex &hx, Derived &dv, std::vector<WalkEntry> &walk, DevIndex &d,
          std::vector<uint2> &tab, std::vector<uint32_t> &bits, std::vector<uint32_t> &fbits,
          std::vector<uint16_t> &pairb, uint32_t tab_u = 0) {
    hx.n = v->n_nodes;
    hx.k = v->k;
    uint64_t nw = (hx.n + 63) / 64;
    for (int c = 0; c < 4; c++) {
        hx.rows[c].assign(v->rows[c], v->rows[c] + nw);
        hx.C[c] = v->C[c];
    }
    hx.lcs.assign(v->lcs, v->lcs + hx.n);
    hx.lcs.resize(hx.n + 256, 0);
    std::string err;
    if (!build_derived(hx, dv, err, true)) return false;
    build_walk_host(dv, hx.n, walk);
    d = host_dev_index(hx, dv, walk);
    {  // two-character rank chunks, as the upload's ext2 option builds them (NTC_EMU_EXT2=1)
        static std::vector<Rank2Chunk> r2;
        const char *e2 = getenv("NTC_EMU_EXT2");
        d.rank2 = nullptr;
        if (e2 && atoi(e2) != 0) {
            build_rank2_host(d, r2);
            d.rank2 = r2.data();
        }
    }
    {  // joint path runs (MsLaneT<true>) unless NTC_EMU_JOINT=0: the upload turns them on only for
       // fragmented path covers, the emulation checks them on every index
        const char *ej = getenv("NTC_EMU_JOINT");
        d.joint = (ej && atoi(ej) == 0) ? 0u : 1u;
        const char *ef = getenv("NTC_EMU_FORKS");  // fork words (joint build): NTC_EMU_FORKS=0 off
        if (ef && atoi(ef) == 0) d.forks = 0;
    }
    const uint32_t U = tab_u ? std::min<uint32_t>(tab_u, std::min<uint32_t>(hx.k, kTabMaxU)) : default_tab_u(hx.n, hx.k, hx.lcs.data());
    d.tab_u = U;
    d.tab_pos = (dv.has_paths && U >= dv.t_jump && hx.n < (1ULL << 31)) ? 1u : 0u;
    build_tab_host(d, U, tab, bits, fbits);
    d.tab = tab.data();
    d.tab_bits = bits.data();
    d.filt_f = fbits.empty() ? 0u : filter_level(U);
    d.filt_bits = fbits.empty() ? nullptr : fbits.data();
    {  // as the upload's auto filter: off with window words; NTC_EMU_FILTER=0/1 forces it
        const char *ef = getenv("NTC_EMU_FILTER"), *ew = getenv("NTC_EMU_WIN");
        const bool win_on = U >= 4 && !(ew && atoi(ew) == 0);
        if (ef ? atoi(ef) == 0 : win_on) {
            d.filt_f = 0;
            d.filt_bits = nullptr;
        }
    }
    d.tab_u = U;
    {  // window words (SCAN): NTC_EMU_WIN=0 off, else on whenever U >= 4 (the upload's auto)
        static std::vector<uint32_t> winb;
        const char *ew = getenv("NTC_EMU_WIN");
        d.win_w = nullptr;
        if (U >= 4 && !(ew && atoi(ew) == 0)) {
            winb.resize(win_words_count(U) * 8);
            for (uint64_t w = 0; w < winb.size(); w++) winb[w] = win_word(bits.data(), U, w >> 3, (uint32_t)(w & 7));
            d.win_w = winb.data();
        }
    }
    d.pair_w = nullptr;
    const char *pe = getenv("NTC_EMU_PAIR_BYTES");
    if (!pe || atoi(pe) != 0) {
        pairb.resize(pair_words_count(U));
        for (uint64_t M = 0; M < pairb.size(); M++) pairb[M] = (uint16_t)pair_word(tab.data() + tab_base(U), U, M);
        d.pair_w = pairb.data();
    }
    return true;
}
}  // namespace

// out[0] = path-cover hash, out[1] = text length, out[2] = paths (host build_paths)
// the upload's default suffix-table depth (derived.cpp default_tab_u) for n nodes with this LCS
extern "C" uint32_t emu_default_tab_u(uint64_t n, uint32_t k, const uint8_t *lcs) { return default_tab_u(n, k, lcs); }

extern "C" int emu_path_cover(const ntc_index_view *v, uint64_t *out) {
    HostIndex hx;
    Derived dv;
    std::vector<WalkEntry> walk;
    DevIndex d{};
    std::vector<uint2> tab;
    std::vector<uint32_t> bits, fbits;
    std::vector<uint16_t> pairb;
    if (!load(v, hx, dv, walk, d, tab, bits, fbits, pairb, 1)) return 1;
    if (!dv.has_paths) return 2;
    out[0] = path_cover_hash(dv.pstream.data(), dv.colex_at.data(), dv.pos_of_node.data(), dv.puniq.data(), hx.n,
                             hx.k, dv.tlen);
    out[1] = dv.tlen;
    out[2] = dv.n_paths;
    return 0;
}

extern "C" int emu_encode(const ntc_index_view *v, const uint8_t *bases, const uint64_t *offs, uint64_t n_reads,
                          uint64_t *rec_out, uint64_t cap, uint64_t *rec_offsets, int64_t *bad, uint32_t *d_out,
                          uint32_t *s_out, int variant, int use_paths, int tab_u) {
    HostIndex hx;
    Derived dv;
    std::vector<WalkEntry> walk;
    std::vector<uint2> tab;
    std::vector<uint32_t> bits, fbits;
    std::vector<uint16_t> pairb;
    DevIndex d;
    if (!load(v, hx, dv, walk, d, tab, bits, fbits, pairb, (uint32_t)tab_u)) return NTC_ERR_FORMAT;
    if (!use_paths) d.has_paths = 0;
    *bad = -1;
    uint64_t tiles = (n_reads + 63) / 64, total = 0;
    rec_offsets[0] = 0;
    // NTC_EMU_SPILL=1: spill footprint of the v4 layout (entries past kEntSlot, records past
    // kRecSlot) -> stderr, for sizing the spill pools
    const bool spill_stats = getenv("NTC_EMU_SPILL") && atoi(getenv("NTC_EMU_SPILL"));
    // secondary entry slots (capi.cpp ent_slots: 16 with joint runs, else 4; NTC_EMU_SLOTS overrides)
    const char *es_env = getenv("NTC_EMU_SLOTS");
    const uint32_t emu_S = es_env ? (uint32_t)atoi(es_env) : (d.joint ? 16u : 4u);
    uint64_t sp_reads_e = 0, sp_ent = 0, sp_reads_r = 0, sp_rec = 0, sp_len_e = 0, sp_len_r = 0, sp_rem_e = 0;
    uint64_t ne_hist[9] = {0};  // reads with ne > 4 + 4 * i
    for (uint64_t t = 0; t < tiles; t++) {
        uint64_t mx = 0;
        for (uint64_t r = t * 64; r < n_reads && r < t * 64 + 64; r++) mx = std::max(mx, offs[r + 1] - offs[r]);
        uint64_t rows = (mx + 31) & ~31ULL;
        std::vector<uint8_t> D(rows * 64 + 64);
        std::vector<uint32_t> S(rows * 64 + 64), F((rows / 32 + 1) * 64);
        std::vector<uint64_t> R(rows * 64 + 64);
        for (uint64_t r = t * 64; r < n_reads && r < t * 64 + 64; r++) {
            uint32_t lane = (uint32_t)(r & 63);
            uint32_t len = (uint32_t)(offs[r + 1] - offs[r]);
            int rc;
            if (variant == 4) {
                // the kernels' layout (k_ms4 / k_parse4 with one read per call): dense group Ed
                // staged through the ECOMB slots with entry 0 carrying the count, S secondary
                // slots, an overflow pool reserved at the first entry past them; 8 record slots
                // then the record pool (capi.cpp encode4_impl)
                // the read at its position-space offset within a 128-byte line (qo = offs[r] mod
                // 512 characters, k_pack's layout), so that traced Q lines match the kernels'
                std::vector<uint64_t> Qt(len / 32 + 3, 0), Qbuf((len + 512) / 32 + 3 + 16, 0);
                uint64_t *Qa = Qbuf.data() + ((16 - (((uintptr_t)Qbuf.data() >> 3) & 15)) & 15);  // 128 B aligned
                const uint32_t q0 = (uint32_t)(offs[r] & 511);
                std::vector<Entry> Ed(kEntSlot), Es(emu_S), Ep(len + 8);
                std::vector<uint4> stage((kStageSlots + 1) * 256);
                std::vector<uint64_t> R2(kRecSlot), Rp(len + 8);
                unsigned long long pcnt = 0, rcnt = 0, status = ~0ull;
                uint32_t obase = 0, rbase = 0;
                rc = pack_read(bases + offs[r], len, Qt.data(), d.absent);
                for (uint32_t i = 0; rc == 0 && i < len; i++)
                    Qa[(q0 + i) >> 5] |= ((Qt[i >> 5] >> (2 * (i & 31))) & 3ull) << (2 * ((q0 + i) & 31));
                uint32_t ne = 0;
                const MsBufs bufs{Qa, Es.data(), Ed.data(), 1, stage.data(), kEntSlot, emu_S, Ep.data(),
                                  Ep.size(), &pcnt, &obase, &status};
                auto run = [&](auto &ms) {
                    trace_phase(0);
                    ms.start(d, q0, len, 0, Qa);
                    for (;;) {
                        trace_step();
                        int st = ms.step(d, bufs);
                        if (st < 0) { rc = st; break; }
                        if (st == 1) break;
                    }
                    if (rc == 0) ms.finish(bufs);
                    ne = ms.ne;
                };
                if (rc == 0) {
                    if (d.joint) {
                        MsLaneT<true> ms;
                        run(ms);
                    } else {
                        MsLaneT<false> ms;
                        run(ms);
                    }
                }
                if (rc == 0 && status != ~0ull) return NTC_ERR_CAPACITY;  // the pool fits every read by construction
                trace_phase(1);
                // k_parse4: the dense group in one load, the count from entry 0
                Entry pre[kEntSlot];
                for (uint32_t j = 0; j < kEntSlot; j++) pre[j] = Ed[j];
                const uint32_t c0 = entry0_count(pre[0]);
                const uint32_t ne2 = c0 == kNeInE0 ? ne : c0;
                if (rc == 0 && ne2 != ne) return NTC_ERR_FORMAT;
                const Entry *E1 = Es.data() - kEntSlot;
                const Entry *E2 = ne2 > kEntSlot + emu_S ? Ep.data() + obase - kEntSlot - emu_S : nullptr;
                const RecPool rp{Rp.data(), Rp.size(), &rcnt, &rbase, &status, 0};
                if (rc == 0)
                    rc = parse_read(d, Qa, q0, E1, ne2, len, R2.data(), nullptr, 1, Ed.data(), 1, pre, E2, emu_S,
                                    &rp);
                trace_read_done();
                if (spill_stats && rc >= 0) {
                    for (int h = 0; h < 9; h++) ne_hist[h] += ne2 > kEntSlot + 4u * (uint32_t)h;
                    if (ne2 > kEntSlot) {
                        sp_reads_e++;
                        sp_ent += ne2 - kEntSlot;
                        sp_len_e += len;
                        sp_rem_e += len - (emu_S ? Es[0].p : Ep[obase].p);  // positions from the first spilled entry on
                    }
                    if ((uint32_t)rc > kRecSlot) {
                        sp_reads_r++;
                        sp_rec += (uint64_t)rc - kRecSlot;
                        sp_len_r += len;
                    }
                }
                if (d_out && rc >= 0)
                    read_ms(d, Qa, q0, E1, ne2, len, d_out + (offs[r] - offs[0]), s_out + (offs[r] - offs[0]),
                            Ed.data(), 1, E2, emu_S);
                if (rc >= 0) {
                    if (status != ~0ull) return NTC_ERR_CAPACITY;
                    if (total + (uint64_t)rc > cap) return NTC_ERR_CAPACITY;
                    for (int jj = 0; jj < rc; jj++)
                        rec_out[total + jj] = jj < (int)kRecSlot ? R2[jj] : Rp[rbase + jj - kRecSlot];
                    total += (uint64_t)rc;
                    rec_offsets[r + 1] = total;
                    continue;
                }
            } else {
                LaneScratch s{D.data() + lane, S.data() + lane, F.data() + lane, R.data() + lane};
                rc = encode_lane(d, bases + offs[r], len, (uint32_t)rows, s);
                if (d_out)
                    for (uint32_t p = 0; p < len; p++) {
                        d_out[offs[r] - offs[0] + p] = D[(uint64_t)p * 64 + lane];
                        s_out[offs[r] - offs[0] + p] = S[(uint64_t)p * 64 + lane];
                    }
            }
            if (rc < 0) {
                *bad = (int64_t)r;
                return -rc;
            }
            if (total + (uint64_t)rc > cap) return NTC_ERR_CAPACITY;
            for (int j = 0; j < rc; j++)
                rec_out[total + j] = R[(uint64_t)j * 64 + lane];
            total += (uint64_t)rc;
            rec_offsets[r + 1] = total;
        }
    }
    if (spill_stats) {
        fprintf(stderr, "ne > 4 + 4i, i = 0..8:");
        for (int h = 0; h < 9; h++) fprintf(stderr, " %llu", (unsigned long long)ne_hist[h]);
        fprintf(stderr, "\n");
    }
    if (spill_stats)
        fprintf(stderr,
                "{\"reads\": %llu, \"bases\": %llu, \"records\": %llu, \"spill_e_reads\": %llu, \"spill_entries\": %llu, "
                "\"spill_e_len\": %llu, \"spill_e_rem\": %llu, \"spill_r_reads\": %llu, \"spill_records\": %llu, "
                "\"spill_r_len\": %llu}\n",
                (unsigned long long)n_reads, (unsigned long long)(offs[n_reads] - offs[0]), (unsigned long long)total,
                (unsigned long long)sp_reads_e, (unsigned long long)sp_ent, (unsigned long long)sp_len_e,
                (unsigned long long)sp_rem_e, (unsigned long long)sp_reads_r, (unsigned long long)sp_rec,
                (unsigned long long)sp_len_r);
    return NTC_OK;
}

extern "C" int emu_decode(const ntc_index_view *v, const uint64_t *recs, uint64_t n, uint8_t *out, uint64_t cap,
                          uint64_t *offs, uint64_t offcap, uint64_t *nreads) {
    HostIndex hx;
    Derived dv;
    std::vector<WalkEntry> walk;
    std::vector<uint2> tab;
    std::vector<uint32_t> bits, fbits;
    std::vector<uint16_t> pairb;
    DevIndex d;
    if (!load(v, hx, dv, walk, d, tab, bits, fbits, pairb, 1)) return NTC_ERR_FORMAT;
    // the kernel's decode (k_dec_rec): blocks of 256 records (NTC_EMU_STAGE_BLOCK), each
    // record's 2-bit codes staged per block (StageWriter), then ASCII per staged word; a read's
    // records are consumed last to first (lib.rs:266)
    std::vector<uint64_t> starts, lens(n), E(n + 1, 0);
    for (uint64_t r = 0; r < n; r++) {
        const uint32_t flag = (uint32_t)(recs[r] >> 56);
        if (flag & 1) starts.push_back(r);
        lens[r] = (flag & 2) ? (flag >> 2) : ((uint32_t)(recs[r] >> 32) & 0xFFFFFF);
        E[r + 1] = E[r] + lens[r];
    }
    const uint64_t total = E[n];
    if (total > cap || starts.size() + 1 > offcap) return NTC_ERR_CAPACITY;
    if (n && (starts.empty() || starts[0] != 0)) return NTC_ERR_FORMAT;
    starts.push_back(n);
    std::vector<uint64_t> g0s(n);
    offs[0] = 0;
    for (size_t i = 0; i + 1 < starts.size(); i++) {
        const uint64_t rb = starts[i], re = starts[i + 1];
        for (uint64_t r = rb; r < re; r++) g0s[r] = E[rb] + (E[re] - E[r + 1]);
        offs[i + 1] = E[re];
    }
    const char *sbe = getenv("NTC_EMU_STAGE_BLOCK");
    const uint64_t stage_block = sbe && atoi(sbe) > 0 ? (uint64_t)atoi(sbe) : 256;
    std::vector<uint64_t> sb(kDecStageWords);
    std::vector<uint32_t> sm(kDecStageWords);
    for (uint64_t b0 = 0; b0 < n; b0 += stage_block) {
        const uint64_t b1 = std::min<uint64_t>(n, b0 + stage_block);
        uint64_t lo = ~0ULL, hi = 0;
        for (uint64_t r = b0; r < b1; r++)
            if (lens[r]) {
                lo = std::min(lo, g0s[r]);
                hi = std::max(hi, g0s[r] + lens[r]);
            }
        if (lo >= hi) continue;
        const uint64_t w_lo = lo >> 5, nw = ((hi - 1) >> 5) - w_lo + 1;
        if (nw > kDecStageWords) {  // direct ASCII
            for (uint64_t r = b0; r < b1; r++) {
                if (!lens[r]) continue;
                const uint64_t w = recs[r];
                if ((w >> 56) & 2) store_codes(out + g0s[r], w, (uint32_t)lens[r]);
                else if (!walk_record(d, (uint32_t)w, (uint32_t)lens[r], out + g0s[r])) return NTC_ERR_FORMAT;
            }
            continue;
        }
        std::fill(sb.begin(), sb.begin() + nw, 0);
        std::fill(sm.begin(), sm.begin() + nw, 0);
        StageWriter sw{sb.data(), sm.data(), w_lo};
        for (uint64_t r = b0; r < b1; r++) {
            if (!lens[r]) continue;
            const uint64_t w = recs[r];
            if ((w >> 56) & 2) sw.put(g0s[r], w, (uint32_t)lens[r]);
            else if (!walk_record_codes(d, (uint32_t)w, (uint32_t)lens[r], g0s[r], sw)) return NTC_ERR_FORMAT;
        }
        for (uint64_t t = 0; t < nw; t++) stage_store_word(out, w_lo + t, sb[t], sm[t]);
    }
    *nreads = starts.size() - 1;
    return NTC_OK;
}

// Wave divergence of k_ms4 (diagnostic): one wave of 64 lanes runs MsLaneT::step (the build
// the upload would pick: joint unless NTC_EMU_JOINT=0) in lock step over the reads, idle
// lanes taking the next read as the kernel's pool hands them out.  out: [0] wave
// iterations, [1] sum over iterations of the distinct entry modes among busy lanes (a "run"
// pending counts as its own mode), [2] lane steps, [3..12] steps per entry mode (Scan, Ext,
// P1, Bs, Brk, First, Enter, BrkLong, ExtFail, run), [13..22] iterations by number of
// distinct modes (1..10).
constexpr int kWaveModes = 10;
template <bool kJoint>
void wave_modes(const DevIndex &d, const uint8_t *bases, const uint64_t *offs, uint64_t n_reads, uint64_t *out) {
    struct Lane {
        MsLaneT<kJoint> ms;
        std::vector<uint64_t> Q;
        std::vector<Entry> Ed, Es, Ep;
        unsigned long long pcnt = 0, status = ~0ull;
        uint32_t obase = 0;
        bool busy = false;
    };
    std::vector<uint4> stage((kStageSlots + 1) * 256);  // lane i stages in slot i (ntc_host_lane)
    std::vector<Lane> L(64);
    uint64_t next = 0;
    for (;;) {
        for (auto &l : L) {
            if (l.busy || next >= n_reads) continue;
            const uint64_t r = next++;
            const uint32_t len = (uint32_t)(offs[r + 1] - offs[r]);
            l.Q.assign(len / 32 + 3, 0);
            l.Ed.assign(kEntSlot, Entry{0, 0, 0, 0});
            l.Es.assign(4, Entry{0, 0, 0, 0});
            l.Ep.assign(len + 8, Entry{0, 0, 0, 0});
            l.pcnt = 0;
            if (len == 0 || pack_read(bases + offs[r], len, l.Q.data(), d.absent) != 0) continue;
            l.ms.start(d, 0, len, 0, l.Q.data());
            l.busy = true;
        }
        uint32_t modes = 0;
        bool any = false;
        for (uint32_t li = 0; li < L.size(); li++) {
            Lane &l = L[li];
            if (!l.busy) continue;
            ntc_host_lane = li;
            any = true;
            const uint32_t m = l.ms.try_run ? (uint32_t)kWaveModes - 1 : l.ms.mode;
            modes |= 1u << m;
            out[3 + m]++;
            out[2]++;
            const MsBufs bufs{l.Q.data(), l.Es.data(), l.Ed.data(), 1, stage.data(), kEntSlot, 4, l.Ep.data(),
                              l.Ep.size(), &l.pcnt, &l.obase, &l.status};
            const int st = l.ms.step(d, bufs);
            if (st != 0) l.busy = false;
        }
        if (!any) break;
        out[0]++;
        const uint32_t dm = (uint32_t)__builtin_popcount(modes);
        out[1] += dm;
        out[3 + kWaveModes + dm - 1]++;
    }
}

extern "C" int emu_wave_modes(const ntc_index_view *v, const uint8_t *bases, const uint64_t *offs, uint64_t n_reads,
                              uint64_t *out) {
    HostIndex hx;
    Derived dv;
    std::vector<WalkEntry> walk;
    std::vector<uint2> tab;
    std::vector<uint32_t> bits, fbits;
    std::vector<uint16_t> pairb;
    DevIndex d;
    if (!load(v, hx, dv, walk, d, tab, bits, fbits, pairb, 0)) return NTC_ERR_FORMAT;
    memset(out, 0, (3 + 2 * kWaveModes) * sizeof(uint64_t));
    if (d.joint) wave_modes<true>(d, bases, offs, n_reads, out);
    else wave_modes<false>(d, bases, offs, n_reads, out);
    return 0;
}
