// extern "C" boundary of libntcomp_gpu.so (include/ntcomp_gpu.h, include/ntcomp_host.h).
// Every entry point returns an ntc_status; HIP failures and reference panics become
// status codes plus ntc_last_error(); nothing aborts across the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <string>
#include <vector>

#include "../../include/ntcomp_gpu.h"
#include "../../include/ntcomp_codec.h"
#include "../../include/ntcomp_host.h"
#include "codec_params.h"
#include "derived.h"
#include "kernels.h"
#include "ntc_internal.h"

using namespace ntc;

namespace {

struct DevBuf {
    void *p = nullptr;
    uint64_t bytes = 0;
};

enum CallKind { kNone = 0, kEncode = 1, kDecode = 2 };

}  // namespace

// device workspace slots of a context (grown by ensure, freed with the context)
enum WsSlot {
    WS_D = 0, WS_S, WS_F, WS_R, WS_RECCOUNT, WS_SCANTMP, WS_TILEBASE, WS_TILEROWS,
    WS_STAGE_BASES, WS_STAGE_OFFS, WS_STAGE_RECS, WS_E, WS_DEC_A, WS_DEC_B, WS_DEC_C,
    WS_DEC_D, WS_Q, WS_E3, WS_NE, WS_COUNTER, WS_R2, WS_ED, WS_WAVECNT, WS_PACK_CHUNKS, WS_PACK_META,
    WS_PACK_PAYLOAD, WS_FA_BASES, WS_FA_OFFS, WS_FA_SCAN, WS_ES, WS_OBASE,
    WS_FQ_RAW, WS_FQ_TILES, WS_FQ_NL, WS_FQ_KEPT, WS_PACK_SEGS,
    WS_UNP_PAY, WS_UNP_MARKS, WS_UNP_ST, WS_UNP_VALS, WS_UNP_RECS, WS_UNP_OUT, WS_COUNT
};

// The device index of one upload: freed with the last context that holds it
// (ntc_index_share lets several contexts on one GPU use one copy).
struct IndexMem {
    int device = 0;
    std::vector<void *> ptrs;
    explicit IndexMem(int d) : device(d) {}
    ~IndexMem() {
        (void)hipSetDevice(device);
        for (void *p : ptrs) (void)hipFree(p);
    }
};

struct ntc_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = true;
    std::string err;
    // index
    bool has_index = false;
    DevIndex dix{};
    std::shared_ptr<IndexMem> index_mem;
    uint64_t index_bytes = 0;
    // workspace buffers (grown, never shrunk)
    DevBuf ws[WS_COUNT];
    unsigned long long *d_status = nullptr;
    // status mailbox in pinned host memory: {status, count a, count b}, written by k_status_box
    // at the end of a device call, so *_status() is one stream sync instead of D2H copies
    uint64_t *h_box = nullptr;
    bool box_valid = false;
    // the records of the last ntc_unpack_streams (in WS_UNP_RECS) and their read / base counts
    uint64_t *unp_d_recs = nullptr;
    uint64_t unp_recs = 0, unp_reads = 0, unp_bases = 0;
    // last call
    CallKind last = kNone;
    uint64_t last_n = 0;           // reads (encode) / records (decode)
    uint64_t *last_out_offs = nullptr;
    uint64_t last_units = 0;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    int encode_variant = 4;
    int last_variant = 0;
    int num_cus = 0;
    Enc4Args last4{};
    // the last v4 encode's arguments: a call that ran out of an overflow pool is re-run
    // with grown pools when its status is read (read_status)
    struct {
        const uint8_t *bases;
        const uint64_t *offs;
        uint64_t n_reads, total_bases, cap;
        uint64_t *rec_out, *rec_offs;
    } call4{};
    uint32_t ent_slots_opt = 0;     // secondary entry slots per read (0: auto, 16 with joint runs, else 4)
    double epool_per_read = 4.0;    // overflow pools: a floor per read (the test hook pool_per_read sets it)
    double rpool_per_read = 1.0;
    double epool_per_base = 0.0;    // and what the last call's reads reserved per base (learn_pool_rates)
    double rpool_per_base = 0.0;
    uint64_t spill_reruns = 0;      // calls re-run with grown pools
    uint32_t tab_u_opt = 0;  // suffix-table depth for the next upload (0 = default_tab_u)
    int tab_u_fallback = 0;  // last upload: the default depth did not fit, U = 14 was used
    int pair_bytes_opt = 1;  // build the SCAN pair bytes at the next upload (0: bitmap tests, A/B)
    int filter_opt = -1;     // SCAN pre-filter at the next upload: -1 auto (off when saturated), 0 off, 1 on
    int64_t filter_density_ppm = -1;  // presence density of the filter level at the last upload
    int joint_opt = -1;      // joint path runs at the next upload: -1 auto (fragmented path cover), 0 off, 1 on
    int path_link_opt = path_link_on() ? 1 : 0;  // path cover: unitigs linked across branches (default) or not
    int win_opt = -1;        // SCAN window words at the next upload: -1 auto (U >= 4), 0 off, 1 on
    int decode_only_opt = 0;  // the next upload builds only what decode needs (walk table): no path
                              // cover, suffix table or SCAN words; encode calls then fail
    bool index_decode_only = false;  // the index in use was uploaded that way
    int ext2_opt = 0;        // build the two-character rank chunks at the next upload (A/B option: 1 measured
                             // slower -- 8 B/node from HBM against 1 B/node of Infinity-Cache-resident rank words)
    uint64_t n_paths = 0, path_text_len = 0;
    int64_t upload_host_us = 0, upload_total_us = 0;  // last ntc_index_upload: host derive / total
    uint64_t max_pass_bases = 1ULL << 30;  // host-buffer calls split into device passes of at most this
    double last_pack_ms = 0;               // last ntc_pack_blocks_device: both packer kernels
    hipEvent_t pack_ev[3] = {nullptr, nullptr, nullptr};
};

namespace {

// work queue heads (kernels.hip WaveQueue: 8, 64 B apart), then the two pool counters
// (kPoolCntE, kPoolCntR: words 64 and 72)
constexpr uint64_t kCounterBytes = 8 * 64 + 2 * 64;


#define HIP_TRY(ctx, expr)                                                                   \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) {                                                              \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                   \
            return NTC_ERR_HIP;                                                              \
        }                                                                                    \
    } while (0)

int set_err(ntc_ctx *ctx, int code, const std::string &msg) {
    if (ctx) ctx->err = msg;
    return code;
}

int ensure(ntc_ctx *ctx, int slot, uint64_t bytes, void **out) {
    DevBuf &b = ctx->ws[slot];
    if (bytes == 0) bytes = 64;
    if (b.bytes < bytes) {
        if (b.p) {
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            HIP_TRY(ctx, hipFree(b.p));
            b.p = nullptr;
            b.bytes = 0;
        }
        uint64_t want = bytes + bytes / 8;  // headroom for slightly larger next calls
        if (hipMalloc(&b.p, want) != hipSuccess) {
            (void)hipGetLastError();
            b.p = nullptr;
            want = bytes;  // no headroom when memory is short
            if (hipMalloc(&b.p, want) != hipSuccess) {
                (void)hipGetLastError();
                b.p = nullptr;
                size_t fr = 0, tot = 0;
                (void)hipMemGetInfo(&fr, &tot);
                return set_err(ctx, NTC_ERR_CAPACITY,
                               "device workspace of " + std::to_string(bytes) + " bytes does not fit (" +
                                   std::to_string(fr) + " bytes free): split the batch");
            }
        }
        b.bytes = want;
    }
    *out = b.p;
    return NTC_OK;
}

const char *status_name(int code) {
    switch (code) {
    case NTC_ERR_INVALID_BASE: return "invalid base (non-ACGT or absent from the index)";
    case NTC_ERR_EMPTY_READ: return "empty read (EncodeError)";
    case NTC_ERR_LENGTH: return "match length >= 2^24";
    case NTC_ERR_CAPACITY: return "output capacity exceeded";
    case NTC_ERR_FORMAT: return "malformed input";
    case NTC_ERR_REFERENCE_PANIC: return "short record longer than k (the reference panics, encode.rs:151-152)";
    default: return "error";
    }
}

// Scratch layout for n_reads reads: either per-tile bases (tile_base, device pointer)
// or uniform rows per tile.
struct Layout {
    const uint64_t *d_tile_base = nullptr;
    uint64_t rows_uniform = 0;
    uint64_t total_rows = 0;
};

int alloc_scratch(ntc_ctx *ctx, uint64_t n_reads, uint64_t total_rows, EncodeArgs &a) {
    void *p;
    int rc;
    const uint64_t slots = total_rows * 64;
    if ((rc = ensure(ctx, WS_D, slots, &p))) return rc;
    a.D = (uint8_t *)p;
    if ((rc = ensure(ctx, WS_S, slots * 4, &p))) return rc;
    a.S = (uint32_t *)p;
    if ((rc = ensure(ctx, WS_F, (total_rows / 32 + 1) * 64 * 4, &p))) return rc;
    a.F = (uint32_t *)p;
    if ((rc = ensure(ctx, WS_R, slots * 8, &p))) return rc;
    a.R = (uint64_t *)p;
    if ((rc = ensure(ctx, WS_RECCOUNT, (n_reads + 1) * 4, &p))) return rc;
    a.rec_count = (uint32_t *)p;
    return NTC_OK;
}

// overflow pool indices are 32-bit (MsLaneT::ob, rbase)
constexpr uint64_t kPoolMax = 0xFFFFFFF0ull;

uint32_t ent_slots(const ntc_ctx *ctx) {
    if (ctx->ent_slots_opt) return ctx->ent_slots_opt;
    // entries per read past the dense 4 (tests/emu NTC_EMU_SPILL, 1 % errors): random genome
    // k = 91 reads rarely spill (6 %, 0.07 % past 8); a strain collection with joint runs and
    // fork hops spills on 98 % of reads.  With the linked path cover (round 6) S91's reads
    // have fewer run entries: 16 secondary slots measured 131.2-131.7 Gbases/s against
    // 129.9-130.9 with 20 (3 runs each, one box); the overflow pool takes the rest
    return ctx->has_index && ctx->dix.joint ? 16u : 4u;
}

// v4: pack -> persistent MS -> parse -> scan -> emit, all in position space.
// total_bases = offs[n] - offs[0] (known to the caller).
int encode4_impl(ntc_ctx *ctx, const uint8_t *d_bases, const uint64_t *d_offs, uint64_t n_reads,
                 uint64_t total_bases, uint64_t *d_rec_out, uint64_t cap, uint64_t *d_rec_offs) {
    if (ctx->index_decode_only)
        return set_err(ctx, NTC_ERR_NO_INDEX, "the index was uploaded for decode only (ctx option decode_only)");
    // k_ms4's query-word cache names 16-byte pairs of the 2-bit stream by a 32-bit index
    // (encode_core.h NTC_QCACHE): a call stays below 2^38 bases (256 Gi, more than HBM holds)
    if (total_bases >= (1ull << 38)) return set_err(ctx, NTC_ERR_CAPACITY, "2^38 bases or more in one call: split the batch");
    Enc4Args a{};
    a.ix = ctx->dix;
    a.bases = d_bases;
    a.offs = d_offs;
    a.n_reads = n_reads;
    a.status = ctx->d_status;
    void *p;
    int rc;
    ctx->call4 = {d_bases, d_offs, n_reads, total_bases, cap, d_rec_out, d_rec_offs};
    // Workspace by need: per read, 4 dense + S secondary entry slots, 8 dense record slots;
    // the rest of a read's entries / records go to overflow pools sized from what earlier
    // calls reserved (a call that runs out is re-run with the pools grown, read_status).
    const uint32_t S = ent_slots(ctx);
    // A read never holds more entries or records than it has positions, so this call's bases
    // bound both pools whatever rate an earlier call (e.g. one of long reads) left behind.
    const uint64_t pos_cap = total_bases + 4 * n_reads + 4096;  // + reservations rounded to 4-entry groups
    auto pool_size = [&](double per_read, double per_base) {
        const double want = std::max(per_read * (double)n_reads, per_base * (double)total_bases);
        return std::min<uint64_t>(std::min<uint64_t>((uint64_t)want + 4096, pos_cap), kPoolMax);
    };
    const uint64_t pcap = pool_size(ctx->epool_per_read, ctx->epool_per_base);
    const uint64_t rcap = pool_size(ctx->rpool_per_read, ctx->rpool_per_base);
    if ((rc = ensure(ctx, WS_Q, (total_bases / 32 + 4) * 8, &p))) return rc;
    a.Q = (uint64_t *)p;
    if ((rc = ensure(ctx, WS_ES, (n_reads + 1) * S * sizeof(Entry), &p))) return rc;
    a.Es = (Entry *)p;
    a.S = S;
    if ((rc = ensure(ctx, WS_E3, pcap * sizeof(Entry), &p))) return rc;
    a.Ep = (Entry *)p;
    a.pcap = pcap;
    if ((rc = ensure(ctx, WS_OBASE, (n_reads + 1) * 8, &p))) return rc;
    a.obase = (uint32_t *)p;
    a.rbase = a.obase + (n_reads + 1);
    if ((rc = ensure(ctx, WS_ED, (n_reads + 1) * kEntSlot * sizeof(Entry), &p))) return rc;
    a.Ed = (Entry *)p;
    if ((rc = ensure(ctx, WS_NE, (n_reads + 1) * 4, &p))) return rc;
    a.ne = (uint32_t *)p;
    if ((rc = ensure(ctx, WS_R, rcap * 8, &p))) return rc;
    a.R = (uint64_t *)p;
    a.rcap = rcap;
    if ((rc = ensure(ctx, WS_R2, (n_reads + 1) * kRecSlot * 8, &p))) return rc;
    a.R2 = (uint64_t *)p;
    if ((rc = ensure(ctx, WS_RECCOUNT, (n_reads + 1) * 4, &p))) return rc;
    a.rec_count = (uint32_t *)p;
    const uint64_t waves = (n_reads + 63) / 64;
    if ((rc = ensure(ctx, WS_WAVECNT, (waves + 1) * 4 + (waves + 2) * 8 + 8, &p))) return rc;
    a.wave_cnt = (uint32_t *)p;
    uint64_t *wave_off = (uint64_t *)(((uintptr_t)(a.wave_cnt + waves + 1) + 7) & ~(uintptr_t)7);
    if ((rc = ensure(ctx, WS_COUNTER, kCounterBytes, &p))) return rc;
    a.counter = (unsigned long long *)p;
    void *tmp;
    if ((rc = ensure(ctx, WS_SCANTMP, scan_tmp_words(n_reads + 1) * 8, &tmp))) return rc;
    HIP_TRY(ctx, hipMemsetAsync(ctx->d_status, 0xFF, 8, ctx->stream));
    HIP_TRY(ctx, hipMemsetAsync(a.counter, 0, kCounterBytes, ctx->stream));
    ctx->box_valid = false;
    ctx->last = kEncode;
    ctx->last_variant = 4;
    ctx->last_n = n_reads;
    ctx->last_out_offs = d_rec_offs;
    ctx->last_units = total_bases;
    ctx->last4 = a;
    HIP_TRY(ctx, hipEventRecord(ctx->ev[0], ctx->stream));
    if (n_reads == 0) {
        HIP_TRY(ctx, hipMemsetAsync(d_rec_offs, 0, 8, ctx->stream));
        for (int i = 1; i < 4; i++) HIP_TRY(ctx, hipEventRecord(ctx->ev[i], ctx->stream));
        return NTC_OK;
    }
    static int bpc = 0;
    if (!bpc) bpc = ms4_blocks_per_cu();
    launch_encode4(a, total_bases, (uint32_t)(ctx->num_cus * bpc), ctx->stream, ctx->ev[3], ctx->ev[1]);
    HIP_TRY(ctx, hipGetLastError());
    launch_emit4(a, wave_off, (uint64_t *)tmp, d_rec_offs, d_rec_out, cap, ctx->stream);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipEventRecord(ctx->ev[2], ctx->stream));
    launch_status_box(ctx->d_status, d_rec_offs + n_reads, (const uint64_t *)(a.counter + kPoolCntE),
                      (const uint64_t *)(a.counter + kPoolCntR), ctx->h_box, ctx->stream);
    HIP_TRY(ctx, hipGetLastError());
    ctx->box_valid = true;
    return NTC_OK;
}

// Pool rates for the next call: what this call's reads reserved (plus a quarter) per input
// base.  Taken from the latest call alone and per base, not per read, so a batch of long
// reads does not inflate the pools of later batches of short ones.
void learn_pool_rates(ntc_ctx *ctx, uint64_t cnt_e, uint64_t cnt_r) {
    const double b = (double)(ctx->call4.total_bases ? ctx->call4.total_bases : 1);
    ctx->epool_per_base = 1.25 * (double)cnt_e / b;
    ctx->rpool_per_base = 1.25 * (double)cnt_r / b;
}

int encode_impl(ntc_ctx *ctx, const uint8_t *d_bases, const uint64_t *d_offs, uint64_t n_reads,
                const Layout &lay, uint64_t *d_rec_out, uint64_t cap, uint64_t *d_rec_offs,
                uint64_t units) {
    if (!ctx->has_index) return set_err(ctx, NTC_ERR_NO_INDEX, "no index uploaded");
    if (ctx->index_decode_only)
        return set_err(ctx, NTC_ERR_NO_INDEX, "the index was uploaded for decode only (ctx option decode_only)");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    ctx->last_variant = ctx->encode_variant;
    EncodeArgs a{};
    a.ix = ctx->dix;
    a.bases = d_bases;
    a.offs = d_offs;
    a.n_reads = n_reads;
    a.tile_base = lay.d_tile_base;
    a.rows_uniform = lay.rows_uniform;
    a.status = ctx->d_status;
    int rc = alloc_scratch(ctx, n_reads, lay.total_rows, a);
    if (rc) return rc;
    void *tmp;
    if ((rc = ensure(ctx, WS_SCANTMP, scan_tmp_words(n_reads + 1) * 8, &tmp))) return rc;
    HIP_TRY(ctx, hipMemsetAsync(ctx->d_status, 0xFF, 8, ctx->stream));
    ctx->box_valid = false;
    ctx->last = kEncode;
    ctx->last_n = n_reads;
    ctx->last_out_offs = d_rec_offs;
    ctx->last_units = units;
    if (n_reads == 0) {
        HIP_TRY(ctx, hipMemsetAsync(d_rec_offs, 0, 8, ctx->stream));
        for (int i = 0; i < 3; i++) HIP_TRY(ctx, hipEventRecord(ctx->ev[i], ctx->stream));
        return NTC_OK;
    }
    HIP_TRY(ctx, hipEventRecord(ctx->ev[0], ctx->stream));
    launch_encode(a, ctx->stream);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipEventRecord(ctx->ev[1], ctx->stream));
    scan_excl_u32(a.rec_count, n_reads, d_rec_offs, (uint64_t *)tmp, ctx->stream);
    EmitArgs e{};
    e.R = a.R;
    e.tile_base = lay.d_tile_base;
    e.rows_uniform = lay.rows_uniform;
    e.rec_count = a.rec_count;
    e.rec_offsets = d_rec_offs;
    e.n_reads = n_reads;
    e.out = d_rec_out;
    e.capacity = cap;
    e.status = ctx->d_status;
    launch_emit(e, ctx->stream);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipEventRecord(ctx->ev[2], ctx->stream));
    return NTC_OK;
}

// A v4 encode that ran out of an overflow pool (status kStatusRegrow): the pool counters
// hold what every read reserved, so the pools grow to that (plus a quarter, remembered per
// read for later calls) and the call runs again on the same inputs.
int regrow_and_rerun(ntc_ctx *ctx) {
    uint64_t cnt[2] = {0, 0};
    HIP_TRY(ctx, hipMemcpy(&cnt[0], ctx->last4.counter + kPoolCntE, 8, hipMemcpyDeviceToHost));
    HIP_TRY(ctx, hipMemcpy(&cnt[1], ctx->last4.counter + kPoolCntR, 8, hipMemcpyDeviceToHost));
    learn_pool_rates(ctx, cnt[0], cnt[1]);
    if ((cnt[0] > kPoolMax || cnt[1] > kPoolMax))
        return set_err(ctx, NTC_ERR_CAPACITY, "entry / record overflow past 2^32 slots: split the batch");
    ctx->spill_reruns++;
    const auto &c = ctx->call4;
    return encode4_impl(ctx, c.bases, c.offs, c.n_reads, c.total_bases, c.rec_out, c.cap, c.rec_offs);
}

int read_status(ntc_ctx *ctx, int64_t *bad_index) {
    for (int attempt = 0;; attempt++) {
        unsigned long long st = 0;
        if (ctx->box_valid) {  // the call's mailbox (k_status_box): one stream sync
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            st = ((volatile uint64_t *)ctx->h_box)[0];
        } else {
            HIP_TRY(ctx, hipMemcpyAsync(&st, ctx->d_status, 8, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        }
        if (st == ~0ULL) {
            if (bad_index) *bad_index = -1;
            if (ctx->box_valid && ctx->last == kEncode && ctx->last_variant == 4)
                learn_pool_rates(ctx, ((volatile uint64_t *)ctx->h_box)[2], ((volatile uint64_t *)ctx->h_box)[3]);
            return NTC_OK;
        }
        if (st == kStatusRegrow) {
            // up to 4 re-runs: the first call on a context learns the entry pool (the parse
            // is skipped while entries overflow), then the record pool; a 10 M-read call on a
            // 177 M-node collection (L31, profiles/round5/big_point_*) ran out after two
            if (ctx->last == kEncode && ctx->last_variant == 4 && attempt < 4) {
                const int rc = regrow_and_rerun(ctx);
                if (rc) return rc;
                continue;
            }
            if (bad_index) *bad_index = -1;
            return set_err(ctx, NTC_ERR_CAPACITY, "entry / record overflow pool exhausted after re-runs");
        }
        int code = (int)(st & 0xFF);
        int64_t idx = (int64_t)(st >> 8);
        if (bad_index) *bad_index = idx;
        char buf[160];
        std::snprintf(buf, sizeof(buf), "%s at index %lld", status_name(code), (long long)idx);
        ctx->err = buf;
        return code;
    }
}


// GPU packer (pack.hip) over the records of n_reads reads in HBM: block b = reads
// [b * block_reads, ...).  Pass 1 on the device, Rice parameters and payload layout on the
// host (glibc f64 math, codec_params.h), pass 2 on the device.  Synchronous.
int pack_blocks_impl(ntc_ctx *ctx, const uint64_t *d_recs, const uint64_t *d_roffs, uint64_t n_reads,
                     uint32_t block_reads, uint8_t *d_payload, uint64_t payload_capacity, ntc_block_meta *meta,
                     uint64_t *payload_bytes, const uint64_t *known_ends = nullptr) {
    *payload_bytes = 0;
    const uint64_t n_blocks = (n_reads + block_reads - 1) / block_reads;
    if (n_blocks == 0) return NTC_OK;
    for (int i = 0; i < 3; i++)
        if (!ctx->pack_ev[i]) HIP_TRY(ctx, hipEventCreate(&ctx->pack_ev[i]));
    uint64_t ends[2] = {0, 0};  // the record offsets' first and last values
    if (known_ends) {
        ends[0] = known_ends[0];
        ends[1] = known_ends[1];
    } else {
        HIP_TRY(ctx, hipMemcpyAsync(&ends[0], d_roffs, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(&ends[1], d_roffs + n_reads, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    if (ends[1] < ends[0]) return set_err(ctx, NTC_ERR_INVALID_ARG, "record offsets decrease");
    void *d_chunks, *d_meta;
    int rc;
    // chunks of block b at rec_begin + rec_begin / 31 + 2 b (pack.hip chunk_base: room for
    // 32 bases in every short record)
    const uint64_t chunk_words = ends[1] + ends[1] / 31 + 2 * n_blocks + 2;
    if ((rc = ensure(ctx, WS_PACK_CHUNKS, chunk_words * 8, &d_chunks))) return rc;
    const uint64_t meta_bytes = n_blocks * (sizeof(PackStats) + sizeof(PackParams) + 32) +
                                pack_stats_scratch_words(n_blocks, block_reads) * 8;
    if ((rc = ensure(ctx, WS_PACK_META, meta_bytes, &d_meta))) return rc;
    PackStats *d_stats = (PackStats *)d_meta;
    PackParams *d_params = (PackParams *)(d_stats + n_blocks);
    uint64_t *d_bits = (uint64_t *)(d_params + n_blocks);
    HIP_TRY(ctx, hipEventRecord(ctx->pack_ev[0], ctx->stream));
    launch_pack_stats(d_recs, d_roffs, n_reads, block_reads, n_blocks, (uint64_t *)d_chunks, chunk_words,
                      d_bits + 4 * n_blocks, d_stats, ctx->stream);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipEventRecord(ctx->pack_ev[1], ctx->stream));
    std::vector<PackStats> st(n_blocks);
    std::vector<PackParams> pp(n_blocks);
    HIP_TRY(ctx, hipMemcpyAsync(st.data(), d_stats, n_blocks * sizeof(PackStats), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    float ms1 = 0;
    HIP_TRY(ctx, hipEventElapsedTime(&ms1, ctx->pack_ev[0], ctx->pack_ev[1]));
    uint64_t words = 0;  // payload words so far (each stream at its exact upper bound)
    for (uint64_t b = 0; b < n_blocks; b++) {
        const PackStats &S = st[b];
        PackParams &P = pp[b];
        ntc_block_meta &M = meta[b];
        std::memset(&M, 0, sizeof(M));
        std::memset(&P, 0, sizeof(P));
        const uint64_t r0 = b * block_reads;
        M.num_records = std::min<uint64_t>(block_reads, n_reads - r0);
        M.n_recs = S.n_recs;
        M.status = NTC_OK;
        if (S.bad) M.status = NTC_ERR_FORMAT;  // a short record past 32 bases (from_2bit panics)
        else if (S.n_recs == 0 || S.n_long == 0 || S.T == 0) M.status = NTC_ERR_EMPTY_READ;  // App. B.3
        if (M.status != NTC_OK) {
            P.skip = 1;
            continue;
        }
        const uint64_t m1 = S.max1 + 2, m4 = S.max4 + 2;
        P.l1 = 63 - __builtin_clzll(m1);
        P.l4 = 63 - __builtin_clzll(m4);
        P.lim1 = (2ULL << P.l1) - m1;
        P.lim4 = (2ULL << P.l4) - m4;  // l4 <= 62
        P.p2 = ntc_rice_log2_b(S.n_long, S.sum2);
        P.p3 = ntc_rice_log2_b(S.n_recs, S.sum3);
        const uint64_t nch = (S.T + 30) / 31;
        const uint64_t bound[4] = {S.n_long * (uint64_t)(P.l1 + 1),
                                   S.n_long * (uint64_t)(1 + P.p2) + (S.sum2 >> P.p2),
                                   S.n_recs * (uint64_t)(1 + P.p3) + (S.sum3 >> P.p3),
                                   nch * (uint64_t)(P.l4 + 1)};
        const uint64_t params[4] = {m1, (uint64_t)P.p2, (uint64_t)P.p3, m4};
        const uint64_t counts[4] = {S.n_long, S.n_long, S.n_recs, nch};
        for (int k = 0; k < 4; k++) {
            P.off[k] = words;
            M.stream[k].offset = words * 8;
            M.stream[k].encoded_size = (bound[k] + 63) / 64;  // refined after pass 2
            M.stream[k].param = params[k];
            M.stream[k].num_u64 = counts[k];
            words += (bound[k] + 63) / 64 + 1;
        }
    }
    *payload_bytes = words * 8;
    if (words * 8 > payload_capacity) return set_err(ctx, NTC_ERR_CAPACITY, "payload_capacity too small");
    // pass 2 in segments (pack.hip k_pack_write): each block's records, then its s4 chunks
    std::vector<PackSeg> segs;
    for (uint64_t b = 0; b < n_blocks; b++) {
        PackParams &P = pp[b];
        P.seg0 = (uint32_t)segs.size();
        if (!P.skip) {
            const PackStats &S = st[b];
            for (uint64_t f = S.rec_begin; f < S.rec_begin + S.n_recs; f += kPackSegRecs)
                segs.push_back(PackSeg{(uint32_t)b, 0u, f, std::min<uint64_t>(kPackSegRecs, S.rec_begin + S.n_recs - f)});
            const uint64_t nch = (S.T + 30) / 31;
            for (uint64_t f = 0; f < nch; f += kPackSegChunks)
                segs.push_back(PackSeg{(uint32_t)b, 1u, f, std::min<uint64_t>(kPackSegChunks, nch - f)});
        }
        P.nseg = (uint32_t)segs.size() - P.seg0;
    }
    void *d_segs;
    if ((rc = ensure(ctx, WS_PACK_SEGS, segs.size() * (sizeof(PackSeg) + 48) + 64, &d_segs))) return rc;
    uint64_t *d_seg_bits = (uint64_t *)((uint8_t *)d_segs + segs.size() * sizeof(PackSeg));
    uint64_t *d_seg_start = d_seg_bits + 3 * segs.size();
    HIP_TRY(ctx, hipMemsetAsync(d_payload, 0, words * 8, ctx->stream));  // shared words and fallback tiles OR into zeros
    HIP_TRY(ctx, hipMemcpyAsync(d_params, pp.data(), n_blocks * sizeof(PackParams), hipMemcpyHostToDevice,
                                ctx->stream));
    if (!segs.empty())
        HIP_TRY(ctx, hipMemcpyAsync(d_segs, segs.data(), segs.size() * sizeof(PackSeg), hipMemcpyHostToDevice,
                                    ctx->stream));
    HIP_TRY(ctx, hipEventRecord(ctx->pack_ev[2], ctx->stream));
    launch_pack_write(d_recs, (const uint64_t *)d_chunks, d_stats, d_params, n_blocks, (const PackSeg *)d_segs,
                      segs.size(), d_seg_bits, d_seg_start, (uint64_t *)d_payload, d_bits, ctx->stream);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipEventRecord(ctx->pack_ev[1], ctx->stream));
    std::vector<uint64_t> bits(n_blocks * 4);
    HIP_TRY(ctx, hipMemcpyAsync(bits.data(), d_bits, n_blocks * 32, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    float ms2 = 0;
    HIP_TRY(ctx, hipEventElapsedTime(&ms2, ctx->pack_ev[2], ctx->pack_ev[1]));
    ctx->last_pack_ms = (double)ms1 + (double)ms2;
    for (uint64_t b = 0; b < n_blocks; b++) {
        if (meta[b].status != NTC_OK) continue;
        for (int k = 0; k < 4; k++) {
            const uint64_t w = (bits[b * 4 + k] + 63) / 64;
            if (w > meta[b].stream[k].encoded_size)
                return set_err(ctx, NTC_ERR_FORMAT, "packer exceeded its stream bound");  // never expected
            meta[b].stream[k].encoded_size = w;
        }
    }
    return NTC_OK;
}

}  // namespace

extern "C" {

int ntc_abi_version(void) { return NTC_ABI_VERSION; }

int ntc_ctx_create(int device, ntc_ctx **out) {
    if (!out) return NTC_ERR_INVALID_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return NTC_ERR_HIP;
    if (device < 0 || device >= ndev) return NTC_ERR_INVALID_ARG;
    ntc_ctx *ctx = new ntc_ctx();
    ctx->device = device;
    // how a host thread waits for the device (A/B hook; HIP's default is auto): "spin",
    // "yield" or "blocking".  Takes effect only before the device's first use in the process.
    if (const char *v = std::getenv("NTC_DEVICE_SCHEDULE")) {
        const unsigned f = std::strcmp(v, "spin") == 0       ? hipDeviceScheduleSpin
                           : std::strcmp(v, "yield") == 0    ? hipDeviceScheduleYield
                           : std::strcmp(v, "blocking") == 0 ? hipDeviceScheduleBlockingSync
                                                             : hipDeviceScheduleAuto;
        if (hipSetDevice(device) == hipSuccess && hipSetDeviceFlags(f) != hipSuccess) (void)hipGetLastError();
    }
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc((void **)&ctx->d_status, 64) != hipSuccess ||
        hipHostMalloc((void **)&ctx->h_box, 64, hipHostMallocDefault) != hipSuccess) {
        delete ctx;
        return NTC_ERR_HIP;
    }
    for (auto &e : ctx->ev)
        if (hipEventCreate(&e) != hipSuccess) {
            delete ctx;
            return NTC_ERR_HIP;
        }
    if (hipDeviceGetAttribute(&ctx->num_cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
        ctx->num_cus <= 0)
        ctx->num_cus = 256;
    if (const char *v = std::getenv("NTC_ENCODE_VARIANT")) {
        int x = std::atoi(v);
        if (x == 1 || x == 4) ctx->encode_variant = x;
    }
    *out = ctx;
    return NTC_OK;
}

void ntc_ctx_destroy(ntc_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (auto &b : ctx->ws)
        if (b.p) (void)hipFree(b.p);
    ctx->index_mem.reset();
    if (ctx->d_status) (void)hipFree(ctx->d_status);
    if (ctx->h_box) (void)hipHostFree(ctx->h_box);
    for (auto &e : ctx->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : ctx->pack_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->stream && ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char *ntc_last_error(const ntc_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int ntc_ctx_set_stream(ntc_ctx *ctx, void *hip_stream) {
    if (!ctx) return NTC_ERR_INVALID_ARG;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->own_stream) HIP_TRY(ctx, hipStreamDestroy(ctx->stream));
    if (hip_stream) {
        ctx->stream = (hipStream_t)hip_stream;
        ctx->own_stream = false;
    } else {
        HIP_TRY(ctx, hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
        ctx->own_stream = true;
    }
    return NTC_OK;
}

int ntc_ctx_synchronize(ntc_ctx *ctx) {
    if (!ctx) return NTC_ERR_INVALID_ARG;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return NTC_OK;
}

int ntc_index_share(ntc_ctx *dst, const ntc_ctx *src) {
    if (!dst || !src) return set_err(dst, NTC_ERR_INVALID_ARG, "null context");
    if (!src->has_index) return set_err(dst, NTC_ERR_NO_INDEX, "the source context holds no index");
    if (src->device != dst->device) return set_err(dst, NTC_ERR_INVALID_ARG, "contexts on different devices");
    if (dst == src) return NTC_OK;
    HIP_TRY(dst, hipSetDevice(dst->device));
    HIP_TRY(dst, hipStreamSynchronize(dst->stream));
    dst->index_mem = src->index_mem;
    dst->dix = src->dix;
    dst->index_bytes = src->index_bytes;
    dst->n_paths = src->n_paths;
    dst->path_text_len = src->path_text_len;
    dst->filter_density_ppm = src->filter_density_ppm;
    dst->tab_u_fallback = src->tab_u_fallback;
    dst->index_decode_only = src->index_decode_only;
    dst->upload_host_us = dst->upload_total_us = 0;
    dst->has_index = true;
    return NTC_OK;
}

}  // extern "C"

// the host half of an upload: the index copied out of the view and its derived tables
// (derived.cpp build_derived), no GPU involved
struct ntc_index_prep {
    HostIndex hx;
    Derived dv;
    int64_t host_us = 0;
};

namespace {
int prepare_index(const ntc_index_view *v, ntc_index_prep &p, std::string &err) {
    const auto t0 = std::chrono::steady_clock::now();
    p.hx.n = v->n_nodes;
    p.hx.k = v->k;
    const uint64_t nw = (v->n_nodes + 63) / 64;
    for (int c = 0; c < 4; c++) {
        p.hx.rows[c].assign(v->rows[c], v->rows[c] + nw);
        p.hx.C[c] = v->C[c];
    }
    p.hx.lcs.assign(v->lcs, v->lcs + v->n_nodes);
    if (!build_derived(p.hx, p.dv, err, false)) return NTC_ERR_FORMAT;
    p.host_us = (int64_t)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0)
                    .count();
    return NTC_OK;
}
bool view_ok(const ntc_index_view *v) {
    if (!v || !v->lcs) return false;
    for (int c = 0; c < 4; c++)
        if (!v->rows[c]) return false;
    return true;
}
int upload_prepared(ntc_ctx *ctx, const ntc_index_prep &prep);
}  // namespace

extern "C" {

int ntc_index_prepare(const ntc_index_view *v, ntc_index_prep **out) {
    if (!out || !view_ok(v)) return NTC_ERR_INVALID_ARG;
    *out = nullptr;
    auto *p = new (std::nothrow) ntc_index_prep();
    if (!p) return NTC_ERR_CAPACITY;
    std::string err;
    const int rc = prepare_index(v, *p, err);
    if (rc) {
        delete p;
        return rc;
    }
    *out = p;
    return NTC_OK;
}

void ntc_index_prep_free(ntc_index_prep *p) { delete p; }

int ntc_index_upload_prepared(ntc_ctx *ctx, const ntc_index_prep *p) {
    if (!ctx || !p) return set_err(ctx, NTC_ERR_INVALID_ARG, "null context or prepared index");
    return upload_prepared(ctx, *p);
}

int ntc_index_upload(ntc_ctx *ctx, const ntc_index_view *v) {
    if (!ctx || !view_ok(v)) return set_err(ctx, NTC_ERR_INVALID_ARG, "null index view");
    ntc_index_prep p;
    std::string err;
    const int rc = prepare_index(v, p, err);
    if (rc) return set_err(ctx, rc, err);
    return upload_prepared(ctx, p);
}

}  // extern "C"

namespace {
int upload_prepared(ntc_ctx *ctx, const ntc_index_prep &prep) {
    const HostIndex &hx = prep.hx;
    const Derived &dv = prep.dv;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const auto t_start = std::chrono::steady_clock::now();
    auto us_since = [&] {
        return prep.host_us + (int64_t)std::chrono::duration_cast<std::chrono::microseconds>(
                                  std::chrono::steady_clock::now() - t_start).count();
    };
    ctx->upload_host_us = prep.host_us;
    // NTC_UPLOAD_TRACE=1: seconds since the start of the device half at each stage (stderr)
    static const bool trace = std::getenv("NTC_UPLOAD_TRACE") != nullptr;
    auto mark = [&](const char *what, bool sync) {
        if (!trace) return;
        if (sync) (void)hipStreamSynchronize(ctx->stream);
        std::fprintf(stderr, "[upload] %-28s %.4f s\n", what,
                     std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count());
    };
    // free a previous index
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    ctx->index_mem = std::make_shared<IndexMem>(ctx->device);  // the previous one goes with its last holder
    ctx->has_index = false;
    ctx->index_bytes = 0;
    const uint64_t n = hx.n;
    auto dalloc = [&](uint64_t bytes, void **p) -> int {
        HIP_TRY(ctx, hipMalloc(p, bytes));
        ctx->index_mem->ptrs.push_back(*p);
        ctx->index_bytes += bytes;
        return NTC_OK;
    };
    void *d_lines, *d_lcs, *d_uniq, *d_walk, *d_walk_a, *d_walk_b, *d_pred, *d_code;
    int rc;
    if ((rc = dalloc(dv.rank.size() * sizeof(uint2), &d_lines))) return rc;
    if ((rc = dalloc(n + 256, &d_lcs))) return rc;
    if ((rc = dalloc(dv.uniq.size() * 4, &d_uniq))) return rc;
    if ((rc = dalloc(n * sizeof(WalkEntry), &d_walk))) return rc;
    HIP_TRY(ctx, hipMalloc(&d_walk_a, n * sizeof(WalkStep)));
    HIP_TRY(ctx, hipMalloc(&d_walk_b, n * sizeof(WalkStep)));
    HIP_TRY(ctx, hipMalloc(&d_pred, n * 4));
    HIP_TRY(ctx, hipMalloc(&d_code, n + 64));
    HIP_TRY(ctx, hipMemcpy(d_lines, dv.rank.data(), dv.rank.size() * sizeof(uint2), hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemset(d_lcs, 0, n + 256));
    HIP_TRY(ctx, hipMemcpy(d_lcs, hx.lcs.data(), n, hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(d_uniq, dv.uniq.data(), dv.uniq.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(d_pred, dv.pred.data(), n * 4, hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(d_code, dv.code.data(), n, hipMemcpyHostToDevice));
    mark("allocations + H2D", false);
    launch_walk_build((const uint32_t *)d_pred, (const uint8_t *)d_code, n, (WalkStep *)d_walk_a,
                      (WalkStep *)d_walk_b, (WalkEntry *)d_walk, ctx->stream);
    HIP_TRY(ctx, hipGetLastError());
    mark("walk table", true);
    // path cover, built on the device (kernels.hip "path cover"; derived.cpp build_paths is
    // the same cover on the host, for emulation)
    void *d_pstream = nullptr, *d_colex_at = nullptr, *d_pos = nullptr, *d_puniq = nullptr;
    bool has_paths = false;
    uint64_t tlen = 0, n_paths = 0;
    const bool dec_only = ctx->decode_only_opt != 0;
    ctx->index_decode_only = false;
    if (!dec_only && n < (1ULL << 31)) {
        const std::vector<uint8_t> dummy = dummy_nodes(hx, dv);
        std::vector<uint32_t> dbits(n / 32 + 2, 0);
        for (uint64_t z = 0; z < n; z++)
            if (dummy[z]) dbits[z >> 5] |= 1u << (z & 31);
        std::vector<void *> tmp;
        auto talloc = [&](uint64_t bytes, void **p) -> int {
            HIP_TRY(ctx, hipMalloc(p, bytes));
            tmp.push_back(*p);
            return NTC_OK;
        };
        auto free_tmp = [&]() {
            (void)hipStreamSynchronize(ctx->stream);
            for (void *p : tmp) (void)hipFree(p);
            tmp.clear();
        };
        void *d_dummy, *d_prv, *d_sta, *d_stb, *d_len, *d_vals, *d_base, *d_stmp, *d_cnt;
        if ((rc = talloc(dbits.size() * 4, &d_dummy)) || (rc = talloc(n * 4, &d_prv)) ||
            (rc = talloc(n * 16, &d_sta)) || (rc = talloc(n * 16, &d_stb)) || (rc = talloc(n * 4, &d_len)) ||
            (rc = talloc(n * 4, &d_vals)) || (rc = talloc((n + 1) * 8, &d_base)) ||
            (rc = talloc(scan_tmp_words(n) * 8, &d_stmp)) || (rc = talloc(16, &d_cnt))) {
            free_tmp();
            return rc;
        }
        HIP_TRY(ctx, hipMemcpy(d_dummy, dbits.data(), dbits.size() * 4, hipMemcpyHostToDevice));
        PathArgs pa{(const uint2 *)d_lines, dv.rwords, (uint32_t)n, hx.k, (const uint8_t *)d_lcs,
                    (const uint32_t *)d_dummy, (const uint32_t *)d_pred, (const uint8_t *)d_code,
                    (const uint32_t *)d_uniq};
        uint32_t *prv = (uint32_t *)d_prv, *cnt = (uint32_t *)d_cnt;
        HIP_TRY(ctx, hipMemsetAsync(prv, 0xFF, n * 4, ctx->stream));
        HIP_TRY(ctx, hipMemsetAsync(cnt, 0, 16, ctx->stream));
        launch_path_edges(pa, prv, ctx->stream);
        if (ctx->path_link_opt) {  // unitigs linked across branches (derived.cpp link_unitigs)
            void *d_want, *d_bpred;
            if ((rc = talloc(n * 4, &d_want)) || (rc = talloc(n * 8, &d_bpred))) {
                free_tmp();
                return rc;
            }
            const uint4 *su = launch_path_rank(prv, (uint32_t)n, (uint4 *)d_sta, (uint4 *)d_stb, ctx->stream);
            HIP_TRY(ctx, hipMemsetAsync(d_len, 0, n * 4, ctx->stream));
            launch_path_lengths(pa, su, prv, (uint32_t *)d_len, (uint32_t *)d_vals, cnt + 2, ctx->stream);
            HIP_TRY(ctx, hipMemsetAsync(d_want, 0xFF, n * 4, ctx->stream));
            HIP_TRY(ctx, hipMemsetAsync(d_bpred, 0xFF, n * 8, ctx->stream));
            launch_path_link(pa, su, (const uint32_t *)d_len, (uint32_t *)d_want, (unsigned long long *)d_bpred, prv,
                             ctx->stream);
        }
        const uint4 *st = launch_path_rank(prv, (uint32_t)n, (uint4 *)d_sta, (uint4 *)d_stb, ctx->stream);
        launch_path_cut(pa, st, prv, cnt, ctx->stream);
        uint32_t cut = 0;
        HIP_TRY(ctx, hipMemcpyAsync(&cut, cnt, 4, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        if (cut) st = launch_path_rank(prv, (uint32_t)n, (uint4 *)d_sta, (uint4 *)d_stb, ctx->stream);
        HIP_TRY(ctx, hipMemsetAsync(d_len, 0, n * 4, ctx->stream));
        launch_path_lengths(pa, st, prv, (uint32_t *)d_len, (uint32_t *)d_vals, cnt + 1, ctx->stream);
        scan_excl_u32((const uint32_t *)d_vals, n, (uint64_t *)d_base, (uint64_t *)d_stmp, ctx->stream);
        uint32_t np32 = 0;
        HIP_TRY(ctx, hipMemcpyAsync(&tlen, (uint64_t *)d_base + n, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(&np32, cnt + 1, 4, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        HIP_TRY(ctx, hipGetLastError());
        n_paths = np32;
        if (tlen + 64 < (1ULL << 31)) {
            // sizes as derived.cpp build_paths: groups read up to k + 64 characters past a node
            const uint64_t n_groups = (tlen + hx.k) / 32 + 8, n_colex = tlen + 8, n_puniq = tlen / 64 + 4;
            if ((rc = dalloc(n_puniq * 8, &d_puniq)) || (rc = dalloc(n_groups * 16, &d_pstream)) ||
                (rc = dalloc(n_colex * 4 + 64, &d_colex_at)) || (rc = dalloc(n * 4, &d_pos))) {
                free_tmp();
                return rc;
            }
            HIP_TRY(ctx, hipMemsetAsync(d_puniq, 0, n_puniq * 8, ctx->stream));
            HIP_TRY(ctx, hipMemsetAsync(d_pstream, 0, n_groups * 16, ctx->stream));
            HIP_TRY(ctx, hipMemsetAsync(d_colex_at, 0xFF, n_colex * 4 + 64, ctx->stream));
            HIP_TRY(ctx, hipMemsetAsync(d_pos, 0xFF, n * 4, ctx->stream));
            launch_path_place(pa, st, prv, (const uint64_t *)d_base, (uint32_t *)d_colex_at, (uint32_t *)d_pos,
                              (uint4 *)d_pstream, (uint64_t *)d_puniq, ctx->stream);
            if (hx.k >= kForkBlockMinK)
                launch_path_forks(pa, st, (const uint32_t *)d_len, (const uint64_t *)d_base, (const uint32_t *)d_pos,
                                  (const uint4 *)d_pstream, (uint32_t *)d_colex_at, ctx->stream);
            HIP_TRY(ctx, hipGetLastError());
            has_paths = true;
        }
        free_tmp();
    }
    mark("path cover", true);
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipFree(d_walk_a));
    HIP_TRY(ctx, hipFree(d_walk_b));
    HIP_TRY(ctx, hipFree(d_pred));
    HIP_TRY(ctx, hipFree(d_code));
    DevIndex &d = ctx->dix;
    d.rank = (const uint2 *)d_lines;
    d.lcs = (const uint8_t *)d_lcs;
    d.uniq = (const uint32_t *)d_uniq;
    d.walk = (const WalkEntry *)d_walk;
    d.rwords = dv.rwords;
    d.n = (uint32_t)n;
    d.k = hx.k;
    d.t_jump = dv.t_jump;
    for (int c = 0; c < 5; c++) d.C[c] = dv.C[c];
    d.has_paths = has_paths ? 1u : 0u;
    d.path_len = has_paths ? (uint32_t)tlen : 0u;
    d.pstream = (const uint4 *)d_pstream;
    d.colex_at = (const uint32_t *)d_colex_at;
    d.pos_of_node = (const uint32_t *)d_pos;
    d.puniq = (const uint64_t *)d_puniq;
    d.forks = has_paths && hx.k >= kForkBlockMinK ? 1u : 0u;
    d.absent = dv.absent;
    // Joint path runs pay off when MS intervals above U hold several nodes for long stretches:
    // genome collections, whose shared regions split the path cover into short unitigs (S91:
    // 1.19 M paths over 70 M nodes).  A cover of long paths (one genome, C91: 2 paths) keeps
    // the lighter k_ms4 build.
    d.joint = has_paths && (ctx->joint_opt == 1 || (ctx->joint_opt < 0 && (uint64_t)n_paths * kJointAutoNodesPerPath > n))
                  ? 1u : 0u;
    if (dec_only) {  // decode reads the walk table alone: no suffix table, SCAN words or rank chunks
        d.rank2 = nullptr;
        d.tab = nullptr;
        d.tab_bits = nullptr;
        d.filt_bits = nullptr;
        d.filt_f = 0;
        d.pair_w = nullptr;
        d.win_w = nullptr;
        d.tab_u = 0;
        d.tab_pos = 0;
        HIP_TRY(ctx, hipGetLastError());
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        ctx->n_paths = 0;
        ctx->path_text_len = 0;
        ctx->index_decode_only = true;
        ctx->has_index = true;
        mark("done (decode only)", false);
        ctx->upload_total_us = us_since();
        return NTC_OK;
    }
    d.rank2 = nullptr;
    if (ctx->ext2_opt) {  // two-character rank lines (8 B per node)
        void *d_r2;
        if ((rc = dalloc(rank2_blocks(n) * 4 * sizeof(Rank2Chunk), &d_r2))) return rc;
        launch_rank2(d, (Rank2Chunk *)d_r2, ctx->stream);
        d.rank2 = (const Rank2Chunk *)d_r2;
    }
    // suffix table, levels 1..U, built on the device from the rank lines
    uint32_t U = ctx->tab_u_opt ? std::min<uint32_t>(ctx->tab_u_opt, std::min<uint32_t>(hx.k, kTabMaxU))
                                : default_tab_u(n, hx.k, hx.lcs.data());
    ctx->tab_u_fallback = 0;
    if (!ctx->tab_u_opt && U > 14) {
        // the density rule's deeper table (U = 15: 11.5 GB against 2.9 GB) only where it fits
        // beside what the device already holds plus an encode workspace (ranks may share a GPU)
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess &&
            (uint64_t)free_b < tab_base(U + 1) * sizeof(uint2) + (64ull << 30)) {
            U = 14;
            ctx->tab_u_fallback = 1;
        }
    }
    void *d_tab, *d_bits, *d_fbits = nullptr;
    if (hipMalloc(&d_tab, tab_base(U + 1) * sizeof(uint2)) != hipSuccess) {
        (void)hipGetLastError();
        if (ctx->tab_u_opt || U <= 14) return set_err(ctx, NTC_ERR_HIP, "suffix table allocation failed");
        U = 14;  // allocation failed at the deeper level: fall back (results never depend on U)
        ctx->tab_u_fallback = 1;
        if ((rc = dalloc(tab_base(U + 1) * sizeof(uint2), &d_tab))) return rc;
    } else {
        ctx->index_mem->ptrs.push_back(d_tab);
        ctx->index_bytes += tab_base(U + 1) * sizeof(uint2);
    }
    const uint32_t F = filter_level(U);
    if ((rc = dalloc(tab_bits_words(U) * 4, &d_bits))) return rc;
    if (F && (rc = dalloc(tab_bits_words(F) * 4, &d_fbits))) return rc;
    d.tab = (const uint2 *)d_tab;
    d.tab_bits = (const uint32_t *)d_bits;
    d.filt_bits = (const uint32_t *)d_fbits;
    d.filt_f = F;
    d.tab_u = U;
    d.tab_pos = (has_paths && U >= dv.t_jump && n < (1ULL << 31)) ? 1u : 0u;
    mark("suffix table allocation", false);
    launch_tab_build(d, U, (uint2 *)d_tab, (uint32_t *)d_bits, F, (uint32_t *)d_fbits, ctx->stream);
    mark("suffix table", true);
    d.win_w = nullptr;
    // SCAN window words (a (U-3)-mer keyed 32-byte entry answers four positions): two lines
    // answer the eight positions of a SCAN unit.  k_ms4 is bound by its lane loads in the
    // CU's vector memory path (TA/TD 93-96 % busy at C91, TCP stalled on pending L2 data), and
    // the L2-resident filter took 18 of them per SCAN: C91 k_ms4 3.70 -> 2.40 ms with window
    // words and no filter.  Auto: on for every U >= 4, both builds.
    const bool win_on = U >= 4 && ctx->win_opt != 0;
    if (win_on) {
        void *d_win;
        if ((rc = dalloc(win_words_count(U) * 32, &d_win))) return rc;
        launch_win_words((const uint32_t *)d_bits, U, (uint32_t *)d_win, ctx->stream);
        d.win_w = (const uint32_t *)d_win;
    }
    ctx->filter_density_ppm = -1;
    if (F) {
        // A filter over a large index is mostly ones (S91's 70 M nodes: 72 % of all 12-mers)
        // and passes most positions, so it costs more lines than it saves: auto mode drops it
        // above kFiltMaxDensityPpm (every SCAN then goes straight to the exact pair words).
        std::vector<uint32_t> fb(tab_bits_words(F));
        HIP_TRY(ctx, hipMemcpyAsync(fb.data(), d_fbits, fb.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        uint64_t ones = 0;
        for (uint32_t x : fb) ones += (uint64_t)__builtin_popcount(x);
        ctx->filter_density_ppm = (int64_t)(ones * 1000000 / ((uint64_t)fb.size() * 32));
        // (auto: off with window words, whose loads do not depend on it)
        const bool on = ctx->filter_opt == 1 ||
                        (ctx->filter_opt < 0 && !win_on && ctx->filter_density_ppm <= kFiltMaxDensityPpm);
        if (!on) d.filt_f = 0;
    }
    d.pair_w = nullptr;
    if (ctx->pair_bytes_opt) {
        void *d_pair;
        if ((rc = dalloc((pair_words_count(U) + 1) / 2 * 4, &d_pair))) return rc;
        launch_pair_words((const uint2 *)d_tab + tab_base(U), U, (uint16_t *)d_pair, ctx->stream);
        d.pair_w = (const uint16_t *)d_pair;
    }
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    ctx->n_paths = n_paths;
    ctx->path_text_len = tlen;
    ctx->has_index = true;
    mark("done", false);
    ctx->upload_total_us = us_since();
    return NTC_OK;
}
}  // namespace

extern "C" {

int ntc_ctx_set_option(ntc_ctx *ctx, const char *key, int64_t value) {
    if (!ctx || !key) return NTC_ERR_INVALID_ARG;
    if (std::strcmp(key, "tab_u") == 0) {  // applies to the next ntc_index_upload
        if (value < 0 || value > (int64_t)kTabMaxU)
            return set_err(ctx, NTC_ERR_INVALID_ARG, "tab_u must be 0 (default) or 1..15");
        ctx->tab_u_opt = (uint32_t)value;
        return NTC_OK;
    }
    if (std::strcmp(key, "pair_bytes") == 0) {  // applies to the next ntc_index_upload
        if (value != 0 && value != 1) return set_err(ctx, NTC_ERR_INVALID_ARG, "pair_bytes must be 0 or 1");
        ctx->pair_bytes_opt = (int)value;
        return NTC_OK;
    }
    if (std::strcmp(key, "filter") == 0) {  // applies to the next ntc_index_upload
        if (value < -1 || value > 1) return set_err(ctx, NTC_ERR_INVALID_ARG, "filter must be -1 (auto), 0 or 1");
        ctx->filter_opt = (int)value;
        return NTC_OK;
    }
    if (std::strcmp(key, "joint") == 0) {  // applies to the next ntc_index_upload
        if (value < -1 || value > 1) return set_err(ctx, NTC_ERR_INVALID_ARG, "joint must be -1 (auto), 0 or 1");
        ctx->joint_opt = (int)value;
        return NTC_OK;
    }
    if (std::strcmp(key, "path_link") == 0) {  // applies to the next ntc_index_upload
        if (value != 0 && value != 1) return set_err(ctx, NTC_ERR_INVALID_ARG, "path_link must be 0 or 1");
        ctx->path_link_opt = (int)value;
        return NTC_OK;
    }
    if (std::strcmp(key, "win") == 0) {  // applies to the next ntc_index_upload
        if (value < -1 || value > 1) return set_err(ctx, NTC_ERR_INVALID_ARG, "win must be -1 (auto), 0 or 1");
        ctx->win_opt = (int)value;
        return NTC_OK;
    }
    if (std::strcmp(key, "decode_only") == 0) {  // applies to the next ntc_index_upload
        if (value != 0 && value != 1) return set_err(ctx, NTC_ERR_INVALID_ARG, "decode_only must be 0 or 1");
        ctx->decode_only_opt = (int)value;
        return NTC_OK;
    }
    if (std::strcmp(key, "warm_dma") == 0) {  // an action: copies of `value` bytes each way, now
        if (value < 1 || value > (1ll << 30)) return set_err(ctx, NTC_ERR_INVALID_ARG, "warm_dma: 1 .. 2^30 bytes");
        HIP_TRY(ctx, hipSetDevice(ctx->device));
        void *h = nullptr, *d = nullptr;
        if (hipHostMalloc(&h, (size_t)value, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            return set_err(ctx, NTC_ERR_HIP, "warm_dma: pinned allocation failed");
        }
        int rc = ensure(ctx, WS_STAGE_BASES, (uint64_t)value, &d);
        if (rc == NTC_OK) {
            if (hipMemcpyAsync(h, d, (size_t)value, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
                hipMemcpyAsync(d, h, (size_t)value, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
                hipStreamSynchronize(ctx->stream) != hipSuccess) {
                (void)hipGetLastError();
                rc = set_err(ctx, NTC_ERR_HIP, "warm_dma: copy failed");
            }
        }
        (void)hipHostFree(h);
        return rc;
    }
    if (std::strcmp(key, "ext2") == 0) {  // applies to the next ntc_index_upload
        if (value != 0 && value != 1) return set_err(ctx, NTC_ERR_INVALID_ARG, "ext2 must be 0 or 1");
        ctx->ext2_opt = (int)value;
        return NTC_OK;
    }
    if (std::strcmp(key, "max_pass_bases") == 0) {  // device workspace ~40 B per base of a pass
        if (value < 1) return set_err(ctx, NTC_ERR_INVALID_ARG, "max_pass_bases must be >= 1");
        ctx->max_pass_bases = (uint64_t)value;
        return NTC_OK;
    }
    if (std::strcmp(key, "ent_slots") == 0) {  // secondary entry slots per read (0: auto)
        if (value < 0 || value > 1024 || (value & 3))
            return set_err(ctx, NTC_ERR_INVALID_ARG, "ent_slots must be 0 (auto) or a multiple of 4 up to 1024");
        ctx->ent_slots_opt = (uint32_t)value;
        return NTC_OK;
    }
    if (std::strcmp(key, "pool_per_read") == 0) {  // test hook: overflow pools per read (entries, records)
        if (value < 0) return set_err(ctx, NTC_ERR_INVALID_ARG, "pool_per_read must be >= 0");
        ctx->epool_per_read = ctx->rpool_per_read = (double)value;
        ctx->epool_per_base = ctx->rpool_per_base = 0.0;
        return NTC_OK;
    }
    if (std::strcmp(key, "encode_variant") == 0) {
        if (value != 1 && value != 4)
            return set_err(ctx, NTC_ERR_INVALID_ARG, "encode_variant must be 4 (default) or 1 (A/B baseline)");
        ctx->encode_variant = (int)value;
        return NTC_OK;
    }
    return set_err(ctx, NTC_ERR_INVALID_ARG, std::string("unknown option ") + key);
}

int ntc_ctx_get_option(const ntc_ctx *ctx, const char *key, int64_t *value) {
    if (!ctx || !key || !value) return NTC_ERR_INVALID_ARG;
    if (std::strcmp(key, "encode_variant") == 0) *value = ctx->encode_variant;
    else if (std::strcmp(key, "tab_u") == 0) *value = ctx->has_index ? ctx->dix.tab_u : ctx->tab_u_opt;
    else if (std::strcmp(key, "pair_bytes") == 0) *value = ctx->has_index ? (ctx->dix.pair_w != nullptr) : ctx->pair_bytes_opt;
    else if (std::strcmp(key, "ext2") == 0) *value = ctx->has_index ? (ctx->dix.rank2 != nullptr) : ctx->ext2_opt;
    else if (std::strcmp(key, "decode_only") == 0) *value = ctx->has_index ? ctx->index_decode_only : ctx->decode_only_opt;
    else if (std::strcmp(key, "filter") == 0) *value = ctx->has_index ? (ctx->dix.filt_f != 0) : ctx->filter_opt;
    else if (std::strcmp(key, "joint") == 0) *value = ctx->has_index ? (int64_t)ctx->dix.joint : ctx->joint_opt;
    else if (std::strcmp(key, "win") == 0) *value = ctx->has_index ? (ctx->dix.win_w != nullptr) : ctx->win_opt;
    else if (std::strcmp(key, "path_link") == 0) *value = ctx->path_link_opt;
    else if (std::strcmp(key, "filter_density_ppm") == 0) *value = ctx->filter_density_ppm;
    else if (std::strcmp(key, "n_paths") == 0) *value = (int64_t)ctx->n_paths;
    else if (std::strcmp(key, "path_text_len") == 0) *value = (int64_t)ctx->path_text_len;
    else if (std::strcmp(key, "path_hash") == 0) {  // test hook: derived.h path_cover_hash of the device cover
        if (!ctx->has_index || !ctx->dix.has_paths) return NTC_ERR_NO_INDEX;
        const uint64_t n = ctx->dix.n, k = ctx->dix.k, tlen = ctx->path_text_len;
        std::vector<uint4> ps((tlen + k) / 32 + 8);
        std::vector<uint32_t> ca(tlen + 8), pn(n);
        std::vector<uint64_t> pu(tlen / 64 + 4);
        if (hipSetDevice(ctx->device) != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess ||
            hipMemcpy(ps.data(), ctx->dix.pstream, ps.size() * 16, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(ca.data(), ctx->dix.colex_at, ca.size() * 4, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(pn.data(), ctx->dix.pos_of_node, pn.size() * 4, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(pu.data(), ctx->dix.puniq, pu.size() * 8, hipMemcpyDeviceToHost) != hipSuccess)
            return NTC_ERR_HIP;
        *value = (int64_t)path_cover_hash(ps.data(), ca.data(), pn.data(), pu.data(), n, (uint32_t)k, tlen);
    }
    else if (std::strcmp(key, "upload_host_us") == 0) *value = ctx->upload_host_us;
    else if (std::strcmp(key, "max_pass_bases") == 0) *value = (int64_t)ctx->max_pass_bases;
    else if (std::strcmp(key, "upload_total_us") == 0) *value = ctx->upload_total_us;
    else if (std::strcmp(key, "tab_u_fallback") == 0) *value = ctx->tab_u_fallback;
    else if (std::strcmp(key, "pack_us") == 0) *value = (int64_t)(ctx->last_pack_ms * 1000.0);
    else if (std::strcmp(key, "ent_slots") == 0) *value = ent_slots(ctx);
    else if (std::strcmp(key, "spill_reruns") == 0) *value = (int64_t)ctx->spill_reruns;
    else if (std::strcmp(key, "pool_entries") == 0) *value = (int64_t)ctx->last4.pcap;  // last call's pools
    else if (std::strcmp(key, "pool_records") == 0) *value = (int64_t)ctx->last4.rcap;
    else if (std::strcmp(key, "workspace_bytes") == 0) {  // device workspace held now (all slots)
        uint64_t t = 0;
        for (const auto &b : ctx->ws) t += b.bytes;
        *value = (int64_t)t;
    }
    else return NTC_ERR_INVALID_ARG;
    return NTC_OK;
}

int ntc_index_info(const ntc_ctx *ctx, uint64_t *n_nodes, uint32_t *k, uint64_t *device_bytes) {
    if (!ctx) return NTC_ERR_INVALID_ARG;
    if (!ctx->has_index) return NTC_ERR_NO_INDEX;
    if (n_nodes) *n_nodes = ctx->dix.n;
    if (k) *k = ctx->dix.k;
    if (device_bytes) *device_bytes = ctx->index_bytes;
    return NTC_OK;
}

int ntc_encode_batch_device(ntc_ctx *ctx, const uint8_t *d_bases, const uint64_t *d_read_offsets,
                            uint64_t n_reads, uint32_t max_read_len, uint64_t *d_rec_out,
                            uint64_t rec_capacity, uint64_t *d_rec_offsets_out) {
    if (!ctx || (!d_read_offsets && n_reads) || !d_rec_offsets_out)
        return set_err(ctx, NTC_ERR_INVALID_ARG, "null argument");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (ctx->encode_variant == 4) {
        if (!ctx->has_index) return set_err(ctx, NTC_ERR_NO_INDEX, "no index uploaded");
        uint64_t total = 0;
        if (n_reads) {
            if (max_read_len > 0) {
                total = n_reads * (uint64_t)max_read_len;  // an upper bound is enough
            } else {
                uint64_t ends[2] = {0, 0};
                HIP_TRY(ctx, hipMemcpyAsync(&ends[0], d_read_offsets, 8, hipMemcpyDeviceToHost, ctx->stream));
                HIP_TRY(ctx, hipMemcpyAsync(&ends[1], d_read_offsets + n_reads, 8, hipMemcpyDeviceToHost, ctx->stream));
                HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
                total = ends[1] - ends[0];
            }
        }
        return encode4_impl(ctx, d_bases, d_read_offsets, n_reads, total, d_rec_out, rec_capacity,
                            d_rec_offsets_out);
    }
    Layout lay;
    const uint64_t tiles = (n_reads + 63) / 64;
    if (max_read_len > 0) {
        lay.rows_uniform = ((uint64_t)max_read_len + 31) & ~31ULL;
        lay.total_rows = tiles * lay.rows_uniform;
    } else if (n_reads > 0) {
        void *rows, *tb, *tmp;
        int rc;
        if ((rc = ensure(ctx, WS_TILEROWS, tiles * 4, &rows))) return rc;
        if ((rc = ensure(ctx, WS_TILEBASE, (tiles + 1) * 8, &tb))) return rc;
        if ((rc = ensure(ctx, WS_SCANTMP, scan_tmp_words(std::max(tiles, n_reads) + 1) * 8, &tmp)))
            return rc;
        launch_tile_rows(d_read_offsets, n_reads, (uint32_t *)rows, ctx->stream);
        scan_excl_u32((const uint32_t *)rows, tiles, (uint64_t *)tb, (uint64_t *)tmp, ctx->stream);
        HIP_TRY(ctx, hipMemcpyAsync(&lay.total_rows, (uint64_t *)tb + tiles, 8, hipMemcpyDeviceToHost,
                                    ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        lay.d_tile_base = (const uint64_t *)tb;
    }
    return encode_impl(ctx, d_bases, d_read_offsets, n_reads, lay, d_rec_out, rec_capacity,
                       d_rec_offsets_out, 0);
}

int ntc_encode_status(ntc_ctx *ctx, int64_t *bad_read, uint64_t *n_records) {
    if (!ctx) return NTC_ERR_INVALID_ARG;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    int rc = read_status(ctx, bad_read);
    if (rc) return rc;
    if (n_records) {
        if (ctx->last != kEncode || !ctx->last_out_offs) return set_err(ctx, NTC_ERR_INVALID_ARG, "no encode call");
        if (ctx->box_valid) *n_records = ((volatile uint64_t *)ctx->h_box)[1];
        else HIP_TRY(ctx, hipMemcpy(n_records, ctx->last_out_offs + ctx->last_n, 8, hipMemcpyDeviceToHost));
    }
    return NTC_OK;
}

namespace {
// one device pass of the v1 (A/B baseline) encoder over all reads
int encode_batch_v1(ntc_ctx *ctx, const uint8_t *bases, const uint64_t *read_offsets, uint64_t n_reads,
                    uint64_t *rec_out, uint64_t rec_capacity, uint64_t *rec_offsets_out, int64_t *bad_read) {
    const uint64_t o0 = read_offsets[0], total = read_offsets[n_reads] - o0;
    // per-tile scratch rows (host knows every length)
    const uint64_t tiles = (n_reads + 63) / 64;
    std::vector<uint64_t> tb(tiles + 1, 0), offs(n_reads + 1);
    for (uint64_t t = 0; t < tiles; t++) {
        uint64_t mx = 0;
        for (uint64_t r = t * 64; r < std::min(n_reads, t * 64 + 64); r++)
            mx = std::max(mx, read_offsets[r + 1] - read_offsets[r]);
        tb[t + 1] = tb[t] + ((mx + 31) & ~31ULL);
    }
    for (uint64_t r = 0; r <= n_reads; r++) offs[r] = read_offsets[r] - o0;
    void *d_bases, *d_offs, *d_tb, *d_recs, *d_roffs;
    int rc;
    if ((rc = ensure(ctx, WS_STAGE_BASES, total + 64, &d_bases))) return rc;
    if ((rc = ensure(ctx, WS_STAGE_OFFS, (n_reads + 1) * 8 * 2, &d_offs))) return rc;
    if ((rc = ensure(ctx, WS_TILEBASE, (tiles + 1) * 8, &d_tb))) return rc;
    if ((rc = ensure(ctx, WS_STAGE_RECS, (total + 1) * 8, &d_recs))) return rc;
    d_roffs = (uint64_t *)d_offs + (n_reads + 1);
    if (total) HIP_TRY(ctx, hipMemcpyAsync(d_bases, bases + o0, total, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(d_offs, offs.data(), (n_reads + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(d_tb, tb.data(), (tiles + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
    Layout lay;
    lay.d_tile_base = (const uint64_t *)d_tb;
    lay.total_rows = tb[tiles];
    rc = encode_impl(ctx, (const uint8_t *)d_bases, (const uint64_t *)d_offs, n_reads, lay, (uint64_t *)d_recs,
                     total + 1, (uint64_t *)d_roffs, total);
    if (rc) return rc;
    rc = read_status(ctx, bad_read);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpy(rec_offsets_out, d_roffs, (n_reads + 1) * 8, hipMemcpyDeviceToHost));
    const uint64_t nrec = rec_offsets_out[n_reads];
    if (nrec > rec_capacity) return set_err(ctx, NTC_ERR_CAPACITY, "rec_capacity smaller than the number of records");
    if (nrec) HIP_TRY(ctx, hipMemcpy(rec_out, d_recs, nrec * 8, hipMemcpyDeviceToHost));
    return NTC_OK;
}
}  // namespace

int ntc_encode_batch(ntc_ctx *ctx, const uint8_t *bases, const uint64_t *read_offsets, uint64_t n_reads,
                     uint64_t *rec_out, uint64_t rec_capacity, uint64_t *rec_offsets_out, int64_t *bad_read) {
    if (bad_read) *bad_read = -1;
    if (!ctx || !read_offsets || !rec_offsets_out || (n_reads && !bases))
        return set_err(ctx, NTC_ERR_INVALID_ARG, "null argument");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    for (uint64_t r = 0; r < n_reads; r++)
        if (read_offsets[r + 1] < read_offsets[r])
            return set_err(ctx, NTC_ERR_INVALID_ARG, "read offsets must be non-decreasing");
    if (!ctx->has_index) return set_err(ctx, NTC_ERR_NO_INDEX, "no index uploaded");
    if (ctx->encode_variant != 4)
        return encode_batch_v1(ctx, bases, read_offsets, n_reads, rec_out, rec_capacity, rec_offsets_out, bad_read);
    // passes of whole reads, at most max_pass_bases each (one read may exceed it alone), so
    // the device workspace stays bounded however large the host batch is
    std::vector<uint64_t> offs, roffs;
    uint64_t r0 = 0, produced = 0;
    rec_offsets_out[0] = 0;
    do {
        uint64_t r1 = std::min(n_reads, r0 + 1);
        if (r1 < n_reads) {  // largest r1 with bases [r0, r1) <= max_pass_bases
            uint64_t lo = r1, hi = n_reads;
            while (lo < hi) {
                const uint64_t mid = (lo + hi + 1) / 2;
                if (read_offsets[mid] - read_offsets[r0] <= ctx->max_pass_bases) lo = mid;
                else hi = mid - 1;
            }
            r1 = lo;
        }
        const uint64_t nr = r1 - r0, o0 = read_offsets[r0], total = read_offsets[r1] - o0;
        offs.resize(nr + 1);
        for (uint64_t r = 0; r <= nr; r++) offs[r] = read_offsets[r0 + r] - o0;
        void *d_bases, *d_offs, *d_recs;
        int rc;
        if ((rc = ensure(ctx, WS_STAGE_BASES, total + 64, &d_bases))) return rc;
        if ((rc = ensure(ctx, WS_STAGE_OFFS, (nr + 1) * 8 * 2, &d_offs))) return rc;
        if ((rc = ensure(ctx, WS_STAGE_RECS, (total + 1) * 8, &d_recs))) return rc;
        uint64_t *d_roffs = (uint64_t *)d_offs + (nr + 1);
        if (total) HIP_TRY(ctx, hipMemcpyAsync(d_bases, bases + o0, total, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(d_offs, offs.data(), (nr + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
        rc = encode4_impl(ctx, (const uint8_t *)d_bases, (const uint64_t *)d_offs, nr, total, (uint64_t *)d_recs,
                          total + 1, d_roffs);
        if (rc) return rc;
        int64_t bad = -1;
        rc = read_status(ctx, &bad);
        if (rc) {
            if (bad_read) *bad_read = bad + (int64_t)r0;
            char buf[160];
            std::snprintf(buf, sizeof(buf), "%s at index %lld", status_name(rc), (long long)(bad + (int64_t)r0));
            ctx->err = buf;
            return rc;
        }
        roffs.resize(nr + 1);
        HIP_TRY(ctx, hipMemcpy(roffs.data(), d_roffs, (nr + 1) * 8, hipMemcpyDeviceToHost));
        const uint64_t nrec = roffs[nr];
        if (produced + nrec > rec_capacity)
            return set_err(ctx, NTC_ERR_CAPACITY, "rec_capacity smaller than the number of records");
        for (uint64_t r = 1; r <= nr; r++) rec_offsets_out[r0 + r] = produced + roffs[r];
        if (nrec) HIP_TRY(ctx, hipMemcpy(rec_out + produced, d_recs, nrec * 8, hipMemcpyDeviceToHost));
        produced += nrec;
        r0 = r1;
    } while (r0 < n_reads);
    return NTC_OK;
}

int ntc_decode_batch_device(ntc_ctx *ctx, const uint64_t *d_recs, uint64_t n_recs, uint8_t *d_bases_out,
                            uint64_t bases_capacity, uint64_t *d_read_offsets_out, uint64_t offsets_capacity) {
    if (!ctx || (!d_recs && n_recs) || !d_read_offsets_out) return set_err(ctx, NTC_ERR_INVALID_ARG, "null argument");
    if (!ctx->has_index) return set_err(ctx, NTC_ERR_NO_INDEX, "no index uploaded");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    void *ws, *tmp;
    int rc;
    const uint64_t n = n_recs;
    // per kDecTileRecs-record tile: pf, pl (sums) then pfs, pls (exclusive scans, totals at [tiles])
    const uint64_t tiles = (n + kDecTileRecs - 1) / kDecTileRecs;
    if ((rc = ensure(ctx, WS_DEC_C, (4 * tiles + 2) * 8, &ws))) return rc;
    uint64_t *pf = (uint64_t *)ws, *pl = pf + tiles, *pfs = pl + tiles, *pls = pfs + tiles + 1;
    if ((rc = ensure(ctx, WS_SCANTMP, (scan_tmp_words(tiles + 1) + 2) * 8, &tmp))) return rc;
    HIP_TRY(ctx, hipMemsetAsync(ctx->d_status, 0xFF, 8, ctx->stream));
    ctx->box_valid = false;
    ctx->last = kDecode;
    ctx->last_n = tiles;
    ctx->last_out_offs = pfs;  // pfs[tiles] = reads, pls[tiles] = bases (ntc_decode_status)
    HIP_TRY(ctx, hipEventRecord(ctx->ev[0], ctx->stream));
    if (n == 0) {
        HIP_TRY(ctx, hipMemsetAsync(pfs, 0, 16, ctx->stream));
        HIP_TRY(ctx, hipMemsetAsync(d_read_offsets_out, 0, 8, ctx->stream));
        for (int i = 1; i < 4; i++) HIP_TRY(ctx, hipEventRecord(ctx->ev[i], ctx->stream));
        return NTC_OK;
    }
    launch_dec_tiles(d_recs, n, pf, pl, pfs, pls, (uint64_t *)tmp, ctx->stream);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipEventRecord(ctx->ev[1], ctx->stream));
    DecWalkArgs wa{};
    wa.ix = ctx->dix;
    wa.recs = d_recs;
    wa.n = n;
    wa.pfs = pfs;
    wa.pls = pls;
    wa.offs_out = d_read_offsets_out;
    wa.offs_capacity = offsets_capacity;
    wa.bases_capacity = bases_capacity;
    wa.out = d_bases_out;
    wa.status = ctx->d_status;
    launch_dec_walk(wa, ctx->stream);
    HIP_TRY(ctx, hipEventRecord(ctx->ev[3], ctx->stream));  // k_dec_rec alone: ev[1] -> ev[3]
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipEventRecord(ctx->ev[2], ctx->stream));
    launch_status_box(ctx->d_status, pfs + tiles, pls + tiles, nullptr, ctx->h_box, ctx->stream);
    HIP_TRY(ctx, hipGetLastError());
    ctx->box_valid = true;
    return NTC_OK;
}

int ntc_decode_status(ntc_ctx *ctx, uint64_t *n_reads, uint64_t *n_bases) {
    if (!ctx) return NTC_ERR_INVALID_ARG;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    int rc = read_status(ctx, nullptr);
    if (ctx->last != kDecode) return set_err(ctx, NTC_ERR_INVALID_ARG, "no decode call");
    uint64_t nr = 0, nb = 0;
    if (ctx->box_valid) {
        nr = ((volatile uint64_t *)ctx->h_box)[1];
        nb = ((volatile uint64_t *)ctx->h_box)[2];
    } else {
        HIP_TRY(ctx, hipMemcpy(&nr, ctx->last_out_offs + ctx->last_n, 8, hipMemcpyDeviceToHost));
        HIP_TRY(ctx, hipMemcpy(&nb, ctx->last_out_offs + (ctx->last_n + 1) + ctx->last_n, 8, hipMemcpyDeviceToHost));
    }
    if (n_reads) *n_reads = nr;
    if (n_bases) *n_bases = nb;
    ctx->last_units = nb;
    return rc;
}

int ntc_decode_batch(ntc_ctx *ctx, const uint64_t *recs, uint64_t n_recs, uint8_t *bases_out,
                     uint64_t bases_capacity, uint64_t *read_offsets_out, uint64_t offsets_capacity,
                     uint64_t *n_reads_out, uint64_t *n_bases_out) {
    if (!ctx || (!recs && n_recs)) return set_err(ctx, NTC_ERR_INVALID_ARG, "null argument");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    uint64_t nreads = 0, nbases = 0;
    for (uint64_t r = 0; r < n_recs; r++) {
        const uint32_t flag = (uint32_t)(recs[r] >> 56);
        nreads += flag & 1;
        nbases += (flag & 2) ? (flag >> 2) : ((uint32_t)(recs[r] >> 32) & 0xFFFFFFu);
    }
    if (n_reads_out) *n_reads_out = nreads;
    if (n_bases_out) *n_bases_out = nbases;
    if (n_recs && !((recs[0] >> 56) & 1)) return set_err(ctx, NTC_ERR_FORMAT, "records do not start a read");
    if (nbases > bases_capacity || nreads + 1 > offsets_capacity || !read_offsets_out || (nbases && !bases_out))
        return set_err(ctx, NTC_ERR_CAPACITY, "decode output buffers too small");
    // passes of whole reads (a pass ends before a `first` record), at most max_pass_bases
    // output bases each unless one read alone is larger
    uint64_t a0 = 0, reads_done = 0, bases_done = 0;
    read_offsets_out[0] = 0;
    std::vector<uint64_t> offs;
    while (a0 < n_recs) {
        uint64_t a1 = a0, pb = 0, pr = 0;
        while (a1 < n_recs) {
            const uint32_t flag = (uint32_t)(recs[a1] >> 56);
            const uint64_t len = (flag & 2) ? (flag >> 2) : ((uint32_t)(recs[a1] >> 32) & 0xFFFFFFu);
            if ((flag & 1) && a1 > a0 && pb + len > ctx->max_pass_bases) break;
            pb += len;
            pr += flag & 1;
            a1++;
        }
        // a read runs to the next `first` record: extend the pass over the rest of this read
        while (a1 < n_recs && !((recs[a1] >> 56) & 1)) {
            const uint32_t flag = (uint32_t)(recs[a1] >> 56);
            pb += (flag & 2) ? (flag >> 2) : ((uint32_t)(recs[a1] >> 32) & 0xFFFFFFu);
            a1++;
        }
        const uint64_t nrec = a1 - a0;
        void *d_recs, *d_out, *d_offs;
        int rc;
        if ((rc = ensure(ctx, WS_STAGE_RECS, (nrec + 1) * 8, &d_recs))) return rc;
        if ((rc = ensure(ctx, WS_STAGE_BASES, pb + 64, &d_out))) return rc;
        if ((rc = ensure(ctx, WS_STAGE_OFFS, (pr + 1) * 8, &d_offs))) return rc;
        HIP_TRY(ctx, hipMemcpyAsync(d_recs, recs + a0, nrec * 8, hipMemcpyHostToDevice, ctx->stream));
        rc = ntc_decode_batch_device(ctx, (const uint64_t *)d_recs, nrec, (uint8_t *)d_out, pb, (uint64_t *)d_offs,
                                     pr + 1);
        if (rc) return rc;
        uint64_t nr = 0, nb = 0;
        rc = ntc_decode_status(ctx, &nr, &nb);
        if (rc) return rc;
        if (nr != pr || nb != pb) return set_err(ctx, NTC_ERR_FORMAT, "decode size mismatch");
        offs.resize(pr + 1);
        HIP_TRY(ctx, hipMemcpy(offs.data(), d_offs, (pr + 1) * 8, hipMemcpyDeviceToHost));
        for (uint64_t r = 1; r <= pr; r++) read_offsets_out[reads_done + r] = bases_done + offs[r];
        if (pb) HIP_TRY(ctx, hipMemcpy(bases_out + bases_done, d_out, pb, hipMemcpyDeviceToHost));
        reads_done += pr;
        bases_done += pb;
        a0 = a1;
    }
    return NTC_OK;
}

int ntc_pack_blocks_device(ntc_ctx *ctx, const uint64_t *d_recs, const uint64_t *d_rec_offsets,
                           uint64_t n_reads, uint32_t block_reads, uint8_t *d_payload,
                           uint64_t payload_capacity, ntc_block_meta *meta, uint64_t *payload_bytes) {
    if (!ctx || !d_rec_offsets || !meta || !payload_bytes || block_reads == 0 || (n_reads && (!d_recs || !d_payload)))
        return set_err(ctx, NTC_ERR_INVALID_ARG, "null argument or block_reads = 0");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    return pack_blocks_impl(ctx, d_recs, d_rec_offsets, n_reads, block_reads, d_payload, payload_capacity, meta,
                            payload_bytes);
}

}  // extern "C"

namespace {
// encode + GPU block packer over reads already in HBM (d_offs: n_reads + 1 offsets, room for
// n_reads + 1 more behind them, where the record offsets go); the tail of
// ntc_encode_pack_batch and ntc_encode_pack_fastq
int encode_pack_staged(ntc_ctx *ctx, const uint8_t *d_bases, const uint64_t *d_offs, uint64_t n_reads, uint64_t total,
                       uint32_t block_reads, ntc_block_meta *meta, uint8_t **payload, uint64_t *payload_bytes,
                       int64_t *bad_read) {
    void *d_recs, *d_payload;
    int rc;
    if ((rc = ensure(ctx, WS_STAGE_RECS, (total + 1) * 8, &d_recs))) return rc;
    uint64_t *d_roffs = (uint64_t *)d_offs + (n_reads + 1);
    rc = encode4_impl(ctx, d_bases, d_offs, n_reads, total, (uint64_t *)d_recs, total + 1, d_roffs);
    if (rc) return rc;
    int64_t bad = -1;
    if ((rc = read_status(ctx, &bad))) {
        if (bad_read) *bad_read = bad;
        return rc;
    }
    // the payload never exceeds the records' 8 B each plus per-stream rounding, except for
    // malformed unary runs: size the device buffer for that and let the packer check
    const uint64_t n_blocks = (n_reads + block_reads - 1) / block_reads;
    uint64_t nrec = 0;  // the status box of the encode call holds it (k_emit4 wrote offsets from 0)
    if (ctx->box_valid) nrec = ((volatile uint64_t *)ctx->h_box)[1];
    else HIP_TRY(ctx, hipMemcpy(&nrec, d_roffs + n_reads, 8, hipMemcpyDeviceToHost));
    const uint64_t ends[2] = {0, nrec};
    uint64_t cap = nrec * 10 + n_blocks * 64 + 64, used = 0;
    for (int attempt = 0;; attempt++) {
        if ((rc = ensure(ctx, WS_PACK_PAYLOAD, cap, &d_payload))) return rc;
        rc = pack_blocks_impl(ctx, (const uint64_t *)d_recs, d_roffs, n_reads, block_reads, (uint8_t *)d_payload,
                              ctx->ws[WS_PACK_PAYLOAD].bytes, meta, &used, ends);
        if (rc != NTC_ERR_CAPACITY || attempt) break;
        cap = used;  // exact requirement from the first pass
    }
    if (rc) return rc;
    uint8_t *h = (uint8_t *)std::malloc(used ? used : 1);
    if (!h) return set_err(ctx, NTC_ERR_CAPACITY, "host payload allocation");
    if (used && hipMemcpy(h, d_payload, used, hipMemcpyDeviceToHost) != hipSuccess) {
        std::free(h);
        return set_err(ctx, NTC_ERR_HIP, "payload copy");
    }
    *payload = h;
    *payload_bytes = used;
    return NTC_OK;
}
}  // namespace

extern "C" {

int ntc_encode_pack_batch(ntc_ctx *ctx, const uint8_t *bases, const uint64_t *read_offsets, uint64_t n_reads,
                          uint32_t block_reads, ntc_block_meta *meta, uint8_t **payload, uint64_t *payload_bytes,
                          int64_t *bad_read) {
    if (bad_read) *bad_read = -1;
    if (!ctx || !read_offsets || !meta || !payload || !payload_bytes || block_reads == 0 || (n_reads && !bases))
        return set_err(ctx, NTC_ERR_INVALID_ARG, "null argument or block_reads = 0");
    *payload = nullptr;
    *payload_bytes = 0;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (!ctx->has_index) return set_err(ctx, NTC_ERR_NO_INDEX, "no index uploaded");
    if (ctx->encode_variant != 4) return set_err(ctx, NTC_ERR_UNSUPPORTED, "encode_pack needs encode_variant 4");
    for (uint64_t r = 0; r < n_reads; r++)
        if (read_offsets[r + 1] < read_offsets[r])
            return set_err(ctx, NTC_ERR_INVALID_ARG, "read offsets must be non-decreasing");
    if (n_reads == 0) return NTC_OK;
    const uint64_t o0 = read_offsets[0], total = read_offsets[n_reads] - o0;
    std::vector<uint64_t> offs(n_reads + 1);
    for (uint64_t r = 0; r <= n_reads; r++) offs[r] = read_offsets[r] - o0;
    void *d_bases, *d_offs;
    int rc;
    if ((rc = ensure(ctx, WS_STAGE_BASES, total + 64, &d_bases))) return rc;
    if ((rc = ensure(ctx, WS_STAGE_OFFS, (n_reads + 1) * 8 * 2, &d_offs))) return rc;
    if (total) HIP_TRY(ctx, hipMemcpyAsync(d_bases, bases + o0, total, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(d_offs, offs.data(), (n_reads + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
    return encode_pack_staged(ctx, (const uint8_t *)d_bases, (const uint64_t *)d_offs, n_reads, total, block_reads,
                              meta, payload, payload_bytes, bad_read);
}

}  // extern "C"

namespace {
// FASTQ text -> bases (WS_STAGE_BASES) + read offsets (WS_STAGE_OFFS, room for the record
// offsets behind them) in HBM, parsed on the device (fastq.hip); synchronous, so the
// structure checks are answered before anything is encoded.  *total = bases kept.
int fastq_stage(ntc_ctx *ctx, const uint8_t *fastq, uint64_t bytes, uint64_t n_reads, void **d_bases, void **d_offs,
                uint64_t *total, int64_t *bad_read) {
    if (bad_read) *bad_read = -1;
    *total = 0;
    // The parse reuses d_status and the mailbox: whatever an earlier encode or decode
    // left there is gone, so its status / counts must not be reported any more.
    ctx->box_valid = false;
    ctx->last = kNone;
    if (bytes >= (1ull << 32)) return set_err(ctx, NTC_ERR_CAPACITY, "FASTQ text of 4 GiB or more: split the batch");
    if (n_reads == 0 && bytes) return set_err(ctx, NTC_ERR_FORMAT, "FASTQ text given for zero reads");
    const uint64_t tiles = fastq_tiles(bytes);
    void *raw, *tl, *nl, *kept, *tmp;
    int rc;
    if ((rc = ensure(ctx, WS_FQ_RAW, bytes + 64, &raw))) return rc;
    if ((rc = ensure(ctx, WS_FQ_TILES, tiles * 4 + (tiles + 1) * 8 + 8, &tl))) return rc;
    if ((rc = ensure(ctx, WS_FQ_NL, 4 * n_reads * 4 + 4, &nl))) return rc;
    if ((rc = ensure(ctx, WS_FQ_KEPT, n_reads * 4 + 4, &kept))) return rc;
    if ((rc = ensure(ctx, WS_SCANTMP, scan_tmp_words(std::max(tiles, n_reads) + 1) * 8, &tmp))) return rc;
    // a sequence line is no longer than its quality line, so bases <= bytes / 2
    if ((rc = ensure(ctx, WS_STAGE_BASES, bytes / 2 + 64, d_bases))) return rc;
    if ((rc = ensure(ctx, WS_STAGE_OFFS, (n_reads + 1) * 8 * 2, d_offs))) return rc;
    FastqArgs a{};
    a.raw = (const uint8_t *)raw;
    a.n_raw = bytes;
    a.n_reads = n_reads;
    a.tile_base = (uint64_t *)tl;
    a.tile_cnt = (uint32_t *)(a.tile_base + tiles + 1);
    a.nl = (uint32_t *)nl;
    a.kept = (uint32_t *)kept;
    a.offs = (uint64_t *)*d_offs;
    a.tmp = (uint64_t *)tmp;
    a.bases = (uint8_t *)*d_bases;
    a.status = ctx->d_status;
    HIP_TRY(ctx, hipMemsetAsync(ctx->d_status, 0xFF, 8, ctx->stream));
    if (bytes) HIP_TRY(ctx, hipMemcpyAsync(raw, fastq, bytes, hipMemcpyHostToDevice, ctx->stream));
    launch_fastq_parse(a, ctx->stream);
    HIP_TRY(ctx, hipGetLastError());
    launch_status_box(ctx->d_status, a.offs + n_reads, nullptr, nullptr, ctx->h_box, ctx->stream);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const uint64_t st = ((volatile uint64_t *)ctx->h_box)[0];
    if (st != ~0ULL) {
        if (bad_read) *bad_read = (int64_t)(st >> 8);
        char buf[160];
        std::snprintf(buf, sizeof(buf), "malformed FASTQ record at index %lld", (long long)(st >> 8));
        return set_err(ctx, (int)(st & 0xFF), buf);
    }
    *total = ((volatile uint64_t *)ctx->h_box)[1];
    return NTC_OK;
}
}  // namespace

extern "C" {

int ntc_fastq_parse(ntc_ctx *ctx, const uint8_t *fastq, uint64_t fastq_bytes, uint64_t n_reads, uint8_t *bases_out,
                    uint64_t bases_capacity, uint64_t *read_offsets_out, uint64_t *n_bases, int64_t *bad_read) {
    if (bad_read) *bad_read = -1;
    if (!ctx || (fastq_bytes && !fastq) || !read_offsets_out) return set_err(ctx, NTC_ERR_INVALID_ARG, "null argument");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    void *d_bases, *d_offs;
    uint64_t total = 0;
    int rc = fastq_stage(ctx, fastq, fastq_bytes, n_reads, &d_bases, &d_offs, &total, bad_read);
    if (rc) return rc;
    if (n_bases) *n_bases = total;
    if (total > bases_capacity || (total && !bases_out))
        return set_err(ctx, NTC_ERR_CAPACITY, "bases_capacity smaller than the bases parsed");
    HIP_TRY(ctx, hipMemcpy(read_offsets_out, d_offs, (n_reads + 1) * 8, hipMemcpyDeviceToHost));
    if (total) HIP_TRY(ctx, hipMemcpy(bases_out, d_bases, total, hipMemcpyDeviceToHost));
    return NTC_OK;
}

int ntc_encode_pack_fastq(ntc_ctx *ctx, const uint8_t *fastq, uint64_t fastq_bytes, uint64_t n_reads,
                          uint32_t block_reads, ntc_block_meta *meta, uint8_t **payload, uint64_t *payload_bytes,
                          uint64_t *n_bases, int64_t *bad_read) {
    if (bad_read) *bad_read = -1;
    if (!ctx || (fastq_bytes && !fastq) || !meta || !payload || !payload_bytes || block_reads == 0)
        return set_err(ctx, NTC_ERR_INVALID_ARG, "null argument or block_reads = 0");
    *payload = nullptr;
    *payload_bytes = 0;
    if (n_bases) *n_bases = 0;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (!ctx->has_index) return set_err(ctx, NTC_ERR_NO_INDEX, "no index uploaded");
    if (ctx->encode_variant != 4) return set_err(ctx, NTC_ERR_UNSUPPORTED, "encode_pack needs encode_variant 4");
    void *d_bases, *d_offs;
    uint64_t total = 0;
    int rc = fastq_stage(ctx, fastq, fastq_bytes, n_reads, &d_bases, &d_offs, &total, bad_read);
    if (rc) return rc;
    if (n_bases) *n_bases = total;
    if (n_reads == 0) return NTC_OK;
    return encode_pack_staged(ctx, (const uint8_t *)d_bases, (const uint64_t *)d_offs, n_reads, total, block_reads,
                              meta, payload, payload_bytes, bad_read);
}

}  // extern "C"

namespace {
// bytes of ">seq.{id}\n" + read + "\n" for ids first_id .. first_id + n_reads - 1
uint64_t fasta_bytes(uint64_t n_reads, uint64_t n_bases, uint64_t first_id) {
    uint64_t need = n_bases + 7 * n_reads;  // 5 + 2 per read, plus the digits
    for (uint64_t lo = 1, d = 1; lo <= first_id + n_reads - 1 && n_reads; lo *= 10, d++) {
        const uint64_t hi = lo > UINT64_MAX / 10 ? UINT64_MAX : lo * 10 - 1;  // ids with d digits: [lo, hi]
        const uint64_t a = std::max(lo, first_id), b = std::min(hi, first_id + n_reads - 1);
        if (a <= b) need += d * (b - a + 1);
        if (hi == UINT64_MAX) break;
    }
    return need;
}

// walk + FASTA text of records already in HBM (d_recs), text D2H into out (need bytes)
int decode_fasta_dev(ntc_ctx *ctx, const uint64_t *d_recs, uint64_t n_recs, uint64_t n_reads, uint64_t n_bases,
                     uint64_t first_id, uint8_t *out, uint64_t need) {
    void *d_bases, *d_offs, *d_scan, *d_out;
    int rc;
    if ((rc = ensure(ctx, WS_FA_BASES, n_bases + 64, &d_bases))) return rc;
    if ((rc = ensure(ctx, WS_FA_OFFS, (n_reads + 2) * 8, &d_offs))) return rc;
    if ((rc = ensure(ctx, WS_FA_SCAN, (2 * (n_reads + 1) + scan_tmp_words(n_reads + 1)) * 8, &d_scan))) return rc;
    if ((rc = ensure(ctx, WS_STAGE_BASES, need + 64, &d_out))) return rc;
    if ((rc = ntc_decode_batch_device(ctx, d_recs, n_recs, (uint8_t *)d_bases, n_bases + 64, (uint64_t *)d_offs,
                                      n_reads + 2)))
        return rc;
    uint64_t *sizes = (uint64_t *)d_scan, *out_offs = sizes + (n_reads + 1), *tmp = out_offs + (n_reads + 1);
    launch_fasta((const uint8_t *)d_bases, (const uint64_t *)d_offs, n_reads, first_id, ctx->d_status, sizes, out_offs,
                 tmp, (uint8_t *)d_out, need, ctx->stream);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipMemcpyAsync(out, d_out, need, hipMemcpyDeviceToHost, ctx->stream));
    uint64_t nr = 0, nb = 0;
    if ((rc = ntc_decode_status(ctx, &nr, &nb))) return rc;  // synchronises
    if (nr != n_reads || nb != n_bases)
        return set_err(ctx, NTC_ERR_FORMAT, "records hold other read / base counts than given");
    return NTC_OK;
}
}  // namespace

namespace ntc {
int reserve_decode(ntc_ctx *ctx, uint64_t pay_bytes, uint64_t n_recs, uint8_t *host, uint64_t host_bytes) {
    if (!ctx) return NTC_ERR_INVALID_ARG;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const uint64_t pw = (pay_bytes + 7) / 8, n_bases = 40 * n_recs, need = fasta_bytes(n_recs, n_bases, 1);
    void *p;
    int rc;
    if ((rc = ensure(ctx, WS_UNP_PAY, pw * 8 + 16, &p))) return rc;
    if ((rc = ensure(ctx, WS_UNP_MARKS, pw * 8 * 8 + 128, &p))) return rc;  // marks + tile tables
    if ((rc = ensure(ctx, WS_UNP_VALS, 3 * n_recs * 8 + 8, &p))) return rc;
    if ((rc = ensure(ctx, WS_UNP_RECS, n_recs * 8 + 8, &p))) return rc;
    if ((rc = ensure(ctx, WS_FA_BASES, n_bases + 64, &p))) return rc;
    if ((rc = ensure(ctx, WS_FA_OFFS, (n_recs + 2) * 8, &p))) return rc;
    if ((rc = ensure(ctx, WS_FA_SCAN, (2 * (n_recs + 1) + scan_tmp_words(n_recs + 1)) * 8, &p))) return rc;
    if ((rc = ensure(ctx, WS_STAGE_BASES, need + 64, &p))) return rc;
    const uint64_t nc = std::min<uint64_t>({host_bytes, need + 64, 4u << 20});
    if (host && nc) {
        HIP_TRY(ctx, hipMemcpyAsync(host, p, nc, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(p, host, nc, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    return NTC_OK;
}
}  // namespace ntc

extern "C" {

int ntc_decode_fasta(ntc_ctx *ctx, const uint64_t *recs, uint64_t n_recs, uint64_t n_reads, uint64_t n_bases,
                     uint64_t first_id, uint8_t *out, uint64_t out_capacity, uint64_t *out_len) {
    if (!ctx || !out_len || (n_recs && !recs) || (n_reads && !out)) return set_err(ctx, NTC_ERR_INVALID_ARG, "null argument");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    *out_len = 0;
    if (!ctx->has_index) return set_err(ctx, NTC_ERR_NO_INDEX, "no index uploaded");
    const uint64_t need = fasta_bytes(n_reads, n_bases, first_id);
    *out_len = need;
    if (need > out_capacity) return set_err(ctx, NTC_ERR_CAPACITY, "out_capacity smaller than the FASTA text");
    if (n_recs == 0) return n_reads ? set_err(ctx, NTC_ERR_FORMAT, "reads without records") : NTC_OK;
    void *d_recs;
    int rc;
    if ((rc = ensure(ctx, WS_STAGE_RECS, n_recs * 8, &d_recs))) return rc;
    HIP_TRY(ctx, hipMemcpyAsync(d_recs, recs, n_recs * 8, hipMemcpyHostToDevice, ctx->stream));
    return decode_fasta_dev(ctx, (const uint64_t *)d_recs, n_recs, n_reads, n_bases, first_id, out, need);
}

int ntc_unpack_streams(ntc_ctx *ctx, const uint8_t *payload, uint64_t payload_bytes, const ntc_block_meta *metas,
                       uint64_t n_blocks, uint64_t *n_blocks_ok, uint64_t *n_reads, uint64_t *n_bases) {
    if (!ctx || (n_blocks && (!metas || !payload)) || !n_blocks_ok) return set_err(ctx, NTC_ERR_INVALID_ARG, "null argument");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    *n_blocks_ok = 0;
    if (n_reads) *n_reads = 0;
    if (n_bases) *n_bases = 0;
    ctx->unp_recs = 0;
    ctx->unp_reads = ctx->unp_bases = 0;
    if (n_blocks == 0) return NTC_OK;
    // stream descriptors: word offsets into the payload, value offsets, record offsets
    std::vector<UnpackStream> st(4 * n_blocks);
    std::vector<uint64_t> roff(n_blocks + 1, 0);
    uint64_t nv = 0;
    const uint64_t pay_words = (payload_bytes + 7) / 8;
    for (uint64_t b = 0; b < n_blocks; b++) {
        for (int i = 0; i < 4; i++) {
            const ntc_stream_meta &m = metas[b].stream[i];
            if ((m.offset & 7) || m.offset / 8 + m.encoded_size > pay_words)
                return set_err(ctx, NTC_ERR_INVALID_ARG, "stream outside the payload or not 8-byte aligned");
            st[4 * b + i] = UnpackStream{m.offset / 8, m.encoded_size, m.num_u64, m.param, nv};
            nv += m.num_u64;
        }
        roff[b + 1] = roff[b] + metas[b].stream[2].num_u64;  // one flag per record
    }
    void *d_pay, *d_marks, *d_st, *d_vals, *d_recs, *d_out;
    int rc;
    if ((rc = ensure(ctx, WS_UNP_PAY, pay_words * 8 + 16, &d_pay))) return rc;
    // the tiles of the streams (their tables after the marks)
    UnpackPlan plan;
    unpack_plan(st.data(), n_blocks, plan);
    if ((rc = ensure(ctx, WS_UNP_MARKS, pay_words * 8 + 128 + unpack_ws_bytes(plan), &d_marks))) return rc;
    void *d_ws = (uint8_t *)d_marks + ((pay_words * 8 + 16 + 63) & ~63ull);
    // the table upload: streams, record offsets, tile lists, stream lists
    const std::vector<UnpTile> *tl[2] = {&plan.mb_tiles, &plan.rice_tiles};
    const std::vector<UnpStreamRef> *sl[2] = {&plan.mb_streams, &plan.rice_streams};
    uint64_t up_bytes = st.size() * sizeof(UnpackStream) + (n_blocks + 1) * 8;
    for (int k = 0; k < 2; k++) up_bytes += tl[k]->size() * sizeof(UnpTile) + sl[k]->size() * sizeof(UnpStreamRef);
    std::vector<uint8_t> up(up_bytes);
    uint64_t at[4];
    {
        uint64_t q = 0;
        std::memcpy(up.data(), st.data(), st.size() * sizeof(UnpackStream));
        q += st.size() * sizeof(UnpackStream);
        std::memcpy(up.data() + q, roff.data(), (n_blocks + 1) * 8);
        q += (n_blocks + 1) * 8;
        for (int k = 0; k < 2; k++) {
            at[2 * k] = q;
            if (!tl[k]->empty()) std::memcpy(up.data() + q, tl[k]->data(), tl[k]->size() * sizeof(UnpTile));
            q += tl[k]->size() * sizeof(UnpTile);
            at[2 * k + 1] = q;
            if (!sl[k]->empty()) std::memcpy(up.data() + q, sl[k]->data(), sl[k]->size() * sizeof(UnpStreamRef));
            q += sl[k]->size() * sizeof(UnpStreamRef);
        }
    }
    if ((rc = ensure(ctx, WS_UNP_ST, up.size(), &d_st))) return rc;
    if ((rc = ensure(ctx, WS_UNP_VALS, nv * 8 + 8, &d_vals))) return rc;
    if ((rc = ensure(ctx, WS_UNP_RECS, roff[n_blocks] * 8 + 8, &d_recs))) return rc;
    uint64_t max_recs = 0;
    for (uint64_t b = 0; b < n_blocks; b++) max_recs = std::max<uint64_t>(max_recs, metas[b].stream[2].num_u64);
    const uint64_t segw = unpack_seg_words(n_blocks, max_recs);
    if ((rc = ensure(ctx, WS_UNP_OUT, n_blocks * 3 * 8 + segw * 8 + 4 * n_blocks * 4 + 8, &d_out))) return rc;
    uint64_t *d_roff = (uint64_t *)((uint8_t *)d_st + st.size() * sizeof(UnpackStream));
    uint64_t *d_out3 = (uint64_t *)d_out, *d_segc = d_out3 + 3 * n_blocks;
    int32_t *d_sst = (int32_t *)(d_segc + segw);
    HIP_TRY(ctx, hipMemcpyAsync(d_pay, payload, payload_bytes, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(d_st, up.data(), up.size(), hipMemcpyHostToDevice, ctx->stream));
    UnpackDev dv{};
    dv.payload = (const uint64_t *)d_pay;
    dv.st = (const UnpackStream *)d_st;
    dv.n_blocks = n_blocks;
    dv.max_recs = max_recs;
    dv.marks = (uint64_t *)d_marks;
    dv.mb_tiles = (const UnpTile *)((uint8_t *)d_st + at[0]);
    dv.mb_streams = (const UnpStreamRef *)((uint8_t *)d_st + at[1]);
    dv.rice_tiles = (const UnpTile *)((uint8_t *)d_st + at[2]);
    dv.rice_streams = (const UnpStreamRef *)((uint8_t *)d_st + at[3]);
    dv.n_mb_tiles = (uint32_t)plan.mb_tiles.size();
    dv.n_rice_tiles = (uint32_t)plan.rice_tiles.size();
    dv.n_mb_streams = (uint32_t)plan.mb_streams.size();
    dv.n_rice_streams = (uint32_t)plan.rice_streams.size();
    dv.ws = d_ws;
    dv.vals = (uint64_t *)d_vals;
    dv.status = d_sst;
    dv.rec_off = d_roff;
    dv.recs = (uint64_t *)d_recs;
    dv.segc = d_segc;
    dv.out3 = d_out3;
    launch_unpack(dv, ctx->stream);
    HIP_TRY(ctx, hipGetLastError());
    std::vector<uint64_t> o3(3 * n_blocks);
    HIP_TRY(ctx, hipMemcpyAsync(o3.data(), d_out3, 3 * n_blocks * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    // the blocks before the first damaged one (decode_block's Err ends the reference's loop,
    // main.rs:202); a block the host already found damaged (meta status) ends it as well
    uint64_t ok = 0, rd = 0, bs = 0;
    for (; ok < n_blocks && o3[3 * ok + 2] == 0 && metas[ok].status == 0; ok++) {
        rd += o3[3 * ok];
        bs += o3[3 * ok + 1];
    }
    *n_blocks_ok = ok;
    if (n_reads) *n_reads = rd;
    if (n_bases) *n_bases = bs;
    ctx->unp_d_recs = (uint64_t *)d_recs;
    ctx->unp_recs = roff[ok];
    ctx->unp_reads = rd;
    ctx->unp_bases = bs;
    return NTC_OK;
}

int ntc_unpacked_records(ntc_ctx *ctx, uint64_t *recs, uint64_t capacity, uint64_t *n_recs) {
    if (!ctx || !n_recs || (capacity && !recs)) return set_err(ctx, NTC_ERR_INVALID_ARG, "null argument");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    *n_recs = ctx->unp_recs;
    if (ctx->unp_recs > capacity) return set_err(ctx, NTC_ERR_CAPACITY, "capacity smaller than the unpacked records");
    if (ctx->unp_recs)
        HIP_TRY(ctx, hipMemcpy(recs, ctx->unp_d_recs, ctx->unp_recs * 8, hipMemcpyDeviceToHost));
    return NTC_OK;
}

int ntc_decode_fasta_unpacked(ntc_ctx *ctx, uint64_t first_id, uint8_t *out, uint64_t out_capacity, uint64_t *out_len) {
    if (!ctx || !out_len) return set_err(ctx, NTC_ERR_INVALID_ARG, "null argument");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    *out_len = 0;
    if (!ctx->has_index) return set_err(ctx, NTC_ERR_NO_INDEX, "no index uploaded");
    const uint64_t need = fasta_bytes(ctx->unp_reads, ctx->unp_bases, first_id);
    *out_len = need;  // (a size query: out_capacity 0)
    if (need > out_capacity) return set_err(ctx, NTC_ERR_CAPACITY, "out_capacity smaller than the FASTA text");
    if (need && !out) return set_err(ctx, NTC_ERR_INVALID_ARG, "null argument");
    if (ctx->unp_recs == 0) return ctx->unp_reads ? set_err(ctx, NTC_ERR_FORMAT, "reads without records") : NTC_OK;
    return decode_fasta_dev(ctx, ctx->unp_d_recs, ctx->unp_recs, ctx->unp_reads, ctx->unp_bases, first_id, out, need);
}

int ntc_last_timing(ntc_ctx *ctx, ntc_timing *out) {
    if (!ctx || !out) return NTC_ERR_INVALID_ARG;
    if (ctx->last == kNone) return set_err(ctx, NTC_ERR_INVALID_ARG, "no call yet");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipEventSynchronize(ctx->ev[2]));
    float a = 0, b = 0;
    std::memset(out, 0, sizeof(*out));
    if ((ctx->last == kEncode && ctx->last_variant == 4) || ctx->last == kDecode) {
        // main = the dominant kernel alone: k_ms4 (ev[3] -> ev[1]) or k_dec_rec (ev[1] -> ev[3])
        float tot = 0, ms = 0;
        HIP_TRY(ctx, hipEventElapsedTime(&tot, ctx->ev[0], ctx->ev[2]));
        if (ctx->last == kDecode) HIP_TRY(ctx, hipEventElapsedTime(&ms, ctx->ev[1], ctx->ev[3]));
        else HIP_TRY(ctx, hipEventElapsedTime(&ms, ctx->ev[3], ctx->ev[1]));
        out->main_ms = ms;
        out->aux_ms = (double)tot - (double)ms;
        out->total_ms = tot;
        out->units = ctx->last_units;
        return NTC_OK;
    }
    HIP_TRY(ctx, hipEventElapsedTime(&a, ctx->ev[0], ctx->ev[1]));
    HIP_TRY(ctx, hipEventElapsedTime(&b, ctx->ev[1], ctx->ev[2]));
    if (ctx->last == kEncode) {
        out->main_ms = a;
        out->aux_ms = b;
    } else {
        out->aux_ms = a;
        out->main_ms = b;
    }
    out->total_ms = (double)a + (double)b;
    out->units = ctx->last_units;
    return NTC_OK;
}

int ntc_device_alloc(ntc_ctx *ctx, uint64_t bytes, void **d_ptr) {
    if (!ctx || !d_ptr) return NTC_ERR_INVALID_ARG;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipMalloc(d_ptr, bytes ? bytes : 64));
    return NTC_OK;
}
int ntc_device_free(ntc_ctx *ctx, void *d_ptr) {
    if (!ctx) return NTC_ERR_INVALID_ARG;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipFree(d_ptr));
    return NTC_OK;
}
int ntc_memcpy_h2d(ntc_ctx *ctx, void *d_dst, const void *h_src, uint64_t bytes) {
    if (!ctx) return NTC_ERR_INVALID_ARG;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return NTC_OK;
}
int ntc_memcpy_d2h(ntc_ctx *ctx, void *h_dst, const void *d_src, uint64_t bytes) {
    if (!ctx) return NTC_ERR_INVALID_ARG;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return NTC_OK;
}

int ntc_debug_matching_statistics(ntc_ctx *ctx, const uint8_t *bases, const uint64_t *read_offsets,
                                  uint64_t n_reads, uint32_t *d_out, uint32_t *start_out) {
    if (!ctx || !read_offsets || !d_out || !start_out) return set_err(ctx, NTC_ERR_INVALID_ARG, "null argument");
    const uint64_t total = read_offsets[n_reads] - read_offsets[0];
    std::vector<uint64_t> recs(total + 1), roffs(n_reads + 1);
    int64_t bad = -1;
    int rc = ntc_encode_batch(ctx, bases, read_offsets, n_reads, recs.data(), total + 1, roffs.data(), &bad);
    if (rc && rc != NTC_ERR_LENGTH) return rc;
    if (ctx->encode_variant == 4) {
        void *dd, *ds;
        if ((rc = ensure(ctx, WS_DEC_A, (total + 1) * 4, &dd))) return rc;
        if ((rc = ensure(ctx, WS_DEC_B, (total + 1) * 4, &ds))) return rc;
        launch_debug_gather4(ctx->last4, (uint32_t *)dd, (uint32_t *)ds, ctx->stream);
        HIP_TRY(ctx, hipGetLastError());
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        HIP_TRY(ctx, hipMemcpy(d_out, dd, total * 4, hipMemcpyDeviceToHost));
        HIP_TRY(ctx, hipMemcpy(start_out, ds, total * 4, hipMemcpyDeviceToHost));
        return NTC_OK;
    }
    DebugArgs g{};
    g.D = (const uint8_t *)ctx->ws[WS_D].p;
    g.S = (const uint32_t *)ctx->ws[WS_S].p;
    g.tile_base = (const uint64_t *)ctx->ws[WS_TILEBASE].p;
    g.offs = (const uint64_t *)ctx->ws[WS_STAGE_OFFS].p;
    g.n_reads = n_reads;
    void *dd, *ds;
    if ((rc = ensure(ctx, WS_DEC_A, (total + 1) * 4, &dd))) return rc;
    if ((rc = ensure(ctx, WS_DEC_B, (total + 1) * 4, &ds))) return rc;
    g.d_out = (uint32_t *)dd;
    g.s_out = (uint32_t *)ds;
    launch_debug_gather(g, ctx->stream);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipMemcpy(d_out, dd, total * 4, hipMemcpyDeviceToHost));
    HIP_TRY(ctx, hipMemcpy(start_out, ds, total * 4, hipMemcpyDeviceToHost));
    return NTC_OK;
}

// ---- host-side index producer / files ---------------------------------------------------
int ntc_build_index(const uint8_t *seqs, const uint64_t *seq_offsets, uint64_t n_seqs, uint32_t k,
                    int add_revcomp, int n_threads, ntc_index_host **out) {
    if (!out || !seq_offsets || (n_seqs && !seqs)) return NTC_ERR_INVALID_ARG;
    if (k < 1 || k > 255) return NTC_ERR_UNSUPPORTED;
    *out = nullptr;
    try {
        auto *h = new ntc_index_host();
        build_index(seqs, seq_offsets, n_seqs, k, add_revcomp != 0, n_threads, h->ix);
        *out = h;
    } catch (const std::exception &e) {
        std::fprintf(stderr, "ntc_build_index: %s\n", e.what());
        return NTC_ERR_FORMAT;
    }
    return NTC_OK;
}

int ntc_build_index_device(ntc_ctx *ctx, const uint8_t *seqs, const uint64_t *seq_offsets, uint64_t n_seqs,
                           uint32_t k, int add_revcomp, ntc_index_host **out) {
    return ntc_build_index_device_ex(ctx, seqs, seq_offsets, n_seqs, k, add_revcomp, nullptr, nullptr, out);
}

int ntc_build_index_device_ex(ntc_ctx *ctx, const uint8_t *seqs, const uint64_t *seq_offsets, uint64_t n_seqs,
                              uint32_t k, int add_revcomp, const ntc_build_opts *opts, ntc_build_stats *stats,
                              ntc_index_host **out) {
    if (!ctx || !out || !seq_offsets || (n_seqs && !seqs)) return set_err(ctx, NTC_ERR_INVALID_ARG, "null argument");
    if (k < 1 || k > 255) return set_err(ctx, NTC_ERR_UNSUPPORTED, "k must be in [1, 255]");
    *out = nullptr;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    for (uint64_t i = 0; i < n_seqs; i++)
        if (seq_offsets[i + 1] < seq_offsets[i]) return set_err(ctx, NTC_ERR_INVALID_ARG, "sequence offsets decrease");
    BuildOpts o;
    if (opts) {
        o.device_budget = opts->device_budget_bytes;
        o.host_budget = opts->host_budget_bytes;
        o.max_partition_keys = opts->max_partition_keys;
        if (opts->temp_dir && *opts->temp_dir) o.temp_dir = opts->temp_dir;
    }
    if (o.temp_dir.empty()) {
        const char *t = std::getenv("TMPDIR");
        o.temp_dir = t && *t ? t : "/tmp";
    }
    auto *h = new ntc_index_host();
    std::string err;
    BuildStats st;
    const bool ok = build_index_device(ctx->stream, seqs, seq_offsets, n_seqs, k, add_revcomp != 0, o, h->ix, st, err);
    if (stats) {
        stats->occurrences = st.occurrences;
        stats->kmers = st.kmers;
        stats->sources = st.sources;
        stats->nodes = st.nodes;
        stats->spilled_bytes = st.spilled_bytes;
        stats->device_budget_bytes = st.device_budget;
        stats->pass_keys = st.pass_keys;
        stats->peak_device_bytes = st.peak_device_bytes;
        stats->kmer_partitions = st.kmer_partitions;
        stats->node_partitions = st.node_partitions;
        stats->compactions = st.compactions;
        stats->seq_uploads = st.seq_uploads;
        stats->seconds = st.seconds;
        stats->seconds_kmers = st.seconds_kmers;
        stats->seconds_sources = st.seconds_sources;
        stats->seconds_nodes = st.seconds_nodes;
        stats->seconds_labels = st.seconds_labels;
        stats->seconds_plan = st.seconds_plan;
        stats->seconds_sort = st.seconds_sort;
    }
    if (!ok) {
        delete h;
        const int code = err.rfind("hip", 0) == 0 ? NTC_ERR_HIP
                         : err.find("allocation") != std::string::npos || err.find("budget") != std::string::npos
                             ? NTC_ERR_CAPACITY
                         : err.find("temp-dir") != std::string::npos || err.find("partition file") != std::string::npos
                             ? NTC_ERR_IO
                             : NTC_ERR_FORMAT;
        return set_err(ctx, code, "ntc_build_index_device: " + err);
    }
    *out = h;
    return NTC_OK;
}

int ntc_index_set_prefix_precalc(ntc_index_host *ix, uint32_t p) {
    if (!ix || p > 12 || p > ix->ix.k) return NTC_ERR_INVALID_ARG;
    ix->ix.prefix_len = p;
    ix->ix.prefix_ranges.clear();
    if (p) prefix_table(ix->ix, p, ix->ix.prefix_ranges);
    return NTC_OK;
}

int ntc_index_prefix_table(const ntc_index_host *ix, uint32_t *p, uint64_t *ranges) {
    if (!ix || !p) return NTC_ERR_INVALID_ARG;
    *p = ix->ix.prefix_len;
    if (ranges && !ix->ix.prefix_ranges.empty())
        std::memcpy(ranges, ix->ix.prefix_ranges.data(), ix->ix.prefix_ranges.size() * 8);
    return NTC_OK;
}

void ntc_index_free(ntc_index_host *ix) { delete ix; }

int ntc_index_view_of(const ntc_index_host *ix, ntc_index_view *v) {
    if (!ix || !v) return NTC_ERR_INVALID_ARG;
    v->n_nodes = ix->ix.n;
    v->k = ix->ix.k;
    v->reserved = 0;
    for (int c = 0; c < 4; c++) {
        v->rows[c] = ix->ix.rows[c].data();
        v->C[c] = ix->ix.C[c];
    }
    v->lcs = ix->ix.lcs.data();
    return NTC_OK;
}

int ntc_index_save(const ntc_index_host *ix, const char *prefix) {
    if (!ix || !prefix) return NTC_ERR_INVALID_ARG;
    std::string err;
    if (!save_index(ix->ix, prefix, err)) {
        std::fprintf(stderr, "ntc_index_save: %s\n", err.c_str());
        return NTC_ERR_IO;
    }
    return NTC_OK;
}

int ntc_index_save_as(const ntc_index_host *ix, const char *prefix, int layout) {
    if (!ix || !prefix || (layout != kIndexOwn && layout != kIndexSbwtRs)) return NTC_ERR_INVALID_ARG;
    std::string err;
    if (!save_index_as(ix->ix, prefix, layout, err)) {
        std::fprintf(stderr, "ntc_index_save_as: %s\n", err.c_str());
        return NTC_ERR_IO;
    }
    return NTC_OK;
}

int ntc_index_load(const char *prefix, ntc_index_host **out) {
    if (!prefix || !out) return NTC_ERR_INVALID_ARG;
    *out = nullptr;
    auto *h = new ntc_index_host();
    std::string err;
    if (!load_index(prefix, h->ix, err)) {
        std::fprintf(stderr, "ntc_index_load: %s\n", err.c_str());
        delete h;
        return NTC_ERR_IO;
    }
    *out = h;
    return NTC_OK;
}

}  // extern "C"
