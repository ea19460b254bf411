// HIP kernels for gfx950 (MI355X): encode (matching statistics + parse + record emit),
// decode (inverse-SBWT walk), the walk-table build and device prefix scans.
// Integer/indexing path: no MFMA.  One GPU lane per read (64 reads per wave); per-read
// scratch is laid out [tile][position][lane] so that every per-position store of a wave
// is one coalesced 64-lane access (DESIGN.md "Kernels").
#include <hip/hip_runtime.h>

#include <cstdint>

#include "encode_core.h"
#include "kernels.h"

namespace ntc {

// ---------------------------------------------------------------------------------
// encode
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_encode(EncodeArgs a) {
    const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (gid >= a.n_reads) return;
    const uint64_t tile = gid >> 6;
    const uint32_t lane = (uint32_t)(gid & 63);
    uint64_t base, rows;
    if (a.tile_base) {
        base = a.tile_base[tile];
        rows = a.tile_base[tile + 1] - base;
    } else {
        base = tile * a.rows_uniform;
        rows = a.rows_uniform;
    }
    const uint64_t beg = a.offs[gid], end = a.offs[gid + 1];
    const uint64_t len64 = end >= beg ? end - beg : 0;
    LaneScratch s;
    s.D = a.D + base * 64 + lane;
    s.S = a.S + base * 64 + lane;
    s.F = a.F + (base >> 5) * 64 + lane;
    s.R = a.R + base * 64 + lane;
    int rc;
    if (end < beg || len64 > 0xFFFFFFFFull) rc = -kErrFormat;
    else rc = encode_lane(a.ix, a.bases + beg, (uint32_t)len64, (uint32_t)rows, s);
    if (rc < 0) {
        atomicMin(a.status, (unsigned long long)((gid << 8) | (uint64_t)(-rc)));
        a.rec_count[gid] = 0;
    } else {
        a.rec_count[gid] = (uint32_t)rc;
    }
}

// ---- encode pipeline --------------------------------------------------------------
// The batch's bases as 2-bit codes (position space: character x = batch position x), 32
// per thread.  Bad bytes (non-ACGT or a character no node ends with) report the read that
// holds them.
__device__ __forceinline__ void pack_report_bad(const Enc4Args &a, const uint8_t *B, uint64_t x0, uint32_t n,
                                                uint32_t absent) {
    for (uint32_t t = 0; t < n; t++) {
        if (!is_acgt(B[x0 + t]) || ((absent >> fast_code(B[x0 + t])) & 1u)) {  // its read
            uint64_t lo = 0, hi = a.n_reads;
            const uint64_t pos = a.offs[0] + x0 + t;
            while (hi - lo > 1) {
                const uint64_t mid = (lo + hi) >> 1;
                if (a.offs[mid] <= pos) lo = mid; else hi = mid;
            }
            atomicMin(a.status, (unsigned long long)((lo << 8) | (uint64_t)kErrInvalidBase));
            return;
        }
    }
}

// 4 ASCII bases -> 8 bits of 2-bit codes (SWAR); ok = all four are A/C/G/T present in the index
__device__ __forceinline__ uint32_t pack4(uint32_t w, uint32_t absent_tab, bool &ok) {
    const uint32_t t = ((w >> 1) ^ (w >> 2)) & 0x03030303u;  // A,C,G,T -> 0,1,2,3 per byte
    ok &= __builtin_amdgcn_perm(0u, 0x54474341u, t) == w;     // code -> "ACGT"[code] round trip
    ok &= __builtin_amdgcn_perm(0u, absent_tab, t) == 0u;     // absent characters
    const uint32_t u = t | (t >> 6);
    return (u | (u >> 12)) & 0xFFu;
}

#ifndef NTC_PACK16
#define NTC_PACK16 1  // k_pack: 16 characters per thread (one coalesced uint4 load, one u32 store)
#endif
#if NTC_PACK16
// Thread t packs characters [16t, 16t + 16) into the 32-bit half t of the 2-bit stream (Q
// word t / 2, low half for even t).  A 16-byte aligned batch start (uniform over the grid)
// takes the fast path: one aligned uint4 load per lane, a wave reading 1 KB contiguous;
// otherwise two aligned loads are realigned per byte.  Halves past the batch's last
// character, up to the end of its last Q word, are written as zero.  `bound` (>= the
// batch's bases) only sizes the grid; the true count is offs[n] - offs[0].
__global__ __launch_bounds__(256) void k_pack(Enc4Args a, uint64_t bound) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t x0 = t * 16;
    const uint64_t total = a.offs[a.n_reads] - a.offs[0];
    (void)bound;
    if (t >= 2 * ((total + 31) / 32)) return;
    uint32_t *Q32 = reinterpret_cast<uint32_t *>(a.Q);
    if (x0 >= total) {
        Q32[t] = 0u;
        return;
    }
    const uint8_t *B = a.bases + a.offs[0];
    const uint32_t absent = a.ix.absent;
    const uint32_t n = total - x0 < 16 ? (uint32_t)(total - x0) : 16u;
    if ((((uintptr_t)B) & 15) == 0 && n == 16) {
        const uint32_t absent_tab = (absent & 1u) | ((absent >> 1) & 1u) << 8 | ((absent >> 2) & 1u) << 16 |
                                    ((absent >> 3) & 1u) << 24;
        const uint4 v = *reinterpret_cast<const uint4 *>(B + x0);
        bool ok = true;
        Q32[t] = pack4(v.x, absent_tab, ok) | pack4(v.y, absent_tab, ok) << 8 | pack4(v.z, absent_tab, ok) << 16 |
                 pack4(v.w, absent_tab, ok) << 24;
        if (!ok) pack_report_bad(a, B, x0, 16, absent);
        return;
    }
    // unaligned start or the last partial chunk: 16-byte blocks never cross a page, so
    // reading a whole block that holds the batch's last byte stays inside its allocation
    const uint8_t *end = B + total;
    const uint8_t *p = B + x0;
    const uintptr_t al = (uintptr_t)p & ~(uintptr_t)15;
    const uint32_t sh = (uint32_t)((uintptr_t)p & 15);
    uint32_t w[8];
#pragma unroll
    for (int q = 0; q < 2; q++) {
        const uint8_t *blk = (const uint8_t *)(al + 16 * q);
        if (blk < end) {
            const uint4 v = *reinterpret_cast<const uint4 *>(blk);
            w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
        } else {
            w[4 * q] = w[4 * q + 1] = w[4 * q + 2] = w[4 * q + 3] = 0x41414141u;
        }
    }
    uint32_t acc = 0;
    bool bad = false;
#pragma unroll
    for (uint32_t c = 0; c < 16; c++) {
        const uint32_t o = sh + c;
        const uint32_t word = o >> 2;
        uint32_t wv = w[0];
#pragma unroll
        for (uint32_t q = 1; q < 8; q++) wv = (word == q) ? w[q] : wv;
        const uint32_t ch = (wv >> (8 * (o & 3))) & 0xFFu;
        if (c < n) {
            bad |= !is_acgt(ch) || ((absent >> fast_code(ch)) & 1u);
            acc |= fast_code(ch) << (2 * c);
        }
    }
    Q32[t] = acc;
    if (bad) pack_report_bad(a, B, x0, n, absent);
}
#else
// Thread b packs characters [32b, 32b + 32).  `bound` (>= the batch's bases) only sizes
// the grid; the true count is offs[n] - offs[0].  A 16-byte aligned batch start (uniform
// over the grid) takes the fast path: two aligned uint4 loads, consecutive lanes reading
// consecutive 32-byte chunks; otherwise three aligned loads are realigned per byte.
__global__ __launch_bounds__(256) void k_pack(Enc4Args a, uint64_t bound) {
    const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t x0 = b * 32;
    if (x0 >= bound) return;
    const uint64_t total = a.offs[a.n_reads] - a.offs[0];
    if (x0 >= total) return;
    const uint8_t *B = a.bases + a.offs[0];
    const uint32_t absent = a.ix.absent;
    const uint32_t n = total - x0 < 32 ? (uint32_t)(total - x0) : 32u;
    if ((((uintptr_t)B) & 15) == 0 && n == 32) {
        const uint32_t absent_tab = (absent & 1u) | ((absent >> 1) & 1u) << 8 | ((absent >> 2) & 1u) << 16 |
                                    ((absent >> 3) & 1u) << 24;
        const uint4 v0 = *reinterpret_cast<const uint4 *>(B + x0);
        const uint4 v1 = *reinterpret_cast<const uint4 *>(B + x0 + 16);
        bool ok = true;
        const uint32_t lo = pack4(v0.x, absent_tab, ok) | pack4(v0.y, absent_tab, ok) << 8 |
                            pack4(v0.z, absent_tab, ok) << 16 | pack4(v0.w, absent_tab, ok) << 24;
        const uint32_t hi = pack4(v1.x, absent_tab, ok) | pack4(v1.y, absent_tab, ok) << 8 |
                            pack4(v1.z, absent_tab, ok) << 16 | pack4(v1.w, absent_tab, ok) << 24;
        a.Q[b] = (uint64_t)lo | ((uint64_t)hi << 32);
        if (!ok) pack_report_bad(a, B, x0, 32, absent);
        return;
    }
    // unaligned start or the last partial chunk: 16-byte blocks never cross a page, so
    // reading a whole block that holds the batch's last byte stays inside its allocation
    const uint8_t *end = B + total;
    const uint8_t *p = B + x0;
    const uintptr_t al = (uintptr_t)p & ~(uintptr_t)15;
    const uint32_t sh = (uint32_t)((uintptr_t)p & 15);
    uint32_t w[12];
#pragma unroll
    for (int q = 0; q < 3; q++) {
        const uint8_t *blk = (const uint8_t *)(al + 16 * q);
        if (blk < end) {
            const uint4 v = *reinterpret_cast<const uint4 *>(blk);
            w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
        } else {
            w[4 * q] = w[4 * q + 1] = w[4 * q + 2] = w[4 * q + 3] = 0x41414141u;
        }
    }
    uint64_t acc = 0;
    bool bad = false;
#pragma unroll
    for (uint32_t t = 0; t < 32; t++) {
        const uint32_t o = sh + t;
        const uint32_t word = o >> 2;
        uint32_t wv = w[0];
#pragma unroll
        for (uint32_t q = 1; q < 12; q++) wv = (word == q) ? w[q] : wv;
        const uint32_t ch = (wv >> (8 * (o & 3))) & 0xFFu;
        if (t < n) {
            bad |= !is_acgt(ch) || ((absent >> fast_code(ch)) & 1u);
            acc |= (uint64_t)fast_code(ch) << (2 * t);
        }
    }
    a.Q[b] = acc;
    if (bad) pack_report_bad(a, B, x0, n, absent);
}
#endif

constexpr uint32_t kPoolChunk = 64;

// Work queues of the persistent kernels: the items are split into kQueues contiguous ranges,
// each with its own head (64 B apart, zeroed per call); block b drains queue b % nq.  One
// head for the whole grid serialises every wave's atomicAdd on one address (device-scope
// atomics on MI355X run at the memory side), which costs milliseconds at 10^5..10^6 grabs.
constexpr uint32_t kQueues = 8;       // = XCDs: consecutive blocks land on different XCDs
constexpr uint32_t kQueueStride = 8;  // u64 words between heads
struct WaveQueue {
    unsigned long long *head;
    uint64_t lo, hi;  // this queue's items
    __device__ WaveQueue(unsigned long long *heads, uint64_t n) {
        const uint32_t nq = gridDim.x < kQueues ? gridDim.x : kQueues, q = blockIdx.x % nq;
        head = heads + (uint64_t)q * kQueueStride;
        lo = n * q / nq;
        hi = n * (q + 1) / nq;
    }
    // next chunk [b, e) for the wave (lane 0 grabs, all lanes get it); false when drained,
    // leaving b and e untouched (the pool stays empty: b == e)
    __device__ bool grab(uint32_t lane, uint32_t chunk, uint64_t &b, uint64_t &e) const {
        unsigned long long got = 0;
        if (lane == 0) got = atomicAdd(head, (unsigned long long)chunk);
        // lane 0's value into scalar registers: the pool bounds stay wave-uniform (SGPRs)
        got = ((unsigned long long)__builtin_amdgcn_readfirstlane((uint32_t)(got >> 32)) << 32) |
              __builtin_amdgcn_readfirstlane((uint32_t)got);
        const uint64_t nb = lo + got;
        if (nb >= hi) return false;
        b = nb;
        e = nb + chunk < hi ? nb + chunk : hi;
        return true;
    }
};

// entries of read r (k_ms4: in entry 0's dk, MsLane::finish; the count array past kNeInE0)
__device__ __forceinline__ uint32_t read_entry_count(const Enc4Args &a, uint64_t r) {
#if NTC_ECOMB
    const uint32_t c = entry0_count(load_entry(a.Ed + r * kEntSlot, 0));
    return c == kNeInE0 ? a.ne[r] : c;
#else
    return a.ne[r];
#endif
}

#ifndef NTC_PARSE_WAVES
#define NTC_PARSE_WAVES 8  // waves per SIMD k_parse4 is compiled for (62 VGPRs, no scratch)
#endif
#ifndef NTC_PARSE_DC
#define NTC_PARSE_DC 1  // k_parse4 holds each read's dense entry group in registers
#endif
// parse of read r (k_parse4's body); returns its record count (0 on error)
__device__ __forceinline__ uint32_t parse_one(const Enc4Args &a, uint64_t r) {
    const uint64_t o0 = a.offs[0], b = a.offs[r], e = a.offs[r + 1];
    const uint64_t P = b - o0;
#if NTC_PARSE_DC && NTC_ECOMB
    // the read's dense group (its first 4 entries, entry 0 with the count) in one round trip
    Entry pre[kEntSlot];
#pragma unroll
    for (uint32_t j = 0; j < kEntSlot; j++) pre[j] = load_entry(a.Ed + r * kEntSlot, (int32_t)j);
    const uint32_t c0 = entry0_count(pre[0]);
    const uint32_t ne = c0 == kNeInE0 ? a.ne[r] : c0;
#else
    const uint32_t ne = read_entry_count(a, r);
    const Entry *pre = nullptr;
#endif
    const RecPool rp{a.R, a.rcap, a.counter + kPoolCntR, a.rbase, a.status, r};
    const Entry *E1 = a.Es + r * a.S - kEntSlot;
    const Entry *E2 = ne > kEntSlot + a.S ? a.Ep + a.obase[r] - kEntSlot - a.S : nullptr;
    const int rc = parse_read(a.ix, a.Q, P, E1, ne, (uint32_t)(e - b), a.R2 + r, nullptr, a.n_reads,
                              a.Ed + r * kEntSlot, 1, pre, E2, a.S, &rp);
    if (rc < 0) {
        atomicMin(a.status, (unsigned long long)((r << 8) | (uint64_t)(-rc)));
        a.rec_count[r] = 0;
        return 0;
    }
    a.rec_count[r] = (uint32_t)rc;
    return (uint32_t)rc;
}

// waves per SIMD k_ms4 is compiled for: without joint runs 7 with the query-word cache (72 VGPRs,
// no scratch, 20 KB of LDS per block; 8 at 64 VGPRs without it, 8 blocks = the CU's 160 KB), with
// them 7 (72 VGPRs, no scratch, 22 KB of LDS).  The
// joint build's lane state fits 72 since round 5 (32-bit read id, the overflow reservation read
// back from obase, the binary search's best interval in LDS, the queue bounds in SGPRs): A/B on
// one box, S91 k_ms4 10.71 -> 10.42 ms at 7 waves; C91 unchanged at 8 (2.69 -> 2.68 ms)
#ifndef NTC_MS_WAVES
#define NTC_MS_WAVES (NTC_QCACHE ? 7 : 8)  // the query-word cache takes 72 VGPRs (encode_core.h)
#endif
#ifndef NTC_MS_WAVES_J
#define NTC_MS_WAVES_J 7
#endif
template <bool kJoint>
__global__ __launch_bounds__(256, kJoint ? NTC_MS_WAVES_J : NTC_MS_WAVES) void k_ms4(Enc4Args a) {
    const uint32_t lane = threadIdx.x & 63;
    if (*a.status != ~0ull) return;  // a read failed to pack: nothing to do
    const uint64_t o0 = a.offs[0];
    uint64_t pool_lo = 0, pool_hi = 0;
    bool exhausted = false, idle = true;
    const WaveQueue wq(a.counter, a.n_reads);
    __shared__ uint4 s_stage[(kStageSlots + 1) * 256];  // MsLane::put_entry write combining, entry 0
    // (joint build) the binary search's best interval: 2 KB per block, 7 blocks per CU at 7 waves
    // per SIMD = 157.5 KB of the 160 KB of LDS
    __shared__ uint2 s_best[kJoint ? 256 : 1];
    // dense slots read-major, secondary slots and the overflow pool sized by need
    const MsBufs bufs{a.Q,    a.Es,    a.Ed,      1,   s_stage, kEntSlot, a.S, a.Ep, a.pcap, a.counter + kPoolCntE,
                      a.obase, a.status, s_best};
    MsLaneT<kJoint> st;
    for (;;) {
        // ---- hand idle lanes the next reads (wave-uniform control flow) ----------------
        const uint64_t want = __ballot(idle);
        if (want) {
            if (pool_lo >= pool_hi && !exhausted) exhausted = !wq.grab(lane, kPoolChunk, pool_lo, pool_hi);
            const uint32_t rank = (uint32_t)__popcll(want & ((1ULL << lane) - 1));
            const uint64_t avail = pool_hi - pool_lo;
            if (idle && rank < avail) {
                const uint64_t rd = pool_lo + rank;
                idle = false;
                const uint64_t b = a.offs[rd], e = a.offs[rd + 1];
                const uint64_t P = b - o0;
                st.start(a.ix, P, (uint32_t)(e - b), rd, e > b ? a.Q : nullptr);
                if (e <= b) {  // empty read (EncodeError, encode.rs:133-135) or bad offsets
                    atomicMin(a.status, (unsigned long long)((rd << 8) | (uint64_t)(e == b ? kErrEmptyRead : kErrFormat)));
                    a.ne[rd] = 0;
                    idle = true;
                }
            }
            const uint64_t took = (uint64_t)__popcll(want);
            pool_lo += took < avail ? took : avail;
        }
        const bool done = __ballot(!idle) == 0 && exhausted;
        if (done) break;
        // ---- one unit of work per busy lane --------------------------------------------
        if (!idle) {
            const int rc = st.step(a.ix, bufs);
            if (rc != 0) {
                if (rc < 0) {
                    atomicMin(a.status, (unsigned long long)(((uint64_t)st.rid << 8) | (uint64_t)(-rc)));
                    a.ne[st.rid] = 0;
                } else if (st.finish(bufs)) {
                    a.ne[st.rid] = st.ne;
                }
                idle = true;
            }
        }
    }
}

__global__ __launch_bounds__(256, NTC_PARSE_WAVES) void k_parse4(Enc4Args a) {
    const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t cnt = 0;
    if (r < a.n_reads) {
        if (*a.status != ~0ull) a.rec_count[r] = 0;
        else cnt = parse_one(a, r);
    }
    // the wave's record total: k_emit4 turns the scanned totals into record offsets
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if ((threadIdx.x & 63) == 0 && r < a.n_reads) a.wave_cnt[r >> 6] = cnt;
}

// record offsets = scanned wave totals + a wave scan of the reads' counts
#ifndef NTC_EMIT_STAGE
#define NTC_EMIT_STAGE 1  // k_emit4 gathers a wave's records in LDS and stores them coalesced
#endif
#if NTC_EMIT_STAGE
constexpr uint32_t kEmitStage = 64 * kRecSlot;  // records a wave stages (more: direct stores)
#endif
__global__ __launch_bounds__(256) void k_emit4(Enc4Args a, const uint64_t *wave_off, uint64_t *rec_offsets,
                                               uint64_t *out, uint64_t capacity) {
    const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    // every load first and unconditional (clamped index): the count, the wave's offset, the
    // status and the first kEmitEarly record slots (record j of read r at R2[j * n_reads + r],
    // coalesced over the wave); a load under a branch or between dependent stores would be
    // its own round trip
    constexpr uint32_t kEmitEarly = 4;
    const uint64_t rc = r < a.n_reads ? r : a.n_reads - 1;
    const uint32_t cnt0 = a.rec_count[rc];
    const uint64_t woff = wave_off[rc >> 6];
    const unsigned long long st = *a.status;
    const uint64_t *slot = a.R2 + rc;
    uint64_t early[kEmitEarly];
#pragma unroll
    for (uint32_t j = 0; j < kEmitEarly; j++) early[j] = slot[(uint64_t)j * a.n_reads];
    const uint32_t cnt = r < a.n_reads ? cnt0 : 0u;
    uint32_t inc = cnt;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += t;
    }
    const uint64_t off = woff + (inc - cnt);
    if (r < a.n_reads) {
        rec_offsets[r] = off;
        if (r + 1 == a.n_reads) rec_offsets[r + 1] = off + cnt;
    }
    const uint32_t ns = cnt < kRecSlot ? cnt : kRecSlot;
#if NTC_EMIT_STAGE
    // The wave's records are one contiguous range [woff, woff + total) of the output.  Each
    // lane's records sit ~31 B apart from its neighbours', so stores straight from the lanes
    // touch every line once per record index; gathered in LDS, the wave stores the range as
    // consecutive 8-byte words (512 B per instruction).
    __shared__ uint64_t s_rec[4][kEmitStage];
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t total = __shfl(inc, 63, 64);
    const bool staged = st == ~0ull && total <= kEmitStage && woff + total <= capacity;  // wave-uniform
    if (staged && r < a.n_reads) {
        uint64_t *dst = s_rec[wv] + (inc - cnt);
#pragma unroll
        for (uint32_t j = 0; j < kEmitEarly; j++)
            if (j < ns) dst[j] = early[j];
        for (uint32_t j = kEmitEarly; j < ns; j++) dst[j] = slot[(uint64_t)j * a.n_reads];
        if (cnt > kRecSlot) {
            const uint64_t *spill = a.R + a.rbase[r] - kRecSlot;
            for (uint32_t j = kRecSlot; j < cnt; j++) dst[j] = spill[j];
        }
    }
    __syncthreads();
    if (staged) {
        for (uint32_t i = lane; i < total; i += 64) out[woff + i] = s_rec[wv][i];
        return;
    }
#endif
    if (r >= a.n_reads) return;
    if (st != ~0ull) return;  // a read failed: the call reports that, no records
    if (off + cnt > capacity) {
        atomicMin(a.status, (unsigned long long)((r << 8) | (uint64_t)kErrCapacity));
        return;
    }
#pragma unroll
    for (uint32_t j = 0; j < kEmitEarly; j++)
        if (j < ns) out[off + j] = early[j];
    for (uint32_t j = kEmitEarly; j < ns; j++) out[off + j] = slot[(uint64_t)j * a.n_reads];
    if (cnt > kRecSlot) {
        const uint64_t *spill = a.R + a.rbase[r] - kRecSlot;
        for (uint32_t j = kRecSlot; j < cnt; j++) out[off + j] = spill[j];
    }
}

// the call's status and up to two counts into the host mailbox (pinned memory): thread t
// writes word t with a vector store; the host reads it after one stream sync
__global__ __launch_bounds__(64) void k_status_box(const unsigned long long *status, const uint64_t *a,
                                                   const uint64_t *b, const uint64_t *c, uint64_t *box) {
    const uint32_t t = threadIdx.x;
    if (t >= 4) return;
    const uint64_t *src = t == 1 ? a : t == 2 ? b : c;
    const uint64_t v = t == 0 ? (uint64_t)*status : (src ? *src : 0);
    box[t] = v;  // per-lane address: a vector store
}
void launch_status_box(const unsigned long long *status, const uint64_t *a, const uint64_t *b, const uint64_t *c,
                       uint64_t *box, hipStream_t s) {
    hipLaunchKernelGGL(k_status_box, dim3(1), dim3(64), 0, s, status, a, b, c, box);
}

// rows of scratch a tile of 64 reads needs = longest read, rounded up to 32
__global__ __launch_bounds__(256) void k_tile_rows(const uint64_t *offs, uint64_t n_reads,
                                                   uint32_t *tile_rows) {
    const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t tile = gid >> 6;
    if (tile * 64 >= n_reads) return;
    uint64_t len = 0;
    if (gid < n_reads) {
        const uint64_t b = offs[gid], e = offs[gid + 1];
        len = e > b ? e - b : 0;
    }
    uint32_t v = len > 0xFFFFFFE0ull ? 0xFFFFFFE0u : (uint32_t)len;
    for (int o = 32; o > 0; o >>= 1) {
        uint32_t t = __shfl_xor(v, o, 64);
        v = t > v ? t : v;
    }
    if ((gid & 63) == 0) tile_rows[tile] = (v + 31) & ~31u;
}

__global__ __launch_bounds__(256) void k_emit(EmitArgs a) {
    const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (gid >= a.n_reads) return;
    const uint64_t tile = gid >> 6;
    const uint32_t lane = (uint32_t)(gid & 63);
    const uint64_t base = a.tile_base ? a.tile_base[tile] : tile * a.rows_uniform;
    const uint32_t cnt = a.rec_count[gid];
    const uint64_t off = a.rec_offsets[gid];
    if (off + cnt > a.capacity) {
        atomicMin(a.status, (unsigned long long)((gid << 8) | (uint64_t)kErrCapacity));
        return;
    }
    const uint64_t *src = a.R + base * 64 + lane;
    for (uint32_t j = 0; j < cnt; j++) a.out[off + j] = src[(uint64_t)j * 64];
}

__global__ __launch_bounds__(256) void k_debug_gather(DebugArgs a) {
    const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (gid >= a.n_reads) return;
    const uint64_t tile = gid >> 6;
    const uint32_t lane = (uint32_t)(gid & 63);
    const uint64_t base = a.tile_base ? a.tile_base[tile] : tile * a.rows_uniform;
    const uint64_t b = a.offs[gid], e = a.offs[gid + 1];
    for (uint64_t p = 0; p < e - b; p++) {
        a.d_out[b + p] = a.D[(base + p) * 64 + lane];
        a.s_out[b + p] = a.S[(base + p) * 64 + lane];
    }
}

// ---- decode index: per 256-record tile, the number of first records and of bases --------
__device__ __forceinline__ void dec_desc(uint64_t w, uint64_t &f, uint64_t &len) {
    const uint32_t flag = (uint32_t)(w >> 56);
    f = flag & 1u;
    len = (flag & 2u) ? (flag >> 2) : ((uint32_t)(w >> 32) & 0xFFFFFFu);
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}


// one wave per tile: 4 coalesced loads per lane, wave sums
__global__ __launch_bounds__(256) void k_dec_tiles(const uint64_t *recs, uint64_t n, uint64_t *pf, uint64_t *pl) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t t = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t * kDecTileRecs >= n) return;  // whole wave
    // all loads unconditional (clamped, masked after): a load under `if (r < n)` is waited for
    // inside its branch, which serialised the tile's eight loads into eight round trips
    uint64_t w[kDecTileRecs / 64];
#pragma unroll
    for (uint32_t q = 0; q < kDecTileRecs / 64; q++) {
        const uint64_t r = t * kDecTileRecs + q * 64 + lane;
        w[q] = recs[r < n ? r : n - 1];
    }
    uint64_t sf = 0, sl = 0;
#pragma unroll
    for (uint32_t q = 0; q < kDecTileRecs / 64; q++) {
        uint64_t f, l;
        dec_desc(w[q], f, l);
        const bool in = t * kDecTileRecs + q * 64 + lane < n;
        sf += in ? f : 0;
        sl += in ? l : 0;
    }
    sf = wave_sum64(sf);
    sl = wave_sum64(sl);
    if (lane == 0) {
        pf[t] = sf;
        pl[t] = sl;
    }
}

__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t &total);

// ---------------------------------------------------------------------------------
// decode
// ---------------------------------------------------------------------------------
// Records are independent once their output offsets are known.  A read's records are
// consumed last to first (lib.rs:266), so record r of read rid lands at start(rid) +
// (end(rid) - E[r + 1]), with E the exclusive scan of lengths in record order and
// start/end(rid) the read's output range.  A block owns one tile of kDecTileRecs records,
// kDecR consecutive ones per thread (coalesced loads, and kDecR independent walk chains per
// lane), and derives E, rid and the reads' ranges from the tile scans (k_dec_tiles) plus a
// block scan; the read open at the tile start and the read running past its end are found
// by scanning records outward.  Output is staged per block (StageWriter): the block's
// records cover a contiguous stretch of output words (with at most a few words shared with
// neighbouring blocks); codes are OR-ed into LDS, then the block writes each word's ASCII
// once.  A block whose stretch exceeds kDecStageWords (very long records) writes ASCII
// directly.
__global__ __launch_bounds__(256) void k_dec_rec(DecWalkArgs a) {
    constexpr uint32_t R = kDecR;
    __shared__ uint64_t s_bits[kDecStageWords];
    __shared__ uint32_t s_mask[kDecStageWords];
    __shared__ uint64_t s_lo[4], s_hi[4];
    __shared__ uint64_t s_start[kDecTileRecs];  // output offset of each read starting in the tile
    __shared__ uint64_t s_open[2];              // start of the read open at the tile start, end of the last read
    __shared__ uint32_t s_failed;
    // Another block may set the status at any time (format errors below), so one load
    // decides for the whole block: waves must not diverge on it before the barriers.
    if (threadIdx.x == 0) s_failed = *(volatile unsigned long long *)a.status != ~0ull;
    __syncthreads();
    if (s_failed) return;
    const uint64_t n = a.n, tiles = (n + kDecTileRecs - 1) / kDecTileRecs, t = blockIdx.x;
    const uint64_t reads = a.pfs[tiles], bases = a.pls[tiles];
    if (reads + 1 > a.offs_capacity || bases > a.bases_capacity) {  // every block: nothing is written
        if (t == 0 && threadIdx.x == 0) atomicMin(a.status, (unsigned long long)kErrCapacity);
        return;
    }
    // the tile's prefixes, loaded before the walk entries below: the wait for them (in-order
    // vmcnt) then leaves the walk loads in flight
    const uint64_t pf_t = a.pfs[t], pl_t = a.pls[t];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t r0 = t * kDecTileRecs, rb = r0 + (uint64_t)threadIdx.x * R;  // this thread's records
    const uint64_t r1 = r0 + kDecTileRecs < n ? r0 + kDecTileRecs : n;
    // Every load below is unconditional (indices clamped into range, results masked after):
    // a load under a branch makes hipcc wait for it inside the branch, which would serialise
    // the records, the walk entries and the scan window into separate round trips.
    uint64_t w[R], f[R], len[R];
#pragma unroll
    for (uint32_t i = 0; i < R; i++) w[i] = a.recs[rb + i < n ? rb + i : n - 1];
    // the first 64-record window of the outward scans (waves 0 and 1)
    const int64_t wi = wave == 0 ? (int64_t)r0 - 64 + lane : (int64_t)(r1 + lane);
    const uint64_t wraw = a.recs[wi < 0 ? 0 : ((uint64_t)wi < n ? (uint64_t)wi : n - 1)];
    // the first walk entry of each long record, issued before the index prologue so that its
    // latency overlaps the scans
    bool is_long[R];
    WalkEntry e0[R];
#pragma unroll
    for (uint32_t i = 0; i < R; i++) {
        if (rb + i >= n) w[i] = 0;
        dec_desc(w[i], f[i], len[i]);
        if (rb + i >= n) f[i] = len[i] = 0;
        is_long[i] = len[i] > 0 && !((w[i] >> 56) & 2) && (uint32_t)w[i] < a.ix.n;
        e0[i] = walk_at(a.ix, is_long[i] ? (uint32_t)w[i] : 0u);
    }
    const uint64_t wpre = (wave == 0 && wi >= 0) || (wave == 1 && (uint64_t)wi < n) ? wraw : 0;
    // E[r] (bases before record r) and the read of r, from the tile scans + a block scan
    uint64_t sf = 0, sl = 0;
#pragma unroll
    for (uint32_t i = 0; i < R; i++) {
        sf += f[i];
        sl += len[i];
    }
    uint64_t tf, tl;
    uint64_t cf = block_excl_scan(sf, tf);
    uint64_t cl = block_excl_scan(sl, tl);
    uint64_t Er[R];
    int64_t li[R];  // read index within the tile (-1: the read open at r0)
    uint64_t rid[R];
#pragma unroll
    for (uint32_t i = 0; i < R; i++) {
        Er[i] = pl_t + cl;
        rid[i] = pf_t + cf + f[i] - 1;  // a record belongs to the last first record at or before it
        li[i] = (int64_t)(cf + f[i]) - 1;
        if (rb + i < n && f[i]) {
            s_start[li[i]] = Er[i];
            if (rid[i] < a.offs_capacity) a.offs_out[rid[i]] = Er[i];  // the read's output offset
        }
        cf += f[i];
        cl += len[i];
    }
    if (wave == 0) {  // start of the read open at r0: back to its first record
        uint64_t acc = 0, base = r0;
        bool open = r0 > 0 && __shfl(f[0], 0, 64) == 0;  // thread 0 holds record r0
        while (open) {
            const int64_t rr = (int64_t)base - 64 + lane;
            uint64_t ff = 0, ll = 0;
            if (rr >= 0) dec_desc(base == r0 ? wpre : a.recs[rr], ff, ll);
            const uint64_t fb = __ballot(ff != 0);
            if (fb) {
                const uint32_t hl = 63u - (uint32_t)__builtin_clzll(fb);  // nearest first record
                acc += wave_sum64(lane >= hl ? ll : 0);
                break;
            }
            acc += wave_sum64(ll);
            if (base <= 64) break;  // no first record before r0 (reported below as a format error)
            base -= 64;
        }
        if (lane == 0) s_open[0] = pl_t - acc;
    } else if (wave == 1) {  // end of the tile's last read: on to the next first record
        uint64_t acc = 0, base = r1;
        while (base < n) {
            const uint64_t rr = base + lane;
            uint64_t ff = 1, ll = 0;
            if (rr < n) dec_desc(base == r1 ? wpre : a.recs[rr], ff, ll);
            const uint64_t fb = __ballot(ff != 0);
            if (fb) {
                const uint32_t fl = (uint32_t)__builtin_ctzll(fb);
                acc += wave_sum64(lane < fl ? ll : 0);
                break;
            }
            acc += wave_sum64(ll);
            base += 64;
        }
        if (lane == 0) s_open[1] = pl_t + tl + acc;
    }
    if (t == 0 && threadIdx.x == 0 && n > 0 && !f[0])
        atomicMin(a.status, (unsigned long long)kErrFormat);  // records must start a read
    if (t + 1 == tiles && threadIdx.x == 0) a.offs_out[reads] = bases;
    __syncthreads();
    uint64_t g0[R];
    uint64_t lo = ~0ULL, hi = 0;
#pragma unroll
    for (uint32_t i = 0; i < R; i++) {
        g0[i] = 0;
        if (rb + i < n) {
            const uint64_t start = li[i] >= 0 ? s_start[li[i]] : s_open[0];
            const uint64_t end = li[i] + 1 < (int64_t)tf ? s_start[li[i] + 1] : s_open[1];
            g0[i] = start + (end - (Er[i] + len[i]));  // a read's records are consumed last to first (lib.rs:266)
        }
        if (len[i]) {
            lo = g0[i] < lo ? g0[i] : lo;
            hi = g0[i] + len[i] > hi ? g0[i] + len[i] : hi;
        }
    }
    // the block's output stretch [lo, hi)
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t l2 = __shfl_xor(lo, o, 64), h2 = __shfl_xor(hi, o, 64);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
    }
    if (lane == 0) {
        s_lo[wave] = lo;
        s_hi[wave] = hi;
    }
    __syncthreads();
    for (int q = 0; q < 4; q++) {
        lo = s_lo[q] < lo ? s_lo[q] : lo;
        hi = s_hi[q] > hi ? s_hi[q] : hi;
    }
    if (lo >= hi) return;  // no characters in this block
    const uint64_t w_lo = lo >> 5, nw = ((hi - 1) >> 5) - w_lo + 1;
    if (nw > kDecStageWords) {  // whole block: direct ASCII
#pragma unroll
        for (uint32_t i = 0; i < R; i++) {
            const uint32_t L = (uint32_t)len[i];
            if (!L) continue;
            if ((w[i] >> 56) & 2) store_codes(a.out + g0[i], w[i], L);
            else if (!walk_record(a.ix, (uint32_t)w[i], L, a.out + g0[i]))
                atomicMin(a.status, (unsigned long long)((rid[i] << 8) | (uint64_t)kErrFormat));
        }
        return;
    }
    for (uint32_t q = threadIdx.x; q < nw; q += 256) {
        s_bits[q] = 0;
        s_mask[q] = 0;
    }
    __syncthreads();
    StageWriter sw{s_bits, s_mask, w_lo};
#pragma unroll
    for (uint32_t i = 0; i < R; i++) {
        const uint32_t L = (uint32_t)len[i];
        if (!L) continue;
        if ((w[i] >> 56) & 2) {
            sw.put(g0[i], w[i], L);
        } else if (!is_long[i]) {
            atomicMin(a.status, (unsigned long long)((rid[i] << 8) | (uint64_t)kErrFormat));
        } else {  // walk_record_codes from the prefetched first entry
            uint32_t end = L;
            walk_put(end, g0[i], sw, e0[i]);
            uint32_t cur = e0[i].jump;
            while (end > 0) {
                if (cur >= a.ix.n) {
                    atomicMin(a.status, (unsigned long long)((rid[i] << 8) | (uint64_t)kErrFormat));
                    break;
                }
                const WalkEntry e = walk_at(a.ix, cur);
                walk_put(end, g0[i], sw, e);
                cur = e.jump;
            }
        }
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < nw; q += 256) stage_store_word(a.out, w_lo + q, s_bits[q], s_mask[q]);
}

// 2-bit output -> ASCII, 32 characters per thread (two 16-byte stores when the output is
// 16-byte aligned, the common case), then re-zero the word for the next call

// ---------------------------------------------------------------------------------
// walk table: W_{2m}(j) = W_m(pred^m(j)) . W_m(j)
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_walk_init(const uint32_t *pred, const uint8_t *code, uint64_t n,
                                                   WalkStep *w) {
    const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    WalkStep e;
    e.chars = code[j];
    e.jump = pred[j];
    e.older = 0;
    w[j] = e;
}

__global__ __launch_bounds__(256) void k_walk_double(const WalkStep *a, WalkStep *b, uint64_t n, uint32_t m) {
    const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const WalkStep x = a[j];
    const WalkStep y = a[x.jump];
    WalkStep o;
    o.chars = y.chars | (x.chars << (2 * m));
    o.jump = y.jump;
    o.older = 0;
    b[j] = o;
}

// 48-step entries: the 16 characters before the 32 of w32[j], from w16 at its jump
__global__ __launch_bounds__(256) void k_walk_ext(WalkStep *w32, const WalkStep *w16, uint64_t n) {
    const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    WalkStep x = w32[j];
    const WalkStep y = w16[x.jump];
    x.older = (uint32_t)y.chars;
    x.jump = y.jump;
    w32[j] = x;
}

// 112-step entries: 48 + 48 + 16 steps (walk_compose)
__global__ __launch_bounds__(256) void k_walk_final(const WalkStep *w48, const WalkStep *w16, uint64_t n,
                                                    WalkEntry *out) {
    const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const WalkStep x = w48[j];
    const WalkStep y = w48[x.jump];
    out[j] = walk_compose(x, y, w16[y.jump]);
}

// ---------------------------------------------------------------------------------
// exclusive prefix scan, out[0..n] (out[n] = total); 256 threads x 16 items per block
// ---------------------------------------------------------------------------------
constexpr int kScanThreads = 256;
constexpr int kScanItems = 16;
constexpr uint64_t kScanTile = (uint64_t)kScanThreads * kScanItems;

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int o) {
    uint32_t lo = __shfl_up((uint32_t)v, o, 64), hi = __shfl_up((uint32_t)(v >> 32), o, 64);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t &total) {
    __shared__ uint64_t wsum[kScanThreads / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t inc = v;
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t t = shfl_up64(inc, o);
        if (lane >= o) inc += t;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint64_t off = 0;
    total = 0;
    for (int w = 0; w < kScanThreads / 64; w++) {
        if (w < wave) off += wsum[w];
        total += wsum[w];
    }
    __syncthreads();
    return off + inc - v;
}

template <class T>
__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const T *in, uint64_t n, uint64_t *part) {
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; j++)
        if (base + j < n) s += (uint64_t)in[base + j];
    uint64_t total;
    block_excl_scan(s, total);
    if (threadIdx.x == 0) part[blockIdx.x] = total;
}

template <class T>
__global__ __launch_bounds__(kScanThreads) void k_scan_apply(const T *in, uint64_t n, const uint64_t *boff,
                                                             uint64_t *out) {
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
    uint64_t v[kScanItems];
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; j++) {
        v[j] = (base + j < n) ? (uint64_t)in[base + j] : 0;
        s += v[j];
    }
    uint64_t total;
    uint64_t run = block_excl_scan(s, total) + (boff ? boff[blockIdx.x] : 0);
#pragma unroll
    for (int j = 0; j < kScanItems; j++) {
        if (base + j < n) out[base + j] = run;
        run += v[j];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kScanThreads - 1) out[n] = run;
}

template <class T>
void scan_excl_t(const T *in, uint64_t n, uint64_t *out, uint64_t *tmp, hipStream_t s) {
    const uint64_t nb = (n + kScanTile - 1) / kScanTile;
    if (nb <= 1) {
        hipLaunchKernelGGL(k_scan_apply<T>, dim3(1), dim3(kScanThreads), 0, s, in, n, nullptr, out);
        return;
    }
    uint64_t *part = tmp, *part_scan = tmp + nb, *tmp2 = part_scan + nb + 1;
    hipLaunchKernelGGL(k_scan_reduce<T>, dim3((uint32_t)nb), dim3(kScanThreads), 0, s, in, n, part);
    scan_excl_t<uint64_t>(part, nb, part_scan, tmp2, s);
    hipLaunchKernelGGL(k_scan_apply<T>, dim3((uint32_t)nb), dim3(kScanThreads), 0, s, in, n,
                       (const uint64_t *)part_scan, out);
}

void launch_dec_tiles(const uint64_t *recs, uint64_t n, uint64_t *pf, uint64_t *pl, uint64_t *pfs, uint64_t *pls,
                      uint64_t *tmp, hipStream_t s) {
    const uint64_t tiles = (n + kDecTileRecs - 1) / kDecTileRecs;
    hipLaunchKernelGGL(k_dec_tiles, dim3((uint32_t)((tiles + 3) / 4)), dim3(256), 0, s, recs, n, pf, pl);
    scan_excl_t<uint64_t>(pf, tiles, pfs, tmp, s);
    scan_excl_t<uint64_t>(pl, tiles, pls, tmp, s);
}

uint64_t scan_tmp_words(uint64_t n) {
    uint64_t w = 0;
    while (true) {
        uint64_t nb = (n + kScanTile - 1) / kScanTile;
        if (nb <= 1) break;
        w += 2 * nb + 1;
        n = nb;
    }
    return w + 8;
}

void scan_excl_u32(const uint32_t *in, uint64_t n, uint64_t *out, uint64_t *tmp, hipStream_t s) {
    scan_excl_t<uint32_t>(in, n, out, tmp, s);
}
void scan_excl_u64(const uint64_t *in, uint64_t n, uint64_t *out, uint64_t *tmp, hipStream_t s) {
    scan_excl_t<uint64_t>(in, n, out, tmp, s);
}

// ---------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------
static inline dim3 grid_for(uint64_t n) { return dim3((uint32_t)((n + 255) / 256)); }

void launch_encode(const EncodeArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(k_encode, grid_for(a.n_reads), dim3(256), 0, s, a);
}
__global__ __launch_bounds__(256) void k_debug_gather4(Enc4Args a, uint32_t *d_out, uint32_t *s_out) {
    const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= a.n_reads) return;
    const uint64_t o0 = a.offs[0], b = a.offs[r], e = a.offs[r + 1];
    const uint64_t P = b - o0;
    const uint32_t ne = read_entry_count(a, r);
    const Entry *E2 = ne > kEntSlot + a.S ? a.Ep + a.obase[r] - kEntSlot - a.S : nullptr;
    read_ms(a.ix, a.Q, P, a.Es + r * a.S - kEntSlot, ne, (uint32_t)(e - b), d_out + P, s_out + P, a.Ed + r * kEntSlot,
            1, E2, a.S);
}

// two-character rank lines (encode_core.h Rank2Chunk): one thread per (block, c1) chunk
__global__ __launch_bounds__(256) void k_rank2(DevIndex ix, Rank2Chunk *out, uint64_t lines) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= lines * 4) return;
    out[i] = rank2_make(ix, i % lines, (int)(i / lines));  // c1-major
}
void launch_rank2(const DevIndex &ix, Rank2Chunk *out, hipStream_t s) {
    const uint64_t lines = rank2_blocks(ix.n);
    hipLaunchKernelGGL(k_rank2, grid_for(lines * 4), dim3(256), 0, s, ix, out, lines);
}

// suffix table level u (4^u entries) from level u - 1
__global__ __launch_bounds__(256) void k_tab_level(DevIndex ix, uint32_t u, const uint2 *prev, uint2 *cur) {
    const uint64_t key = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (key >> (2 * u)) return;
    cur[key] = tab_make(ix, u, key, prev, ix.tab_pos && u == ix.tab_u);
}

__global__ __launch_bounds__(256) void k_tab_bits(const uint2 *top, uint32_t U, uint32_t *bits) {  // level U
    const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (w >= tab_bits_words(U)) return;
    if (U >= 3) {
        bits[w] = tab_bits_word(top, w);
    } else {
        uint32_t b = 0;
        for (uint32_t key = 0; key < (1u << (2 * U)); key++) b |= (uint32_t)tab_long(top[key]) << key;
        bits[0] = b;
    }
}

__global__ __launch_bounds__(256) void k_pair_words(const uint2 *top, uint32_t U, uint32_t *out) {
    const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;  // two pair words per thread
    const uint64_t cnt = pair_words_count(U);
    if (2 * w >= cnt) return;
    uint32_t v = pair_word(top, U, 2 * w);
    if (2 * w + 1 < cnt) v |= pair_word(top, U, 2 * w + 1) << 16;
    out[w] = v;
}

void launch_pair_words(const uint2 *top, uint32_t U, uint16_t *out, hipStream_t s) {
    hipLaunchKernelGGL(k_pair_words, grid_for((pair_words_count(U) + 1) / 2), dim3(256), 0, s, top, U,
                       (uint32_t *)out);
}

// window words (encode_core.h win_word): one 32-bit word per thread, from the level-U
// presence bitmap (32 MB at U = 14, L2 / Infinity-Cache resident while this runs)
__global__ __launch_bounds__(256) void k_win_words(const uint32_t *bits, uint32_t U, uint32_t *out) {
    const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (w >= win_words_count(U) * 8) return;
    out[w] = win_word(bits, U, w >> 3, (uint32_t)(w & 7));
}

void launch_win_words(const uint32_t *bits, uint32_t U, uint32_t *out, hipStream_t s) {
    hipLaunchKernelGGL(k_win_words, grid_for(win_words_count(U) * 8), dim3(256), 0, s, bits, U, out);
}

void launch_tab_build(const DevIndex &ix, uint32_t U, uint2 *tab, uint32_t *bits, uint32_t F, uint32_t *fbits,
                      hipStream_t s) {
    for (uint32_t u = 1; u <= U; u++) {
        const uint64_t cnt = 1ULL << (2 * u);
        hipLaunchKernelGGL(k_tab_level, grid_for(cnt), dim3(256), 0, s, ix, u, u > 1 ? tab + tab_base(u - 1) : tab,
                           tab + tab_base(u));
    }
    hipLaunchKernelGGL(k_tab_bits, grid_for(tab_bits_words(U)), dim3(256), 0, s, (const uint2 *)(tab + tab_base(U)),
                       U, bits);
    if (F)
        hipLaunchKernelGGL(k_tab_bits, grid_for(tab_bits_words(F)), dim3(256), 0, s,
                           (const uint2 *)(tab + tab_base(F)), F, fbits);
}

void launch_debug_gather4(const Enc4Args &a, uint32_t *d_out, uint32_t *s_out, hipStream_t s) {
    hipLaunchKernelGGL(k_debug_gather4, grid_for(a.n_reads), dim3(256), 0, s, a, d_out, s_out);
}

int ms4_blocks_per_cu() {
    int blocks = 0;
    int bj = 0;  // both builds: the grid must fit either
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_ms4<false>, 256, 0) != hipSuccess || blocks <= 0 ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&bj, k_ms4<true>, 256, 0) != hipSuccess || bj <= 0)
        blocks = 4;
    return bj < blocks ? bj : blocks;
}

void launch_encode4(const Enc4Args &a, uint64_t total, uint32_t ms_blocks, hipStream_t s, hipEvent_t ev_ms_begin,
                    hipEvent_t ev_ms_end) {
    hipLaunchKernelGGL(k_pack, grid_for((total + 31) / 32 * (NTC_PACK16 ? 2 : 1)), dim3(256), 0, s, a, total);
    (void)hipEventRecord(ev_ms_begin, s);
    const uint64_t need = (a.n_reads + 255) / 256;
    if (a.ix.joint)
        hipLaunchKernelGGL(k_ms4<true>, dim3(need < ms_blocks ? (uint32_t)need : ms_blocks), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(k_ms4<false>, dim3(need < ms_blocks ? (uint32_t)need : ms_blocks), dim3(256), 0, s, a);
    (void)hipEventRecord(ev_ms_end, s);
    hipLaunchKernelGGL(k_parse4, grid_for(a.n_reads), dim3(256), 0, s, a);
}

void launch_emit4(const Enc4Args &a, uint64_t *wave_off, uint64_t *tmp, uint64_t *rec_offsets, uint64_t *out,
                  uint64_t capacity, hipStream_t s) {
    scan_excl_u32(a.wave_cnt, (a.n_reads + 63) / 64, wave_off, tmp, s);
    hipLaunchKernelGGL(k_emit4, grid_for(a.n_reads), dim3(256), 0, s, a, (const uint64_t *)wave_off, rec_offsets,
                       out, capacity);
}

void launch_tile_rows(const uint64_t *offs, uint64_t n_reads, uint32_t *tile_rows, hipStream_t s) {
    uint64_t threads = ((n_reads + 63) / 64) * 64;
    hipLaunchKernelGGL(k_tile_rows, grid_for(threads), dim3(256), 0, s, offs, n_reads, tile_rows);
}
void launch_emit(const EmitArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(k_emit, grid_for(a.n_reads), dim3(256), 0, s, a);
}
void launch_debug_gather(const DebugArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(k_debug_gather, grid_for(a.n_reads), dim3(256), 0, s, a);
}
void launch_dec_walk(const DecWalkArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(k_dec_rec, dim3((uint32_t)((a.n + kDecTileRecs - 1) / kDecTileRecs)), dim3(256), 0, s,
                       a);
}
void launch_walk_build(const uint32_t *pred, const uint8_t *code, uint64_t n, WalkStep *a, WalkStep *b,
                       WalkEntry *out, hipStream_t s) {
    hipLaunchKernelGGL(k_walk_init, grid_for(n), dim3(256), 0, s, pred, code, n, a);
    for (uint32_t m = 1; m < 32; m *= 2) {
        hipLaunchKernelGGL(k_walk_double, grid_for(n), dim3(256), 0, s, (const WalkStep *)a, b, n, m);
        WalkStep *t = a;
        a = b;
        b = t;
    }
    // a = 32-step entries, b = 16-step entries
    hipLaunchKernelGGL(k_walk_ext, grid_for(n), dim3(256), 0, s, a, (const WalkStep *)b, n);
    hipLaunchKernelGGL(k_walk_final, grid_for(n), dim3(256), 0, s, (const WalkStep *)a, (const WalkStep *)b, n, out);
}


// ---- path cover (derived.cpp build_paths, in parallel) ---------------------------------
// Edge z -> y when z is alone in its (k-1)-suffix group with one label and neither node
// is a dummy; every node then has at most one path in- and out-edge, so the components
// are simple paths and cycles.  List ranking by pointer jumping gives each node its start
// and distance; cycles are cut at their smallest node and ranked again.
__device__ __forceinline__ bool path_dummy(const uint32_t *bits, uint32_t z) { return (bits[z >> 5] >> (z & 31)) & 1u; }

__global__ __launch_bounds__(256) void k_path_edges(PathArgs a, uint32_t *prv) {
    const uint32_t z = blockIdx.x * 256u + threadIdx.x;
    if (z >= a.n || path_dummy(a.dummy, z)) return;
    const bool head = a.k < 2 || a.lcs[z] < a.k - 1;
    const bool alone = a.k < 2 || z + 1 == a.n || a.lcs[z + 1] < a.k - 1;
    if (!head || !alone) return;
    uint2 w[4];
    uint32_t m = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        w[c] = a.rank[(uint64_t)c * a.rwords + (z >> 5)];
        m |= ((w[c].y >> (z & 31)) & 1u) << c;
    }
    if (m == 0 || (m & (m - 1))) return;
    const int c = __builtin_ctz(m);
    const uint32_t y = rank_word(w[c], z);
    if (!path_dummy(a.dummy, y)) prv[y] = z;
}

// ---- unitig linking (derived.cpp link_unitigs, in parallel) ------------------------------
// After k_path_edges + one ranking (st) and the unitig lengths (len[start]): each unitig's
// last node t names its preferred successor y (a unitig's first node; the shortest unitig,
// then the smallest node) and offers itself to every successor y with the key (its unitig's
// length, t), kept by a 64-bit atomicMin; t -> y becomes a path edge when both choose each
// other.  Nodes on pure cycles (their rank reached no start) take no part, as on the host.
__global__ __launch_bounds__(256) void k_link_want(PathArgs a, const uint4 *st, const uint32_t *prv,
                                                   const uint32_t *len, uint32_t *want,
                                                   unsigned long long *best_pred) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t == 0 || t >= a.n || path_dummy(a.dummy, t)) return;
    const uint4 e = st[t];
    if (prv[e.x] != 0xFFFFFFFFu) return;  // on a cycle
    const uint32_t L = len[e.x];
    if (e.y + 1 != L) return;  // not its unitig's last node
    uint32_t h = t;
    while (h > 0 && a.lcs[h] >= a.k - 1) h--;  // the (k-1)-suffix group's first node holds the labels
    const unsigned long long mine = (unsigned long long)L << 32 | t;
    unsigned long long best = ~0ull;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const uint2 w = a.rank[(uint64_t)c * a.rwords + (h >> 5)];
        if (!((w.y >> (h & 31)) & 1u)) continue;
        const uint32_t y = rank_word(w, h);
        if (path_dummy(a.dummy, y) || prv[y] != 0xFFFFFFFFu) continue;
        const unsigned long long ky = (unsigned long long)len[y] << 32 | y;  // y starts its unitig
        best = ky < best ? ky : best;
        atomicMin(best_pred + y, mine);
    }
    if (best != ~0ull) want[t] = (uint32_t)best;
}

__global__ __launch_bounds__(256) void k_link_apply(const uint4 *st, const uint32_t *len, const uint32_t *want,
                                                    const unsigned long long *best_pred, uint32_t n, uint32_t *prv) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= n) return;
    const uint32_t y = want[t];
    if (y == 0xFFFFFFFFu) return;
    if (best_pred[y] == ((unsigned long long)len[st[t].x] << 32 | t)) prv[y] = t;  // one winner per y
}

void launch_path_link(const PathArgs &a, const uint4 *st, const uint32_t *len, uint32_t *want,
                      unsigned long long *best_pred, uint32_t *prv, hipStream_t s) {
    hipLaunchKernelGGL(k_link_want, grid_for(a.n), dim3(256), 0, s, a, st, (const uint32_t *)prv, len, want, best_pred);
    hipLaunchKernelGGL(k_link_apply, grid_for(a.n), dim3(256), 0, s, st, len, (const uint32_t *)want,
                       (const unsigned long long *)best_pred, a.n, prv);
}

__global__ __launch_bounds__(256) void k_path_rank_init(const uint32_t *prv, uint32_t n, uint4 *st) {
    const uint32_t z = blockIdx.x * 256u + threadIdx.x;
    if (z >= n) return;
    const uint32_t p = prv[z];
    st[z] = p == 0xFFFFFFFFu ? make_uint4(z, 0, z, 0) : make_uint4(p, 1, min(z, p), 0);
}

__global__ __launch_bounds__(256) void k_path_rank_step(const uint4 *in, uint32_t n, uint4 *out) {
    const uint32_t z = blockIdx.x * 256u + threadIdx.x;
    if (z >= n) return;
    const uint4 e = in[z];
    const uint4 f = in[e.x];
    out[z] = make_uint4(f.x, e.y + f.y, min(e.z, f.z), 0);
}

__global__ __launch_bounds__(256) void k_path_cut(PathArgs a, const uint4 *st, uint32_t *prv, uint32_t *flag) {
    const uint32_t z = blockIdx.x * 256u + threadIdx.x;
    if (z == 0 || z >= a.n || path_dummy(a.dummy, z)) return;
    const uint4 e = st[z];
    // only z itself writes prv[z]; a node whose rank did not end at a start is on a cycle
    if (e.z == z && prv[e.x] != 0xFFFFFFFFu) {
        prv[z] = 0xFFFFFFFFu;
        *flag = 1;
    }
}

// path length = max rank + 1 over the path's nodes.  A wave's nodes mostly lie on one path
// (a few paths cover the whole graph), so the max is taken per distinct path in the wave
// first: one atomicMax per (wave, path) instead of one per node on the same few addresses.
__global__ __launch_bounds__(256) void k_path_len(PathArgs a, const uint4 *st, uint32_t *len) {
    const uint32_t z = blockIdx.x * 256u + threadIdx.x;
    const bool valid = !(z == 0 || z >= a.n || path_dummy(a.dummy, z));
    uint32_t key = 0xFFFFFFFFu, val = 0;
    if (valid) {
        const uint4 e = st[z];
        key = e.x;
        val = e.y + 1;
    }
    uint64_t todo = __ballot(valid);
    while (todo) {
        const uint32_t lead = (uint32_t)__builtin_ctzll(todo);
        const uint32_t k0 = __shfl(key, lead, 64);
        const bool mine = valid && key == k0;
        uint32_t v = mine ? val : 0u;
        for (int o = 32; o > 0; o >>= 1) {
            const uint32_t t = __shfl_xor(v, o, 64);
            v = t > v ? t : v;
        }
        if ((threadIdx.x & 63) == lead) atomicMax(len + k0, v);
        todo &= ~__ballot(mine);
    }
}

__global__ __launch_bounds__(256) void k_path_vals(PathArgs a, const uint32_t *prv, const uint32_t *len,
                                                   uint32_t *vals, uint32_t *n_paths) {
    const uint32_t z = blockIdx.x * 256u + threadIdx.x;
    if (z >= a.n) return;
    const bool start = z > 0 && !path_dummy(a.dummy, z) && prv[z] == 0xFFFFFFFFu;
    vals[z] = start ? len[z] + a.k : 0;
    const uint64_t ballot = __ballot(start);
    if (start && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(ballot)) atomicAdd(n_paths, (uint32_t)__popcll(ballot));
}

__device__ __forceinline__ void path_put(uint4 *pstream, uint64_t t, uint32_t c) {
    const uint32_t o = (uint32_t)(t & 31);
    uint32_t *w = reinterpret_cast<uint32_t *>(pstream + (t >> 5)) + (o < 16 ? 0 : 1);
    atomicOr(w, (c & 3u) << (2 * (o & 15)));
}

__global__ __launch_bounds__(256) void k_path_place(PathArgs a, const uint4 *st, const uint32_t *prv,
                                                    const uint64_t *base, uint32_t *colex_at, uint32_t *pos_of_node,
                                                    uint4 *pstream, uint64_t *puniq) {
    const uint32_t z = blockIdx.x * 256u + threadIdx.x;
    if (z == 0 || z >= a.n || path_dummy(a.dummy, z)) return;
    const uint4 e = st[z];
    const uint64_t pos = base[e.x] + e.y;
    const uint32_t u = (a.uniq[z >> 5] >> (z & 31)) & 1u;
    colex_at[pos] = z | (u << 31);
    pos_of_node[z] = (uint32_t)pos;
    const uint64_t end = pos + a.k - 1;  // the node's k-mer ends at text position end
    atomicOr(reinterpret_cast<uint32_t *>(pstream + (end >> 5)) + 2, 1u << (end & 31));
    if (u) atomicOr(reinterpret_cast<unsigned long long *>(puniq + (pos >> 6)), 1ull << (pos & 63));
    if (prv[z] != 0xFFFFFFFFu) {
        path_put(pstream, end, a.code[z]);
    } else {  // a path start: all k characters of its k-mer, walking back k - 1 predecessors
        uint32_t t = z;
        for (int64_t i = (int64_t)a.k - 1; i >= 0; i--) {
            path_put(pstream, pos + (uint64_t)i, a.code[t]);
            t = a.pred[t];
        }
    }
}

// fork blocks after each path end (derived.cpp build_paths, encode_core.h fork_block): run
// after k_path_place, so that every real node's path position and all path text are known
__global__ __launch_bounds__(256) void k_path_forks(PathArgs a, const uint4 *st, const uint32_t *len,
                                                    const uint64_t *base, const uint32_t *pos_of_node,
                                                    const uint4 *pstream, uint32_t *colex_at) {
    const uint32_t z = blockIdx.x * 256u + threadIdx.x;
    if (z == 0 || z >= a.n || path_dummy(a.dummy, z)) return;
    const uint4 e = st[z];
    if (e.y + 1 != len[e.x]) return;  // not its path's last node
    const uint64_t pos = base[e.x] + e.y;
    uint32_t h = z;
    while (h > 0 && a.lcs[h] >= a.k - 1) h--;  // the (k-1)-suffix group's first node holds the labels
    uint4 *blk = reinterpret_cast<uint4 *>(colex_at + fork_block(pos + 1));
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const uint2 w = a.rank[(uint64_t)c * a.rwords + (h >> 5)];
        uint32_t v = 0xFFFFFFFFu;
        if ((w.y >> (h & 31)) & 1u) {
            const uint32_t y = rank_word(w, h);
            if (!path_dummy(a.dummy, y)) v = pos_of_node[y];
        }
        uint64_t chars = 0;
        uint32_t ends = 0;
        if (v != 0xFFFFFFFFu) path_text32(pstream, (uint64_t)v + a.k - 1, chars, ends);
        blk[c] = make_uint4(v, (uint32_t)chars, (uint32_t)(chars >> 32), ends);
    }
}

void launch_path_forks(const PathArgs &a, const uint4 *st, const uint32_t *len, const uint64_t *base,
                       const uint32_t *pos_of_node, const uint4 *pstream, uint32_t *colex_at, hipStream_t s) {
    hipLaunchKernelGGL(k_path_forks, grid_for(a.n), dim3(256), 0, s, a, st, len, base, pos_of_node, pstream, colex_at);
}

void launch_path_edges(const PathArgs &a, uint32_t *prv, hipStream_t s) {
    hipLaunchKernelGGL(k_path_edges, grid_for(a.n), dim3(256), 0, s, a, prv);
}

uint4 *launch_path_rank(const uint32_t *prv, uint32_t n, uint4 *a, uint4 *b, hipStream_t s) {
    hipLaunchKernelGGL(k_path_rank_init, grid_for(n), dim3(256), 0, s, prv, n, a);
    // 2^rounds >= n: every path is ranked to its start, every cycle's minimum is found
    int rounds = 1;
    while ((1ull << rounds) < (uint64_t)n) rounds++;
    for (int r = 0; r < rounds; r++) {
        hipLaunchKernelGGL(k_path_rank_step, grid_for(n), dim3(256), 0, s, (const uint4 *)a, n, b);
        std::swap(a, b);
    }
    return a;
}

void launch_path_cut(const PathArgs &a, const uint4 *st, uint32_t *prv, uint32_t *flag, hipStream_t s) {
    hipLaunchKernelGGL(k_path_cut, grid_for(a.n), dim3(256), 0, s, a, st, prv, flag);
}

void launch_path_lengths(const PathArgs &a, const uint4 *st, const uint32_t *prv, uint32_t *len, uint32_t *vals,
                         uint32_t *n_paths, hipStream_t s) {
    hipLaunchKernelGGL(k_path_len, grid_for(a.n), dim3(256), 0, s, a, st, len);
    hipLaunchKernelGGL(k_path_vals, grid_for(a.n), dim3(256), 0, s, a, prv, (const uint32_t *)len, vals, n_paths);
}

void launch_path_place(const PathArgs &a, const uint4 *st, const uint32_t *prv, const uint64_t *base,
                       uint32_t *colex_at, uint32_t *pos_of_node, uint4 *pstream, uint64_t *puniq, hipStream_t s) {
    hipLaunchKernelGGL(k_path_place, grid_for(a.n), dim3(256), 0, s, a, st, prv, base, colex_at, pos_of_node, pstream,
                       puniq);
}

}  // namespace ntc
