// Native encode pipeline of the CLI: `ntcomp encode -i P reads.fq > encoded.dat`
// (src/main.rs:141-181), file in, encoded.dat out, with every stage overlapped:
//
//   reader   batches of blocks_per_batch x 65,536 reads (main.rs:152) into a ring of
//            pinned host buffers.  A plain FASTQ (mapped) goes as text: the reader's gang
//            copies it into the buffer while counting newlines and looking for blank lines
//            (fq_copy_scan), and cuts the batch after the last whole block's last line, so
//            the GPU parses it (ntc_encode_pack_fastq).  Anything else -- compressed input,
//            FASTA, a batch with a blank line from there on -- is parsed by the host pool
//            (ntc_fastx_next_batch_into); reads past the last whole block of a batch carry
//            into the next buffer.  Either way every block but the file's last holds
//            exactly 65,536 reads, and the last holds num_records % 65,536 (main.rs:174-177).
//   GPU      one driver thread per context, batches dealt round-robin:
//            ntc_encode_pack_fastq / ntc_encode_pack_batch = H2D, (parse,) encode kernels,
//            GPU block packer, D2H of the four coded streams per block (the u64 records
//            never leave HBM).
//   deflate  the host pool gzips each block's streams (ntc_deflate_block) -- the only
//            codec step left on the CPU.
//   writer   the calling thread writes the file header (lib.rs:52-67) and the blocks in
//            file order; a block the reference drops (no long or no short record,
//            write_block_to errs and main.rs:170 ignores it -- App. B.3) is skipped.
#include <emmintrin.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ntcomp_codec.h"
#include "../../include/ntcomp_gpu.h"
#include "../../include/ntcomp_host.h"
#include "../../include/ntcomp_pipeline.h"
#include "ntc_internal.h"

namespace {

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// Pinned host memory: 2 MB pages, touched, then registered with HIP (hipHostRegister runs at
// ~25 GB/s, hipHostMalloc at ~4 GB/s on the box: scripts/ingest_bw.cpp, profiles/round4).
// Freed buffers stay registered in a process-wide pool (up to kPinnedPoolMax bytes) and are
// handed out again, so pipelines that grow and drop buffers per batch neither pay the
// registration again nor register a range the process just unregistered.
constexpr size_t kPinnedPoolMax = 8ull << 30;
struct PinnedPool {
    std::mutex mu;
    std::map<void *, size_t> size_of;       // every buffer handed out or pooled
    std::multimap<size_t, void *> idle;     // pooled: size -> buffer
    size_t idle_bytes = 0;
};
PinnedPool &pinned_pool() {
    static PinnedPool *p = new PinnedPool();  // never destroyed: buffers live until the process ends
    return *p;
}
// decode: the streams decoded on the host pool instead of the GPU (NTC_HOST_UNPACK=1)
bool host_unpack_on() {
    const char *h = std::getenv("NTC_HOST_UNPACK");
    return h && std::atoi(h) > 0;
}

void *pinned_alloc(size_t n) {
    const size_t sz = (std::max<size_t>(n, 1) + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
    PinnedPool &P = pinned_pool();
    {
        std::lock_guard<std::mutex> g(P.mu);
        auto it = P.idle.lower_bound(sz);
        if (it != P.idle.end() && it->first <= 2 * sz + (64u << 20)) {  // not a far larger one
            void *q = it->second;
            P.idle_bytes -= it->first;
            P.idle.erase(it);
            return q;
        }
    }
    void *q = mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (q == MAP_FAILED) return nullptr;
    madvise(q, sz, MADV_HUGEPAGE);
    std::memset(q, 0, sz);  // real pages before they are pinned
    if (hipHostRegister(q, sz, hipHostRegisterPortable) != hipSuccess) {
        (void)hipGetLastError();
        munmap(q, sz);
        return nullptr;
    }
    std::lock_guard<std::mutex> g(P.mu);
    P.size_of[q] = sz;
    return q;
}
void pinned_free(void *q) {
    if (!q) return;
    PinnedPool &P = pinned_pool();
    std::vector<std::pair<void *, size_t>> drop;
    {
        std::lock_guard<std::mutex> g(P.mu);
        auto it = P.size_of.find(q);
        if (it == P.size_of.end()) return;
        P.idle.emplace(it->second, q);
        P.idle_bytes += it->second;
        while (P.idle_bytes > kPinnedPoolMax && !P.idle.empty()) {  // the largest idle ones go
            auto big = std::prev(P.idle.end());
            drop.emplace_back(big->second, big->first);
            P.idle_bytes -= big->first;
            P.size_of.erase(big->second);
            P.idle.erase(big);
        }
    }
    for (auto &d : drop) {
        (void)hipHostUnregister(d.first);
        munmap(d.first, d.second);
    }
}

struct Batch {  // one pinned buffer of the ring
    uint8_t *bases = nullptr;
    uint64_t *offs = nullptr;
    uint64_t cap_bases = 0, cap_reads = 0;
    uint8_t *text = nullptr;  // plain FASTQ text for the GPU parse (text_len bytes, n_process records)
    uint64_t text_cap = 0, text_len = 0;
    bool is_text = false;
    uint64_t n_reads = 0;    // reads in the buffer (carry + new)
    uint64_t n_process = 0;  // reads handed to the GPU (whole blocks, or all at the end)
    uint64_t first_read = 0; // file index of the buffer's first read
    uint64_t first_block = 0;
    bool busy = false;
};

// Copy n bytes of FASTQ text into dst (16-byte aligned) and scan them on the way: the
// newlines, and the first line inside the piece that starts with '\n' or '\r' (a blank
// line, which the host parser skips between records; the piece's first byte is the caller's).
struct FqScan {
    uint64_t nl = 0;
    size_t blank = SIZE_MAX;  // offset of the first blank line's first byte, or SIZE_MAX
};
template <bool kCopy>
FqScan fq_copy_scan(const uint8_t *src, uint8_t *dst, size_t n) {
    FqScan r;
    const __m128i NL = _mm_set1_epi8('\n'), CR = _mm_set1_epi8('\r');
    uint64_t carry = 0;  // the byte before this 64-byte block is '\n'
    size_t i = 0;
    for (; i + 64 <= n; i += 64) {
        uint64_t mnl = 0, mcr = 0;
        for (int k = 0; k < 4; k++) {
            const __m128i x = _mm_loadu_si128((const __m128i *)(src + i + 16 * k));
            if (kCopy) _mm_stream_si128((__m128i *)(dst + i + 16 * k), x);
            mnl |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(x, NL)) << (16 * k);
            mcr |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(x, CR)) << (16 * k);
        }
        const uint64_t bad = ((mnl << 1) | carry) & (mnl | mcr);
        if (bad && r.blank == SIZE_MAX) r.blank = i + (size_t)__builtin_ctzll(bad);
        carry = mnl >> 63;
        r.nl += (uint64_t)__builtin_popcountll(mnl);
    }
    if (kCopy) _mm_sfence();
    for (; i < n; i++) {
        const uint8_t c = src[i];
        if (kCopy) dst[i] = c;
        if (carry && (c == '\n' || c == '\r') && r.blank == SIZE_MAX) r.blank = i;
        carry = c == '\n';
        r.nl += c == '\n';
    }
    return r;
}

// byte position just past the target-th newline (1-based) of p[0, n), or n
size_t nth_newline_end(const uint8_t *p, size_t n, uint64_t target) {
    const __m128i NL = _mm_set1_epi8('\n');
    size_t i = 0;
    for (; i + 64 <= n; i += 64) {
        uint64_t m = 0;
        for (int k = 0; k < 4; k++)
            m |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i *)(p + i + 16 * k)), NL))
                 << (16 * k);
        const uint64_t c = (uint64_t)__builtin_popcountll(m);
        if (c < target) {
            target -= c;
            continue;
        }
        for (; target > 1; target--) m &= m - 1;
        return i + (size_t)__builtin_ctzll(m) + 1;
    }
    for (; i < n; i++)
        if (p[i] == '\n' && --target == 0) return i + 1;
    return n;
}

struct BlockOut {  // a deflated block (its four streams' parts), or a dropped one
    uint8_t *part[4] = {nullptr, nullptr, nullptr, nullptr};
    uint64_t len[4] = {0, 0, 0, 0};
    int status = NTC_OK;
    int left = 0;  // parts not yet deflated
};

struct Shared {
    std::mutex mu;
    std::condition_variable cv;
    int error = NTC_OK;
    std::string msg;
    int64_t bad_read = -1;
    void fail(int code, const std::string &m, int64_t bad = -1) {
        std::lock_guard<std::mutex> g(mu);
        if (error == NTC_OK) {
            error = code;
            msg = m;
            bad_read = bad;
        }
        cv.notify_all();
    }
};

}  // namespace

extern "C" {

int ntc_encode_file(ntc_ctx *const *ctxs, int n_ctx, const char *in_path, int out_fd, const ntc_pipeline_opts *opts,
                    ntc_pipeline_stats *stats) {
    if (!ctxs || n_ctx <= 0 || !in_path || out_fd < 0) return NTC_ERR_INVALID_ARG;
    for (int i = 0; i < n_ctx; i++)
        if (!ctxs[i]) return NTC_ERR_INVALID_ARG;
    ntc_pipeline_opts o{};
    if (opts) o = *opts;
    const int T = o.threads > 0 ? o.threads : ntc_host_threads();
    const uint32_t BR = 65536;  // main.rs:152
    // 4 blocks per GPU call and 64 Mi-base buffers: the first batch is on the GPU after
    // ~30 ms and the pinned ring stays small (10 M x 150 bp: pipeline 0.59 -> 0.32 s against
    // 16 blocks and 256 Mi bases, scripts/pipe_bench.py on one MI355X box)
    const uint64_t per_batch = (uint64_t)(o.blocks_per_batch > 0 ? o.blocks_per_batch : 4) * BR;
    const uint64_t cap_bases = o.batch_bases > 0 ? o.batch_bases : (64ull << 20);
    const int engine = o.deflate_engine;
    ntc_pipeline_stats S{};
    const auto t0 = Clock::now();
    // NTC_PIPE_TRACE=n: the first n batches' (and blocks') events on stderr, ms from the start
    const char *etr = std::getenv("NTC_PIPE_TRACE");
    const uint64_t etrace_n = etr ? (uint64_t)std::atoll(etr) : 0;
    auto etrace = [&](const char *what, uint64_t b) {
        if (b < etrace_n) std::fprintf(stderr, "[pipe] %8.3f ms %s %llu\n", 1e3 * secs(t0, Clock::now()), what,
                                       (unsigned long long)b);
    };

    ntc_fastx *fx = nullptr;
    int rc = ntc_fastx_open(in_path, &fx);
    if (rc) return rc;
    ntc_fastx_set_threads(fx, T);
    // a mapped plain FASTQ goes to the GPU as text
    uint64_t text_n = 0;
    const uint8_t *text = o.host_parse ? nullptr : ntc::fastx_mapped(fx, &text_n);

    // pinned ring: the GPU threads hold at most n_ctx buffers, the reader fills one more.
    // A slot's base buffer (the large part, ~320 MB) is pinned by the reader when it first
    // fills the slot, so only the first one delays the first batch (pinning runs at a few
    // GB/s); the offsets are pinned here.
    const int NB = n_ctx + 2;
    std::vector<Batch> ring((size_t)NB);
    for (auto &b : ring) {
        b.cap_bases = cap_bases + BR * 1024ull;  // a carry of < 65,536 reads sits in front
        b.cap_reads = per_batch + BR + 1;
        if (!(b.offs = (uint64_t *)pinned_alloc(b.cap_reads * 8))) {
            for (auto &x : ring) pinned_free(x.offs);
            ntc_fastx_close(fx);
            return NTC_ERR_HIP;
        }
    }
    std::atomic<double> t_pin{0};
    S.alloc_s = secs(t0, Clock::now());
    Shared sh;
    std::vector<std::deque<int>> gpu_q((size_t)n_ctx);  // per context: ring indices in batch order
    bool reader_done = false;
    uint64_t total_blocks = 0;    // known once the reader is done
    std::atomic<double> t_parse{0}, t_gpu{0}, t_deflate{0}, t_write{0};
    // deflate tasks (one per stream of a block: ntc_deflate_stream) and blocks in progress
    struct Task {
        std::shared_ptr<uint8_t> payload;  // the GPU call's host payload (ntc_buffer_free)
        ntc_block_meta meta;
        uint64_t block;
        int stream;
    };
    std::deque<Task> tasks;
    std::map<uint64_t, BlockOut> done;
    uint64_t pending_tasks = 0;
    uint64_t writer_at = 0;  // the block the writer waits for
    const uint64_t max_pending = (uint64_t)T * 8 + 64;  // bound on blocks queued or finished but unwritten

    auto add_time = [](std::atomic<double> &a, double d) {
        double cur = a.load();
        while (!a.compare_exchange_weak(cur, cur + d)) {
        }
    };

    // ---- reader ---------------------------------------------------------------------------
    // A buffer that cannot hold a whole 65,536-read block (long reads) grows until it does.
    auto grow = [&](Batch &b, uint64_t need_bases, uint64_t keep_bases, uint64_t keep_reads) -> bool {
        if (need_bases <= b.cap_bases) return true;
        const uint64_t cap = std::max(need_bases, b.cap_bases * 2);
        uint8_t *nbuf = (uint8_t *)pinned_alloc(cap);
        if (!nbuf) return false;
        if (keep_bases) std::memcpy(nbuf, b.bases, keep_bases);
        pinned_free(b.bases);
        b.bases = nbuf;
        b.cap_bases = cap;
        (void)keep_reads;
        return true;
    };
    // GPU-parse reader state.  Mapped: the next batch's text starts at text_pos (a record
    // start).  Streamed (a decoder's output): the text after the last cut, carry_n bytes at
    // carry_p in the previous batch's buffer, goes first into the next one.
    const bool streamed = !text && !o.host_parse && ntc::fastx_streamed_fastq(fx);
    uint64_t text_pos = 0;
    const uint8_t *carry_p = nullptr;
    uint64_t carry_n = 0;
    bool stream_eof = false;
    double rec_bytes = 320;  // text bytes per record so far (a guess for 150 bp reads until known)
    std::atomic<uint64_t> text_batches{0};
    // the reader's gang: 8 threads copy + scan at ~45 GB/s on the box, as fast as 16 for the
    // pipeline and at less CPU beside the deflate pool (scripts/rt_sweep.sh); NTC_READ_THREADS
    // is the A/B hook
    const char *rt_env = std::getenv("NTC_READ_THREADS");
    const int RT = std::max(1, rt_env ? std::atoi(rt_env) : std::min(T, 8));
    if (text) {  // bytes per record from the first MiB
        const size_t m = (size_t)std::min<uint64_t>(text_n, 1u << 20);
        uint64_t nl = 0;
        for (size_t i = 0; i < m; i++) nl += text[i] == '\n';
        rec_bytes = nl >= 4 ? 4.0 * (double)m / (double)nl : (double)m + 1;
    }
    // Fill b with the text of the next whole blocks (or the input's end): 1 = filled, 0 = no
    // input left, -1 = hand over to the host parser (a blank line before the cut, a line
    // count that is not a multiple of 4 at the end, a block too large for one call), -2 = the
    // decoder failed
    auto fill_text = [&](ntc::Gang &gang, Batch &b, bool &eof) -> int {
        const uint64_t kMaxText = (1ull << 32) - (64u << 20);  // ntc_encode_pack_fastq takes < 4 GiB
        uint64_t want_cap = (uint64_t)((double)per_batch * rec_bytes * 1.03) + (256u << 10);
        std::vector<FqScan> sc;
        for (;;) {
            if (!streamed) {
                if (text_pos >= text_n) return 0;
                if (text[text_pos] != '@') return -1;
            }
            // room for the carried text plus more (a batch read with a doubled buffer can leave a
            // carry larger than this batch's estimate)
            if (streamed) want_cap = std::max<uint64_t>(want_cap, carry_n + (4u << 20));
            want_cap = std::min(want_cap, kMaxText);
            if (streamed && carry_n >= want_cap) return -1;  // more than 4 GiB without one block
            if (b.text_cap < want_cap) {
                const auto ta = Clock::now();
                uint8_t *nt = (uint8_t *)pinned_alloc(want_cap);
                if (!nt) return -1;
                if (carry_n && carry_p == b.text) {  // growing the buffer that holds the carry
                    std::memcpy(nt, carry_p, carry_n);
                    carry_p = nt;
                }
                pinned_free(b.text);
                b.text = nt;
                b.text_cap = want_cap;
                t_pin = t_pin.load() + secs(ta, Clock::now());
            }
            uint64_t len;
            const uint8_t *src;
            if (!streamed) {
                len = std::min(text_n - text_pos, want_cap);
                src = text + text_pos;
            } else {
                if (carry_n && carry_p != b.text) std::memcpy(b.text, carry_p, carry_n);
                bool io_err = false;
                len = carry_n + ntc::fastx_stream_read(fx, b.text + carry_n, want_cap - carry_n, &io_err);
                if (io_err) return -2;
                stream_eof = len < want_cap;
                carry_p = b.text;  // all of it unused until the cut
                carry_n = len;
                if (len == 0) return 0;
                if (b.text[0] != '@') return -1;
                src = b.text;
            }
            constexpr uint64_t kPiece = 1u << 20;
            const uint64_t np = (len + kPiece - 1) / kPiece;
            sc.assign(np, FqScan{});
            std::atomic<uint64_t> next{0};
            gang.run([&](int) {
                for (uint64_t q; (q = next.fetch_add(1)) < np;) {
                    const uint64_t a = q * kPiece, e = std::min(len, a + kPiece);
                    sc[q] = streamed ? fq_copy_scan<false>(src + a, nullptr, e - a)
                                     : fq_copy_scan<true>(src + a, b.text + a, e - a);
                }
            });
            uint64_t nl = 0, blank = UINT64_MAX;  // the first blank line in the text read
            for (uint64_t q = 0; q < np; q++) {
                const uint64_t a = q * kPiece;
                if (blank == UINT64_MAX && a && src[a - 1] == '\n' && (src[a] == '\n' || src[a] == '\r')) blank = a;
                if (blank == UINT64_MAX && sc[q].blank != SIZE_MAX) blank = a + sc[q].blank;
                nl += sc[q].nl;
            }
            eof = streamed ? stream_eof : text_pos + len == text_n;
            // the text read ends the input with whole records and no blank line: all of it
            // goes; otherwise whole blocks of the complete records, cut after the last one's
            // last line
            const uint64_t lines = nl + (eof && src[len - 1] != '\n');
            const bool whole = eof && lines % 4 == 0 && blank == UINT64_MAX;
            const uint64_t recs = whole ? lines / 4 : nl / 4;
            uint64_t n = 0, cut = len;
            if (whole && recs <= per_batch) {
                n = recs;
            } else {
                n = std::min<uint64_t>(recs, per_batch) / BR * BR;
                if (n == 0) {  // not one whole block in the text read: read more, or give up
                    if (eof || len < want_cap || want_cap >= kMaxText) return -1;
                    want_cap *= 2;
                    continue;
                }
                // the batch ends after newline 4 n: find the piece holding it
                uint64_t before = 0, q = 0;
                while (before + sc[q].nl < 4 * n) before += sc[q++].nl;
                const uint64_t a = q * kPiece;
                cut = a + nth_newline_end(src + a, std::min(len, a + kPiece) - a, 4 * n - before);
                eof = false;
            }
            if (blank < cut) return -1;  // the batch holds a blank line: the host parser takes it
            b.text_len = cut;
            b.n_reads = b.n_process = n;
            rec_bytes = (double)cut / (double)std::max<uint64_t>(n, 1);
            if (streamed) {
                carry_p = b.text + cut;
                carry_n = len - cut;
                eof = eof || (stream_eof && carry_n == 0);
            } else {
                text_pos += cut;
                eof = eof || text_pos == text_n;
            }
            return 1;
        }
    };
    std::thread reader([&] {
        uint64_t next_read = 0, next_block = 0, batch_no = 0;
        int prev = -1;
        uint64_t carry = 0;  // reads at the tail of ring[prev] past its processed blocks
        bool as_text = text != nullptr || streamed;
        std::unique_ptr<ntc::Gang> gang(as_text ? new ntc::Gang(RT) : nullptr);
        for (;;) {
            int bi;
            {
                std::unique_lock<std::mutex> g(sh.mu);
                bi = (int)(batch_no % (uint64_t)NB);
                sh.cv.wait(g, [&] { return sh.error != NTC_OK || !ring[(size_t)bi].busy; });
                if (sh.error != NTC_OK) break;
            }
            Batch &b = ring[(size_t)bi];
            b.is_text = false;
            if (as_text) {
                const auto tp = Clock::now();
                bool eof = false;
                const int r = fill_text(*gang, b, eof);
                add_time(t_parse, secs(tp, Clock::now()));
                if (r > 0) {
                    if (batch_no == 0) S.first_batch_s = secs(t0, Clock::now());
                    b.is_text = true;
                    b.first_read = next_read;
                    b.first_block = next_block;
                    next_read += b.n_process;
                    next_block += (b.n_process + BR - 1) / BR;
                    text_batches++;
                    etrace("read batch", batch_no);
                    {
                        std::lock_guard<std::mutex> g(sh.mu);
                        b.busy = true;
                        gpu_q[(size_t)(batch_no % (uint64_t)n_ctx)].push_back(bi);
                        batch_no++;
                        sh.cv.notify_all();
                    }
                    if (eof) break;
                    continue;
                }
                if (r == 0) break;
                if (r == -2) {
                    sh.fail(NTC_ERR_IO, "FASTX input: malformed or unreadable");
                    break;
                }
                as_text = false;  // the host parser goes on from the first record not sent
                if (streamed) {
                    ntc::fastx_stream_unread(fx, carry_p, carry_n);
                    carry_n = 0;
                } else {
                    ntc::fastx_seek_mapped(fx, text_pos);
                }
            }
            if (!b.bases) {
                const auto ta = Clock::now();
                if (!(b.bases = (uint8_t *)pinned_alloc(b.cap_bases))) {
                    sh.fail(NTC_ERR_HIP, "pinned host allocation failed");
                    break;
                }
                t_pin = t_pin.load() + secs(ta, Clock::now());  // the reader alone writes it
            }
            uint64_t used = 0;  // bases in b
            b.offs[0] = 0;
            if (carry) {  // the previous buffer's unprocessed reads go first
                const Batch &p = ring[(size_t)prev];
                const uint64_t a0 = p.offs[p.n_process], a1 = p.offs[p.n_reads];
                if (!grow(b, (a1 - a0) * 2 + (64u << 20), 0, 0)) {
                    sh.fail(NTC_ERR_CAPACITY, "pinned host allocation failed");
                    break;
                }
                std::memcpy(b.bases, p.bases + a0, a1 - a0);
                for (uint64_t r = 0; r <= carry; r++) b.offs[r] = p.offs[p.n_process + r] - a0;
                used = a1 - a0;
            }
            b.n_reads = carry;
            bool eof = false, bad = false;
            const auto tp = Clock::now();
            for (;;) {  // fill: at least one whole block (or the end of the input)
                const uint64_t room = b.cap_bases - used;
                const uint64_t want = per_batch - b.n_reads, max_b = room / 2;
                uint64_t got = 0;
                const int r = ntc_fastx_next_batch_into(fx, want, max_b, b.bases + used, room, b.offs + b.n_reads, &got);
                if (r) {
                    sh.fail(r, r == NTC_ERR_CAPACITY ? "a read longer than half the batch buffer (raise batch_bases)"
                                                     : "FASTX input: malformed or unreadable");
                    bad = true;
                    break;
                }
                if (used)
                    for (uint64_t i = 0; i <= got; i++) b.offs[b.n_reads + i] += used;
                b.n_reads += got;
                const uint64_t nb = b.offs[b.n_reads] - used;
                used = b.offs[b.n_reads];
                if (got == 0 || (got < want && nb < max_b)) {
                    eof = true;
                    break;
                }
                if (b.n_reads >= BR || b.n_reads == per_batch) break;
                // fewer than 65,536 reads filled half the buffer: grow it and read on
                if (!grow(b, b.cap_bases * 2, used, b.n_reads)) {
                    sh.fail(NTC_ERR_CAPACITY, "pinned host allocation failed");
                    bad = true;
                    break;
                }
            }
            add_time(t_parse, secs(tp, Clock::now()));
            if (bad) break;
            if (batch_no == 0) S.first_batch_s = secs(t0, Clock::now());
            b.n_process = eof ? b.n_reads : (b.n_reads / BR) * BR;
            b.first_read = next_read;
            b.first_block = next_block;
            const uint64_t nblk = (b.n_process + BR - 1) / BR;
            carry = b.n_reads - b.n_process;
            prev = bi;
            next_read += b.n_process;
            next_block += nblk;
            if (b.n_process) {
                std::lock_guard<std::mutex> g(sh.mu);
                b.busy = true;
                gpu_q[(size_t)(batch_no % (uint64_t)n_ctx)].push_back(bi);
                batch_no++;
                sh.cv.notify_all();
            }
            if (eof && carry == 0) break;
        }
        std::lock_guard<std::mutex> g(sh.mu);
        S.reader_done_s = secs(t0, Clock::now());
        reader_done = true;
        total_blocks = next_block;
        S.reads = next_read;
        sh.cv.notify_all();
    });

    // ---- GPU drivers --------------------------------------------------------------------------
    std::vector<std::thread> gpus;
    for (int c = 0; c < n_ctx; c++)
        gpus.emplace_back([&, c] {
            for (;;) {
                int bi;
                {
                    std::unique_lock<std::mutex> g(sh.mu);
                    sh.cv.wait(g, [&] { return sh.error != NTC_OK || !gpu_q[(size_t)c].empty() || reader_done; });
                    if (sh.error != NTC_OK) return;
                    if (gpu_q[(size_t)c].empty()) {
                        if (reader_done) return;
                        continue;
                    }
                    bi = gpu_q[(size_t)c].front();
                    gpu_q[(size_t)c].pop_front();
                    // backpressure: do not run far ahead of the deflate pool and writer (the
                    // batch holding the writer's next block always goes)
                    sh.cv.wait(g, [&] {
                        return sh.error != NTC_OK || pending_tasks < max_pending ||
                               ring[(size_t)bi].first_block <= writer_at;
                    });
                    if (sh.error != NTC_OK) return;
                }
                Batch &b = ring[(size_t)bi];
                const uint64_t nblk = (b.n_process + BR - 1) / BR;
                std::vector<ntc_block_meta> metas(nblk);
                uint8_t *payload = nullptr;
                uint64_t plen = 0;
                int64_t bad = -1;
                uint64_t nb = 0;
                const auto tg = Clock::now();
                const int r = b.is_text ? ntc_encode_pack_fastq(ctxs[c], b.text, b.text_len, b.n_process, BR,
                                                                metas.data(), &payload, &plen, &nb, &bad)
                                        : ntc_encode_pack_batch(ctxs[c], b.bases, b.offs, b.n_process, BR,
                                                                metas.data(), &payload, &plen, &bad);
                add_time(t_gpu, secs(tg, Clock::now()));
                if (r) {
                    ntc_buffer_free(payload);
                    if (b.is_text && r == NTC_ERR_FORMAT)  // as the host parser reports it
                        sh.fail(r, "FASTX input: malformed or unreadable");
                    else
                        sh.fail(r, std::string("encode: ") + ntc_last_error(ctxs[c]),
                                bad >= 0 ? (int64_t)b.first_read + bad : -1);
                    return;
                }
                std::shared_ptr<uint8_t> pl(payload, ntc_buffer_free);
                etrace("gpu done, first block", b.first_block);
                std::lock_guard<std::mutex> g(sh.mu);
                S.gpu_done_s = secs(t0, Clock::now());
                S.bases += b.is_text ? nb : b.offs[b.n_process] - b.offs[0];
                b.busy = false;
                for (uint64_t k = 0; k < nblk; k++) {  // streams of the largest payload first
                    const bool ok = metas[k].status == NTC_OK;
                    BlockOut &bo = done[b.first_block + k];
                    bo.status = metas[k].status;
                    bo.left = ok ? 4 : 1;
                    int order[4] = {0, 1, 2, 3};
                    std::sort(order, order + 4, [&](int x, int y) {
                        return metas[k].stream[x].encoded_size > metas[k].stream[y].encoded_size;
                    });
                    for (int q = 0; q < (ok ? 4 : 1); q++) tasks.push_back(Task{pl, metas[k], b.first_block + k, order[q]});
                    pending_tasks++;
                }
                sh.cv.notify_all();
            }
        });

    // ---- deflate pool ----------------------------------------------------------------------------
    std::vector<std::thread> pool;
    for (int t = 0; t < T; t++)
        pool.emplace_back([&] {
            for (;;) {
                Task task;
                {
                    std::unique_lock<std::mutex> g(sh.mu);
                    sh.cv.wait(g, [&] { return sh.error != NTC_OK || !tasks.empty(); });
                    if (sh.error != NTC_OK) return;
                    if (tasks.empty()) return;
                    task = std::move(tasks.front());
                    tasks.pop_front();
                }
                uint8_t *data = nullptr;
                uint64_t len = 0;
                const auto td = Clock::now();
                const int status = task.meta.status;
                if (status == NTC_OK) {
                    const int r = ntc_deflate_stream(&task.meta, task.stream, task.payload.get(), engine, &data, &len);
                    if (r) {
                        sh.fail(r, "deflate failed");
                        return;
                    }
                } else if (status != NTC_ERR_EMPTY_READ) {
                    sh.fail(status, "malformed block");
                    return;
                }
                task.payload.reset();
                add_time(t_deflate, secs(td, Clock::now()));
                std::lock_guard<std::mutex> g(sh.mu);
                BlockOut &bo = done[task.block];
                bo.part[task.stream] = data;
                bo.len[task.stream] = len;
                if (--bo.left == 0) sh.cv.notify_all();
            }
        });

    // ---- writer (this thread) ------------------------------------------------------------------------
    auto write_all = [&](const uint8_t *p, uint64_t n) -> bool {
        while (n) {
            const ssize_t w = ::write(out_fd, p, n);
            if (w <= 0) return false;
            p += w;
            n -= (uint64_t)w;
        }
        return true;
    };
    uint8_t header[32];
    ntc_file_header(header);
    if (!write_all(header, 32)) sh.fail(NTC_ERR_IO, "write failed");
    S.bytes_out = 32;
    for (uint64_t blk = 0;; blk++) {
        BlockOut out;
        {
            std::unique_lock<std::mutex> g(sh.mu);
            sh.cv.wait(g, [&] {
                return sh.error != NTC_OK || (done.count(blk) && done[blk].left == 0) ||
                       (reader_done && blk >= total_blocks && !done.count(blk));
            });
            if (sh.error != NTC_OK) break;
            if (!done.count(blk)) break;  // all blocks written
            out = done[blk];
            done.erase(blk);
            pending_tasks--;
            writer_at = blk + 1;
            sh.cv.notify_all();
        }
        const auto tw = Clock::now();
        if (out.status == NTC_OK) {
            for (int q = 0; q < 4; q++) {
                if (!write_all(out.part[q], out.len[q])) sh.fail(NTC_ERR_IO, "write failed");
                S.bytes_out += out.len[q];
            }
            S.blocks++;
        } else {
            S.dropped_blocks++;
        }
        for (int q = 0; q < 4; q++) ntc_buffer_free(out.part[q]);
        add_time(t_write, secs(tw, Clock::now()));
        etrace("written block", blk);
    }
    {
        std::lock_guard<std::mutex> g(sh.mu);
        if (sh.error == NTC_OK) {
            sh.error = -1;  // stop the workers (no more tasks will come)
        }
        sh.cv.notify_all();
    }
    etrace("all written", 0);
    reader.join();
    for (auto &t : gpus) t.join();
    for (auto &t : pool) t.join();
    etrace("threads joined", 0);
    for (auto &kv : done)
        for (int q = 0; q < 4; q++) ntc_buffer_free(kv.second.part[q]);
    for (auto &b : ring) {
        pinned_free(b.bases);
        pinned_free(b.offs);
        pinned_free(b.text);
    }
    etrace("buffers freed", 0);
    ntc_fastx_close(fx);
    etrace("input closed", 0);
    const int result = sh.error == -1 ? NTC_OK : sh.error;
    S.alloc_s += t_pin.load();
    S.parse_s = t_parse.load();
    S.gpu_s = t_gpu.load();
    S.deflate_s = t_deflate.load();
    S.write_s = t_write.load();
    S.wall_s = secs(t0, Clock::now());
    S.threads = T;
    S.gpu_parsed = (int32_t)text_batches.load();
    S.bad_read = sh.bad_read;
    std::snprintf(S.error, sizeof(S.error), "%s", result == NTC_OK ? "" : sh.msg.c_str());
    if (stats) *stats = S;
    return result;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------
// Native decode pipeline of the CLI: `ntcomp decode -i P encoded.dat > out.fasta`
// (src/main.rs:183-211), every stage overlapped:
//
//   extents  the file is mapped; the blocks' extents and record counts come from their
//            32-byte headers alone (block_size of each stream; the flag stream's num_u64 =
//            records).  A truncated block ends the input, as read_exact ends decode_block.
//   unzip    the host pool inflates each block's four streams (ntc_read_block_streams)
//            straight into the batch's pinned payload buffer.
//   GPU      one driver thread per context, batches dealt round-robin:
//            ntc_unpack_streams = H2D of the streams, Rice / minimal-binary decode and
//            zip_block_contents on the device (unpack.hip), the batch's read count back;
//            then, once the reads of the batches before fix its ">seq.N" numbering,
//            ntc_decode_fasta_unpacked = the inverse-SBWT walk, the FASTA text formatted on
//            the GPU, D2H of the text.
//   writer   the calling thread writes the batches' text in file order (a regular file:
//            pwrite at the batch's offset; otherwise write), the next batches' GPU work
//            running meanwhile.  Batches are numbered by whichever thread completes a read
//            count.
// NTC_HOST_UNPACK=1: the pool decodes each block into u64 records (ntc_read_block_into),
// counting its reads, and ntc_decode_fasta takes the records.
// A damaged block ends the output after the blocks before it (decode_block's Err ends the
// reference's loop, main.rs:202).
// ---------------------------------------------------------------------------------------
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>

namespace {

struct DBlock {
    uint64_t a, len;   // byte range of the block
    uint64_t n_recs;   // records (the flag stream's num_u64)
    uint64_t pay;      // bytes of its four inflated streams (8 x encoded_size each)
    bool bad;          // a header that cannot describe its gzip stream: damaged, never sized
};

struct DSlot {  // one batch in flight
    uint64_t *recs = nullptr;
    uint64_t cap_recs = 0;
    uint8_t *pay = nullptr;  // GPU unpack: the blocks' inflated streams
    uint64_t cap_pay = 0, n_pay = 0;
    std::vector<ntc_block_meta> metas;
    uint8_t *text = nullptr;
    uint64_t cap_text = 0;
    uint64_t batch = ~0ULL;  // batch held, ~0 = free
    uint64_t first_block = 0, n_blocks = 0;
    uint64_t n_recs = 0, n_reads = 0, n_bases = 0, text_len = 0;
    uint64_t first_id = 0;
    uint64_t finished = 0;   // blocks of this batch unzipped or found damaged
    int bad_block = -1;      // first damaged block (index in the batch)
    bool buffer = false;     // recs sized for the batch
    bool ready = false;      // complete + first_id known: the GPU may take it
    bool unpacked = false;   // GPU unpack: the batch's reads and bases are known
    bool decoded = false;
};

void count_reads(const uint64_t *r, uint64_t n, uint64_t *reads, uint64_t *bases) {
    uint64_t rd = 0, bs = 0;  // first flags and bases of records (flag byte = bits 56..63)
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t w = r[i];
        const uint32_t flag = (uint32_t)(w >> 56);
        rd += flag & 1;
        bs += (flag & 2) ? (flag >> 2) : ((w >> 32) & 0xFFFFFFu);
    }
    *reads += rd;
    *bases += bs;
}

uint64_t digits_total(uint64_t first, uint64_t n) {  // decimal digits of first .. first + n - 1
    uint64_t tot = 0;
    for (uint64_t lo = 1, d = 1; n && lo <= first + n - 1; lo *= 10, d++) {
        const uint64_t hi = lo > UINT64_MAX / 10 ? UINT64_MAX : lo * 10 - 1;
        const uint64_t a = std::max(lo, first), b = std::min(hi, first + n - 1);
        if (a <= b) tot += d * (b - a + 1);
        if (hi == UINT64_MAX) break;
    }
    return tot;
}

}  // namespace

extern "C" {

int ntc_decode_file(ntc_ctx *const *ctxs, int n_ctx, const char *in_path, int out_fd, const ntc_pipeline_opts *opts,
                    ntc_pipeline_stats *stats) {
    if (!ctxs || n_ctx <= 0 || !in_path || out_fd < 0) return NTC_ERR_INVALID_ARG;
    for (int i = 0; i < n_ctx; i++)
        if (!ctxs[i]) return NTC_ERR_INVALID_ARG;
    ntc_pipeline_opts o{};
    if (opts) o = *opts;
    const int T = o.threads > 0 ? o.threads : ntc_host_threads();
    // two blocks per GPU call: ~21 MB of text per batch keeps the pinned ring small and the
    // writer (the bound: ~8 GB/s into one file's page cache) busy from the first 20 ms
    const uint64_t bpb = (uint64_t)(o.blocks_per_batch > 0 ? o.blocks_per_batch : 2);
    ntc_pipeline_stats S{};
    const auto t0 = Clock::now();

    // ---- map + extents ------------------------------------------------------------------
    const int fd = ::open(in_path, O_RDONLY);
    if (fd < 0) return NTC_ERR_IO;
    struct stat st;
    if (fstat(fd, &st) != 0) {
        ::close(fd);
        return NTC_ERR_IO;
    }
    const uint64_t fsize = (uint64_t)st.st_size;
    const uint8_t *data = nullptr;
    if (fsize) {
        data = (const uint8_t *)mmap(nullptr, fsize, PROT_READ, MAP_PRIVATE, fd, 0);
        if (data == MAP_FAILED) {
            ::close(fd);
            return NTC_ERR_IO;
        }
        madvise((void *)data, fsize, MADV_SEQUENTIAL);
    }
    ::close(fd);
    auto le32 = [&](uint64_t p) { return (uint64_t)data[p] | (uint64_t)data[p + 1] << 8 | (uint64_t)data[p + 2] << 16 |
                                         (uint64_t)data[p + 3] << 24; };
    // A block's buffers are sized from its headers before anything is inflated, so each
    // header is checked against its own gzip stream first: the ISIZE trailer must equal
    // 8 x encoded_size, which deflate cannot exceed 1032 x block_size, and stream 2 (Rice: one
    // bit per value at least) bounds num_u64.  A block that fails is damaged -- the output ends
    // before it, as the reference's loop ends at decode_block's Err (main.rs:202) -- instead of
    // a pinned allocation sized from garbage.
    std::vector<DBlock> blocks;
    for (uint64_t pos = 32; pos < fsize;) {  // after the 32-byte file header (main.rs:196-198)
        uint64_t p = pos, nrec = 0, pay = 0;
        bool whole = true, bad = false;
        for (int s = 0; s < 4 && whole; s++) {
            if (p + 32 > fsize) {
                whole = false;
                break;
            }
            const uint64_t bs = le32(p), enc = le32(p + 12);
            if (s == 2) nrec = le32(p + 8);
            if (bs < 18 || p + 32 + bs > fsize || le32(p + 32 + bs - 4) != ((8 * enc) & 0xFFFFFFFFULL) ||
                8 * enc > 1032 * bs || (s == 2 && nrec > 64 * enc))
                bad = true;
            pay += 8 * enc;
            p += 32 + bs;
            if (p > fsize) whole = false;
        }
        if (!whole) break;
        // a bad block is sized as nothing; the unzip pool reports it damaged
        blocks.push_back(bad ? DBlock{pos, p - pos, 0, 0, true} : DBlock{pos, p - pos, nrec, pay, false});
        pos = p;
    }
    // NTC_FIRST_BATCH_BLOCKS=n: batch 0 holds n blocks, the others blocks_per_batch.  A
    // one-block first batch (the writer -- the pipeline's bound -- starting sooner) measured
    // no better on the box: the first write still came at ~20 ms, pipeline 0.160-0.198 s
    // against 0.166-0.178 s (profiles/round6/e2e_first_batch/), so the default stays bpb.
    const char *fbe = std::getenv("NTC_FIRST_BATCH_BLOCKS");
    const uint64_t b0n = std::max<uint64_t>(1, std::min<uint64_t>(bpb, fbe ? (uint64_t)std::atoll(fbe) : bpb));
    auto batch_first = [&](uint64_t b) -> uint64_t { return b == 0 ? 0 : b0n + (b - 1) * bpb; };
    auto batch_of = [&](uint64_t blk) -> uint64_t { return blk < b0n ? 0 : 1 + (blk - b0n) / bpb; };
    auto batch_end = [&](uint64_t b) -> uint64_t { return std::min<uint64_t>(blocks.size(), batch_first(b + 1)); };
    const uint64_t n_batches = blocks.empty() ? 0 : batch_of(blocks.size() - 1) + 1;
    S.alloc_s = secs(t0, Clock::now());

    const int NB = n_ctx + 2;
    std::vector<DSlot> slots((size_t)NB);
    // the streams decoded on the GPU (default) or on the host pool (NTC_HOST_UNPACK=1): the
    // 10 M-read decode pipeline ran at 8.0 against 7.6 Gbases/s on one MI355X box, the pool's
    // thread-time 0.11 against 0.64 s (profiles/round5/e2e_dec_*)
    const bool gpu_unpack = !host_unpack_on();
    // NTC_PIPE_TRACE=n: the first n batches' events on stderr (ms from the call's start)
    const char *tr = std::getenv("NTC_PIPE_TRACE");
    const uint64_t trace_n = tr ? (uint64_t)std::atoll(tr) : 0;
    auto trace = [&](const char *what, uint64_t b) {
        if (b < trace_n) std::fprintf(stderr, "[pipe] %8.3f ms batch %llu %s\n", 1e3 * secs(t0, Clock::now()),
                                      (unsigned long long)b, what);
    };
    Shared sh;
    uint64_t next_task = 0;       // next block to unzip
    uint64_t next_id = 1;         // main.rs:204: seq.{i+1}
    int64_t stop_batch = -1;      // batch holding the first damaged block (output ends in it)
    std::atomic<double> t_unzip{0}, t_gpu{0}, t_write{0}, t_pin{0};
    auto add_time = [](std::atomic<double> &a, double d) {
        double cur = a.load();
        while (!a.compare_exchange_weak(cur, cur + d)) {
        }
    };
    auto slot_of = [&](uint64_t b) -> DSlot & { return slots[(size_t)(b % (uint64_t)NB)]; };
    // pinned buffers are sized per batch (grown in the claiming thread, outside the lock)
    auto ensure_pinned = [&](void **p, uint64_t *cap, uint64_t need) -> bool {
        if (need <= *cap) return true;
        const auto tp = Clock::now();
        struct Acc {
            std::atomic<double> &a;
            Clock::time_point t;
            ~Acc() {
                double cur = a.load(), d = secs(t, Clock::now());
                while (!a.compare_exchange_weak(cur, cur + d)) {
                }
            }
        } acc{t_pin, tp};
        pinned_free(*p);
        *p = nullptr;
        *cap = 0;
        const uint64_t want = need + need / 8 + 4096;
        if (!(*p = pinned_alloc(want))) return false;
        *cap = want;
        return true;
    };

    // ">seq.N" numbering: batch a gets first_id once every batch before it has its read count
    // (host unpack: the batch is complete; GPU unpack: the device has decoded its streams).
    // Whichever thread completes a count numbers the batches as far ahead as they allow, so
    // their GPU work overlaps the writes of the batches before them (round 5's first version
    // numbered them in the writer's loop only: a batch's text then waited for the write of
    // the one before it, 3.1 ms per batch where the write takes 2).
    uint64_t next_assign = 0;
    auto assign_ahead = [&]() {  // under sh.mu
        while (next_assign < n_batches) {
            if (stop_batch >= 0 && (int64_t)next_assign > stop_batch) break;
            DSlot &sl = slot_of(next_assign);
            if (sl.batch != next_assign || sl.finished != sl.n_blocks) break;
            if (gpu_unpack && !sl.unpacked) break;
            if (!gpu_unpack && sl.bad_block >= 0) {  // only the blocks before the damaged one
                uint64_t n = 0;
                for (int i = 0; i < sl.bad_block; i++) n += blocks[sl.first_block + (uint64_t)i].n_recs;
                sl.n_recs = n;
                sl.n_reads = sl.n_bases = 0;
                count_reads(sl.recs, n, &sl.n_reads, &sl.n_bases);
            }
            sl.first_id = next_id;
            next_id += sl.n_reads;
            sl.ready = true;
            next_assign++;
            sh.cv.notify_all();
        }
    };
    // ---- GPU drivers ---------------------------------------------------------------------------
    // A batch is complete when all of its blocks are in (or every block before its first
    // damaged one, once no task of it is still running).  The assigner (below, in the
    // writer's loop) fixes first_id in batch order.
    std::vector<std::thread> gpus;
    for (int c = 0; c < n_ctx; c++)
        gpus.emplace_back([&, c] {
            // While the pool inflates the first batches: one tiny unpack (an empty block) and
            // one tiny decode (a one-base read), so the first real calls find the unpacker's
            // and the formatter's code objects loaded (HIP loads them at a kernel's first
            // launch: ~10 ms on the first batch's path otherwise)
            if (gpu_unpack && !std::getenv("NTC_NO_WARM")) {
                ntc_block_meta m0{};
                uint64_t ok = 0, nr = 0, nbs = 0, len = 0, brecs = 0, bpay = 0;
                uint8_t pay0[8] = {0}, txt[64];
                const uint64_t rec1 = (uint64_t)(1u | 2u | (1u << 2)) << 56;  // first, short, 1 base "A"
                // (the larger of this context's first two batches: batch 0 is one block)
                for (uint64_t b2 = (uint64_t)c; b2 < n_batches && b2 <= (uint64_t)c + (uint64_t)n_ctx; b2 += (uint64_t)n_ctx) {
                    uint64_t r2 = 0, p2 = 0;
                    for (uint64_t i = batch_first(b2); i < batch_end(b2); i++) {
                        r2 += blocks[i].n_recs;
                        p2 += blocks[i].pay;
                    }
                    brecs = std::max(brecs, r2);
                    bpay = std::max(bpay, p2);
                }
                // ... and the device workspaces sized for the first batches (hipMalloc'd here)
                trace("warm-up start", c);
                const int w1 = ntc_unpack_streams(ctxs[c], pay0, 8, &m0, 1, &ok, &nr, &nbs);
                trace("warm-up unpack", c);
                const int w2 = w1 ? w1 : ntc_decode_fasta(ctxs[c], &rec1, 1, 1, 1, 1, txt, sizeof(txt), &len);
                trace("warm-up decode", c);
                const int w3 = w2 ? w2 : ntc::reserve_decode(ctxs[c], bpay, brecs, nullptr, 0);
                trace("warm-up reserve", c);
                if (w3) {
                    sh.fail(NTC_ERR_HIP, std::string("decode: ") + ntc_last_error(ctxs[c]));
                    return;
                }
            }
            for (uint64_t b = (uint64_t)c;; b += (uint64_t)n_ctx) {
                DSlot *slp;
                if (gpu_unpack) {
                    // the batch's streams decoded on the device as soon as every block of it is
                    // inflated (or found damaged): its read count numbers the batches after it
                    {
                        std::unique_lock<std::mutex> g(sh.mu);
                        sh.cv.wait(g, [&] {
                            return sh.error != NTC_OK || b >= n_batches || (stop_batch >= 0 && (int64_t)b > stop_batch) ||
                                   (slot_of(b).batch == b && slot_of(b).finished == slot_of(b).n_blocks);
                        });
                        if (sh.error != NTC_OK || b >= n_batches || (stop_batch >= 0 && (int64_t)b > stop_batch)) return;
                        slp = &slot_of(b);
                    }
                    DSlot &sl = *slp;
                    const uint64_t nb = sl.bad_block >= 0 ? (uint64_t)sl.bad_block : sl.n_blocks;
                    const auto tg = Clock::now();
                    uint64_t ok = 0, nr = 0, nbs = 0;
                    const int rc = ntc_unpack_streams(ctxs[c], sl.pay, sl.n_pay, sl.metas.data(), nb, &ok, &nr, &nbs);
                    add_time(t_gpu, secs(tg, Clock::now()));
                    if (rc) {
                        sh.fail(rc, std::string("decode: ") + ntc_last_error(ctxs[c]));
                        return;
                    }
                    {
                        std::unique_lock<std::mutex> g(sh.mu);
                        if (ok < nb) {  // a block the device could not decode: the output ends before it
                            sl.bad_block = (int)ok;
                            if (stop_batch < 0 || (int64_t)b < stop_batch) stop_batch = (int64_t)b;
                        }
                        sl.n_reads = nr;
                        sl.n_bases = nbs;
                        sl.unpacked = true;
                        trace("unpacked", b);
                        assign_ahead();
                        sh.cv.notify_all();
                        sh.cv.wait(g, [&] { return sh.error != NTC_OK || sl.ready; });
                        if (sh.error != NTC_OK) return;
                    }
                    const uint64_t need = sl.n_bases + 7 * sl.n_reads + digits_total(sl.first_id, sl.n_reads) + 64;
                    const auto tf = Clock::now();
                    if (!ensure_pinned((void **)&sl.text, &sl.cap_text, need)) {
                        sh.fail(NTC_ERR_HIP, "pinned host allocation failed");
                        return;
                    }
                    uint64_t len = 0;
                    const int rf = ntc_decode_fasta_unpacked(ctxs[c], sl.first_id, sl.text, sl.cap_text, &len);
                    add_time(t_gpu, secs(tf, Clock::now()));
                    if (rf) {
                        sh.fail(rf, std::string("decode: ") + ntc_last_error(ctxs[c]));
                        return;
                    }
                    std::lock_guard<std::mutex> g(sh.mu);
                    sl.text_len = len;
                    sl.decoded = true;
                    trace("decoded", b);
                    S.gpu_done_s = secs(t0, Clock::now());
                    sh.cv.notify_all();
                    continue;
                }
                {
                    std::unique_lock<std::mutex> g(sh.mu);
                    sh.cv.wait(g, [&] {
                        return sh.error != NTC_OK || b >= n_batches || (stop_batch >= 0 && (int64_t)b > stop_batch) ||
                               (slot_of(b).batch == b && slot_of(b).ready);
                    });
                    if (sh.error != NTC_OK || b >= n_batches || (stop_batch >= 0 && (int64_t)b > stop_batch)) return;
                    slp = &slot_of(b);
                }
                DSlot &sl = *slp;
                const uint64_t nrec = sl.n_recs;
                const uint64_t need = sl.n_bases + 7 * sl.n_reads + digits_total(sl.first_id, sl.n_reads) + 64;
                const auto tg = Clock::now();
                if (!ensure_pinned((void **)&sl.text, &sl.cap_text, need)) {
                    sh.fail(NTC_ERR_HIP, "pinned host allocation failed");
                    return;
                }
                uint64_t len = 0;
                const int rc = ntc_decode_fasta(ctxs[c], sl.recs, nrec, sl.n_reads, sl.n_bases, sl.first_id, sl.text,
                                                sl.cap_text, &len);
                add_time(t_gpu, secs(tg, Clock::now()));
                if (rc) {
                    sh.fail(rc, std::string("decode: ") + ntc_last_error(ctxs[c]));
                    return;
                }
                std::lock_guard<std::mutex> g(sh.mu);
                sl.text_len = len;
                sl.decoded = true;
                trace("decoded", b);
                S.gpu_done_s = secs(t0, Clock::now());
                sh.cv.notify_all();
            }
        });

    // ---- pinned buffers of the first batches, allocated in parallel -----------------------------
    // (each is mapped, touched and registered: ~10 ms for a batch's 21 MB of text, which the
    // first batch would otherwise wait for in turn; later batches reuse them).  The text size
    // is a guess from the records (48 bytes each: C91's reads take 41); a batch that needs
    // more regrows its buffer as before.
    {
        std::vector<std::thread> pre;
        for (uint64_t j = 0; j < (uint64_t)NB && j < n_batches; j++)
            pre.emplace_back([&, j] {
                uint64_t nr = 0, np = 0;
                for (uint64_t i = batch_first(j); i < batch_end(j); i++) {
                    nr += blocks[i].n_recs;
                    np += blocks[i].pay;
                }
                DSlot &sl = slots[(size_t)j];
                const bool ok = (gpu_unpack ? ensure_pinned((void **)&sl.pay, &sl.cap_pay, np + 8)
                                            : ensure_pinned((void **)&sl.recs, &sl.cap_recs, nr * 8 + 8)) &&
                                ensure_pinned((void **)&sl.text, &sl.cap_text, nr * 48 + (1u << 20));
                if (!ok) sh.fail(NTC_ERR_HIP, "pinned host allocation failed");
            });
        for (auto &t : pre) t.join();
    }

    // ---- unzip pool ------------------------------------------------------------------------
    // Blocks are taken in file order; the first block of a batch claims the batch's slot
    // (free once the writer is done with batch b - NB) and sizes its record buffer.  Past a
    // damaged block no later batch is started; the rest of its own batch is still unzipped
    // so that the batch completes (only the blocks before the damaged one are decoded).
    std::vector<std::thread> pool;
    for (int t = 0; t < T; t++)
        pool.emplace_back([&] {
            for (;;) {
                uint64_t blk, b;
                bool first;
                {
                    std::unique_lock<std::mutex> g(sh.mu);
                    auto exhausted = [&] {
                        return sh.error != NTC_OK || next_task >= blocks.size() ||
                               (stop_batch >= 0 && (int64_t)batch_of(next_task) > stop_batch);
                    };
                    sh.cv.wait(g, [&] {
                        if (exhausted()) return true;
                        const uint64_t nb = batch_of(next_task);
                        const DSlot &sl = slot_of(nb);
                        return sl.batch == nb || sl.batch == ~0ULL;
                    });
                    if (exhausted()) return;
                    blk = next_task++;
                    b = batch_of(blk);
                    DSlot &sl = slot_of(b);
                    first = sl.batch != b;
                    if (first) {
                        DSlot fresh;
                        fresh.recs = sl.recs;
                        fresh.cap_recs = sl.cap_recs;
                        fresh.pay = sl.pay;
                        fresh.cap_pay = sl.cap_pay;
                        fresh.text = sl.text;
                        fresh.cap_text = sl.cap_text;
                        fresh.metas.swap(sl.metas);
                        sl = std::move(fresh);
                        sl.batch = b;
                        sl.first_block = batch_first(b);
                        sl.n_blocks = batch_end(b) - sl.first_block;
                        for (uint64_t i = 0; i < sl.n_blocks; i++) {
                            sl.n_recs += blocks[sl.first_block + i].n_recs;
                            sl.n_pay += blocks[sl.first_block + i].pay;
                        }
                        sl.metas.assign(sl.n_blocks, ntc_block_meta{});
                    }
                }
                DSlot &sl = slot_of(b);
                if (first) {  // size the batch's pinned record / stream buffer outside the lock
                    const bool okp = gpu_unpack ? ensure_pinned((void **)&sl.pay, &sl.cap_pay, sl.n_pay + 8)
                                                : ensure_pinned((void **)&sl.recs, &sl.cap_recs, sl.n_recs * 8 + 8);
                    if (!okp) {
                        sh.fail(NTC_ERR_HIP, "pinned host allocation failed");
                        return;
                    }
                    std::lock_guard<std::mutex> g(sh.mu);
                    sl.buffer = true;
                    sh.cv.notify_all();
                } else {
                    std::unique_lock<std::mutex> g(sh.mu);
                    sh.cv.wait(g, [&] { return sh.error != NTC_OK || sl.buffer; });
                    if (sh.error != NTC_OK) return;
                }
                uint64_t off = 0, poff = 0;
                for (uint64_t i = sl.first_block; i < blk; i++) {
                    off += blocks[i].n_recs;
                    poff += blocks[i].pay;
                }
                const auto tu = Clock::now();
                uint64_t used = 0, nr = 0, numr = 0, reads = 0, bases = 0;
                const DBlock &db = blocks[blk];
                int rc;
                if (db.bad) {
                    rc = NTC_ERR_FORMAT;
                    if (gpu_unpack) sl.metas[blk - sl.first_block].status = rc;
                } else if (gpu_unpack) {  // inflate only: the streams are decoded on the GPU
                    ntc_block_meta &m = sl.metas[blk - sl.first_block];
                    rc = ntc_read_block_streams(data + db.a, db.len, &used, sl.pay + poff, db.pay, &m);
                    if (rc == NTC_OK && (m.n_recs != db.n_recs || used != db.len)) rc = NTC_ERR_FORMAT;
                    for (int i = 0; i < 4; i++) m.stream[i].offset += poff;
                    if (rc != NTC_OK) m.status = rc;
                } else {
                    rc = ntc_read_block_into(data + db.a, db.len, &used, sl.recs + off, db.n_recs, &nr, &numr);
                    if (rc == NTC_OK && (nr != db.n_recs || used != db.len)) rc = NTC_ERR_FORMAT;
                    if (rc == NTC_OK) count_reads(sl.recs + off, nr, &reads, &bases);
                }
                add_time(t_unzip, secs(tu, Clock::now()));
                std::lock_guard<std::mutex> g(sh.mu);
                const int bi = (int)(blk - sl.first_block);
                if (rc != NTC_OK) {
                    if (sl.bad_block < 0 || bi < sl.bad_block) sl.bad_block = bi;
                    if (stop_batch < 0 || (int64_t)b < stop_batch) stop_batch = (int64_t)b;
                } else {
                    sl.n_reads += reads;  // recounted below when the batch holds a damaged block
                    sl.n_bases += bases;
                }
                sl.finished++;
                if (blk + 1 == blocks.size() || (stop_batch >= 0 && sl.finished == sl.n_blocks))
                    S.reader_done_s = secs(t0, Clock::now());
                if (sl.finished == sl.n_blocks) trace("inflated", b);
                if (!gpu_unpack && sl.finished == sl.n_blocks) assign_ahead();
                sh.cv.notify_all();
            }
        });

    // ---- assigner + writer (this thread) ------------------------------------------------------------
    struct stat ost;
    // pwrite only into a regular file opened without O_APPEND (Linux pwrite ignores the
    // offset under O_APPEND); the shared file offset is moved past the text at the end, so
    // `{ decode a; decode b; } > out` keeps both outputs as the reference's stdout does
    const int fl = fcntl(out_fd, F_GETFL);
    const bool seekable = fstat(out_fd, &ost) == 0 && S_ISREG(ost.st_mode) && fl >= 0 && !(fl & O_APPEND) &&
                          lseek(out_fd, 0, SEEK_CUR) >= 0;
    off_t out_pos = seekable ? lseek(out_fd, 0, SEEK_CUR) : 0;
    // one writer: buffered writes into one file serialise on its inode lock, and on the GPU
    // box one thread's pwrite put 1.6 GB into the page cache at 12.6 GB/s against 10.4 from
    // 8 threads at their own offsets and 1.9 through a shared mapping
    // (profiles/round5/write_bw_box.jsonl, scripts/write_bw.cpp)
    auto write_text = [&](const uint8_t *p, uint64_t n) -> bool {
        while (n) {
            const ssize_t w = seekable ? ::pwrite(out_fd, p, n, out_pos) : ::write(out_fd, p, n);
            if (w <= 0) return false;
            p += w;
            n -= (uint64_t)w;
            out_pos += w;
        }
        return true;
    };
    for (uint64_t b = 0; b < n_batches; b++) {
        DSlot *slp;
        {
            std::unique_lock<std::mutex> g(sh.mu);
            sh.cv.wait(g, [&] {
                if (sh.error != NTC_OK) return true;
                if (stop_batch >= 0 && (int64_t)b > stop_batch) return true;
                assign_ahead();
                const DSlot &sl = slot_of(b);
                return sl.batch == b && sl.decoded;
            });
            if (sh.error != NTC_OK || (stop_batch >= 0 && (int64_t)b > stop_batch)) break;
            slp = &slot_of(b);
        }
        const auto tw = Clock::now();
        if (!write_text(slp->text, slp->text_len)) sh.fail(NTC_ERR_IO, "write failed");
        add_time(t_write, secs(tw, Clock::now()));
        std::lock_guard<std::mutex> g(sh.mu);
        if (b == 0) S.first_batch_s = secs(t0, Clock::now());
        trace("written", b);
        S.reads += slp->n_reads;
        S.bases += slp->n_bases;
        S.bytes_out += slp->text_len;
        S.blocks += slp->bad_block >= 0 ? (uint64_t)slp->bad_block : slp->n_blocks;
        const bool last = stop_batch >= 0 && (int64_t)b == stop_batch;
        slp->batch = ~0ULL;  // free the slot
        sh.cv.notify_all();
        if (last) break;
    }
    {
        std::lock_guard<std::mutex> g(sh.mu);
        if (sh.error == NTC_OK) sh.error = -1;  // stop the workers
        sh.cv.notify_all();
    }
    for (auto &t : pool) t.join();
    for (auto &t : gpus) t.join();
    for (auto &sl : slots) {
        pinned_free(sl.recs);
        pinned_free(sl.pay);
        pinned_free(sl.text);
    }
    if (data) munmap((void *)data, fsize);
    if (seekable) (void)lseek(out_fd, out_pos, SEEK_SET);
    const int result = sh.error == -1 ? NTC_OK : sh.error;
    S.dropped_blocks = blocks.size() - S.blocks;  // after a damaged block (or none)
    S.alloc_s += t_pin.load();
    S.parse_s = t_unzip.load();
    S.gpu_s = t_gpu.load();
    S.write_s = t_write.load();
    S.wall_s = secs(t0, Clock::now());
    S.threads = T;
    S.bad_read = -1;
    if (result != NTC_OK)
        std::snprintf(S.error, sizeof(S.error), "%s", sh.msg.c_str());
    else if (stop_batch >= 0)  // not an error for the reference either: its loop just ends
        std::snprintf(S.error, sizeof(S.error), "damaged block %llu: output ends before it",
                      (unsigned long long)S.blocks);
    if (stats) *stats = S;
    return result;
}

}  // extern "C"
