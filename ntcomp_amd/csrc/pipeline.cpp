// Native encode pipeline of the CLI: `ntcomp encode -i P reads.fq > encoded.dat`
// (src/main.rs:141-181), file in, encoded.dat out, with every stage overlapped:
//
//   reader   FASTX batches of blocks_per_batch x 65,536 reads (main.rs:152) into a ring of
//            pinned host buffers (ntc_fastx_next_batch_into: plain FASTQ is mapped and
//            parsed by the host pool).  Reads past the last whole block of a batch carry
//            into the next buffer, so every block but the file's last holds exactly 65,536
//            reads, and the last holds num_records % 65,536 (main.rs:174-177).
//   GPU      one driver thread per context, batches dealt round-robin:
//            ntc_encode_pack_batch = H2D, encode kernels, GPU block packer, D2H of the four
//            coded streams per block (the u64 records never leave HBM).
//   deflate  the host pool gzips each block's streams (ntc_deflate_block) -- the only
//            codec step left on the CPU.
//   writer   the calling thread writes the file header (lib.rs:52-67) and the blocks in
//            file order; a block the reference drops (no long or no short record,
//            write_block_to errs and main.rs:170 ignores it -- App. B.3) is skipped.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
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

namespace {

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

struct Batch {  // one pinned buffer of the ring
    uint8_t *bases = nullptr;
    uint64_t *offs = nullptr;
    uint64_t cap_bases = 0, cap_reads = 0;
    uint64_t n_reads = 0;    // reads in the buffer (carry + new)
    uint64_t n_process = 0;  // reads handed to the GPU (whole blocks, or all at the end)
    uint64_t first_read = 0; // file index of the buffer's first read
    uint64_t first_block = 0;
    bool busy = false;
};

struct BlockOut {  // a deflated block, or a dropped one
    uint8_t *data = nullptr;
    uint64_t len = 0;
    int status = NTC_OK;
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
    const uint64_t per_batch = (uint64_t)(o.blocks_per_batch > 0 ? o.blocks_per_batch : 16) * BR;
    const uint64_t cap_bases = o.batch_bases > 0 ? o.batch_bases : (256ull << 20);
    const int engine = o.deflate_engine;
    ntc_pipeline_stats S{};
    const auto t0 = Clock::now();

    ntc_fastx *fx = nullptr;
    int rc = ntc_fastx_open(in_path, &fx);
    if (rc) return rc;
    ntc_fastx_set_threads(fx, T);

    // pinned ring: the GPU threads hold at most n_ctx buffers, the reader fills one more
    const int NB = n_ctx + 2;
    std::vector<Batch> ring((size_t)NB);
    for (auto &b : ring) {
        b.cap_bases = cap_bases + BR * 1024ull;  // a carry of < 65,536 reads sits in front
        b.cap_reads = per_batch + BR + 1;
        if (hipHostMalloc((void **)&b.bases, b.cap_bases, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void **)&b.offs, b.cap_reads * 8, hipHostMallocDefault) != hipSuccess) {
            for (auto &x : ring) {
                if (x.bases) (void)hipHostFree(x.bases);
                if (x.offs) (void)hipHostFree(x.offs);
            }
            ntc_fastx_close(fx);
            return NTC_ERR_HIP;
        }
    }

    S.alloc_s = secs(t0, Clock::now());
    Shared sh;
    std::vector<std::deque<int>> gpu_q((size_t)n_ctx);  // per context: ring indices in batch order
    bool reader_done = false;
    uint64_t total_blocks = 0;    // known once the reader is done
    std::atomic<double> t_parse{0}, t_gpu{0}, t_deflate{0}, t_write{0};
    // deflate tasks and finished blocks
    struct Task {
        std::shared_ptr<std::vector<uint8_t>> payload;
        ntc_block_meta meta;
        uint64_t block;
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
        uint8_t *nbuf = nullptr;
        if (hipHostMalloc((void **)&nbuf, cap, hipHostMallocDefault) != hipSuccess) return false;
        if (keep_bases) std::memcpy(nbuf, b.bases, keep_bases);
        (void)hipHostFree(b.bases);
        b.bases = nbuf;
        b.cap_bases = cap;
        (void)keep_reads;
        return true;
    };
    std::thread reader([&] {
        uint64_t next_read = 0, next_block = 0, batch_no = 0;
        int prev = -1;
        uint64_t carry = 0;  // reads at the tail of ring[prev] past its processed blocks
        for (;;) {
            int bi;
            {
                std::unique_lock<std::mutex> g(sh.mu);
                bi = (int)(batch_no % (uint64_t)NB);
                sh.cv.wait(g, [&] { return sh.error != NTC_OK || !ring[(size_t)bi].busy; });
                if (sh.error != NTC_OK) break;
            }
            Batch &b = ring[(size_t)bi];
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
                const auto tg = Clock::now();
                const int r = ntc_encode_pack_batch(ctxs[c], b.bases, b.offs, b.n_process, BR, metas.data(), &payload,
                                                    &plen, &bad);
                add_time(t_gpu, secs(tg, Clock::now()));
                if (r) {
                    ntc_buffer_free(payload);
                    sh.fail(r, std::string("encode: ") + ntc_last_error(ctxs[c]),
                            bad >= 0 ? (int64_t)b.first_read + bad : -1);
                    return;
                }
                auto pl = std::make_shared<std::vector<uint8_t>>(payload, payload + plen);
                ntc_buffer_free(payload);
                std::lock_guard<std::mutex> g(sh.mu);
                S.gpu_done_s = secs(t0, Clock::now());
                S.bases += b.offs[b.n_process] - b.offs[0];
                b.busy = false;
                for (uint64_t k = 0; k < nblk; k++) {
                    tasks.push_back(Task{pl, metas[k], b.first_block + k});
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
                BlockOut out;
                const auto td = Clock::now();
                out.status = task.meta.status;
                if (out.status == NTC_OK) {
                    const int r = ntc_deflate_block(&task.meta, task.payload->data(), engine, &out.data, &out.len);
                    if (r) {
                        sh.fail(r, "deflate failed");
                        return;
                    }
                } else if (out.status != NTC_ERR_EMPTY_READ) {
                    sh.fail(out.status, "malformed block");
                    return;
                }
                task.payload.reset();
                add_time(t_deflate, secs(td, Clock::now()));
                std::lock_guard<std::mutex> g(sh.mu);
                done[task.block] = out;
                sh.cv.notify_all();
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
            sh.cv.wait(g, [&] { return sh.error != NTC_OK || done.count(blk) || (reader_done && blk >= total_blocks); });
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
            if (!write_all(out.data, out.len)) sh.fail(NTC_ERR_IO, "write failed");
            S.bytes_out += out.len;
            S.blocks++;
        } else {
            S.dropped_blocks++;
        }
        ntc_buffer_free(out.data);
        add_time(t_write, secs(tw, Clock::now()));
    }
    {
        std::lock_guard<std::mutex> g(sh.mu);
        if (sh.error == NTC_OK) {
            sh.error = -1;  // stop the workers (no more tasks will come)
        }
        sh.cv.notify_all();
    }
    reader.join();
    for (auto &t : gpus) t.join();
    for (auto &t : pool) t.join();
    for (auto &kv : done) ntc_buffer_free(kv.second.data);
    for (auto &b : ring) {
        (void)hipHostFree(b.bases);
        (void)hipHostFree(b.offs);
    }
    ntc_fastx_close(fx);
    const int result = sh.error == -1 ? NTC_OK : sh.error;
    S.parse_s = t_parse.load();
    S.gpu_s = t_gpu.load();
    S.deflate_s = t_deflate.load();
    S.write_s = t_write.load();
    S.wall_s = secs(t0, Clock::now());
    S.threads = T;
    S.bad_read = sh.bad_read;
    std::snprintf(S.error, sizeof(S.error), "%s", result == NTC_OK ? "" : sh.msg.c_str());
    if (stats) *stats = S;
    return result;
}

}  // extern "C"
