// Host-side internal types shared by the builder, index I/O and the C ABI.
#pragma once
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace ntc {

// SBWT subset matrix + LCS in host memory (the form kbo::build / load_sbwt hand over).
struct HostIndex {
    uint64_t n = 0;
    uint32_t k = 0;
    std::vector<uint64_t> rows[4];  // ceil(n/64) words each, LSB-first
    uint64_t C[4] = {0, 0, 0, 0};
    std::vector<uint8_t> lcs;       // n bytes
    // -p/--prefix-precalc lookup table (sbwt PrefixLookupTable): [start, end) per p-mer
    uint32_t prefix_len = 0;
    std::vector<uint64_t> prefix_ranges;  // 2 * 4^prefix_len words
};
// colex interval of every p-mer, first character most significant (index_io.cpp)
void prefix_table(const HostIndex &ix, uint32_t p, std::vector<uint64_t> &ranges);

void build_index(const uint8_t *seqs, const uint64_t *offs, uint64_t nseqs, uint32_t k,
                 bool revcomp, int threads, HostIndex &out);
bool save_index(const HostIndex &ix, const std::string &prefix, std::string &err);
bool load_index(const std::string &prefix, HostIndex &ix, std::string &err);  // either layout
enum { kIndexOwn = 0, kIndexSbwtRs = 1 };  // ntc_index_save_as layouts (index_io.cpp)
bool save_index_as(const HostIndex &ix, const std::string &prefix, int layout, std::string &err);

// T - 1 helper threads that run one job at a time together with the caller (pipeline.cpp:
// the reader's copy + scan of each batch; pgzip.cpp: the symbol conversion of each read;
// spawning threads per batch costs ~1 ms a batch): run(f) calls f(t) on every thread,
// t = 0 the caller, and returns when all are done.
struct Gang {
    std::mutex mu;
    std::condition_variable go, done;
    std::function<void(int)> job;
    uint64_t gen = 0;
    int running = 0;
    bool stop = false;
    std::vector<std::thread> th;
    explicit Gang(int T) {
        for (int t = 1; t < T; t++)
            th.emplace_back([this, t] {
                uint64_t seen = 0;
                for (;;) {
                    std::function<void(int)> j;
                    {
                        std::unique_lock<std::mutex> g(mu);
                        go.wait(g, [&] { return stop || gen != seen; });
                        if (stop) return;
                        seen = gen;
                        j = job;
                    }
                    j(t);
                    std::lock_guard<std::mutex> g(mu);
                    if (--running == 0) done.notify_all();
                }
            });
    }
    int size() const { return (int)th.size() + 1; }
    void run(const std::function<void(int)> &f) {
        {
            std::lock_guard<std::mutex> g(mu);
            job = f;
            running = (int)th.size();
            gen++;
        }
        go.notify_all();
        f(0);
        std::unique_lock<std::mutex> g(mu);
        done.wait(g, [&] { return running == 0; });
    }
    ~Gang() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        go.notify_all();
        for (auto &x : th) x.join();
    }
};

}  // namespace ntc

struct ntc_fastx;
struct ntc_block_meta;
struct ntc_ctx;
namespace ntc {
// a plain FASTQ that ntc_fastx_open mapped: its bytes (null for any other input), and
// moving the mapped parser to byte pos (a record start) -- pipeline.cpp's GPU-parse reader
const uint8_t *fastx_mapped(ntc_fastx *fx, uint64_t *size);
void fastx_seek_mapped(ntc_fastx *fx, uint64_t pos);
// a FASTQ read through a decoder (gzip, BGZF, bz2, xz, zstd) or a pipe: the next decoded
// bytes into dst (up to cap; fewer only at the end of input), and bytes handed back so the
// host parser goes on from them (the GPU-parse reader's fallback)
bool fastx_streamed_fastq(ntc_fastx *fx);
uint64_t fastx_stream_read(ntc_fastx *fx, uint8_t *dst, uint64_t cap, bool *io_error);
void fastx_stream_unread(ntc_fastx *fx, const uint8_t *src, uint64_t n);

// Parallel inflate of a non-BGZF gzip file (pgzip.cpp): null when the file is not gzip.
// pgz_read: cap bytes into dst (fewer only at the end), 1 filled, 0 the end, -1 an error
// (corrupt or truncated data, a CRC or ISIZE mismatch).
// the GPU unpacker's block decode on the host (block_codec.cpp; the sanitizer stand-in)
int unpack_block_host(const ::ntc_block_meta &m, const uint8_t *payload, std::vector<uint64_t> &recs);
// The decode pipeline's device workspaces sized ahead for a batch of about n_recs records in
// pay_bytes of inflated streams (capi.cpp): hipMalloc'd while the first batch inflates
// rather than on its path.  Estimates: at most 3 values and one read per record, 48 bytes of
// FASTA per record; a batch that needs more grows them as before.  host (pinned, host_bytes)
// takes one copy each way of up to 4 MiB: the process's first large copies start the DMA
// engines (7.7 ms before the first batch's text came back otherwise).
int reserve_decode(::ntc_ctx *ctx, uint64_t pay_bytes, uint64_t n_recs, uint8_t *host, uint64_t host_bytes);
struct PgzReader;
PgzReader *pgz_open(const char *path, int threads);
int pgz_read(PgzReader *r, char *dst, size_t cap, size_t *got);
void pgz_close(PgzReader *r);
}  // namespace ntc

struct ntc_index_host {
    ntc::HostIndex ix;
};
