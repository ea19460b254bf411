// Sanitizer driver (tests/san, CPU only): runs the library's host code -- FASTX ingest
// (fastx.cpp: plain / gzip / BGZF / bz2 / xz / zstd), the block codec (block_codec.cpp),
// index files (index_io.cpp), the threaded host builder (sbwt_build.cpp) and the native
// file pipelines' host threads (pipeline.cpp, GPU stage stubbed by gpu_stub.cpp) -- built
// with -fsanitize=address,undefined or -fsanitize=thread (Makefile).  Each command prints
// one line of results; tests/test_sanitizers.py compares them with the production library
// and fails on any sanitizer report.
#include <fcntl.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ntcomp_codec.h"
#include "../../include/ntcomp_host.h"
#include "../../include/ntcomp_pipeline.h"
#include "../../ntcomp_amd/csrc/ntc_internal.h"

extern "C" {
struct orc_index;
orc_index *orc_index_new(uint64_t n, uint32_t k, const uint64_t *rowA, const uint64_t *rowC, const uint64_t *rowG,
                         const uint64_t *rowT, const uint64_t *Carr, const uint8_t *lcs, uint32_t precalc);
void orc_index_free(orc_index *ix);
}
ntc_ctx *stub_ctx_new(const orc_index *ix);
void stub_ctx_free(ntc_ctx *c);

static uint64_t fnv(uint64_t h, const void *p, size_t n) {
    const uint8_t *b = (const uint8_t *)p;
    for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 0x100000001b3ULL;
    return h;
}

static std::vector<uint8_t> slurp(const char *path) {
    std::vector<uint8_t> v;
    FILE *f = std::fopen(path, "rb");
    if (!f) return v;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) v.insert(v.end(), buf, buf + n);
    std::fclose(f);
    return v;
}

// fastx PATH THREADS MAX_READS MAX_BASES INTO(0/1)
static int cmd_fastx(char **a) {
    ntc_fastx *fx = nullptr;
    int rc = ntc_fastx_open(a[0], &fx);
    uint64_t reads = 0, bases = 0, batches = 0, h = 0xcbf29ce484222325ULL;
    if (rc == 0) {
        ntc_fastx_set_threads(fx, std::atoi(a[1]));
        const uint64_t mr = std::strtoull(a[2], nullptr, 10), mb = std::strtoull(a[3], nullptr, 10);
        const bool into = std::atoi(a[4]) != 0;
        std::vector<uint8_t> buf(into ? mb + (1 << 20) : 0);
        std::vector<uint64_t> offs(into ? mr + 1 : 0);
        for (;;) {
            const uint8_t *b = nullptr;
            const uint64_t *o = nullptr;
            uint64_t n = 0;
            if (into) {
                rc = ntc_fastx_next_batch_into(fx, mr, mb, buf.data(), buf.size(), offs.data(), &n);
                b = buf.data();
                o = offs.data();
            } else {
                rc = ntc_fastx_next_batch(fx, mr, mb, &b, &o, &n);
            }
            if (rc || n == 0) break;
            batches++;
            for (uint64_t r = 0; r < n; r++) {
                const uint64_t L = o[r + 1] - o[r];
                h = fnv(h, &L, 8);
                h = fnv(h, b + o[r], L);
            }
            reads += n;
            bases += o[n] - o[0];
        }
        ntc_fastx_close(fx);
    }
    std::printf("rc=%d reads=%llu bases=%llu hash=%016llx\n", rc, (unsigned long long)reads,
                (unsigned long long)bases, (unsigned long long)h);
    return 0;
}

// blocks PATH: every block of an encoded.dat (after the 32-byte file header)
static int cmd_blocks(char **a) {
    std::vector<uint8_t> d = slurp(a[0]);
    uint64_t pos = d.size() >= 32 ? 32 : d.size(), blocks = 0, recs_total = 0, h = 0xcbf29ce484222325ULL;
    int rc = 0;
    while (pos < d.size()) {
        uint64_t used = 0, nrec = 0, num = 0;
        uint64_t *recs = nullptr;
        rc = ntc_read_block(d.data() + pos, d.size() - pos, &used, &recs, &nrec, &num);
        if (rc) break;
        h = fnv(h, recs, nrec * 8);
        h = fnv(h, &num, 8);
        ntc_buffer_free(recs);
        recs_total += nrec;
        blocks++;
        pos += used;
    }
    std::printf("rc=%d blocks=%llu recs=%llu hash=%016llx\n", rc, (unsigned long long)blocks,
                (unsigned long long)recs_total, (unsigned long long)h);
    return 0;
}

static uint64_t index_hash(const ntc::HostIndex &ix) {
    uint64_t h = 0xcbf29ce484222325ULL;
    h = fnv(h, &ix.n, 8);
    h = fnv(h, &ix.k, 4);
    h = fnv(h, ix.C, 32);
    for (int c = 0; c < 4; c++) h = fnv(h, ix.rows[c].data(), ix.rows[c].size() * 8);
    return fnv(h, ix.lcs.data(), ix.lcs.size());
}

// index PREFIX [SAVE_PREFIX LAYOUT PREFIX_LEN]
static int cmd_index(char **a, int n) {
    ntc::HostIndex ix;
    std::string err;
    const bool ok = ntc::load_index(a[0], ix, err);
    if (ok && n >= 4) {
        ix.prefix_len = (uint32_t)std::atoi(a[3]);
        if (ix.prefix_len) ntc::prefix_table(ix, ix.prefix_len, ix.prefix_ranges);
        if (!ntc::save_index_as(ix, a[1], std::atoi(a[2]), err)) {
            std::printf("rc=save %s\n", err.c_str());
            return 0;
        }
    }
    std::printf("rc=%d n=%llu hash=%016llx\n", ok ? 0 : 1, (unsigned long long)ix.n,
                ok ? (unsigned long long)index_hash(ix) : 0ULL);
    return 0;
}

// build FASTX K THREADS: the threaded host builder on every sequence of the file
static int cmd_build(char **a) {
    ntc_fastx *fx = nullptr;
    if (ntc_fastx_open(a[0], &fx)) return 2;
    std::vector<uint8_t> seq;
    std::vector<uint64_t> offs{0};
    for (;;) {
        const uint8_t *b;
        const uint64_t *o;
        uint64_t n = 0;
        if (ntc_fastx_next_batch(fx, 1 << 16, 1 << 26, &b, &o, &n) || !n) break;
        for (uint64_t r = 0; r < n; r++) {
            seq.insert(seq.end(), b + o[r], b + o[r + 1]);
            offs.push_back(seq.size());
        }
    }
    ntc_fastx_close(fx);
    ntc::HostIndex ix;
    ntc::build_index(seq.data(), offs.data(), offs.size() - 1, (uint32_t)std::atoi(a[1]), true, std::atoi(a[2]), ix);
    std::printf("rc=0 n=%llu hash=%016llx\n", (unsigned long long)ix.n, (unsigned long long)index_hash(ix));
    return 0;
}

// encode|decode PREFIX IN OUT THREADS BPB NCTX [DEFLATE [HOST_PARSE [REPS]]]
// REPS > 0 (the host-ceiling build, -DNTC_STUB_MEMO): the pipeline's own batch sizes, one
// untimed run that fills the stub's memo, then REPS timed runs; wall = the fastest
static int cmd_pipe(bool enc, char **a, int n) {
    ntc::HostIndex ix;
    std::string err;
    if (!ntc::load_index(a[0], ix, err)) {
        std::printf("rc=index %s\n", err.c_str());
        return 0;
    }
    orc_index *o = orc_index_new(ix.n, ix.k, ix.rows[0].data(), ix.rows[1].data(), ix.rows[2].data(),
                                 ix.rows[3].data(), ix.C, ix.lcs.data(), 8);
    const int nctx = std::atoi(a[5]);
    std::vector<ntc_ctx *> ctxs;
    for (int i = 0; i < nctx; i++) ctxs.push_back(stub_ctx_new(o));
    const int reps = n >= 9 ? std::atoi(a[8]) : 0;
    ntc_pipeline_opts opts{};
    opts.threads = std::atoi(a[3]);
    opts.blocks_per_batch = std::atoi(a[4]);
    opts.batch_bases = enc && reps == 0 ? (1u << 20) : 0;  // small ring buffers: many batches, buffer growth
    opts.deflate_engine = n >= 7 ? std::atoi(a[6]) : NTC_DEFLATE_ZLIB;
    opts.host_parse = n >= 8 ? std::atoi(a[7]) : 0;
    ntc_pipeline_stats st{};
    int rc = 0;
    double best = 1e30;
    for (int rep = 0; rep <= reps; rep++) {
        const int fd = ::open(a[2], O_WRONLY | O_CREAT | O_TRUNC, 0644);
        const auto t0 = std::chrono::steady_clock::now();
        st = ntc_pipeline_stats{};
        rc = enc ? ntc_encode_file(ctxs.data(), nctx, a[1], fd, &opts, &st)
                 : ntc_decode_file(ctxs.data(), nctx, a[1], fd, &opts, &st);
        ::close(fd);
        const double w = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (rep > 0 && w < best) best = w;
        if (rc) break;
    }
    if (reps > 0)
        std::printf("wall=%.4f gbases_s=%.3f parse_s=%.4f gpu_s=%.4f deflate_s=%.4f write_s=%.4f alloc_s=%.4f "
                    "first_batch_s=%.4f reader_done_s=%.4f ",
                    best, st.bases / best / 1e9, st.parse_s, st.gpu_s, st.deflate_s, st.write_s, st.alloc_s,
                    st.first_batch_s, st.reader_done_s);
    for (auto *c : ctxs) stub_ctx_free(c);
    orc_index_free(o);
    std::printf("rc=%d reads=%llu bases=%llu blocks=%llu dropped=%llu bad=%lld text=%d\n", rc,
                (unsigned long long)st.reads, (unsigned long long)st.bases, (unsigned long long)st.blocks,
                (unsigned long long)st.dropped_blocks, (long long)st.bad_read, st.gpu_parsed);
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const std::string c = argv[1];
    char **a = argv + 2;
    const int n = argc - 2;
    if (c == "fastx" && n >= 5) return cmd_fastx(a);
    if (c == "blocks" && n >= 1) return cmd_blocks(a);
    if (c == "index" && n >= 1) return cmd_index(a, n);
    if (c == "build" && n >= 3) return cmd_build(a);
    if ((c == "encode" || c == "decode") && n >= 6) return cmd_pipe(c == "encode", a, n);
    std::fprintf(stderr, "usage: san_driver fastx|blocks|index|build|encode|decode ...\n");
    return 2;
}
