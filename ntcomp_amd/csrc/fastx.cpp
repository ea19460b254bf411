// FASTA / FASTQ ingest for the CLI (include/ntcomp_host.h "FASTX").
//
// Replaces needletail::parse_fastx_file + SequenceRecord::normalize(true) as the reference
// uses them (src/main.rs:51-62 build input, :158-163 encode input): plain, gzip, bzip2,
// xz or zstd input, detected from the magic bytes like needletail's niffler (zlib's gz* reads
// plain and gzip; bzip2, xz and zstd go through libbz2.so.1 / liblzma.so.5 / libzstd.so.1,
// loaded at run time -- the
// image has their runtime libraries but no headers, so the few stable entry points and
// stream structs used are declared below), FASTA records (">" header, sequence over any number of lines)
// and FASTQ records ("@" header, sequence, "+", quality).  normalize(iupac = true) is
// restated from needletail [ext, recalled, needletail 0.6]: A C G T N - kept; a c g ->
// upper case; t u U -> T; n -> N; . ~ -> -; IUPAC B D H V R Y S W K M kept (lower case
// upper-cased); whitespace dropped; anything else -> N.  Record names are not kept (the
// reference discards them on encode, main.rs:158-166).
//
// Feed rate: a producer thread inflates (or reads) 8 MiB chunks into a small ring while
// the caller's thread scans records in place (memchr per line, branch-free table
// normalisation into one growing buffer), so a gzip input is bound by inflate alone.
#include <dlfcn.h>
#include <emmintrin.h>
#include <zlib.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/ntcomp_host.h"

namespace {

uint8_t norm_table[256];
bool norm_init = false;

void init_norm() {
    if (norm_init) return;
    for (int c = 0; c < 256; c++) norm_table[c] = 'N';
    for (const char *p = "ACGTN-"; *p; p++) norm_table[(uint8_t)*p] = (uint8_t)*p;
    norm_table[(uint8_t)'a'] = 'A';
    norm_table[(uint8_t)'c'] = 'C';
    norm_table[(uint8_t)'g'] = 'G';
    norm_table[(uint8_t)'t'] = 'T';
    norm_table[(uint8_t)'u'] = 'T';
    norm_table[(uint8_t)'U'] = 'T';
    norm_table[(uint8_t)'n'] = 'N';
    norm_table[(uint8_t)'.'] = '-';
    norm_table[(uint8_t)'~'] = '-';
    for (const char *p = "BDHVRYSWKM"; *p; p++) {
        norm_table[(uint8_t)*p] = (uint8_t)*p;
        norm_table[(uint8_t)(*p - 'A' + 'a')] = (uint8_t)*p;
    }
    for (const char *p = " \t\r\n"; *p; p++) norm_table[(uint8_t)*p] = 0;  // dropped
    norm_init = true;
}

constexpr size_t kChunk = 8u << 20;
constexpr size_t kRing = 4;

// ---- byte sources ---------------------------------------------------------------------
struct ByteReader {  // read up to n decoded bytes: > 0 bytes, 0 at the end, < 0 on error
    virtual ~ByteReader() {}
    virtual int read(char *dst, unsigned n) = 0;
};

struct GzReader : ByteReader {  // plain or gzip (zlib's transparent gz* reader)
    gzFile f;
    explicit GzReader(gzFile file) : f(file) {}
    ~GzReader() override { gzclose(f); }
    int read(char *dst, unsigned n) override { return gzread(f, dst, n); }
};

// Stream decoders over a FILE*: feed kIn-byte blocks of the compressed file to a decoder
template <class Codec>
struct StreamReader : ByteReader {
    static constexpr size_t kIn = 1u << 20;
    FILE *f;
    Codec codec;
    std::vector<char> in = std::vector<char>(kIn);
    bool ok = false;
    explicit StreamReader(FILE *file) : f(file) { ok = codec.init(); }
    ~StreamReader() override {
        codec.end();
        std::fclose(f);
    }
    bool eof_in = false, ended = false;  // input exhausted; the last decoded stream is complete
    int read(char *dst, unsigned n) override {
        if (!ok) return -1;
        codec.set_out(dst, n);
        while (codec.out_left() > 0) {
            if (codec.in_left() == 0) {
                if (eof_in) break;
                const size_t got = std::fread(in.data(), 1, kIn, f);
                if (got == 0) {
                    if (std::ferror(f)) return -1;
                    eof_in = true;
                }
                codec.set_in(in.data(), got);
                if (got == 0 && ended) break;  // clean end after a complete stream
            }
            const unsigned before = codec.out_left();
            const size_t in_before = codec.in_left();
            const int rc = codec.step(eof_in);
            if (rc < 0) return -1;
            ended = rc == 1 || (ended && codec.out_left() == before && codec.in_left() == in_before);
            if (rc == 0 && codec.out_left() == before && codec.in_left() == in_before && eof_in) {
                if (!ended) return -1;  // truncated input
                break;
            }
        }
        return (int)(n - codec.out_left());
    }
};

// libbz2 (bzlib.h ABI): concatenated streams are decoded one after another
struct BzStream {
    char *next_in;
    unsigned avail_in, total_in_lo32, total_in_hi32;
    char *next_out;
    unsigned avail_out, total_out_lo32, total_out_hi32;
    void *state;
    void *(*bzalloc)(void *, int, int);
    void (*bzfree)(void *, void *);
    void *opaque;
};
struct Bz2Codec {
    int (*init_fn)(BzStream *, int, int) = nullptr;
    int (*dec_fn)(BzStream *) = nullptr;
    int (*end_fn)(BzStream *) = nullptr;
    BzStream z{};
    bool live = false;
    bool init() {
        void *h = dlopen("libbz2.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("libbz2.so.1.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return false;
        init_fn = (int (*)(BzStream *, int, int))dlsym(h, "BZ2_bzDecompressInit");
        dec_fn = (int (*)(BzStream *))dlsym(h, "BZ2_bzDecompress");
        end_fn = (int (*)(BzStream *))dlsym(h, "BZ2_bzDecompressEnd");
        if (!init_fn || !dec_fn || !end_fn) return false;
        std::memset(&z, 0, sizeof(z));
        live = init_fn(&z, 0, 0) == 0;
        return live;
    }
    void end() {
        if (live) end_fn(&z);
        live = false;
    }
    void set_in(char *p, size_t n) { z.next_in = p; z.avail_in = (unsigned)n; }
    void set_out(char *p, unsigned n) { z.next_out = p; z.avail_out = n; }
    size_t in_left() const { return z.avail_in; }
    unsigned out_left() const { return z.avail_out; }
    int step(bool) {  // 0 progress, 1 a stream ended, -1 error
        const int rc = dec_fn(&z);
        if (rc == 4) {  // BZ_STREAM_END: a following stream (pbzip2) starts a new decoder
            char *ni = z.next_in, *no = z.next_out;
            const unsigned ai = z.avail_in, ao = z.avail_out;
            end_fn(&z);
            std::memset(&z, 0, sizeof(z));
            live = init_fn(&z, 0, 0) == 0;
            z.next_in = ni;
            z.avail_in = ai;
            z.next_out = no;
            z.avail_out = ao;
            return live ? 1 : -1;
        }
        return rc == 0 ? 0 : -1;  // BZ_OK
    }
};

// liblzma (lzma/base.h ABI, stable since 5.0): xz with concatenated streams
struct LzmaStream {
    const uint8_t *next_in;
    size_t avail_in;
    uint64_t total_in;
    uint8_t *next_out;
    size_t avail_out;
    uint64_t total_out;
    const void *allocator;
    void *internal;
    void *reserved_ptr1, *reserved_ptr2, *reserved_ptr3, *reserved_ptr4;
    uint64_t reserved_int1, reserved_int2;
    size_t reserved_int3, reserved_int4;
    int reserved_enum1, reserved_enum2;
};
struct XzCodec {
    int (*dec_init)(LzmaStream *, uint64_t, uint32_t) = nullptr;
    int (*code_fn)(LzmaStream *, int) = nullptr;
    void (*end_fn)(LzmaStream *) = nullptr;
    LzmaStream z{};
    bool live = false;
    bool init() {
        void *h = dlopen("liblzma.so.5", RTLD_NOW | RTLD_LOCAL);
        if (!h) return false;
        dec_init = (int (*)(LzmaStream *, uint64_t, uint32_t))dlsym(h, "lzma_stream_decoder");
        code_fn = (int (*)(LzmaStream *, int))dlsym(h, "lzma_code");
        end_fn = (void (*)(LzmaStream *))dlsym(h, "lzma_end");
        if (!dec_init || !code_fn || !end_fn) return false;
        std::memset(&z, 0, sizeof(z));                       // LZMA_STREAM_INIT
        live = dec_init(&z, ~0ULL, 0x08u /* LZMA_CONCATENATED */) == 0;
        return live;
    }
    void end() {
        if (live) end_fn(&z);
        live = false;
    }
    void set_in(char *p, size_t n) { z.next_in = (const uint8_t *)p; z.avail_in = n; }
    void set_out(char *p, unsigned n) { z.next_out = (uint8_t *)p; z.avail_out = n; }
    size_t in_left() const { return z.avail_in; }
    unsigned out_left() const { return (unsigned)z.avail_out; }
    int step(bool finished) {
        const int rc = code_fn(&z, finished ? 3 /* LZMA_FINISH */ : 0 /* LZMA_RUN */);
        if (rc == 1) return 1;  // LZMA_STREAM_END
        return rc == 0 ? 0 : -1;
    }
};

// libzstd (zstd.h streaming ABI, stable since 1.0): concatenated frames decode one after
// another through the same stream
struct ZstdIn {
    const void *src;
    size_t size, pos;
};
struct ZstdOut {
    void *dst;
    size_t size, pos;
};
struct ZstdCodec {
    void *(*create_fn)() = nullptr;
    size_t (*free_fn)(void *) = nullptr;
    size_t (*dec_fn)(void *, ZstdOut *, ZstdIn *) = nullptr;
    unsigned (*is_error)(size_t) = nullptr;
    void *ds = nullptr;
    ZstdIn zi{nullptr, 0, 0};
    ZstdOut zo{nullptr, 0, 0};
    bool init() {
        void *h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return false;
        create_fn = (void *(*)())dlsym(h, "ZSTD_createDStream");
        free_fn = (size_t(*)(void *))dlsym(h, "ZSTD_freeDStream");
        dec_fn = (size_t(*)(void *, ZstdOut *, ZstdIn *))dlsym(h, "ZSTD_decompressStream");
        is_error = (unsigned (*)(size_t))dlsym(h, "ZSTD_isError");
        if (!create_fn || !free_fn || !dec_fn || !is_error) return false;
        ds = create_fn();  // a new DStream starts a frame without ZSTD_initDStream
        return ds != nullptr;
    }
    void end() {
        if (ds) free_fn(ds);
        ds = nullptr;
    }
    void set_in(char *p, size_t n) { zi = ZstdIn{p, n, 0}; }
    void set_out(char *p, unsigned n) { zo = ZstdOut{p, n, 0}; }
    size_t in_left() const { return zi.size - zi.pos; }
    unsigned out_left() const { return (unsigned)(zo.size - zo.pos); }
    int step(bool) {  // 0 progress, 1 a frame ended, -1 error
        const size_t rc = dec_fn(ds, &zo, &zi);
        if (is_error(rc)) return -1;
        return rc == 0 ? 1 : 0;
    }
};

// gzip through libdeflate (libdeflate.so.0, ~4x zlib's inflate rate on this image): whole
// members at once, so the compressed file is read into memory and each member inflates into
// one buffer (a BGZF member's size is in its header; otherwise the output size is guessed
// from the last ISIZE, mod 2^32, and grown on LIBDEFLATE_INSUFFICIENT_SPACE).  Used for
// files up to kDeflateMaxFile compressed bytes; larger ones stream through zlib.
constexpr uint64_t kDeflateMaxFile = 2ull << 30;
struct DeflateReader : ByteReader {
    void *(*alloc_fn)() = nullptr;
    void (*free_fn)(void *) = nullptr;
    int (*gz_fn)(void *, const void *, size_t, void *, size_t, size_t *, size_t *) = nullptr;
    void *dec = nullptr;
    std::vector<unsigned char> comp;
    size_t ci = 0;  // next member
    char *out = nullptr;
    size_t out_n = 0, out_pos = 0, cap = 0;
    bool ok = false;
    DeflateReader(FILE *f, uint64_t size) {
        void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (h) {
            alloc_fn = (void *(*)())dlsym(h, "libdeflate_alloc_decompressor");
            free_fn = (void (*)(void *))dlsym(h, "libdeflate_free_decompressor");
            gz_fn = (int (*)(void *, const void *, size_t, void *, size_t, size_t *, size_t *))dlsym(
                h, "libdeflate_gzip_decompress_ex");
        }
        if (alloc_fn && free_fn && gz_fn && (dec = alloc_fn())) {
            comp.resize(size);
            ok = std::fread(comp.data(), 1, size, f) == size;
        }
        std::fclose(f);
    }
    ~DeflateReader() override {
        if (dec) free_fn(dec);
        for (void *d : pool) free_fn(d);
        std::free(out);
    }
    static uint32_t le32(const unsigned char *p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }
    // BGZF member at m (left bytes on): its size, or 0 when it is not one
    static size_t bgzf_size(const unsigned char *m, size_t left) {
        if (left < 26 || m[0] != 0x1F || m[1] != 0x8B || !(m[3] & 4) || (m[10] | m[11] << 8) < 6 || m[12] != 'B' ||
            m[13] != 'C')
            return 0;
        const size_t bsize = (size_t)(m[16] | m[17] << 8) + 1;
        return bsize >= 26 && bsize <= left ? bsize : 0;
    }
    // BGZF: the next run of up to kBatch members, inflated in parallel into out at the offsets
    // their ISIZE trailers give (bgzip's 64 KB members are independent).  1 done, 0 not BGZF here
    // (or a single member), -1 error
    static constexpr size_t kBatch = 256;
    std::vector<void *> pool;
    int next_bgzf_batch() {
        std::vector<size_t> at, sz, off(1, 0);
        size_t c = ci;
        while (at.size() < kBatch && c < comp.size()) {
            const size_t b = bgzf_size(comp.data() + c, comp.size() - c);
            if (!b) break;
            at.push_back(c);
            sz.push_back(b);
            off.push_back(off.back() + le32(comp.data() + c + b - 4));
            c += b;
        }
        if (at.size() < 2) return 0;
        if (off.back() + 1 > cap) {
            std::free(out);
            cap = std::max<size_t>(off.back() + 1, kBatch << 16);
            out = (char *)std::malloc(cap);
            if (!out) return -1;
        }
        const unsigned T = std::max(1u, std::min<unsigned>(8, std::thread::hardware_concurrency()));
        while (pool.size() < T) {
            void *d = alloc_fn();
            if (!d) return -1;
            pool.push_back(d);
        }
        bool bad = false;
        std::mutex mu;
        auto work = [&](unsigned t) {
            for (size_t i = t; i < at.size(); i += T) {
                size_t used = 0, got = 0;
                const int rc = gz_fn(pool[t], comp.data() + at[i], sz[i], out + off[i], off[i + 1] - off[i], &used, &got);
                if (rc != 0 || used != sz[i] || got != off[i + 1] - off[i]) {
                    std::lock_guard<std::mutex> g(mu);
                    bad = true;
                }
            }
        };
        std::vector<std::thread> th;
        for (unsigned t = 1; t < T; t++) th.emplace_back(work, t);
        work(0);
        for (auto &x : th) x.join();
        if (bad) return -1;
        ci = c;
        out_n = off.back();
        out_pos = 0;
        return 1;
    }
    // the member at ci into out: 1 done, 0 no member left, -1 error
    int next_member() {
        const size_t left = comp.size() - ci;
        if (left == 0) return 0;
        const int rb = next_bgzf_batch();
        if (rb != 0) return rb;
        const unsigned char *m = comp.data() + ci;
        if (left < 18 || m[0] != 0x1F || m[1] != 0x8B) return -1;
        uint64_t want;
        if (const size_t bsize = bgzf_size(m, left)) {  // BGZF: the member's size, its ISIZE exact
            want = le32(m + bsize - 4);
        } else {
            // the last member's ISIZE + j 2^32 >= what is left (inflated >= its input - headers)
            want = le32(comp.data() + comp.size() - 4);
            while (want + 64 < left) want += 1ull << 32;
        }
        for (;;) {
            if (want + 1 > cap) {
                std::free(out);
                cap = want + 1;
                out = (char *)std::malloc(cap);
                if (!out) return -1;
            }
            size_t in_used = 0, got = 0;
            const int rc = gz_fn(dec, m, left, out, cap, &in_used, &got);
            if (rc == 0) {
                ci += in_used;
                out_n = got;
                out_pos = 0;
                return 1;
            }
            // 3 = INSUFFICIENT_SPACE (a multi-member file's earlier, larger member): grow
            if (rc != 3 || want > (uint64_t)left * 1100 + (1u << 20)) return -1;
            want = want * 2 + (1u << 20);
        }
    }
    int read(char *dst, unsigned n) override {  // fills dst across (BGZF's 64 KB) members
        unsigned done = 0;
        while (done < n) {
            if (out_pos == out_n) {
                const int rc = next_member();
                if (rc < 0) return -1;
                if (rc == 0) break;
                continue;
            }
            const size_t t = std::min<size_t>(n - done, out_n - out_pos);
            std::memcpy(dst + done, out + out_pos, t);
            out_pos += t;
            done += (unsigned)t;
        }
        return (int)done;
    }
};

// the reader for a path, by its first bytes; *rc = NTC_ERR_IO / NTC_ERR_UNSUPPORTED on failure
ByteReader *open_reader(const char *path, int *rc) {
    unsigned char m[6] = {0};
    FILE *f = std::fopen(path, "rb");
    if (!f) {
        *rc = NTC_ERR_IO;
        return nullptr;
    }
    const size_t got = std::fread(m, 1, 6, f);
    std::rewind(f);
    ByteReader *r = nullptr;
    if (got >= 3 && m[0] == 'B' && m[1] == 'Z' && m[2] == 'h') {
        auto *b = new StreamReader<Bz2Codec>(f);
        if (!b->ok) { delete b; *rc = NTC_ERR_UNSUPPORTED; return nullptr; }
        r = b;
    } else if (got >= 6 && std::memcmp(m, "\xFD" "7zXZ\0", 6) == 0) {
        auto *x = new StreamReader<XzCodec>(f);
        if (!x->ok) { delete x; *rc = NTC_ERR_UNSUPPORTED; return nullptr; }
        r = x;
    } else if (got >= 4 && m[0] == 0x28 && m[1] == 0xB5 && m[2] == 0x2F && m[3] == 0xFD) {
        auto *z = new StreamReader<ZstdCodec>(f);
        if (!z->ok) { delete z; *rc = NTC_ERR_UNSUPPORTED; return nullptr; }
        r = z;
    } else {
        if (got >= 3 && m[0] == 0x1F && m[1] == 0x8B && m[2] == 8) {
            std::fseek(f, 0, SEEK_END);
            const long size = std::ftell(f);
            std::rewind(f);
            if (size > 0 && (uint64_t)size <= kDeflateMaxFile && !std::getenv("NTC_FASTX_ZLIB")) {
                auto *d = new DeflateReader(f, (uint64_t)size);  // closes f
                if (d->ok) return d;
                delete d;
                f = nullptr;
            }
        }
        if (f) std::fclose(f);
        gzFile g = gzopen(path, "rb");
        if (!g) {
            *rc = NTC_ERR_IO;
            return nullptr;
        }
        gzbuffer(g, 1u << 20);
        r = new GzReader(g);
    }
    return r;
}

// Producer: decoded chunks from a ByteReader, bounded queue of kRing chunks.
struct ChunkSource {
    ByteReader *f;
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::vector<char>> full;
    std::vector<std::vector<char>> spare;
    bool done = false, stop = false, error = false;

    explicit ChunkSource(ByteReader *reader) : f(reader) { th = std::thread([this] { run(); }); }
    ~ChunkSource() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv.notify_all();
        th.join();
    }
    void run() {
        for (;;) {
            std::vector<char> c;
            {
                std::unique_lock<std::mutex> g(mu);
                cv.wait(g, [&] { return stop || full.size() < kRing; });
                if (stop) return;
                if (!spare.empty()) {
                    c.swap(spare.back());
                    spare.pop_back();
                }
            }
            c.resize(kChunk);
            const int got = f->read(c.data(), (unsigned)kChunk);
            std::lock_guard<std::mutex> g(mu);
            if (got < 0) error = true;
            if (got <= 0) {
                done = true;
                cv.notify_all();
                return;
            }
            c.resize((size_t)got);
            full.push_back(std::move(c));
            cv.notify_all();
        }
    }
    // next chunk into `out` (swapped); false at end of input
    bool take(std::vector<char> &out, bool &err) {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return !full.empty() || done; });
        err = error;
        if (full.empty()) return false;
        out.swap(full.front());
        full.pop_front();
        cv.notify_all();
        return true;
    }
    void give_back(std::vector<char> &c) {
        std::lock_guard<std::mutex> g(mu);
        if (spare.size() < kRing) spare.push_back(std::move(c));
    }
};

}  // namespace

struct ntc_fastx {
    ByteReader *f = nullptr;
    ChunkSource *src = nullptr;
    std::vector<char> buf;  // unparsed bytes live in [pos, end)
    std::vector<char> chunk;
    size_t pos = 0, end = 0;
    bool eof = false, io_error = false;
    int format = 0;  // '>' FASTA, '@' FASTQ
    bool have_pending = false;  // FASTA: the next record's '>' line was already consumed
    // current batch
    std::vector<uint8_t> bases;
    size_t nb = 0;
    std::vector<uint64_t> offsets;

    // append the next chunk behind the unparsed tail; false at end of input (a missing
    // final newline is supplied once so the last line always ends in '\n')
    bool fill() {
        if (eof) return false;
        const size_t tail = end - pos;
        if (!src->take(chunk, io_error)) {
            eof = true;
            if (tail && buf[end - 1] != '\n') {
                if (end == buf.size()) buf.resize(buf.size() + 1);
                buf[end++] = '\n';
                return true;
            }
            return false;
        }
        if (pos) std::memmove(buf.data(), buf.data() + pos, tail);
        pos = 0;
        end = tail;
        if (buf.size() < end + chunk.size()) buf.resize(end + chunk.size() + (1u << 16));
        std::memcpy(buf.data() + end, chunk.data(), chunk.size());
        end += chunk.size();
        src->give_back(chunk);
        return true;
    }
    const char *find_nl(size_t from) const {
        return (const char *)std::memchr(buf.data() + from, '\n', end - from);
    }
    void append_seq(const char *s, size_t n) {
        if (nb + n > bases.size()) bases.resize(std::max(bases.size() * 2, nb + n + (1u << 20)));
        uint8_t *d = bases.data() + nb;
        size_t i = 0, j = 0;
        // fast path: 16 bytes at a time while every byte is already one of A C G T
        const __m128i cA = _mm_set1_epi8('A'), cC = _mm_set1_epi8('C'), cG = _mm_set1_epi8('G'),
                      cT = _mm_set1_epi8('T');
        for (; i + 16 <= n; i += 16) {
            const __m128i x = _mm_loadu_si128((const __m128i *)(s + i));
            const __m128i ok = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(x, cA), _mm_cmpeq_epi8(x, cC)),
                                            _mm_or_si128(_mm_cmpeq_epi8(x, cG), _mm_cmpeq_epi8(x, cT)));
            if (_mm_movemask_epi8(ok) == 0xFFFF) {
                _mm_storeu_si128((__m128i *)(d + j), x);
                j += 16;
                continue;
            }
            for (size_t t = i; t < i + 16; t++) {  // this block holds something else
                const uint8_t v = norm_table[(uint8_t)s[t]];
                d[j] = v;
                j += v != 0;
            }
        }
        for (; i < n; i++) {
            const uint8_t v = norm_table[(uint8_t)s[i]];
            d[j] = v;
            j += v != 0;
        }
        nb += j;
    }
    // next FASTQ record's sequence appended; 0 ok, 1 end of input, <0 format error
    int next_fastq() {
        for (;;) {
            while (pos < end && (buf[pos] == '\n' || buf[pos] == '\r')) pos++;
            if (pos == end) {
                if (!fill()) return 1;
                continue;
            }
            if (buf[pos] != '@') return -1;
            const char *h = find_nl(pos);
            const char *se = h ? find_nl((size_t)(h - buf.data()) + 1) : nullptr;
            const char *pe = se ? find_nl((size_t)(se - buf.data()) + 1) : nullptr;
            const char *qe = pe ? find_nl((size_t)(pe - buf.data()) + 1) : nullptr;
            if (!qe) {
                if (!fill()) return -1;  // truncated record
                continue;
            }
            if (se[1] != '+') return -1;
            append_seq(h + 1, (size_t)(se - h - 1));
            pos = (size_t)(qe - buf.data()) + 1;
            return 0;
        }
    }
    // next FASTA record's sequence (any number of lines) appended
    int next_fasta() {
        if (!have_pending) {
            for (;;) {  // skip blank lines, then expect a header
                while (pos < end && (buf[pos] == '\n' || buf[pos] == '\r')) pos++;
                if (pos < end) break;
                if (!fill()) return 1;
            }
            if (buf[pos] != '>') return -1;
            for (;;) {
                const char *h = find_nl(pos);
                if (h) {
                    pos = (size_t)(h - buf.data()) + 1;
                    break;
                }
                pos = end;  // a header longer than the buffer: drop what we have
                if (!fill()) return 0;
            }
        }
        have_pending = false;
        bool mid_line = false;  // a sequence line continues across a refill
        for (;;) {
            if (pos == end && !fill()) return 0;
            if (!mid_line && buf[pos] == '>') {
                // the next record's header: consume it now
                for (;;) {
                    const char *h = find_nl(pos);
                    if (h) {
                        pos = (size_t)(h - buf.data()) + 1;
                        break;
                    }
                    pos = end;
                    if (!fill()) break;
                }
                have_pending = true;
                return 0;
            }
            const char *nl = find_nl(pos);
            const size_t stop = nl ? (size_t)(nl - buf.data()) : end;
            append_seq(buf.data() + pos, stop - pos);
            pos = nl ? stop + 1 : end;
            mid_line = !nl;
        }
    }
};

extern "C" {

int ntc_fastx_open(const char *path, ntc_fastx **out) {
    if (!path || !out) return NTC_ERR_INVALID_ARG;
    *out = nullptr;
    init_norm();
    int orc = NTC_OK;
    ByteReader *f = open_reader(path, &orc);
    if (!f) return orc;
    auto *fx = new ntc_fastx();
    fx->f = f;
    fx->src = new ChunkSource(f);
    // detect the format from the first non-whitespace character
    for (;;) {
        if (fx->pos == fx->end && !fx->fill()) break;
        const char c = fx->buf[fx->pos];
        if (c == '\n' || c == '\r' || c == ' ') {
            fx->pos++;
            continue;
        }
        fx->format = c;
        break;
    }
    if (fx->io_error || (fx->format != '>' && fx->format != '@' && fx->format != 0)) {
        const int rc = fx->io_error ? NTC_ERR_IO : NTC_ERR_FORMAT;
        ntc_fastx_close(fx);
        return rc;
    }
    if (fx->format == 0) fx->format = '>';  // empty input
    *out = fx;
    return NTC_OK;
}

int ntc_fastx_next_batch(ntc_fastx *fx, uint64_t max_reads, uint64_t max_bases, const uint8_t **bases,
                         const uint64_t **offsets, uint64_t *n_reads) {
    if (!fx || !bases || !offsets || !n_reads || max_reads == 0) return NTC_ERR_INVALID_ARG;
    fx->nb = 0;
    fx->offsets.assign(1, 0);
    fx->offsets.reserve(max_reads + 1);
    while (fx->offsets.size() - 1 < max_reads && fx->nb < max_bases) {
        const int rc = fx->format == '@' ? fx->next_fastq() : fx->next_fasta();
        if (rc == 1) break;
        if (rc < 0) return fx->io_error ? NTC_ERR_IO : NTC_ERR_FORMAT;  // a truncated stream is an I/O error
        fx->offsets.push_back(fx->nb);
    }
    if (fx->io_error) return NTC_ERR_IO;
    *bases = fx->bases.data();
    *offsets = fx->offsets.data();
    *n_reads = fx->offsets.size() - 1;
    return NTC_OK;
}

int ntc_fasta_format(const uint8_t *bases, const uint64_t *offsets, uint64_t n_reads, uint64_t first_id,
                     uint8_t **out, uint64_t *out_len) {
    if (!out || !out_len || (n_reads && (!offsets || !bases))) return NTC_ERR_INVALID_ARG;
    const uint64_t total = n_reads ? offsets[n_reads] - offsets[0] : 0;
    uint8_t *buf = (uint8_t *)std::malloc(total + n_reads * 28 + 1);
    if (!buf) return NTC_ERR_CAPACITY;
    uint8_t *w = buf;
    char num[24];
    for (uint64_t r = 0; r < n_reads; r++) {
        const int nl = std::snprintf(num, sizeof(num), "%llu", (unsigned long long)(first_id + r));
        std::memcpy(w, ">seq.", 5);
        std::memcpy(w + 5, num, (size_t)nl);
        w += 5 + nl;
        *w++ = '\n';
        const uint64_t len = offsets[r + 1] - offsets[r];
        std::memcpy(w, bases + (offsets[r] - offsets[0]), len);
        w += len;
        *w++ = '\n';
    }
    *out = buf;
    *out_len = (uint64_t)(w - buf);
    return NTC_OK;
}

void ntc_fastx_close(ntc_fastx *fx) {
    if (!fx) return;
    delete fx->src;  // joins the producer before the file goes away
    delete fx->f;
    delete fx;
}

}  // extern "C"
