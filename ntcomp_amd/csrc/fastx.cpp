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
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ntcomp_host.h"
#include "ntc_internal.h"

namespace {

uint8_t norm_table[256];

void fill_norm();
// once per process, thread-safe: ntc_fastx_open may run on several threads at once
void init_norm() {
    static std::once_flag once;
    std::call_once(once, fill_norm);
}
void fill_norm() {
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
}

// growable byte buffer without zero-fill (std::vector::resize would touch every new byte)
struct RawBuf {
    uint8_t *p = nullptr;
    size_t cap = 0;
    RawBuf() = default;
    RawBuf(const RawBuf &) = delete;
    RawBuf &operator=(const RawBuf &) = delete;
    RawBuf(RawBuf &&o) noexcept : p(o.p), cap(o.cap) { o.p = nullptr, o.cap = 0; }
    ~RawBuf() { std::free(p); }
    uint8_t *data() { return p; }
    size_t size() const { return cap; }
    // room for n bytes, keeping the first keep
    void reserve_keep(size_t n, size_t keep) {
        if (n <= cap) return;
        size_t want = std::max(n, cap + cap / 2);
        uint8_t *q;
        if (want >= (8u << 20)) {  // large: 2 MB aligned, transparent huge pages (512x fewer faults)
            want = (want + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
            q = (uint8_t *)std::aligned_alloc(2u << 20, want);
            if (q) madvise(q, want, MADV_HUGEPAGE);
        } else {
            q = (uint8_t *)std::malloc(want);
        }
        if (!q) throw std::bad_alloc();
        if (keep) std::memcpy(q, p, keep);
        std::free(p);
        p = q;
        cap = want;
    }
};

// normalize(true) of n bytes into d (d has room for n); returns the bytes kept
size_t norm_copy(const char *s, size_t n, uint8_t *d) {
    size_t i = 0, j = 0;
    // fast path: 16 bytes at a time while every byte is already one of A C G T
    const __m128i cA = _mm_set1_epi8('A'), cC = _mm_set1_epi8('C'), cG = _mm_set1_epi8('G'), cT = _mm_set1_epi8('T');
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
    return j;
}

// line length without a trailing '\r' (needletail strips CRLF endings)
inline size_t line_len(const char *b, const char *e) { return (size_t)(e - b) - (e > b && e[-1] == '\r'); }

// ---- plain FASTQ through mmap, parsed in parallel -------------------------------------
// A batch's byte range is cut into T pieces at record starts (a line beginning with '@'
// whose next-but-one line begins with '+': a quality line that begins with '@' is followed
// by a header and a sequence line, so it never qualifies); each piece is parsed by its own
// thread, and every piece must end exactly where the next begins, else the range is parsed
// again by one thread.  Same records, same errors as the streaming parser.
struct FqPiece {
    RawBuf bases;
    std::vector<uint64_t> ends;    // per record: bases up to and including it
    std::vector<uint64_t> starts;  // per record: byte position of its '@'
    size_t stop = 0;               // byte position after the last record parsed (blank lines skipped)
    int err = 0;                   // 0 ok, NTC_ERR_FORMAT
};

// records starting in [from, limit) of p[0..n); a record may run past limit
void parse_fq_range(const char *p, size_t n, size_t from, size_t limit, FqPiece &o) {
    size_t pos = from;
    o.ends.clear();
    o.starts.clear();
    o.err = 0;
    uint64_t nb = 0;
    for (;;) {
        while (pos < n && (p[pos] == '\n' || p[pos] == '\r')) pos++;
        if (pos >= limit || pos >= n) break;
        if (p[pos] != '@') {
            o.err = NTC_ERR_FORMAT;
            break;
        }
        const char *e = p + n;
        const char *h = (const char *)std::memchr(p + pos, '\n', n - pos);
        const char *se = h ? (const char *)std::memchr(h + 1, '\n', (size_t)(e - h - 1)) : nullptr;
        const char *pe = se ? (const char *)std::memchr(se + 1, '\n', (size_t)(e - se - 1)) : nullptr;
        if (!pe) {  // truncated record
            o.err = NTC_ERR_FORMAT;
            break;
        }
        const char *qe = (const char *)std::memchr(pe + 1, '\n', (size_t)(e - pe - 1));
        if (!qe) qe = e;  // the last line may lack its newline
        if (se[1] != '+' || line_len(h + 1, se) != line_len(pe + 1, qe)) {
            o.err = NTC_ERR_FORMAT;
            break;
        }
        const size_t L = (size_t)(se - h - 1);
        o.bases.reserve_keep(nb + L + (1u << 16), nb);
        nb += norm_copy(h + 1, L, o.bases.data() + nb);
        o.starts.push_back(pos);
        o.ends.push_back(nb);
        pos = (size_t)(qe - p) + (qe < e);
    }
    while (pos < n && (p[pos] == '\n' || p[pos] == '\r')) pos++;
    o.stop = pos;
}

// first record start at or after c and before limit (limit if none)
size_t fq_record_start(const char *p, size_t n, size_t c, size_t limit) {
    if (c > 0 && p[c - 1] != '\n') {
        const char *nl = (const char *)std::memchr(p + c, '\n', n - c);
        if (!nl) return limit;
        c = (size_t)(nl - p) + 1;
    }
    while (c < limit) {
        if (p[c] == '@') {
            const char *l1 = (const char *)std::memchr(p + c, '\n', n - c);
            const char *l2 = l1 ? (const char *)std::memchr(l1 + 1, '\n', n - (size_t)(l1 + 1 - p)) : nullptr;
            if (l2 && l2 + 1 < p + n && l2[1] == '+') return c;
        }
        const char *nl = (const char *)std::memchr(p + c, '\n', n - c);
        if (!nl) return limit;
        c = (size_t)(nl - p) + 1;
    }
    return limit;
}

constexpr size_t kChunk = 8u << 20;
constexpr size_t kRing = 4;

// ---- byte sources ---------------------------------------------------------------------
struct ByteReader {  // read up to n decoded bytes: > 0 bytes, 0 at the end, < 0 on error
    virtual ~ByteReader() {}
    virtual int read(char *dst, unsigned n) = 0;
    // cap bytes into dst (fewer only at the end): 1 filled, 0 the end was met, -1 error
    virtual int read_into(char *dst, size_t cap, size_t *got) {
        *got = 0;
        while (*got < cap) {
            const int r = read(dst + *got, (unsigned)std::min<size_t>(cap - *got, 1u << 30));
            if (r < 0) return -1;
            if (r == 0) return 0;
            *got += (size_t)r;
        }
        return 1;
    }
};

struct GzReader : ByteReader {  // plain or gzip (zlib's transparent gz* reader)
    gzFile f;
    explicit GzReader(gzFile file) : f(file) {}
    ~GzReader() override { gzclose(f); }
    int read(char *dst, unsigned n) override {
        const int got = gzread(f, dst, n);
        if (got <= 0) {  // gzread reports a truncated member as a clean end: ask gzerror
            int err = Z_OK;
            gzerror(f, &err);
            if (err != Z_OK) return -1;
        }
        return got;
    }
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

// gzip through libdeflate (libdeflate.so.0, ~4x zlib's inflate rate on this image).
//  * BGZF (bgzip: members of <= 64 KB carrying their size): the compressed file streams
//    through a bounded window (kWindow) and runs of up to kBatch members inflate in
//    parallel into one buffer at the offsets their ISIZE trailers give.
//  * Other gzip files up to kWholeMax compressed bytes: read whole, each member inflated
//    into one buffer sized from its ISIZE guess (the last member's ISIZE, mod 2^32), capped
//    at kOutCap; a member that does not fit, or any libdeflate failure, hands the stream
//    to zlib's gzread from the same point (the bytes already delivered are skipped), so a
//    valid file never fails here.  Larger gzip files stream through zlib directly.
//  * Bytes after the last member that are not a gzip member end the input, as gzread does.
constexpr uint64_t kWholeMax = 256ull << 20;
constexpr uint64_t kOutCap = 2ull << 30;
constexpr size_t kWindow = 32u << 20;
struct DeflateReader : ByteReader {
    void *(*alloc_fn)() = nullptr;
    void (*free_fn)(void *) = nullptr;
    int (*gz_fn)(void *, const void *, size_t, void *, size_t, size_t *, size_t *) = nullptr;
    void *dec = nullptr;
    std::string path;
    FILE *f = nullptr;
    bool bgzf = false, in_eof = false;
    std::vector<unsigned char> comp;  // whole file, or the BGZF window [ci, comp_end)
    size_t ci = 0, comp_end = 0;
    char *out = nullptr;
    size_t out_n = 0, out_pos = 0, cap = 0;
    uint64_t delivered = 0, members = 0;
    GzReader *zfall = nullptr;  // zlib takes over after a libdeflate failure
    bool ok = false;
    DeflateReader(const char *p, FILE *file, uint64_t size, bool is_bgzf) : path(p), f(file), bgzf(is_bgzf) {
        void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (h) {
            alloc_fn = (void *(*)())dlsym(h, "libdeflate_alloc_decompressor");
            free_fn = (void (*)(void *))dlsym(h, "libdeflate_free_decompressor");
            gz_fn = (int (*)(void *, const void *, size_t, void *, size_t, size_t *, size_t *))dlsym(
                h, "libdeflate_gzip_decompress_ex");
        }
        if (!(alloc_fn && free_fn && gz_fn && (dec = alloc_fn()))) return;
        if (bgzf) {
            comp.resize(kWindow);
            ok = true;
        } else {
            comp.resize(size);
            ok = std::fread(comp.data(), 1, size, f) == size;
            comp_end = size;
            in_eof = true;
        }
    }
    ~DeflateReader() override {
        if (dec) free_fn(dec);
        for (void *d : pool) free_fn(d);
        std::free(out);
        delete zfall;
        if (f) std::fclose(f);
    }
    static uint32_t le32(const unsigned char *p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }
    // BGZF member at m (left bytes on): its size, or 0 when it is not one
    static size_t bgzf_size(const unsigned char *m, size_t left) {
        if (left < 18 || m[0] != 0x1F || m[1] != 0x8B || !(m[3] & 4) || (m[10] | m[11] << 8) < 6 || m[12] != 'B' ||
            m[13] != 'C')
            return 0;
        const size_t bsize = (size_t)(m[16] | m[17] << 8) + 1;
        return bsize >= 26 ? bsize : 0;
    }
    // BGZF window: keep [ci, comp_end) and top it up from the file
    bool refill() {
        if (in_eof) return true;
        if (ci) {
            std::memmove(comp.data(), comp.data() + ci, comp_end - ci);
            comp_end -= ci;
            ci = 0;
        }
        while (comp_end < comp.size()) {
            const size_t got = std::fread(comp.data() + comp_end, 1, comp.size() - comp_end, f);
            if (got == 0) {
                if (std::ferror(f)) return false;
                in_eof = true;
                break;
            }
            comp_end += got;
        }
        return true;
    }
    // The next run of up to kBatch BGZF members, inflated in parallel (bgzip's members are
    // independent).  1 done, 0 no member here, -1 error
    static constexpr size_t kBatch = 256;
    std::vector<void *> pool;
    int next_bgzf_batch() {
        std::vector<size_t> at, sz, off(1, 0);
        for (int pass = 0; pass < 2; pass++) {
            at.clear();
            sz.clear();
            off.assign(1, 0);
            size_t c = ci;
            bool short_window = false;
            while (at.size() < kBatch && c < comp_end) {
                const size_t b = bgzf_size(comp.data() + c, comp_end - c);
                if (!b) break;
                if (b > comp_end - c) {  // the member runs past the window
                    short_window = true;
                    break;
                }
                at.push_back(c);
                sz.push_back(b);
                off.push_back(off.back() + le32(comp.data() + c + b - 4));
                c += b;
            }
            if (pass == 0 && (at.size() < kBatch && (short_window || c == comp_end)) && !in_eof) {
                if (!refill()) return -1;
                continue;
            }
            break;
        }
        if (at.empty()) return 0;
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
        for (unsigned t = 1; t < T && t < at.size(); t++) th.emplace_back(work, t);
        work(0);
        for (auto &x : th) x.join();
        if (bad) return -1;
        ci = at.back() + sz.back();
        members += at.size();
        out_n = off.back();
        out_pos = 0;
        return 1;
    }
    // the member at ci into out: 1 done, 0 end of input, -1 error (zlib takes over)
    int next_member() {
        if (bgzf) {
            if (comp_end - ci < 26 && !in_eof && !refill()) return -1;
            if (ci == comp_end) return 0;
            const int rb = next_bgzf_batch();
            if (rb != 0) return rb;
            // not a BGZF member here: the rest goes through zlib
            return -1;
        }
        const size_t left = comp_end - ci;
        if (left == 0) return 0;
        const unsigned char *m = comp.data() + ci;
        if (left < 18 || m[0] != 0x1F || m[1] != 0x8B) return members ? 0 : -1;  // trailing bytes end it
        // the last member's ISIZE + j 2^32 >= what is left (inflated >= its input - headers)
        uint64_t want = le32(comp.data() + comp_end - 4);
        while (want + 64 < left) want += 1ull << 32;
        for (;;) {
            if (want > kOutCap) return -1;
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
                members++;
                out_n = got;
                out_pos = 0;
                return 1;
            }
            if (rc != 3) return -1;  // 3 = INSUFFICIENT_SPACE: an earlier, larger member
            want = want * 2 + (1u << 20);
        }
    }
    // BGZF straight into the caller's buffer: the whole members from ci whose inflated sizes
    // (ISIZE) fit in room, inflated in parallel at their offsets (one pass over up to ~one
    // window); bytes written, 0 when the next member does not fit or is not BGZF, -1 on error
    int64_t inflate_members_into(char *dst, size_t room) {
        if (comp_end - ci < kWindow / 2 && !in_eof && !refill()) return -1;
        std::vector<size_t> at, sz, off(1, 0);
        for (size_t c = ci; c < comp_end;) {
            const size_t b = bgzf_size(comp.data() + c, comp_end - c);
            if (!b || b > comp_end - c) break;  // not BGZF here, or past the window
            const uint32_t isz = le32(comp.data() + c + b - 4);
            if (off.back() + isz > room) break;
            at.push_back(c);
            sz.push_back(b);
            off.push_back(off.back() + isz);
            c += b;
        }
        if (at.empty()) return 0;
        const unsigned T = (unsigned)std::max(1, std::min(16, ntc_host_threads()));
        while (pool.size() < T) {
            void *d = alloc_fn();
            if (!d) return -1;
            pool.push_back(d);
        }
        std::atomic<bool> bad{false};
        std::atomic<size_t> next{0};
        auto work = [&](unsigned t) {
            for (size_t i; (i = next.fetch_add(8)) < at.size();)  // 8 members (~0.5 MB) a grab
                for (size_t j = i; j < std::min(at.size(), i + 8); j++) {
                    size_t used = 0, got = 0;
                    const int rc = gz_fn(pool[t], comp.data() + at[j], sz[j], dst + off[j], off[j + 1] - off[j], &used,
                                         &got);
                    if (rc != 0 || used != sz[j] || got != off[j + 1] - off[j]) bad = true;
                }
        };
        std::vector<std::thread> th;
        for (unsigned t = 1; t < T && t * 8 < at.size(); t++) th.emplace_back(work, t);
        work(0);
        for (auto &x : th) x.join();
        // libdeflate rejected a member (or its sizes disagree): nothing is delivered, and the
        // buffered path takes the same members, falling back to zlib as read() does
        if (bad) return 0;
        ci = at.back() + sz.back();
        members += at.size();
        delivered += off.back();
        return (int64_t)off.back();
    }
    int read_into(char *dst, size_t cap, size_t *got) override {
        *got = 0;
        while (*got < cap) {
            if (out_pos < out_n) {  // the rest of a batch the buffered path inflated
                const size_t t = std::min(cap - *got, out_n - out_pos);
                std::memcpy(dst + *got, out + out_pos, t);
                out_pos += t;
                *got += t;
                delivered += t;
                continue;
            }
            if (bgzf && !zfall) {
                const int64_t w = inflate_members_into(dst + *got, cap - *got);
                if (w < 0) return -1;
                if (w > 0) {
                    *got += (size_t)w;
                    continue;
                }
            }
            // the buffered path: a member larger than the room, a non-BGZF tail, the end
            const int r = read(dst + *got, (unsigned)std::min<size_t>(cap - *got, 1u << 30));
            if (r < 0) return -1;
            if (r == 0) return 0;
            *got += (size_t)r;
        }
        return 1;
    }
    // hand the rest of the stream to zlib: reopen, skip what was delivered
    bool to_zlib() {
        gzFile g = gzopen(path.c_str(), "rb");
        if (!g) return false;
        gzbuffer(g, 1u << 20);
        zfall = new GzReader(g);
        std::vector<char> skip(1u << 20);
        uint64_t left = delivered;
        while (left) {
            const int got = zfall->read(skip.data(), (unsigned)std::min<uint64_t>(left, skip.size()));
            if (got <= 0) return false;
            left -= (uint64_t)got;
        }
        return true;
    }
    int read(char *dst, unsigned n) override {  // fills dst across members
        if (zfall) return zfall->read(dst, n);
        unsigned done = 0;
        while (done < n) {
            if (out_pos == out_n) {
                const int rc = next_member();
                if (rc < 0) {
                    if (!to_zlib()) return -1;
                    const int more = zfall->read(dst + done, n - done);
                    if (more < 0) return -1;
                    return (int)(done + (unsigned)more);
                }
                if (rc == 0) break;
                continue;
            }
            const size_t t = std::min<size_t>(n - done, out_n - out_pos);
            std::memcpy(dst + done, out + out_pos, t);
            out_pos += t;
            done += (unsigned)t;
            delivered += t;
        }
        return (int)done;
    }
};

// One gzip member (or several concatenated) that is not BGZF, inflated in parallel
// (pgzip.cpp): the reference's own `.fastq.gz` input (README.md:30), which one zlib stream
// inflated at ~0.6 GB/s of text on one thread.
struct ParallelGzReader : ByteReader {
    ntc::PgzReader *r;
    explicit ParallelGzReader(ntc::PgzReader *x) : r(x) {}
    ~ParallelGzReader() override { ntc::pgz_close(r); }
    int read_into(char *dst, size_t cap, size_t *got) override { return ntc::pgz_read(r, dst, cap, got); }
    int read(char *dst, unsigned n) override {
        size_t got = 0;
        const int rc = ntc::pgz_read(r, dst, n, &got);
        return rc < 0 ? -1 : (int)got;
    }
};
// compressed size from which a non-BGZF gzip goes to the parallel inflater (NTC_PGZ_MIN)
uint64_t pgz_min_bytes() {
    const char *e = std::getenv("NTC_PGZ_MIN");
    return e ? (uint64_t)std::atoll(e) : (4ull << 20);
}

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
        if (got >= 3 && m[0] == 0x1F && m[1] == 0x8B && m[2] == 8 && !std::getenv("NTC_FASTX_ZLIB")) {
            unsigned char h[18] = {0};
            const size_t hn = std::fread(h, 1, 18, f);
            std::fseek(f, 0, SEEK_END);
            const long size = std::ftell(f);
            std::rewind(f);
            const bool bgzf = hn == 18 && DeflateReader::bgzf_size(h, 18) != 0;
            if (!bgzf && size > 0 && (uint64_t)size >= pgz_min_bytes()) {
                if (ntc::PgzReader *pr = ntc::pgz_open(path, std::max(1, std::min(16, ntc_host_threads())))) {
                    std::fclose(f);
                    return new ParallelGzReader(pr);
                }
            }
            if (size > 0 && (bgzf || (uint64_t)size <= kWholeMax)) {
                auto *d = new DeflateReader(path, f, (uint64_t)size, bgzf);  // owns f
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

    bool direct = false;    // the producer stopped: the consumer reads f itself (read_direct)
    size_t front_off = 0;   // direct: bytes of full.front() already handed out

    explicit ChunkSource(ByteReader *reader) : f(reader) { th = std::thread([this] { run(); }); }
    ~ChunkSource() {
        if (direct) return;
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv.notify_all();
        th.join();
    }
    // Stop the producer; the chunks it made are handed out first.  Then the consumer's own
    // thread decodes straight into its buffer (the GPU-parse reader: BGZF members inflate in
    // parallel into the pinned batch, no chunk copies).
    void go_direct() {
        if (direct) return;
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv.notify_all();
        th.join();
        direct = true;
    }
    // direct: up to cap bytes into dst (fewer only at the end of input); -1 on error
    int64_t read_direct(char *dst, size_t cap) {
        go_direct();
        size_t got = 0;
        while (got < cap && !full.empty()) {
            std::vector<char> &c = full.front();
            const size_t t = std::min(cap - got, c.size() - front_off);
            std::memcpy(dst + got, c.data() + front_off, t);
            got += t;
            front_off += t;
            if (front_off == c.size()) {
                full.pop_front();
                front_off = 0;
            }
        }
        if (error) return -1;
        if (got < cap && !done) {
            size_t g = 0;
            const int rc = f->read_into(dst + got, cap - got, &g);
            got += g;
            if (rc < 0) {
                error = true;
                return -1;
            }
            if (rc == 0) done = true;
        }
        return (int64_t)got;
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
        if (direct) {  // the producer is gone: hand out what it left, then read here
            err = error;
            if (!full.empty()) {
                if (front_off) full.front().erase(full.front().begin(), full.front().begin() + (long)front_off);
                front_off = 0;
                out.swap(full.front());
                full.pop_front();
                return true;
            }
            if (done || error) return false;
            out.resize(kChunk);
            const int got = f->read(out.data(), (unsigned)kChunk);
            if (got < 0) error = true;
            if (got <= 0) {
                done = true;
                err = error;
                return false;
            }
            out.resize((size_t)got);
            return true;
        }
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
        if (direct) return;
        std::lock_guard<std::mutex> g(mu);
        if (spare.size() < kRing) spare.push_back(std::move(c));
    }
};

}  // namespace

struct ntc_fastx {
    // plain FASTQ: the file mapped, parsed in parallel pieces (parse_fq_range)
    const char *mm = nullptr;
    size_t mm_n = 0, mm_pos = 0;
    double avg_rec = 0;  // bytes per record so far
    int threads = 1;
    std::vector<FqPiece> pieces;
    ByteReader *f = nullptr;
    ChunkSource *src = nullptr;
    std::vector<char> buf;  // unparsed bytes live in [pos, end)
    std::vector<char> chunk;
    size_t pos = 0, end = 0;
    bool eof = false, io_error = false;
    int format = 0;  // '>' FASTA, '@' FASTQ
    bool have_pending = false;  // FASTA: the next record's '>' line was already consumed
    // current batch
    RawBuf bases;
    size_t nb = 0;
    std::vector<uint64_t> offsets;

    // one batch from the mapping: up to max_reads reads / about max_bases bases
    int mm_batch(uint64_t max_reads, uint64_t max_bases, uint8_t *dst, uint64_t dst_cap, uint64_t *dst_offs) {
        uint64_t reads = 0;
        nb = 0;
        while (reads < max_reads && nb < max_bases && mm_pos < mm_n) {
            const uint64_t want = max_reads - reads;
            if (avg_rec <= 0) {  // probe the record size on a few records
                FqPiece probe;
                parse_fq_range(mm, mm_n, mm_pos, std::min(mm_n, mm_pos + (64u << 10)), probe);
                avg_rec = probe.starts.size() > 1 ? (double)(probe.starts.back() - probe.starts[0]) /
                                                        (double)(probe.starts.size() - 1)
                                                  : 512.0;
            }
            const size_t region = (size_t)std::min<double>((double)(mm_n - mm_pos),
                                                           (double)want * avg_rec * 1.02 + (256u << 10));
            const size_t lim = mm_pos + region;
            const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)threads, region >> 20));
            if ((int)pieces.size() < T) pieces.resize((size_t)T);
            std::vector<size_t> cut((size_t)T + 1);
            cut[0] = mm_pos;
            cut[(size_t)T] = lim;
            for (int t = 1; t < T; t++)
                cut[(size_t)t] = std::max(cut[(size_t)t - 1], fq_record_start(mm, mm_n, mm_pos + region * (size_t)t / (size_t)T, lim));
            // size every piece's buffers here: allocating inside the workers serialises them on
            // the address-space lock that their page faults need too
            for (int t = 0; t < T; t++) {
                const size_t bytes = cut[(size_t)t + 1] - cut[(size_t)t];
                const size_t recs = (size_t)((double)bytes / std::max(avg_rec, 16.0) * 1.25) + 1024;
                pieces[(size_t)t].bases.reserve_keep(bytes / 2 + (1u << 20), 0);
                pieces[(size_t)t].ends.reserve(recs);
                pieces[(size_t)t].starts.reserve(recs);
            }
            auto work = [&](int t) { parse_fq_range(mm, mm_n, cut[(size_t)t], cut[(size_t)t + 1], pieces[(size_t)t]); };
            std::vector<std::thread> th;
            for (int t = 1; t < T; t++) th.emplace_back(work, t);
            work(0);
            for (auto &x : th) x.join();
            int np = T;
            for (int t = 0; t + 1 < T; t++)
                if (pieces[(size_t)t].err || pieces[(size_t)t].stop != cut[(size_t)t + 1]) {
                    np = -1;  // a piece did not end where the next begins: parse [mm_pos, lim) in one
                    break;
                }
            if (np < 0) {
                np = 1;
                parse_fq_range(mm, mm_n, mm_pos, lim, pieces[0]);
            }
            // take records in order up to the limits; the first record not taken restarts there
            size_t next_pos = pieces[(size_t)np - 1].stop;
            int err = 0;
            std::vector<uint64_t> take((size_t)np, 0), base0((size_t)np, 0), boff((size_t)np, 0);
            for (int t = 0; t < np; t++) {
                FqPiece &pc = pieces[(size_t)t];
                base0[(size_t)t] = reads;
                boff[(size_t)t] = nb;
                uint64_t k = 0;
                while (k < pc.ends.size() && reads + k < max_reads && nb + (k ? pc.ends[k - 1] : 0) < max_bases) k++;
                take[(size_t)t] = k;
                reads += k;
                nb += k ? pc.ends[k - 1] : 0;
                if (k < pc.ends.size()) {
                    next_pos = pc.starts[k];
                    np = t + 1;
                    break;
                }
                if (pc.err) {
                    err = pc.err;
                    np = t + 1;
                    break;
                }
            }
            // copy out in parallel
            if (!dst) {
                bases.reserve_keep(nb + 64, boff[0]);
                if (offsets.size() < reads + 1) offsets.resize(reads + 1);
            } else if (nb > dst_cap) {
                return NTC_ERR_CAPACITY;
            }
            uint8_t *B = dst ? dst : bases.data();
            uint64_t *O = dst ? dst_offs : offsets.data();
            O[0] = 0;
            auto copy = [&](int t) {
                FqPiece &pc = pieces[(size_t)t];
                const uint64_t k = take[(size_t)t];
                if (!k) return;
                std::memcpy(B + boff[(size_t)t], pc.bases.data(), pc.ends[k - 1]);
                for (uint64_t i = 0; i < k; i++) O[base0[(size_t)t] + i + 1] = boff[(size_t)t] + pc.ends[i];
            };
            th.clear();
            for (int t = 1; t < np; t++) th.emplace_back(copy, t);
            copy(0);
            for (auto &x : th) x.join();

            if (err) return err;
            const size_t used = next_pos - mm_pos;
            mm_pos = next_pos;
            if (reads) avg_rec = 0.5 * avg_rec + 0.5 * (double)used / (double)std::max<uint64_t>(1, reads - base0[0]);
            if (used == 0) break;  // nothing parsed (end of data)
        }
        mm_reads = reads;
        return NTC_OK;
    }
    uint64_t mm_reads = 0;
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
        bases.reserve_keep(nb + n + (1u << 20), nb);
        nb += norm_copy(s, n, bases.data() + nb);
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
            if (se[1] != '+' || line_len(h + 1, se) != line_len(pe + 1, qe)) return -1;  // needletail: equal lengths
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

int ntc_host_threads(void) {
    static const int cached = [] {  // once, thread-safe (inputs may open on several threads at once)
        int n = 0;
        if (const char *v = std::getenv("NTC_THREADS")) n = std::atoi(v);
        if (n <= 0) {
            cpu_set_t set;
            n = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : (int)std::thread::hardware_concurrency();
            if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {  // cgroup v2 CPU quota
                char q[32] = {0};
                unsigned long long period = 0;
                if (std::fscanf(f, "%31s %llu", q, &period) == 2 && std::strcmp(q, "max") != 0 && period) {
                    const unsigned long long quota = std::strtoull(q, nullptr, 10);
                    const int lim = (int)((quota + period - 1) / period);
                    if (lim > 0 && lim < n) n = lim;
                }
                std::fclose(f);
            }
        }
        return std::max(1, n);
    }();
    return cached;
}

int ntc_fastx_set_threads(ntc_fastx *fx, int n_threads) {
    if (!fx) return NTC_ERR_INVALID_ARG;
    fx->threads = n_threads > 0 ? n_threads : ntc_host_threads();
    return NTC_OK;
}

// A plain (uncompressed) FASTQ file is mapped and parsed in parallel; anything else streams.
static ntc_fastx *open_mapped_fastq(const char *path) {
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) return nullptr;
    struct stat st;
    if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode) || st.st_size < 4) {
        ::close(fd);
        return nullptr;
    }
    const size_t n = (size_t)st.st_size;
    const unsigned char *m = (const unsigned char *)mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) return nullptr;
    const bool compressed = (m[0] == 0x1F && m[1] == 0x8B) || (m[0] == 'B' && m[1] == 'Z' && m[2] == 'h') ||
                            (m[0] == 0xFD && m[1] == '7') || (m[0] == 0x28 && m[1] == 0xB5);
    size_t i = 0;
    while (i < n && (m[i] == '\n' || m[i] == '\r' || m[i] == ' ')) i++;
    if (compressed || i == n || m[i] != '@') {
        munmap((void *)m, n);
        return nullptr;
    }
    madvise((void *)m, n, MADV_SEQUENTIAL);
    auto *fx = new ntc_fastx();
    fx->mm = (const char *)m;
    fx->mm_n = n;
    fx->mm_pos = 0;
    fx->format = '@';
    fx->threads = ntc_host_threads();
    return fx;
}

int ntc_fastx_open(const char *path, ntc_fastx **out) {
    if (!path || !out) return NTC_ERR_INVALID_ARG;
    *out = nullptr;
    init_norm();
    if (!std::getenv("NTC_FASTX_STREAM"))
        if (ntc_fastx *fx = open_mapped_fastq(path)) {
            *out = fx;
            return NTC_OK;
        }
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

}  // extern "C"

namespace ntc {
const uint8_t *fastx_mapped(ntc_fastx *fx, uint64_t *size) {
    if (!fx || !fx->mm) return nullptr;
    if (size) *size = fx->mm_n;
    return (const uint8_t *)fx->mm;
}
void fastx_seek_mapped(ntc_fastx *fx, uint64_t pos) {
    if (fx && fx->mm) fx->mm_pos = std::min<size_t>((size_t)pos, fx->mm_n);
}
bool fastx_streamed_fastq(ntc_fastx *fx) { return fx && !fx->mm && fx->src && fx->format == '@'; }
uint64_t fastx_stream_read(ntc_fastx *fx, uint8_t *dst, uint64_t cap, bool *io_error) {
    uint64_t got = 0;
    while (got < cap) {
        if (fx->pos < fx->end) {  // what the format check (or an unread) left in the buffer
            const size_t t = (size_t)std::min<uint64_t>(fx->end - fx->pos, cap - got);
            std::memcpy(dst + got, fx->buf.data() + fx->pos, t);
            fx->pos += t;
            got += t;
            continue;
        }
        if (fx->eof) break;
        const int64_t r = fx->src->read_direct((char *)dst + got, (size_t)(cap - got));
        if (r < 0) {
            fx->io_error = true;
            fx->eof = true;
            break;
        }
        got += (uint64_t)r;
        if (got < cap) fx->eof = true;  // read_direct fills the room unless the input ended
    }
    if (io_error) *io_error = fx->io_error;
    return got;
}
void fastx_stream_unread(ntc_fastx *fx, const uint8_t *src, uint64_t n) {
    const size_t tail = fx->end - fx->pos;
    std::vector<char> nb((size_t)n + tail + 1 + (1u << 16));
    std::memcpy(nb.data(), src, (size_t)n);
    std::memcpy(nb.data() + n, fx->buf.data() + fx->pos, tail);
    fx->buf.swap(nb);
    fx->pos = 0;
    fx->end = (size_t)n + tail;
    // fill() supplies a missing final newline when it meets the end of input; the end was
    // met already, so supply it here
    if (fx->eof && fx->end && fx->buf[fx->end - 1] != '\n') fx->buf[fx->end++] = '\n';
}
}  // namespace ntc

extern "C" {

int ntc_fastx_next_batch(ntc_fastx *fx, uint64_t max_reads, uint64_t max_bases, const uint8_t **bases,
                         const uint64_t **offsets, uint64_t *n_reads) {
    if (!fx || !bases || !offsets || !n_reads || max_reads == 0) return NTC_ERR_INVALID_ARG;
    if (fx->mm) {
        const int rc = fx->mm_batch(max_reads, max_bases, nullptr, 0, nullptr);
        if (rc) return rc;
        if (fx->offsets.empty()) fx->offsets.assign(1, 0);
        *bases = fx->bases.data();
        *offsets = fx->offsets.data();
        *n_reads = fx->mm_reads;
        return NTC_OK;
    }
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

int ntc_fastx_next_batch_into(ntc_fastx *fx, uint64_t max_reads, uint64_t max_bases, uint8_t *bases,
                              uint64_t bases_capacity, uint64_t *offsets, uint64_t *n_reads) {
    if (!fx || !bases || !offsets || !n_reads || max_reads == 0) return NTC_ERR_INVALID_ARG;
    *n_reads = 0;
    if (fx->mm) {
        const int rc = fx->mm_batch(max_reads, max_bases, bases, bases_capacity, offsets);
        if (rc) return rc;
        *n_reads = fx->mm_reads;
        if (!fx->mm_reads) offsets[0] = 0;
        return NTC_OK;
    }
    const uint8_t *b;
    const uint64_t *o;
    uint64_t n;
    const int rc = ntc_fastx_next_batch(fx, max_reads, max_bases, &b, &o, &n);
    if (rc) return rc;
    if (o[n] > bases_capacity) return NTC_ERR_CAPACITY;
    std::memcpy(bases, b, o[n]);
    std::memcpy(offsets, o, (n + 1) * 8);
    *n_reads = n;
    return NTC_OK;
}

void ntc_fastx_close(ntc_fastx *fx) {
    if (!fx) return;
    if (fx->mm) {
        munmap((void *)fx->mm, fx->mm_n);
        delete fx;
        return;
    }
    delete fx->src;  // joins the producer before the file goes away
    delete fx->f;
    delete fx;
}

}  // extern "C"
