// FASTA / FASTQ ingest for the CLI (include/ntcomp_host.h "FASTX").
//
// Replaces needletail::parse_fastx_file + SequenceRecord::normalize(true) as the reference
// uses them (src/main.rs:51-62 build input, :158-163 encode input): plain or gzip input
// (zlib's gz* reads both), FASTA records (">" header, sequence over any number of lines)
// and FASTQ records ("@" header, sequence, "+", quality).  normalize(iupac = true) is
// restated from needletail [ext, recalled, needletail 0.6]: A C G T N - kept; a c g ->
// upper case; t u U -> T; n -> N; . ~ -> -; IUPAC B D H V R Y S W K M kept (lower case
// upper-cased); whitespace dropped; anything else -> N.  Record names are not kept (the
// reference discards them on encode, main.rs:158-166).
#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
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

}  // namespace

struct ntc_fastx {
    gzFile f = nullptr;
    std::vector<char> buf;  // read-ahead
    size_t pos = 0, end = 0;
    bool eof = false;
    int format = 0;  // 0 unknown, '>' FASTA, '@' FASTQ
    bool have_pending = false;  // FASTA: the next record's '>' line was already consumed
    // current batch
    std::vector<uint8_t> bases;
    std::vector<uint64_t> offsets;

    bool fill() {
        if (eof) return false;
        if (pos > 0 && pos < end) std::memmove(buf.data(), buf.data() + pos, end - pos);
        end -= pos;
        pos = 0;
        if (buf.size() < (1u << 22)) buf.resize(1u << 22);
        if (end == buf.size()) buf.resize(buf.size() * 2);
        const int got = gzread(f, buf.data() + end, (unsigned)(buf.size() - end));
        if (got <= 0) {
            eof = true;
            return false;
        }
        end += (size_t)got;
        return true;
    }
    // one line without its terminator; false at end of input
    bool line(std::string &out) {
        out.clear();
        for (;;) {
            const char *b = buf.data() + pos;
            const char *nl = (const char *)std::memchr(b, '\n', end - pos);
            if (nl) {
                out.append(b, nl - b);
                pos = (size_t)(nl - buf.data()) + 1;
                if (!out.empty() && out.back() == '\r') out.pop_back();
                return true;
            }
            out.append(b, end - pos);
            pos = end;
            if (!fill()) return !out.empty();
        }
    }
    void append_seq(const std::string &s) {
        for (unsigned char c : s) {
            const uint8_t v = norm_table[c];
            if (v) bases.push_back(v);
        }
    }
    // next record's normalized sequence appended to `bases`; 0 = ok, 1 = end, <0 error
    int next() {
        std::string l;
        if (format == '>') {
            if (!have_pending) {
                do {
                    if (!line(l)) return 1;
                } while (l.empty());
                if (l[0] != '>') return -1;
            }
            have_pending = false;
            while (line(l)) {
                if (!l.empty() && l[0] == '>') {
                    have_pending = true;
                    break;
                }
                append_seq(l);
            }
            return 0;
        }
        // FASTQ
        do {
            if (!line(l)) return 1;
        } while (l.empty());
        if (l[0] != '@') return -1;
        std::string seq, plus, qual;
        if (!line(seq) || !line(plus) || plus.empty() || plus[0] != '+') return -1;
        if (!line(qual)) return -1;
        append_seq(seq);
        return 0;
    }
};

extern "C" {

int ntc_fastx_open(const char *path, ntc_fastx **out) {
    if (!path || !out) return NTC_ERR_INVALID_ARG;
    *out = nullptr;
    init_norm();
    gzFile f = gzopen(path, "rb");
    if (!f) return NTC_ERR_IO;
    gzbuffer(f, 1u << 20);
    auto *fx = new ntc_fastx();
    fx->f = f;
    fx->buf.resize(1u << 22);
    // detect the format from the first non-empty character
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
    if (fx->format != '>' && fx->format != '@' && !(fx->eof && fx->pos == fx->end)) {
        gzclose(f);
        delete fx;
        return NTC_ERR_FORMAT;
    }
    if (fx->format == 0) fx->format = '>';  // empty input
    *out = fx;
    return NTC_OK;
}

int ntc_fastx_next_batch(ntc_fastx *fx, uint64_t max_reads, uint64_t max_bases, const uint8_t **bases,
                         const uint64_t **offsets, uint64_t *n_reads) {
    if (!fx || !bases || !offsets || !n_reads || max_reads == 0) return NTC_ERR_INVALID_ARG;
    fx->bases.clear();
    fx->offsets.assign(1, 0);
    while (fx->offsets.size() - 1 < max_reads && fx->bases.size() < max_bases) {
        const int rc = fx->next();
        if (rc == 1) break;
        if (rc < 0) return NTC_ERR_FORMAT;
        fx->offsets.push_back(fx->bases.size());
    }
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
    if (fx->f) gzclose(fx->f);
    delete fx;
}

}  // extern "C"
