/*
 * ntcomp_oracle.c -- TEST INFRASTRUCTURE ONLY.  A faithful, single-threaded CPU
 * restatement of tmaklin/ntcomp's encode/decode hot path.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load this file's library;
 * the product (ntcomp_amd/, libntcomp_gpu.so) never links, loads or calls it.
 *
 * PARITY STATUS: UNPINNED against the real reference.  The reference is Rust and its
 * index semantics live in crates absent from this image (sbwt 0.3.11, kbo 0.5.1,
 * bitnuc 0.2.11 -- Cargo.lock:1358-1361, 740-743, 145-148; no toolchain, no sources,
 * no network).  Its only test (tests/fasta_data.rs:28-101) pins round-trip identity.
 * This oracle is pinned instead against the fixtures in tests/golden/, produced by the
 * independent brute-force restatement tests/golden/make_golden.py.
 *
 * It performs the SAME index operations, in the same order, as the reference:
 *   - StreamingIndex::matching_statistics   [ext sbwt] called at lib.rs:172-173:
 *       extend_right = 2 ranks, contract_left = linear LCS scan, one level at a time
 *   - encode_sequence                        lib.rs:163-230 (incl. the access_kmer
 *       assert of lib.rs:181-183 and the jump loop lib.rs:193-203)
 *   - left_extend_kmer                       lib.rs:94-128 (4 x search() per step)
 *   - encode_dictionary                      encode.rs:129-166 (access_kmer for short
 *       records + bitnuc::as_2bit)
 *   - decode_sequence                        lib.rs:254-318 (access_kmer +
 *       left_extend_kmer2, lib.rs:130-161)
 *   - SbwtIndex::search with the 8-mer prefix lookup table (cli.rs:46 default -p 8)
 * so its single-thread run is the CPU baseline that bench.py reports (kind "port").
 *
 * Build: make -C oracle   (gcc -O2 -shared -fPIC)
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_ERR_INVALID_BASE (-1)
#define ORC_ERR_EMPTY (-2)
#define ORC_ERR_CAPACITY (-3)
#define ORC_ERR_LENGTH (-4)
#define ORC_ERR_PANIC (-5)
#define ORC_ERR_ARG (-6)

typedef struct {
    uint64_t lo, hi;
} range_t;

typedef struct orc_index {
    uint64_t n;
    uint32_t k;
    uint32_t precalc;
    uint64_t nwords;
    uint64_t *rows[4];   /* copies of the 4 subset-matrix bit rows */
    uint64_t *cum[4];    /* ones before word w (rank directory)     */
    uint64_t *sel[4];    /* word index holding one #(s*64)          */
    uint64_t nsel[4];
    uint64_t C[4];
    uint8_t *lcs;
    range_t *prefix;     /* 4^precalc intervals, (0,0) when empty  */
} orc_index;

static inline int code_of(uint8_t b) {
    switch (b) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    default: return -1;
    }
}
static const uint8_t ALPHA[4] = {'A', 'C', 'G', 'T'};

/* rank_c(i) = #sets in [0,i) containing c  (simple-sds BitVector::rank). */
static inline uint64_t rank1(const orc_index *ix, int c, uint64_t i) {
    uint64_t w = i >> 6, b = i & 63;
    uint64_t r = ix->cum[c][w];
    if (b) r += (uint64_t)__builtin_popcountll(ix->rows[c][w] & ((1ULL << b) - 1));
    return r;
}

/* select_c(r) = position of the r-th (0-based) set containing c. */
static inline uint64_t select1(const orc_index *ix, int c, uint64_t r) {
    uint64_t w = ix->sel[c][r >> 6];
    while (w + 1 < ix->nwords + 1 && ix->cum[c][w + 1] <= r) w++;
    uint64_t x = ix->rows[c][w];
    uint64_t rem = r - ix->cum[c][w];
    while (rem--) x &= x - 1;
    return (w << 6) + (uint64_t)__builtin_ctzll(x);
}

static inline range_t extend_right(const orc_index *ix, range_t I, int c) {
    range_t J;
    J.lo = ix->C[c] + rank1(ix, c, I.lo);
    J.hi = ix->C[c] + rank1(ix, c, I.hi);
    return J;
}

/* StreamingIndex::contract_left [ext sbwt]: widen I to every node sharing the last t
 * characters. */
static inline range_t contract_left(const orc_index *ix, range_t I, uint32_t t) {
    while (I.lo > 0 && ix->lcs[I.lo] >= t) I.lo--;
    while (I.hi < ix->n && ix->lcs[I.hi] >= t) I.hi++;
    return I;
}

/* SbwtIndex::search: prefix lookup table, then extend_right per character. */
static int search(const orc_index *ix, const int *codes, uint32_t len, range_t *out) {
    range_t I = {0, ix->n};
    uint32_t i = 0;
    if (ix->prefix && len >= ix->precalc) {
        uint64_t key = 0;
        for (; i < ix->precalc; i++) key = (key << 2) | (uint64_t)codes[i];
        I = ix->prefix[key];
        if (I.hi <= I.lo) return 0;
    }
    for (; i < len; i++) {
        I = extend_right(ix, I, codes[i]);
        if (I.hi <= I.lo) return 0;
    }
    *out = I;
    return 1;
}

/* SbwtIndex::access_kmer: inverse walk, k selects, '$' below the root. */
static void access_kmer(const orc_index *ix, uint64_t j, uint8_t *out) {
    uint32_t k = ix->k;
    for (int64_t t = (int64_t)k - 1; t >= 0; t--) {
        if (j == 0) {
            out[t] = '$';
            continue;
        }
        int c = 3;
        while (c > 0 && ix->C[c] > j) c--;
        out[t] = ALPHA[c];
        j = select1(ix, c, j - ix->C[c]);
    }
}

orc_index *orc_index_new(uint64_t n, uint32_t k, const uint64_t *rowA, const uint64_t *rowC,
                         const uint64_t *rowG, const uint64_t *rowT, const uint64_t *Carr,
                         const uint8_t *lcs, uint32_t precalc) {
    orc_index *ix = (orc_index *)calloc(1, sizeof(orc_index));
    if (!ix) return NULL;
    ix->n = n;
    ix->k = k;
    ix->nwords = (n + 63) / 64;
    const uint64_t *src[4] = {rowA, rowC, rowG, rowT};
    for (int c = 0; c < 4; c++) {
        ix->rows[c] = (uint64_t *)calloc(ix->nwords + 1, 8);
        memcpy(ix->rows[c], src[c], ix->nwords * 8);
        if (n & 63) ix->rows[c][ix->nwords - 1] &= (1ULL << (n & 63)) - 1;
        ix->cum[c] = (uint64_t *)calloc(ix->nwords + 2, 8);
        uint64_t s = 0;
        for (uint64_t w = 0; w <= ix->nwords; w++) {
            ix->cum[c][w] = s;
            if (w < ix->nwords) s += (uint64_t)__builtin_popcountll(ix->rows[c][w]);
        }
        ix->cum[c][ix->nwords + 1] = s;
        ix->nsel[c] = s / 64 + 1;
        ix->sel[c] = (uint64_t *)calloc(ix->nsel[c], 8);
        uint64_t w = 0;
        for (uint64_t q = 0; q < ix->nsel[c]; q++) {
            uint64_t r = q * 64;
            while (w + 1 <= ix->nwords && ix->cum[c][w + 1] <= r) w++;
            ix->sel[c][q] = w;
        }
        ix->C[c] = Carr[c];
    }
    ix->lcs = (uint8_t *)malloc(n ? n : 1);
    memcpy(ix->lcs, lcs, n);
    ix->precalc = precalc;
    if (precalc > 0 && precalc <= k && precalc <= 12) {
        uint64_t np = 1ULL << (2 * precalc);
        ix->prefix = (range_t *)calloc(np, sizeof(range_t));
        int codes[16];
        for (uint64_t key = 0; key < np; key++) {
            for (uint32_t i = 0; i < precalc; i++)
                codes[i] = (int)((key >> (2 * (precalc - 1 - i))) & 3);
            range_t I = {0, n};
            int ok = 1;
            for (uint32_t i = 0; i < precalc; i++) {
                I = extend_right(ix, I, codes[i]);
                if (I.hi <= I.lo) { ok = 0; break; }
            }
            if (ok) ix->prefix[key] = I;
        }
    } else {
        ix->precalc = 0;
    }
    return ix;
}

void orc_index_free(orc_index *ix) {
    if (!ix) return;
    for (int c = 0; c < 4; c++) {
        free(ix->rows[c]);
        free(ix->cum[c]);
        free(ix->sel[c]);
    }
    free(ix->lcs);
    free(ix->prefix);
    free(ix);
}

uint64_t orc_rank(const orc_index *ix, int c, uint64_t i) { return rank1(ix, c, i); }
uint64_t orc_select(const orc_index *ix, int c, uint64_t r) { return select1(ix, c, r); }
void orc_access_kmer(const orc_index *ix, uint64_t j, uint8_t *out) { access_kmer(ix, j, out); }

/* StreamingIndex::matching_statistics [ext sbwt], lib.rs:172-173. */
static int ms_codes(const orc_index *ix, const int *codes, uint64_t len, uint32_t *out_d,
                    uint64_t *out_lo) {
    uint32_t d = 0;
    range_t I = {0, ix->n};
    for (uint64_t p = 0; p < len; p++) {
        int c = codes[p];
        while (d > 0) {
            range_t J = extend_right(ix, I, c);
            if (J.hi > J.lo) break;
            I = contract_left(ix, I, d - 1);
            d -= 1;
        }
        range_t J = extend_right(ix, I, c);
        if (J.hi > J.lo) {
            I = J;
            d = d + 1 < ix->k ? d + 1 : ix->k;
        }
        out_d[p] = d;
        out_lo[p] = I.lo;
    }
    return 0;
}

int orc_matching_statistics(const orc_index *ix, const uint8_t *q, uint64_t len, uint32_t *out_d,
                            uint64_t *out_lo) {
    int *codes = (int *)malloc((len ? len : 1) * sizeof(int));
    for (uint64_t p = 0; p < len; p++) {
        codes[p] = code_of(q[p]);
        if (codes[p] < 0) { free(codes); return ORC_ERR_INVALID_BASE; }
    }
    ms_codes(ix, codes, len, out_d, out_lo);
    free(codes);
    return ORC_OK;
}

/* left_extend_kmer, lib.rs:94-128.  kmer buffer holds the extended string right-aligned
 * in buf[..end); returns the extended length. */
static uint32_t left_extend_kmer(const orc_index *ix, int *buf, uint64_t end, uint32_t klen,
                                 const int *ref, uint64_t ref_len, uint64_t max_ext, int check_ref,
                                 int *scratch) {
    uint32_t k = ix->k;
    uint64_t ext = 0;
    uint32_t len = klen; /* kmer.len() */
    while (ext < max_ext) {
        /* new_kmer = c . kmer[0 .. kmer.len() - (ext+1)]  (a k-mer) */
        int nhits = 0, hit_c = -1;
        uint64_t hit_size = 0;
        const int *kstart = buf + (end - len);
        for (int c = 0; c < 4; c++) {
            scratch[0] = c;
            memcpy(scratch + 1, kstart, (size_t)(len - (ext + 1)) * sizeof(int));
            range_t r;
            if (search(ix, scratch, (uint32_t)(1 + len - (ext + 1)), &r)) {
                if (nhits == 0) { hit_c = c; hit_size = r.hi - r.lo; }
                nhits++;
            }
        }
        (void)k;
        if (nhits > 0) {
            int seq_matches = check_ref ? (hit_c == ref[ref_len - len - 1]) : 1;
            if (seq_matches && nhits == 1 && hit_size == 1) {
                buf[end - len - 1] = hit_c;
                len += 1;
            } else {
                break;
            }
        } else {
            break;
        }
        ext += 1;
    }
    return len;
}

typedef struct {
    uint64_t len;
    uint64_t lo;
} dict_t;

/* encode_sequence (lib.rs:163-230) + encode_dictionary (encode.rs:129-166) for one read. */
static int64_t encode_read_codes(const orc_index *ix, const int *codes, uint64_t n,
                                 uint64_t *rec_out, uint64_t cap, uint32_t *d, uint64_t *lo,
                                 int *extbuf, dict_t *kept, uint8_t *kmer) {
    uint32_t k = ix->k;
    if (n == 0) return ORC_ERR_EMPTY;
    ms_codes(ix, codes, n, d, lo);
    for (uint64_t p = 0; p < n; p++)
        if (d[p] == 0) return ORC_ERR_INVALID_BASE; /* lib.rs:207 would never terminate */
    uint64_t i = n, nk = 0;
    int *scratch = extbuf + n + 1;
    while (i > 0) {
        uint64_t st = lo[i - 1];
        if (d[i - 1] == k && i > (uint64_t)k + 1) {
            access_kmer(ix, st, kmer); /* lib.rs:181-183 */
            for (uint32_t t = 0; t < k; t++)
                if (kmer[t] != ALPHA[codes[i - k + t]]) return ORC_ERR_PANIC;
            memcpy(extbuf + (i - k), codes + (i - k), (size_t)k * sizeof(int));
            uint32_t new_len = left_extend_kmer(ix, extbuf, i, k, codes, i, i - k - 1, 1, scratch);
            uint64_t match_len = new_len;
            uint64_t old_i = i;
            for (;;) {
                if (d[i - 1] < match_len) {
                    uint64_t old_ms = d[i - 1];
                    i -= old_ms;
                    match_len -= old_ms;
                } else {
                    d[old_i - 1] = (uint32_t)(new_len - (match_len - 1));
                    kept[nk].len = d[old_i - 1];
                    kept[nk].lo = lo[old_i - 1];
                    nk++;
                    break;
                }
            }
        } else {
            kept[nk].len = d[i - 1];
            kept[nk].lo = lo[i - 1];
            nk++;
            if (i > d[i - 1]) {
                i -= d[i - 1] - 1;
            } else {
                break;
            }
        }
        if (i > 0) i -= 1;
        else break;
    }
    uint64_t total = 0, mx = 0;
    for (uint64_t r = 0; r < nk; r++) {
        total += kept[r].len;
        if (kept[r].len > mx) mx = kept[r].len;
    }
    if (mx >= (1ULL << 24)) return ORC_ERR_LENGTH; /* lib.rs:226 */
    if (total != n) return ORC_ERR_PANIC;          /* lib.rs:227 */
    if (nk > cap) return ORC_ERR_CAPACITY;
    /* encode_dictionary */
    for (uint64_t r = 0; r < nk; r++) {
        uint64_t first = (r == 0);
        uint64_t w;
        if (kept[r].len > 11) {
            w = (kept[r].lo & 0xFFFFFFFFULL) | ((kept[r].len & 0xFFFFFFULL) << 32) | (first << 56);
        } else {
            if (kept[r].len > k) return ORC_ERR_PANIC; /* kmer[(k - len)..k] underflows */
            access_kmer(ix, kept[r].lo, kmer);
            uint64_t bits = 0;
            for (uint64_t j = 0; j < kept[r].len; j++) {
                int c = code_of(kmer[k - kept[r].len + j]);
                if (c < 0) return ORC_ERR_PANIC; /* as_2bit(b"$") errors */
                bits |= (uint64_t)c << (2 * j);
            }
            w = (bits & 0x00FFFFFFFFFFFFFFULL) | (((first + 2) | (kept[r].len << 2)) << 56);
        }
        rec_out[r] = w;
    }
    return (int64_t)nk;
}

/* Encode a batch of reads; rec_offsets[n_reads+1].  Returns total records or <0. */
int64_t orc_encode_batch(const orc_index *ix, const uint8_t *bases, const uint64_t *offsets,
                         uint64_t n_reads, uint64_t *rec_out, uint64_t cap, uint64_t *rec_offsets,
                         int64_t *bad_read) {
    uint64_t maxlen = 0;
    for (uint64_t r = 0; r < n_reads; r++) {
        uint64_t L = offsets[r + 1] - offsets[r];
        if (L > maxlen) maxlen = L;
    }
    uint64_t M = maxlen + 1;
    int *codes = (int *)malloc(M * sizeof(int));
    uint32_t *d = (uint32_t *)malloc(M * sizeof(uint32_t));
    uint64_t *lo = (uint64_t *)malloc(M * sizeof(uint64_t));
    int *extbuf = (int *)malloc((2 * M + 8) * sizeof(int));
    dict_t *kept = (dict_t *)malloc(M * sizeof(dict_t));
    uint8_t *kmer = (uint8_t *)malloc(ix->k + 1);
    int64_t total = 0, ret = 0;
    if (bad_read) *bad_read = -1;
    rec_offsets[0] = 0;
    for (uint64_t r = 0; r < n_reads; r++) {
        uint64_t L = offsets[r + 1] - offsets[r];
        const uint8_t *q = bases + offsets[r];
        for (uint64_t p = 0; p < L; p++) {
            codes[p] = code_of(q[p]);
            if (codes[p] < 0) { ret = ORC_ERR_INVALID_BASE; break; }
        }
        if (ret == 0) {
            int64_t nr = encode_read_codes(ix, codes, L, rec_out + total, cap - (uint64_t)total, d,
                                           lo, extbuf, kept, kmer);
            if (nr < 0) ret = nr;
            else total += nr;
        }
        if (ret) {
            if (bad_read) *bad_read = (int64_t)r;
            break;
        }
        rec_offsets[r + 1] = (uint64_t)total;
    }
    free(codes); free(d); free(lo); free(extbuf); free(kept); free(kmer);
    return ret ? ret : total;
}

/* decode_sequence (lib.rs:254-318).  Writes reads back-to-back into out (cap bytes) with
 * read_offsets[n_reads+1]; returns total bases or <0. */
int64_t orc_decode(const orc_index *ix, const uint64_t *recs, uint64_t n_recs, uint8_t *out,
                   uint64_t cap, uint64_t *read_offsets, uint64_t off_cap, uint64_t *n_reads_out) {
    uint32_t k = ix->k;
    /* pass 1: segment lengths so the reversed assembly can be written in place */
    uint64_t total = 0, nreads = 0;
    for (uint64_t r = 0; r < n_recs; r++) {
        uint8_t flag = (uint8_t)(recs[r] >> 56);
        total += (flag & 2) ? (uint64_t)(flag >> 2) : ((recs[r] >> 32) & 0xFFFFFF);
        if (flag & 1) nreads++;
    }
    if (total > cap || nreads + 1 > off_cap) return ORC_ERR_CAPACITY;
    /* the reference iterates records in reverse, builds each read left-to-right and
     * pushes it on its 'first' record, then reverses the list of reads */
    uint64_t maxext = 64;
    int *buf = NULL;
    int *scratch = (int *)malloc(((size_t)k + 8) * sizeof(int));
    uint8_t *kmer = (uint8_t *)malloc(k + 1);
    /* read boundaries in forward order: read starts at each first-flag record */
    uint64_t *rstart = (uint64_t *)malloc((nreads + 1) * sizeof(uint64_t));
    uint64_t nr = 0;
    for (uint64_t r = 0; r < n_recs; r++)
        if ((recs[r] >> 56) & 1) rstart[nr++] = r;
    rstart[nr] = n_recs;
    uint64_t pos = 0;
    read_offsets[0] = 0;
    for (uint64_t rd = 0; rd < nr; rd++) {
        for (uint64_t r = rstart[rd + 1]; r-- > rstart[rd];) {
            uint64_t rec = recs[r];
            uint8_t flag = (uint8_t)(rec >> 56);
            if ((flag & 2) == 0) {
                uint64_t colex = rec & 0xFFFFFFFFULL;
                uint64_t slen = (rec >> 32) & 0xFFFFFF;
                access_kmer(ix, colex, kmer);
                if (slen > k) {
                    if (slen + 8 > maxext) {
                        maxext = 2 * slen + 8;
                        free(buf);
                        buf = NULL;
                    }
                    if (!buf) buf = (int *)malloc(maxext * sizeof(int));
                    uint64_t end = maxext;
                    for (uint32_t t = 0; t < k; t++) {
                        int c = code_of(kmer[t]);
                        if (c < 0) { free(buf); free(scratch); free(kmer); free(rstart); return ORC_ERR_PANIC; }
                        buf[end - k + t] = c;
                    }
                    uint32_t got = left_extend_kmer(ix, buf, end, k, NULL, 0, slen - k, 0, scratch);
                    if (got != slen) { free(buf); free(scratch); free(kmer); free(rstart); return ORC_ERR_PANIC; }
                    for (uint64_t t = 0; t < slen; t++) out[pos + t] = ALPHA[buf[end - slen + t]];
                } else {
                    memcpy(out + pos, kmer + (k - slen), slen);
                }
                pos += slen;
            } else {
                uint64_t len = flag >> 2;
                uint64_t bits = rec & 0x00FFFFFFFFFFFFFFULL;
                for (uint64_t j = 0; j < len; j++) out[pos + j] = ALPHA[(bits >> (2 * j)) & 3];
                pos += len;
            }
        }
        read_offsets[rd + 1] = pos;
    }
    free(buf); free(scratch); free(kmer); free(rstart);
    *n_reads_out = nr;
    return (int64_t)pos;
}
