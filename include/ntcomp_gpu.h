/*
 * ntcomp_gpu.h -- C ABI of libntcomp_gpu.so, the MI355X (gfx950) encode/decode hot path
 * of ntcomp.  Plain C types only: pointers, sizes, status codes.  No torch, no HIP types.
 *
 * What each entry point replaces in the reference (tmaklin/ntcomp, Rust):
 *
 *   ntc_index_upload        the in-memory (SbwtIndexVariant, LcsArray) pair returned by
 *                           kbo::index::load_sbwt (src/main.rs:149, :190) -- uploaded once
 *                           per GPU and kept resident in HBM.
 *   ntc_encode_batch[_device]
 *                           ntcomp::encode_sequence (src/lib.rs:163-230) FUSED with
 *                           ntcomp::encode::encode_dictionary (src/encode.rs:129-166), over
 *                           a batch of reads: the per-read loop of src/main.rs:162-173.
 *                           Output is the u64 record stream, per read rightmost segment
 *                           first with the `first` flag on it, bit-identical to
 *                           encode_dictionary's, ready for write_block_to (src/lib.rs:232).
 *   ntc_decode_batch[_device]
 *                           ntcomp::decode_sequence (src/lib.rs:254-318) over the records
 *                           of one or more blocks (what decode_block, src/lib.rs:320-368,
 *                           calls after unzipping a block).
 *
 * Error behaviour: the reference panics (unwrap / assert!) or, for a base absent from
 * the index, never terminates (lib.rs:206-207 with d = 0 underflows).  Across this ABI
 * every such case is a status code; nothing aborts:
 *   NTC_ERR_EMPTY_READ    encode.rs:133-135 / lib.rs:224 (EncodeError on empty input)
 *   NTC_ERR_INVALID_BASE  non-ACGT byte, or a base the index does not contain
 *   NTC_ERR_LENGTH        a match length >= 2^24 (assert at lib.rs:226)
 *   NTC_ERR_REFERENCE_PANIC  a short record (len <= 11) longer than k, possible only for
 *                         k <= 10: encode.rs:151-152 slices kmer[(k - len)..k] and panics
 *
 * Threading: one ntc_ctx per GPU, driven by one host thread at a time.  Contexts on
 * different devices are independent.  The index is read-only once uploaded.
 */
#ifndef NTCOMP_GPU_H
#define NTCOMP_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NTC_ABI_VERSION 1

typedef enum ntc_status {
    NTC_OK = 0,
    NTC_ERR_INVALID_ARG = 1,
    NTC_ERR_INVALID_BASE = 2,
    NTC_ERR_EMPTY_READ = 3,
    NTC_ERR_LENGTH = 4,
    NTC_ERR_CAPACITY = 5,
    NTC_ERR_HIP = 6,
    NTC_ERR_NO_INDEX = 7,
    NTC_ERR_FORMAT = 8,
    NTC_ERR_IO = 9,
    NTC_ERR_UNSUPPORTED = 10,
    NTC_ERR_REFERENCE_PANIC = 11
} ntc_status;

typedef struct ntc_ctx ntc_ctx;

/* A host-memory view of an SBWT subset-matrix index + LCS array (sbwt 0.3.11 semantics,
 * SURVEY.md Appendix A.1): n nodes in colex order, node 0 = root $^k.
 *   rows[c]  (c = A,C,G,T): ceil(n/64) little-endian u64 words; bit j%64 of word j/64
 *            set <=> node j's label set contains c.
 *   C[c]     = 1 + #labels with a character < c (= first node ending with c).
 *   lcs[j]   = longest common suffix of nodes j-1 and j (lcs[0] = 0); k <= 255.      */
typedef struct ntc_index_view {
    uint64_t n_nodes;
    uint32_t k;
    uint32_t reserved;
    const uint64_t *rows[4];
    uint64_t C[4];
    const uint8_t *lcs;
} ntc_index_view;

/* Per-call device timings (milliseconds, HIP events on the context's stream). */
typedef struct ntc_timing {
    double total_ms;      /* first launch -> last launch of the call           */
    double main_ms;       /* the dominant kernel: encode k_ms4 / decode walk     */
    double aux_ms;        /* everything else (tiling, scans, record emit)       */
    uint64_t units;       /* bases processed (encode: input, decode: output)   */
    uint64_t records;     /* records produced (encode) / consumed (decode)     */
} ntc_timing;

int ntc_abi_version(void);

int ntc_ctx_create(int device, ntc_ctx **out);
void ntc_ctx_destroy(ntc_ctx *ctx);
const char *ntc_last_error(const ntc_ctx *ctx);
/* Optional: launch on a caller-owned hipStream_t (passed as void*); NULL = own stream. */
int ntc_ctx_set_stream(ntc_ctx *ctx, void *hip_stream);
int ntc_ctx_synchronize(ntc_ctx *ctx);
/* Tuning / diagnostics.  "encode_variant": 4 (default: packed bases, suffix table for
 * positions whose U-mer is absent, persistent matching-statistics kernel with dynamic
 * read assignment and path runs, separate parse) or 1 (the first design: one lane per
 * read walking every position, kept for A/B).  "tab_u": suffix-table depth U for the
 * NEXT ntc_index_upload (0 = default ceil(log4 n) + 2 capped at min(k, 14); results
 * never depend on it).  "max_pass_bases" (default 2^30): ntc_encode_batch /
 * ntc_decode_batch run in device passes of whole reads holding at most this many bases
 * (device workspace is ~40 B per base of a pass; results never depend on it).
 * "joint" for the NEXT upload: -1 (default, auto: on when the path cover averages fewer
 * than 4096 nodes per path, i.e. a genome collection), 0 or 1: joint path runs over
 * multi-node matching-statistics intervals (results never depend on it; after an upload
 * get_option returns the setting in use).  "win" (-1 auto = on for U >= 4 / 0 / 1): SCAN
 * window words, 4^(U-3) x 32 B, four positions per line.  Also "filter" (-1 auto = on only
 * without window words and below 60 % density / 0 / 1: SCAN pre-filter), "ext2" (0 / 1:
 * two-character rank chunks), "pair_bytes" (0 / 1), same rules.  "decode_only" (0 default
 * / 1) for the NEXT upload: build only what decoding reads (the walk table), none of the
 * encoder's path cover, suffix table or SCAN words; encode calls on that index then fail
 * with NTC_ERR_NO_INDEX (after the upload get_option returns whether the index in use is
 * decode-only; ntc_index_share passes it on).
 * "warm_dma" (bytes, 1 .. 2^30) is an action: one device-to-host and one host-to-device copy
 * of that size through a temporary pinned buffer, now -- the process's first large copies
 * start the DMA engines (≈ 8 ms on the MI355X box), which the CLI does beside the index
 * preparation instead of on the first batch's path.
 * Read-only: "n_paths", "path_text_len" (the path cover built on the device at upload),
 * "path_hash" (test hook: FNV-1a of the cover arrays, derived.h path_cover_hash),
 * "tab_u" (after an upload: the depth in use), "tab_u_fallback" (1: the default depth 15
 * did not fit in free HBM, 14 was used), "pack_us" (last GPU block packer call, both
 * kernels), "upload_host_us" / "upload_total_us"
 * (last upload: host-side derivation / whole call).  Env NTC_ENCODE_VARIANT sets the
 * default variant at ntc_ctx_create.                                                 */
int ntc_ctx_set_option(ntc_ctx *ctx, const char *key, int64_t value);
int ntc_ctx_get_option(const ntc_ctx *ctx, const char *key, int64_t *value);

/* Upload the index once; builds the device-side rank words, the unique-predecessor
 * bitvector, the path cover, the suffix table (+ presence bitmaps) and the inverse-walk
 * jump table in HBM (DESIGN.md "Data layout in HBM").  About 3 GB at n = 10 M, k = 91. */
int ntc_index_upload(ntc_ctx *ctx, const ntc_index_view *ix);
/* ntc_index_upload in two halves, so a caller can derive the host tables (no GPU) while
 * contexts are being created: ntc_index_prepare copies the view and builds them;
 * ntc_index_upload_prepared puts them on ctx's device (any number of contexts / devices;
 * same device index as ntc_index_upload).  Free with ntc_index_prep_free.              */
typedef struct ntc_index_prep ntc_index_prep;
int ntc_index_prepare(const ntc_index_view *ix, ntc_index_prep **out);
int ntc_index_upload_prepared(ntc_ctx *ctx, const ntc_index_prep *prep);
void ntc_index_prep_free(ntc_index_prep *prep);
/* dst uses src's device index (both contexts on one GPU): no second upload, no second copy
 * in HBM; the index is freed with the last context holding it.  Each context keeps its own
 * stream and workspace, so two contexts on one GPU overlap one call's copies and host work
 * with the other's kernels (the CLI's contexts per GPU).                                  */
int ntc_index_share(ntc_ctx *dst, const ntc_ctx *src);
int ntc_index_info(const ntc_ctx *ctx, uint64_t *n_nodes, uint32_t *k, uint64_t *device_bytes);

/* ---- encode ---------------------------------------------------------------------- */
/* Host buffers: bases = reads back to back (ASCII, already normalize()d to upper case);
 * read_offsets[n_reads+1].  On success rec_offsets_out[n_reads+1] delimits each read's
 * records inside rec_out.  Synchronous.  On a per-read error *bad_read (if non-NULL)
 * receives the first failing read index.                                            */
int ntc_encode_batch(ntc_ctx *ctx, const uint8_t *bases, const uint64_t *read_offsets,
                     uint64_t n_reads, uint64_t *rec_out, uint64_t rec_capacity,
                     uint64_t *rec_offsets_out, int64_t *bad_read);

/* Device buffers (HBM-resident, e.g. from hipMalloc or a torch tensor); read_offsets
 * index d_bases directly.  Asynchronous on the context stream when max_read_len > 0 (an
 * upper bound on every read's length, e.g. 150); with max_read_len = 0 the library
 * first sizes its scratch from the offsets (one small device->host read).  Call
 * ntc_encode_status() (which synchronises) for the verdict.  rec_capacity must be >=
 * the total number of records (total bases is always enough).  The workspace is sized
 * by need: when a call runs out of an overflow pool (reads with many entries or
 * records), ntc_encode_status grows the pools and runs the call again on the same
 * buffers, so d_bases, d_read_offsets and the outputs must stay valid and unchanged until
 * ntc_encode_status returns (option "spill_reruns" counts such re-runs).              */
int ntc_encode_batch_device(ntc_ctx *ctx, const uint8_t *d_bases, const uint64_t *d_read_offsets,
                            uint64_t n_reads, uint32_t max_read_len, uint64_t *d_rec_out,
                            uint64_t rec_capacity, uint64_t *d_rec_offsets_out);
int ntc_encode_status(ntc_ctx *ctx, int64_t *bad_read, uint64_t *n_records);

/* ---- decode ---------------------------------------------------------------------- */
/* recs: the u64 records of whole reads (one or more blocks, in file order).  Writes the
 * reads back to back into bases_out and read_offsets_out[n_reads+1].  Synchronous.
 * NTC_ERR_CAPACITY if bases_capacity / offsets_capacity are too small (the required
 * sizes are returned in *n_bases_out and *n_reads_out).                              */
int ntc_decode_batch(ntc_ctx *ctx, const uint64_t *recs, uint64_t n_recs, uint8_t *bases_out,
                     uint64_t bases_capacity, uint64_t *read_offsets_out,
                     uint64_t offsets_capacity, uint64_t *n_reads_out, uint64_t *n_bases_out);
/* Device variant; asynchronous; verdict + sizes via ntc_decode_status().             */
int ntc_decode_batch_device(ntc_ctx *ctx, const uint64_t *d_recs, uint64_t n_recs,
                            uint8_t *d_bases_out, uint64_t bases_capacity,
                            uint64_t *d_read_offsets_out, uint64_t offsets_capacity);
int ntc_decode_status(ntc_ctx *ctx, uint64_t *n_reads, uint64_t *n_bases);
/* decode_sequence and the decode command's output lines (src/lib.rs:254-318,
 * src/main.rs:203-209) in one device pass: the records of whole reads (host buffer) in,
 * ">seq.{first_id + r}\n{read r}\n" for every read out (host buffer), the FASTA text
 * formatted on the GPU.  n_reads / n_bases: what the records hold (first flags; record
 * lengths) -- they size the device buffers and are checked against the decode
 * (NTC_ERR_FORMAT if they differ).  *out_len = the text's bytes (the size needed on
 * NTC_ERR_CAPACITY).  Synchronous.                                                      */
int ntc_decode_fasta(ntc_ctx *ctx, const uint64_t *recs, uint64_t n_recs, uint64_t n_reads, uint64_t n_bases,
                     uint64_t first_id, uint8_t *out, uint64_t out_capacity, uint64_t *out_len);

/* Timings of the last encode/decode call (synchronises). */
int ntc_last_timing(ntc_ctx *ctx, ntc_timing *out);

/* Device memory helpers for callers without their own allocator (bench, tests). */
int ntc_device_alloc(ntc_ctx *ctx, uint64_t bytes, void **d_ptr);
int ntc_device_free(ntc_ctx *ctx, void *d_ptr);
int ntc_memcpy_h2d(ntc_ctx *ctx, void *d_dst, const void *h_src, uint64_t bytes);
int ntc_memcpy_d2h(ntc_ctx *ctx, void *h_dst, const void *d_src, uint64_t bytes);

/* Diagnostics: the k-bounded matching statistics of each position (d, colex start of
 * the interval) exactly as StreamingIndex::matching_statistics (lib.rs:172-173) returns
 * them; host buffers sized to the total number of bases.                             */
int ntc_debug_matching_statistics(ntc_ctx *ctx, const uint8_t *bases,
                                  const uint64_t *read_offsets, uint64_t n_reads,
                                  uint32_t *d_out, uint32_t *start_out);

#ifdef __cplusplus
}
#endif
#endif
