/*
 * abi_check.c -- a C99 consumer of libntcomp_gpu.so that sees nothing but the headers in include/.
 *
 * It stands where the reference's Rust FFI would: the struct layouts are
 * checked at compile time against the #[repr(C)] declarations given there, and with a data
 * directory (written by tests/test_abi_c.py) it drives the path the reference's call sites
 * take -- src/main.rs:149 (index), :166-170 (encode_sequence + encode_dictionary, then
 * write_block_to per block), src/lib.rs:320-365 (decode_block -> decode_sequence) -- through
 * the C ABI alone:
 *   ntc_index_upload -> ntc_encode_batch -> ntc_write_block -> ntc_read_block ->
 *   ntc_decode_batch, and ntc_encode_pack_batch -> ntc_deflate_block (GPU packer),
 * comparing with the committed golden records and reads.
 *
 *   abi_check --layout     print the layouts + ABI version (no GPU call)
 *   abi_check DIR          run the round trip on device 0 (DIR: meta.txt + *.bin)
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ntcomp_codec.h"
#include "ntcomp_gpu.h"
#include "ntcomp_host.h"
#include "ntcomp_pipeline.h"

/* #[repr(C)] NtcIndexView: u64, u32, u32, [*const u64; 4], [u64; 4], *const u8 */
_Static_assert(sizeof(void *) == 8, "64-bit target");
_Static_assert(offsetof(ntc_index_view, n_nodes) == 0, "n_nodes");
_Static_assert(offsetof(ntc_index_view, k) == 8, "k");
_Static_assert(offsetof(ntc_index_view, reserved) == 12, "reserved");
_Static_assert(offsetof(ntc_index_view, rows) == 16, "rows");
_Static_assert(offsetof(ntc_index_view, C) == 48, "C");
_Static_assert(offsetof(ntc_index_view, lcs) == 80, "lcs");
_Static_assert(sizeof(ntc_index_view) == 88, "ntc_index_view");
/* #[repr(C)] NtcTiming: f64, f64, f64, u64, u64 */
_Static_assert(offsetof(ntc_timing, total_ms) == 0 && offsetof(ntc_timing, main_ms) == 8 &&
                   offsetof(ntc_timing, aux_ms) == 16 && offsetof(ntc_timing, units) == 24 &&
                   offsetof(ntc_timing, records) == 32 && sizeof(ntc_timing) == 40,
               "ntc_timing");
/* #[repr(C)] NtcStreamMeta: 4 x u64; NtcBlockMeta: [NtcStreamMeta; 4], u64, u64, i32, u32 */
_Static_assert(sizeof(ntc_stream_meta) == 32 && offsetof(ntc_stream_meta, offset) == 24, "ntc_stream_meta");
_Static_assert(offsetof(ntc_block_meta, stream) == 0 && offsetof(ntc_block_meta, num_records) == 128 &&
                   offsetof(ntc_block_meta, n_recs) == 136 && offsetof(ntc_block_meta, status) == 144 &&
                   offsetof(ntc_block_meta, reserved) == 148 && sizeof(ntc_block_meta) == 152,
               "ntc_block_meta");
/* #[repr(C)] NtcPipelineOpts: i32, i32, u64, i32, i32; NtcPipelineStats: 5 x u64, 9 x f64, i32,
 * i32, i64, [c_char; 256] */
_Static_assert(offsetof(ntc_pipeline_opts, batch_bases) == 8 && offsetof(ntc_pipeline_opts, deflate_engine) == 16 &&
                   offsetof(ntc_pipeline_opts, host_parse) == 20 && sizeof(ntc_pipeline_opts) == 24,
               "ntc_pipeline_opts");
_Static_assert(offsetof(ntc_pipeline_stats, parse_s) == 40 && offsetof(ntc_pipeline_stats, wall_s) == 72 &&
                   offsetof(ntc_pipeline_stats, alloc_s) == 80 && offsetof(ntc_pipeline_stats, threads) == 112 &&
                   offsetof(ntc_pipeline_stats, gpu_parsed) == 116 &&
                   offsetof(ntc_pipeline_stats, bad_read) == 120 && offsetof(ntc_pipeline_stats, error) == 128 &&
                   sizeof(ntc_pipeline_stats) == 384,
               "ntc_pipeline_stats");
_Static_assert(offsetof(ntc_build_opts, host_budget_bytes) == 8 && offsetof(ntc_build_opts, temp_dir) == 16 &&
                   offsetof(ntc_build_opts, max_partition_keys) == 24 && sizeof(ntc_build_opts) == 32,
               "ntc_build_opts");
_Static_assert(offsetof(ntc_build_stats, peak_device_bytes) == 56 && offsetof(ntc_build_stats, kmer_partitions) == 64 &&
                   offsetof(ntc_build_stats, seq_uploads) == 76 && offsetof(ntc_build_stats, seconds) == 80 &&
                   offsetof(ntc_build_stats, seconds_sort) == 128 && sizeof(ntc_build_stats) == 136,
               "ntc_build_stats");
/* the status enum crosses the boundary as a C int (Rust: c_int) */
_Static_assert(sizeof(ntc_status) == sizeof(int), "ntc_status");

static void *slurp(const char *dir, const char *name, size_t *len) {
    char path[4096];
    snprintf(path, sizeof(path), "%s/%s", dir, name);
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    void *p = malloc(n > 0 ? (size_t)n : 1);
    if (p && n > 0 && fread(p, 1, (size_t)n, f) != (size_t)n) {
        free(p);
        p = NULL;
    }
    fclose(f);
    *len = (size_t)n;
    return p;
}

#define CHECK(cond, ...)                      \
    do {                                      \
        if (!(cond)) {                        \
            fprintf(stderr, "abi_check: ");   \
            fprintf(stderr, __VA_ARGS__);     \
            fprintf(stderr, "\n");            \
            return 1;                         \
        }                                     \
    } while (0)

static int run(const char *dir) {
    unsigned long long n, k, c[4], n_reads, n_recs;
    char path[4096];
    snprintf(path, sizeof(path), "%s/meta.txt", dir);
    FILE *mf = fopen(path, "r");
    CHECK(mf, "missing %s", path);
    int got = fscanf(mf, "%llu %llu %llu %llu %llu %llu %llu %llu", &n, &k, &c[0], &c[1], &c[2], &c[3], &n_reads,
                     &n_recs);
    fclose(mf);
    CHECK(got == 8, "bad meta.txt");
    size_t lr, ll, lb, lo, le;
    uint64_t *rows = (uint64_t *)slurp(dir, "rows.bin", &lr);
    uint8_t *lcs = (uint8_t *)slurp(dir, "lcs.bin", &ll);
    uint8_t *bases = (uint8_t *)slurp(dir, "bases.bin", &lb);
    uint64_t *offs = (uint64_t *)slurp(dir, "offs.bin", &lo);
    uint64_t *expect = (uint64_t *)slurp(dir, "recs.bin", &le);
    const uint64_t words = (n + 63) / 64;
    CHECK(rows && lcs && bases && offs && expect, "missing data files");
    CHECK(lr == 4 * words * 8 && ll == n && lo == (n_reads + 1) * 8 && le == n_recs * 8, "data sizes");

    ntc_ctx *ctx = NULL;
    CHECK(ntc_ctx_create(0, &ctx) == NTC_OK, "ntc_ctx_create");
    ntc_index_view v;
    memset(&v, 0, sizeof(v));
    v.n_nodes = n;
    v.k = (uint32_t)k;
    for (int i = 0; i < 4; i++) {
        v.rows[i] = rows + (size_t)i * words;
        v.C[i] = c[i];
    }
    v.lcs = lcs;
    CHECK(ntc_index_upload(ctx, &v) == NTC_OK, "ntc_index_upload: %s", ntc_last_error(ctx));

    /* encode (src/main.rs:162-173) */
    const uint64_t cap = offs[n_reads] + 1;
    uint64_t *recs = (uint64_t *)malloc(cap * 8), *roffs = (uint64_t *)malloc((n_reads + 1) * 8);
    int64_t bad = 0;
    CHECK(ntc_encode_batch(ctx, bases, offs, n_reads, recs, cap, roffs, &bad) == NTC_OK && bad == -1,
          "ntc_encode_batch: %s", ntc_last_error(ctx));
    CHECK(roffs[n_reads] == n_recs && memcmp(recs, expect, n_recs * 8) == 0, "records differ from the goldens");

    /* write_block_to (lib.rs:232) -> decode_block's container half (lib.rs:320-363) */
    uint8_t *blk = NULL;
    uint64_t blk_len = 0, used = 0, nr = 0, nrec = 0;
    uint64_t *back = NULL;
    CHECK(ntc_write_block(recs, n_recs, n_reads, &blk, &blk_len) == NTC_OK, "ntc_write_block");
    CHECK(ntc_read_block(blk, blk_len, &used, &back, &nr, &nrec) == NTC_OK, "ntc_read_block");
    CHECK(used == blk_len && nr == n_recs && nrec == n_reads && memcmp(back, expect, n_recs * 8) == 0,
          "block round trip");

    /* the GPU packer path: same container bytes as the host codec */
    ntc_block_meta meta;
    uint8_t *payload = NULL, *blk2 = NULL;
    uint64_t plen = 0, blk2_len = 0;
    CHECK(ntc_encode_pack_batch(ctx, bases, offs, n_reads, 65536, &meta, &payload, &plen, &bad) == NTC_OK,
          "ntc_encode_pack_batch: %s", ntc_last_error(ctx));
    CHECK(ntc_deflate_block(&meta, payload, NTC_DEFLATE_ZLIB, &blk2, &blk2_len) == NTC_OK, "ntc_deflate_block");
    CHECK(blk2_len == blk_len && memcmp(blk, blk2, blk_len) == 0, "GPU-packed block differs from the host block");

    /* decode_sequence (lib.rs:254-318) */
    uint8_t *out = (uint8_t *)malloc(offs[n_reads] + 1);
    uint64_t *ooffs = (uint64_t *)malloc((n_reads + 1) * 8);
    uint64_t dr = 0, db = 0;
    CHECK(ntc_decode_batch(ctx, back, nr, out, offs[n_reads] + 1, ooffs, n_reads + 1, &dr, &db) == NTC_OK,
          "ntc_decode_batch: %s", ntc_last_error(ctx));
    CHECK(dr == n_reads && db == offs[n_reads] && memcmp(out, bases, db) == 0 &&
              memcmp(ooffs, offs, (n_reads + 1) * 8) == 0,
          "decode(encode(x)) != x");

    /* the error surface is a status code, never an abort */
    const uint8_t bad_read[3] = {'A', 'X', 'C'};
    const uint64_t bad_offs[2] = {0, 3};
    CHECK(ntc_encode_batch(ctx, bad_read, bad_offs, 1, recs, cap, roffs, &bad) == NTC_ERR_INVALID_BASE && bad == 0,
          "invalid base status");

    ntc_buffer_free(blk);
    ntc_buffer_free(blk2);
    ntc_buffer_free(back);
    ntc_buffer_free(payload);
    ntc_ctx_destroy(ctx);
    free(rows), free(lcs), free(bases), free(offs), free(expect), free(recs), free(roffs), free(out), free(ooffs);
    printf("abi_check: OK (%llu reads, %llu records, k = %llu)\n", n_reads, n_recs, k);
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 2 || strcmp(argv[1], "--layout") == 0) {
        printf("{\"abi_version\": %d, \"ntc_index_view\": %zu, \"ntc_timing\": %zu, \"ntc_block_meta\": %zu}\n",
               ntc_abi_version(), sizeof(ntc_index_view), sizeof(ntc_timing), sizeof(ntc_block_meta));
        return ntc_abi_version() == NTC_ABI_VERSION ? 0 : 1;
    }
    return run(argv[1]);
}
