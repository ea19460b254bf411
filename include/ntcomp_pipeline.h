/*
 * ntcomp_pipeline.h -- the CLI's native file-to-file drivers (libntcomp_gpu.so).
 *
 *   ntc_encode_file   src/main.rs:141-181 (`ntcomp encode -i P reads > encoded.dat`):
 *                     FASTX batches -> GPU encode + block packer on every context ->
 *                     deflate on the host pool -> file header + blocks, in file order.
 *                     A plain FASTQ goes to the GPU as text, cut at block boundaries,
 *                     and is parsed there (ntc_encode_pack_fastq); a batch with a blank
 *                     line, and every compressed or FASTA input, is parsed on the host.
 *   ntc_decode_file   src/main.rs:183-211 (`ntcomp decode -i P encoded.dat > out.fasta`):
 *                     blocks inflated + stream-decoded on the host pool -> GPU walk and
 *                     FASTA formatting on every context -> ">seq.N" records in file order.
 *
 * Behaviour kept from the reference: blocks of 65,536 reads (main.rs:152), the last block's
 * header carries num_records % 65,536 (main.rs:176), a block with no long or no short
 * record is not written (write_block_to errs and main.rs:170 drops it).
 * Errors are status codes (the reference panics or, for bases absent from the index, never
 * terminates): the first failing read's file index is in stats->bad_read.
 */
#ifndef NTCOMP_PIPELINE_H
#define NTCOMP_PIPELINE_H

#include <stdint.h>

#include "ntcomp_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ntc_pipeline_opts {
    int32_t threads;          /* host pool (parse, deflate); <= 0: ntc_host_threads()        */
    int32_t blocks_per_batch; /* 65,536-read blocks per GPU call; <= 0: 4 (encode), 2 (decode) */
    uint64_t batch_bases;     /* encode: bases per pinned batch buffer; 0: 64 Mi (grows for long reads) */
    int32_t deflate_engine;   /* NTC_DEFLATE_ZLIB (0), _LIBDEFLATE (1) or _ADAPTIVE (2)        */
    int32_t host_parse;       /* encode, plain FASTQ: 0 = the text goes to the GPU, which parses
                                 it (ntc_encode_pack_fastq); 1 = parsed by the host pool      */
} ntc_pipeline_opts;

typedef struct ntc_pipeline_stats {
    uint64_t reads, bases, blocks, dropped_blocks, bytes_out;
    double parse_s, gpu_s, deflate_s, write_s; /* thread-seconds per stage                  */
    double wall_s;
    double alloc_s;                            /* seconds spent pinning host buffers        */
    double first_batch_s, reader_done_s, gpu_done_s; /* timeline from the call's start       */
    int32_t threads;
    int32_t gpu_parsed;                        /* encode: batches parsed on the GPU (FASTQ text) */
    int64_t bad_read;                          /* file index of the failing read, or -1     */
    char error[256];
} ntc_pipeline_stats;

/* ctxs: n_ctx contexts with the index uploaded (one per GPU; two on one device are allowed).
 * Writes encoded.dat to out_fd (not closed).                                              */
int ntc_encode_file(ntc_ctx *const *ctxs, int n_ctx, const char *in_path, int out_fd, const ntc_pipeline_opts *opts,
                    ntc_pipeline_stats *stats);

/* Reads encoded.dat at in_path (mapped), writes FASTA to out_fd (not closed): ">seq.i\n"
 * + bases + "\n" per read, i from 1 across the file (main.rs:204).  opts->threads sizes the
 * inflate pool, opts->blocks_per_batch the GPU call (<= 0: 2; batch_bases and
 * deflate_engine are unused).  A truncated block ends the input like read_exact (main.rs:199); a damaged block
 * (bad gzip member or stream sizes) ends the output after the blocks before it and still
 * returns NTC_OK, as decode_block's Err just ends the reference's loop (main.rs:202): the
 * caller sees it in stats->dropped_blocks (> 0) and stats->error.  stats: reads, bases,
 * blocks decoded, dropped_blocks = whole blocks not decoded, bytes_out = FASTA bytes,
 * parse_s = inflate CPU time summed over threads, gpu_s, write_s, wall_s, alloc_s = block
 * scan + pinned allocation seconds, first_batch_s / reader_done_s / gpu_done_s = when the
 * first batch was written / the last block inflated / the last GPU call returned.            */
int ntc_decode_file(ntc_ctx *const *ctxs, int n_ctx, const char *in_path, int out_fd, const ntc_pipeline_opts *opts,
                    ntc_pipeline_stats *stats);

#ifdef __cplusplus
}
#endif
#endif
