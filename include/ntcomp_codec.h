/*
 * ntcomp_codec.h -- block container of encoded.dat (libntcomp_gpu.so).
 *
 *   ntc_file_header   encode_file_header(0,0,0,0)           src/lib.rs:52-67 (32 zero bytes)
 *   ntc_write_block   write_block_to(u64_encoding, num_records, sink)   src/lib.rs:232-252
 *                     (split_encoded_dictionary + compress_block x4, src/encode.rs:96-229)
 *                     = ntc_pack_block + ntc_deflate_block
 *   ntc_pack_block    the part of write_block_to before deflate: split_encoded_dictionary
 *                     (src/encode.rs:168-229), rice_encode / minimal_binary_encode
 *                     (src/encode.rs:59-94) and the bytes compress_block hands to
 *                     deflate_bytes (src/encode.rs:107-109), per stream
 *   ntc_pack_blocks_device
 *                     the same on the GPU, for every block of a batch of encoded reads
 *                     (records already in HBM, straight from ntc_encode_batch_device)
 *   ntc_deflate_block the rest of compress_block: gzip each stream (deflate_bytes,
 *                     src/encode.rs:49-57) and prefix its 32-byte BlockHeader
 *                     (src/lib.rs:37-50, src/encode.rs:113-120)
 *   ntc_read_block    decode_block's container half: 4 x (32-byte header, gzip payload),
 *                     decompress_block x4 + zip_block_contents      src/lib.rs:320-363,
 *                     src/decode.rs:79-149 -- returns the u64 records that
 *                     decode_sequence (ntc_decode_batch) consumes.
 * Buffers returned through uint8_t** / uint64_t** are freed with ntc_buffer_free.
 */
#ifndef NTCOMP_CODEC_H
#define NTCOMP_CODEC_H

#include <stdint.h>

#include "ntcomp_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One coded stream of a block, before deflate: 8 * encoded_size payload bytes at
 * `offset`, the u64 code words in the byte order compress_block gives deflate (each word
 * big-endian: the MSB-first bit stream of dsi-bitstream's BE BufBitWriter). */
typedef struct ntc_stream_meta {
    uint64_t num_u64;      /* values in the stream          (BlockHeader.num_u64)      */
    uint64_t encoded_size; /* u64 code words                (BlockHeader.encoded_size) */
    uint64_t param;        /* Rice log2_b, or minimal-binary max = max value + 2
                              (BlockHeader.rice_param)                                 */
    uint64_t offset;       /* byte offset of the payload in the caller's payload buffer */
} ntc_stream_meta;

/* The four streams of one block: [0] colex ranks (minimal binary), [1] match lengths
 * (Rice), [2] flag bytes (Rice), [3] short-record bases in 31-base 2-bit chunks (minimal
 * binary).  status = NTC_ERR_EMPTY_READ when s1 or s4 is empty: the reference's
 * minimal_binary_encode errs and write_block_to writes nothing (src/encode.rs:80,
 * src/lib.rs:242-250; main.rs:170 ignores the error -- SURVEY App. B.3).             */
typedef struct ntc_block_meta {
    ntc_stream_meta stream[4];
    uint64_t num_records; /* BlockHeader.num_records (reads in the block; main.rs:170,176) */
    uint64_t n_recs;      /* u64 records of the block                                   */
    int32_t status;
    uint32_t reserved;
} ntc_block_meta;

#define NTC_DEFLATE_ZLIB 0       /* system zlib, level 6                                  */
#define NTC_DEFLATE_LIBDEFLATE 1 /* libdeflate.so.0, level 6 (~3x faster; other deflate
                                    bytes, same inflated content)                       */
#define NTC_DEFLATE_ADAPTIVE 2   /* libdeflate level 6 where it compresses: a stream whose
                                    first 32 KiB carry >= 7.9 bits of order-0 entropy per
                                    byte (s1's colex ids and s4's bases are such: level 6
                                    shrinks them by < 0.1 %) goes out as stored deflate
                                    blocks, as zlib's own stored-block fallback would write
                                    it; half the CPU of NTC_DEFLATE_LIBDEFLATE, same streams
                                    after inflate, within 0.1 % of its size              */

void ntc_file_header(uint8_t out[32]);
/* NTC_ERR_EMPTY_READ when the block has no long or no short records (see above). */
int ntc_write_block(const uint64_t *recs, uint64_t n_recs, uint64_t num_records, uint8_t **out,
                    uint64_t *out_len);
/* Host packer: *payload (freed with ntc_buffer_free) holds the four streams back to back,
 * meta->stream[s].offset relative to it.  Returns meta->status.                       */
int ntc_pack_block(const uint64_t *recs, uint64_t n_recs, uint64_t num_records, ntc_block_meta *meta,
                   uint8_t **payload, uint64_t *payload_len);
/* Header + gzip member per stream, the bytes write_block_to writes.  payload is the base
 * the meta offsets are relative to.  engine: NTC_DEFLATE_ZLIB, _LIBDEFLATE or _ADAPTIVE
 * (NTC_ERR_UNSUPPORTED if libdeflate.so.0 is missing).  Returns meta->status when the
 * block is dropped (nothing written).                                                  */
int ntc_deflate_block(const ntc_block_meta *meta, const uint8_t *payload, int engine, uint8_t **out,
                      uint64_t *out_len);
/* One stream's part of ntc_deflate_block (its 32-byte header + gzip member): a block's
 * bytes are streams 0..3 concatenated, so a pool can deflate them in parallel.          */
int ntc_deflate_stream(const ntc_block_meta *meta, int stream, const uint8_t *payload, int engine, uint8_t **out,
                       uint64_t *out_len);
/* Parses one block at data[0..len).  NTC_ERR_IO on a clean end of input (no bytes left),
 * NTC_ERR_FORMAT on a damaged block (decode_block's Err, which ends the reference's
 * decode loop, src/main.rs:202).                                                      */
int ntc_read_block(const uint8_t *data, uint64_t len, uint64_t *consumed, uint64_t **recs,
                   uint64_t *n_recs, uint64_t *num_records);
/* The same into a caller buffer of capacity records (NTC_ERR_CAPACITY, with *n_recs the
 * block's count, when it does not fit).  Inflate through libdeflate when present.       */
int ntc_read_block_into(const uint8_t *data, uint64_t len, uint64_t *consumed, uint64_t *recs, uint64_t capacity,
                        uint64_t *n_recs, uint64_t *num_records);
void ntc_buffer_free(void *p);

/* ---- GPU packer ---------------------------------------------------------------------- */
/* Blocks of a batch of encoded reads: block b = reads [b * block_reads,
 * min((b + 1) * block_reads, n_reads)), num_records = its read count (the caller passes
 * block_reads = 65536, main.rs:152; a final partial block carries n_reads % 65536 as
 * main.rs:176 does).  d_recs / d_rec_offsets[n_reads + 1] are device buffers as
 * ntc_encode_batch_device writes them (offsets relative to d_recs).  Writes every
 * block's four payloads into d_payload (device, payload_capacity bytes) and n_blocks
 * metas into the HOST array meta (offsets relative to d_payload; each stream gets room
 * for an exact upper bound of its code, so payloads have small gaps).  *payload_bytes =
 * bytes used (on NTC_ERR_CAPACITY: bytes needed; about 1-2 B per record is typical).
 * Synchronous: the Rice parameters are computed on the host (glibc log/exp as the
 * reference's f64 math) from a first device pass.                                     */
int ntc_pack_blocks_device(ntc_ctx *ctx, const uint64_t *d_recs, const uint64_t *d_rec_offsets,
                           uint64_t n_reads, uint32_t block_reads, uint8_t *d_payload,
                           uint64_t payload_capacity, ntc_block_meta *meta, uint64_t *payload_bytes);
/* Host reads -> packed blocks in one call: ntc_encode_batch's device pass (one pass,
 * however many bases) + ntc_pack_blocks_device, so the u64 records never leave HBM: the
 * CLI's path (src/main.rs:162-177: encode_sequence + encode_dictionary per read, then
 * write_block_to per 65,536 reads, up to deflate).  meta: ceil(n_reads / block_reads)
 * entries.  *payload (host, freed with ntc_buffer_free) holds every block's streams at
 * the meta offsets; hand each block to ntc_deflate_block.                              */
int ntc_encode_pack_batch(ntc_ctx *ctx, const uint8_t *bases, const uint64_t *read_offsets, uint64_t n_reads,
                          uint32_t block_reads, ntc_block_meta *meta, uint8_t **payload, uint64_t *payload_bytes,
                          int64_t *bad_read);

/* ---- GPU unpacker (the inverse of the packer) ------------------------------------------ */
/* decode_block (src/lib.rs:320-368) split at inflate.  ntc_read_block_streams (host): one
 * block's four stream headers at data[0..len) and their gzip members inflated into
 * payload[0..capacity) (stream i at meta->stream[i].offset, 8-byte aligned, exactly
 * encoded_size words each: the big-endian words compress_block wrote); meta->n_recs = the
 * block's records (its flag stream's values), num_records its header field.  Returns what
 * ntc_read_block_into returns for a block it cannot read (NTC_ERR_IO at a clean end,
 * NTC_ERR_FORMAT damaged, NTC_ERR_CAPACITY past capacity).
 * ntc_unpack_streams (GPU): payload[0..payload_bytes) holding n_blocks blocks' streams at
 * their metas' offsets -> the blocks' u64 records in the context's device memory, in
 * block order: rice_decode / minimal_binary_decode / zip_block_contents
 * (src/decode.rs:51-149) on the device.  *n_blocks_ok = the blocks before the first
 * damaged one (a meta with status != 0, or one the device cannot decode: decode_block's
 * Err ends the reference's loop, main.rs:202); *n_reads / *n_bases = what those blocks'
 * records hold.  Synchronous.
 * ntc_unpacked_records: those records to the host (tests).  ntc_decode_fasta_unpacked:
 * ntc_decode_fasta of those records without their trip through host memory (*out_len =
 * the text's bytes; NTC_ERR_CAPACITY past out_capacity, so capacity 0 asks the size).    */
int ntc_read_block_streams(const uint8_t *data, uint64_t len, uint64_t *consumed, uint8_t *payload,
                           uint64_t capacity, ntc_block_meta *meta);
int ntc_unpack_streams(ntc_ctx *ctx, const uint8_t *payload, uint64_t payload_bytes, const ntc_block_meta *metas,
                       uint64_t n_blocks, uint64_t *n_blocks_ok, uint64_t *n_reads, uint64_t *n_bases);
int ntc_unpacked_records(ntc_ctx *ctx, uint64_t *recs, uint64_t capacity, uint64_t *n_recs);
int ntc_decode_fasta_unpacked(ntc_ctx *ctx, uint64_t first_id, uint8_t *out, uint64_t out_capacity,
                              uint64_t *out_len);

/* ---- FASTQ parsed on the GPU ------------------------------------------------------------ */
/* The CLI's ingest (src/main.rs:158-163: needletail records + normalize(true)) for plain
 * FASTQ, done on the device: fastq[0, fastq_bytes) is the text of exactly n_reads records of
 * 4 lines each ('@' header, sequence, '+' line, quality as long as the sequence after one
 * '\r' is stripped from each; the last line may lack its newline) and nothing else -- no
 * blank lines, which the host parser (ntc_fastx_*) skips between records and the caller
 * sends there.  Bases are the sequence lines normalised as ntc_fastx does.  Text under
 * 4 GiB per call.  NTC_ERR_FORMAT (bad_read = the first failing record) if the text is not
 * that.  Synchronous; fastq should be pinned host memory for full PCIe speed.
 *   ntc_fastq_parse        bases + read_offsets[n_reads + 1] back to the host (tests, tools);
 *                          *n_bases = bases parsed (NTC_ERR_CAPACITY past bases_capacity)
 *   ntc_encode_pack_fastq  ntc_encode_pack_batch on the parsed reads, which never leave
 *                          HBM: same metas and payload as parsing on the host and calling
 *                          ntc_encode_pack_batch; *n_bases = bases encoded              */
int ntc_fastq_parse(ntc_ctx *ctx, const uint8_t *fastq, uint64_t fastq_bytes, uint64_t n_reads, uint8_t *bases_out,
                    uint64_t bases_capacity, uint64_t *read_offsets_out, uint64_t *n_bases, int64_t *bad_read);
int ntc_encode_pack_fastq(ntc_ctx *ctx, const uint8_t *fastq, uint64_t fastq_bytes, uint64_t n_reads,
                          uint32_t block_reads, ntc_block_meta *meta, uint8_t **payload, uint64_t *payload_bytes,
                          uint64_t *n_bases, int64_t *bad_read);

#ifdef __cplusplus
}
#endif
#endif
