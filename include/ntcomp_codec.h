/*
 * ntcomp_codec.h -- host-side block container of encoded.dat (libntcomp_gpu.so).
 *
 *   ntc_file_header   encode_file_header(0,0,0,0)           src/lib.rs:52-67 (32 zero bytes)
 *   ntc_write_block   write_block_to(u64_encoding, num_records, sink)   src/lib.rs:232-252
 *                     (split_encoded_dictionary + compress_block x4, src/encode.rs:96-229)
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

void ntc_file_header(uint8_t out[32]);
/* NTC_ERR_EMPTY_READ when the block has no long or no short records: the reference's
 * minimal_binary_encode errors on an empty stream and write_block_to writes nothing
 * (src/encode.rs:80, src/lib.rs:242-250; main.rs:170 ignores the error -- SURVEY B.3). */
int ntc_write_block(const uint64_t *recs, uint64_t n_recs, uint64_t num_records, uint8_t **out,
                    uint64_t *out_len);
/* Parses one block at data[0..len).  NTC_ERR_IO on a clean end of input (no bytes left),
 * NTC_ERR_FORMAT on a damaged block (decode_block's Err, which ends the reference's
 * decode loop, src/main.rs:202).                                                      */
int ntc_read_block(const uint8_t *data, uint64_t len, uint64_t *consumed, uint64_t **recs,
                   uint64_t *n_recs, uint64_t *num_records);
void ntc_buffer_free(void *p);

#ifdef __cplusplus
}
#endif
#endif
