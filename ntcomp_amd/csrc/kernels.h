// Kernel argument structs and launchers (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "encode_core.h"

namespace ntc {

struct HostIndex;
// GPU index build (build.hip): the host builder's index (sbwt_build.cpp), built on stream s
// in bucket-range partitions whose passes fit device_budget (0: 85 % of the free HBM);
// sorted partitions wait in host memory up to host_budget (0: no limit), past it in files
// under temp_dir.  max_partition_keys caps a pass (test hook, 0: from the budget).
struct BuildOpts {
    uint64_t device_budget = 0, host_budget = 0, max_partition_keys = 0;
    std::string temp_dir;
};
struct BuildStats {
    uint64_t occurrences = 0, kmers = 0, sources = 0, nodes = 0;
    uint64_t spilled_bytes = 0, device_budget = 0, pass_keys = 0, peak_device_bytes = 0;
    uint32_t kmer_partitions = 0, node_partitions = 0, compactions = 0, seq_uploads = 0;
    double seconds = 0, seconds_kmers = 0, seconds_sources = 0, seconds_nodes = 0, seconds_labels = 0;
    double seconds_plan = 0, seconds_sort = 0;  // the occurrence histogram (sequence upload included); sorts
};
bool build_index_device(hipStream_t s, const uint8_t *seqs, const uint64_t *offs, uint64_t n_seqs, uint32_t k,
                        bool revcomp, const BuildOpts &o, HostIndex &out, BuildStats &st, std::string &err);

struct EncodeArgs {
    DevIndex ix;
    const uint8_t *bases;
    const uint64_t *offs;        // [n_reads+1], absolute into bases
    uint64_t n_reads;
    const uint64_t *tile_base;   // [tiles+1] scratch rows per tile, or null => uniform
    uint64_t rows_uniform;       // multiple of 32
    uint8_t *D;
    uint32_t *S;
    uint32_t *F;
    uint64_t *R;
    uint32_t *rec_count;
    unsigned long long *status;  // min over (read << 8 | code); ~0 = ok
};

struct Enc4Args {
    DevIndex ix;
    const uint8_t *bases;
    const uint64_t *offs;        // [n_reads+1], absolute into bases
    uint64_t n_reads;
    uint64_t *Q;                 // packed bases, position space (2 bits, 32 per word)
    Entry *Es;                   // the next S entries of each read (secondary slots, ent_ptr)
    uint32_t S;                  // secondary slots per read (multiple of 4)
    Entry *Ep;                   // overflow pool of entries (reservations, MsLaneT::reserve)
    uint64_t pcap;               // its entries (< 2^32)
    uint32_t *obase;             // each overflowing read's entry reservation
    Entry *Ed;                   // first kEntSlot entries of each read (dense slots, ent_ptr)
    uint32_t *ne;                // entries per read
    uint64_t *R;                 // records past kRecSlot: reservations (parse_read's RecPool)
    uint64_t rcap;               // its records (< 2^32)
    uint32_t *rbase;             // each overflowing read's record reservation
    uint64_t *R2;                // first kRecSlot records of each read (dense slots)
    uint32_t *rec_count;
    uint32_t *wave_cnt;          // records of each wave's 64 reads (k_parse4 -> scan -> k_emit4)
    unsigned long long *status;
    unsigned long long *counter; // work queue heads of k_ms4 (WaveQueue, zeroed per call), then
                                 // the entry and record pool counters (kPoolCounters)
};
// the pools' reservation counters: words 64 and 72 of the counter area (past the 8 queue
// heads, 64 B apart), zeroed with them per call
constexpr uint32_t kPoolCntE = 64, kPoolCntR = 72;

struct EmitArgs {
    const uint64_t *R;           // [tile][j][lane]
    const uint64_t *tile_base;
    uint64_t rows_uniform;
    const uint32_t *rec_count;
    const uint64_t *rec_offsets;
    uint64_t n_reads;
    uint64_t *out;
    uint64_t capacity;
    unsigned long long *status;
};

struct DebugArgs {
    const uint8_t *D;
    const uint32_t *S;
    const uint64_t *tile_base;
    uint64_t rows_uniform;
    const uint64_t *offs;
    uint64_t n_reads;
    uint32_t *d_out;
    uint32_t *s_out;
};

// decode tiles: k_dec_rec's block of 256 threads owns kDecTileRecs consecutive records, kDecR
// per thread (independent walk chains per lane).  4: 126 VGPRs, 4 waves/SIMD = 16 chains per
// SIMD (2: 84 VGPRs, 5 waves = 10 chains); D91 k_dec_rec 0.935 -> 0.900 ms, SD91 1.117 ->
// 1.103 ms (A/B on one box, round 3)
#ifndef NTC_DEC_R
#define NTC_DEC_R 4
#endif
constexpr uint32_t kDecR = NTC_DEC_R;
constexpr uint32_t kDecTileRecs = 256 * kDecR;

struct DecWalkArgs {
    DevIndex ix;
    const uint64_t *recs;
    uint64_t n;
    const uint64_t *pfs;         // per kDecTileRecs-record tile: first records before it [tiles + 1]
    const uint64_t *pls;         // per tile: bases before it [tiles + 1]
    uint64_t *offs_out;          // each read's output offset [nreads + 1] (written here)
    uint64_t offs_capacity;
    uint64_t bases_capacity;
    uint8_t *out;
    unsigned long long *status;
};

// GPU block packer (pack.hip): per 65,536-read block, stream totals, then the four coded
// streams of write_block_to (src/lib.rs:232-252) before deflate
struct PackStats {
    uint64_t n_recs, n_long, max1, sum2, sum3, T, max4, bad, rec_begin;
};
struct PackParams {
    uint64_t off[4];      // word offsets of s1..s4 in the payload
    uint64_t lim1, lim4;  // minimal-binary limits 2^(l+1) - max
    int32_t p2, p3, l1, l4;
    uint32_t skip, pad;   // skip: the block is dropped (App. B.3) or malformed
    uint32_t seg0, nseg;  // the block's pass-2 segments [seg0, seg0 + nseg): records first, then s4 chunks
};
// a workgroup's share of pass 2: kind 0 = records [first, first + count) (absolute indices,
// streams s1-s3), kind 1 = s4 chunks [first, first + count) of the block
struct PackSeg {
    uint32_t block, kind;
    uint64_t first, count;
};
constexpr uint64_t kPackSegRecs = 16384, kPackSegChunks = 16384;
// pass 1 (stream totals + s4 chunks) in segments of 4096 reads: chunks (chunk_words words,
// zeroed here) as pack.hip chunk_base lays them out, scratch: pack_stats_scratch_words()
uint64_t pack_stats_scratch_words(uint64_t n_blocks, uint32_t block_reads);
void launch_pack_stats(const uint64_t *recs, const uint64_t *roffs, uint64_t n_reads, uint32_t block_reads,
                       uint64_t n_blocks, uint64_t *chunks, uint64_t chunk_words, uint64_t *scratch,
                       PackStats *stats, hipStream_t s);
// pass 2 over n_segs segments: their code lengths, each block's segment offsets (seg_bits /
// seg_start: 3 words per segment), then every segment's codes in parallel
void launch_pack_write(const uint64_t *recs, const uint64_t *chunks, const PackStats *stats,
                       const PackParams *params, uint64_t n_blocks, const PackSeg *segs, uint64_t n_segs,
                       uint64_t *seg_bits, uint64_t *seg_start, uint64_t *payload, uint64_t *bits_out,
                       hipStream_t s);

// decode output as FASTA text on the GPU (fasta.hip): ">seq.{first_id + r}\n{read r}\n";
// sizes / out_offs: n + 1 words, tmp: scan_tmp_words(n) words; out_offs[n] = total bytes.
// Nothing is written unless the decode status is clear (~0) and the text fits out_cap.
// GPU block unpacker (unpack.hip): stream i of block b is entry 4 b + i (s1 colex, s2 length,
// s3 flag, s4 short-base chunks), its inflated big-endian words at payload[word_off ...]
struct UnpackStream {
    uint64_t word_off;  // u64 words into the payload (and into the marks scratch)
    uint64_t nwords;    // encoded_size
    uint64_t n;         // num_u64 values
    uint64_t param;     // Rice parameter / minimal-binary max
    uint64_t val_off;   // its values at vals[val_off ...]
};
// The streams run in tiles (a workgroup each): tile k of a list is tile `tile` of stream si,
// which is entry `stream` of the list's streams; a stream's tiles are contiguous, from
// first_tile.  unpack_plan lists the minimal-binary (s1, s4) and Rice (s2, s3) tiles from the
// host copy of the stream table.
struct UnpTile {
    uint32_t si, tile, stream, pad;
};
struct UnpStreamRef {
    uint32_t si, first_tile, n_tiles, pad;
};
struct UnpackPlan {
    std::vector<UnpTile> mb_tiles, rice_tiles;
    std::vector<UnpStreamRef> mb_streams, rice_streams;
};
void unpack_plan(const UnpackStream *st, uint64_t n_blocks, UnpackPlan &plan);
uint64_t unpack_ws_bytes(const UnpackPlan &plan);  // the tiles' tables (ws)
// streams -> values (status[4 b + i]), zip -> records of block b at recs[rec_off[b] ...];
// out3[3 b .. 3 b + 2] = reads, bases, status.  marks: as many words as the payload; segc:
// unpack_seg_words(n_blocks, the largest block's records) words
struct UnpackDev {
    const uint64_t *payload;
    const UnpackStream *st;
    uint64_t n_blocks, max_recs;
    uint64_t *marks;
    const UnpTile *mb_tiles, *rice_tiles;  // the plan's lists, on the device
    const UnpStreamRef *mb_streams, *rice_streams;
    uint32_t n_mb_tiles, n_rice_tiles, n_mb_streams, n_rice_streams;
    void *ws;
    uint64_t *vals;
    int32_t *status;
    const uint64_t *rec_off;
    uint64_t *recs, *segc, *out3;
};
void launch_unpack(const UnpackDev &d, hipStream_t s);
uint64_t unpack_seg_words(uint64_t n_blocks, uint64_t max_recs);
void launch_fasta(const uint8_t *d_bases, const uint64_t *d_offs, uint64_t n, uint64_t first_id,
                  const unsigned long long *d_status, uint64_t *sizes, uint64_t *out_offs, uint64_t *tmp, uint8_t *out,
                  uint64_t out_cap, hipStream_t s);

// plain FASTQ text of n_reads whole 4-line records -> normalised bases + read offsets
// (fastq.hip).  tile_cnt: fastq_tiles(n_raw) words, tile_base: tiles + 1 (its last word =
// the newlines found), nl: 4 n_reads, kept: n_reads, offs: n_reads + 1, tmp:
// scan_tmp_words(max(tiles, n_reads) + 1), bases: room for the sequence lines' bytes.
// status (preset to ~0) gets read << 8 | NTC_ERR_FORMAT for the first malformed record;
// then no base is written.
struct FastqArgs {
    const uint8_t *raw;
    uint64_t n_raw, n_reads;
    uint32_t *tile_cnt;
    uint64_t *tile_base;
    uint32_t *nl;
    uint32_t *kept;
    uint64_t *offs;
    uint64_t *tmp;
    uint8_t *bases;
    unsigned long long *status;
};
uint64_t fastq_tiles(uint64_t n_raw);
void launch_fastq_parse(const FastqArgs &a, hipStream_t s);

void launch_encode(const EncodeArgs &a, hipStream_t s);
void launch_encode4(const Enc4Args &a, uint64_t total, uint32_t ms_blocks, hipStream_t s,
                    hipEvent_t ev_ms_begin, hipEvent_t ev_ms_end);
// record offsets (rec_offsets[0..n], written here) from the per-wave counts, then records
void launch_emit4(const Enc4Args &a, uint64_t *wave_off, uint64_t *tmp, uint64_t *rec_offsets, uint64_t *out,
                  uint64_t capacity, hipStream_t s);
int ms4_blocks_per_cu();
void launch_debug_gather4(const Enc4Args &a, uint32_t *d_out, uint32_t *s_out, hipStream_t s);
void launch_pair_words(const uint2 *top, uint32_t U, uint16_t *out, hipStream_t s);
void launch_win_words(const uint32_t *bits, uint32_t U, uint32_t *out, hipStream_t s);
void launch_tab_build(const DevIndex &ix, uint32_t U, uint2 *tab, uint32_t *bits, uint32_t F, uint32_t *fbits,
                      hipStream_t s);
void launch_tile_rows(const uint64_t *offs, uint64_t n_reads, uint32_t *tile_rows, hipStream_t s);
void launch_emit(const EmitArgs &a, hipStream_t s);
void launch_debug_gather(const DebugArgs &a, hipStream_t s);
// decode: per 256-record tile sums (firsts, bases) and their exclusive scans (pfs, pls:
// tiles + 1 words each; pf, pl: tiles words each; tmp: scan_tmp_words(tiles)), then the
// walk kernel, which derives every record's read and output offset itself
void launch_dec_tiles(const uint64_t *recs, uint64_t n, uint64_t *pf, uint64_t *pl, uint64_t *pfs, uint64_t *pls,
                      uint64_t *tmp, hipStream_t s);
void launch_dec_walk(const DecWalkArgs &a, hipStream_t s);
void launch_rank2(const DevIndex &ix, Rank2Chunk *out, hipStream_t s);
void launch_status_box(const unsigned long long *status, const uint64_t *a, const uint64_t *b, const uint64_t *c,
                       uint64_t *box, hipStream_t s);
void launch_walk_build(const uint32_t *pred, const uint8_t *code, uint64_t n, WalkStep *a, WalkStep *b,
                       WalkEntry *out, hipStream_t s);
uint64_t scan_tmp_words(uint64_t n);

// Path cover on the device (derived.cpp build_paths, same cover): unitigs of the real
// k-mers, laid out by start node.  Orchestrated by ntc_index_upload.
struct PathArgs {
    const uint2 *rank;       // rank words [4][rwords]
    uint32_t rwords;
    uint32_t n, k;
    const uint8_t *lcs;
    const uint32_t *dummy;   // bit z: node z is a dummy
    const uint32_t *pred;    // inverse-walk predecessor
    const uint8_t *code;     // last character of each node
    const uint32_t *uniq;    // bit z: z's (k-1)-suffix group is {z}
};
// prv[y] = the path predecessor of y, or 0xFFFFFFFF (prv must be preset to all ones)
void launch_path_edges(const PathArgs &a, uint32_t *prv, hipStream_t s);
// list ranking by pointer jumping: st[z] = {start node, distance, min node on the way, 0};
// returns the buffer (a or b) holding the result
uint4 *launch_path_rank(const uint32_t *prv, uint32_t n, uint4 *a, uint4 *b, hipStream_t s);
// unitig linking (derived.cpp link_unitigs): st = the ranking of the unitig edges in prv,
// len[start] = unitig lengths (launch_path_lengths), want preset to all ones, best_pred to
// all ones (64-bit); adds the chosen t -> y edges to prv
void launch_path_link(const PathArgs &a, const uint4 *st, const uint32_t *len, uint32_t *want,
                      unsigned long long *best_pred, uint32_t *prv, hipStream_t s);
// fork blocks after each path end (k >= kForkBlockMinK), after launch_path_place
void launch_path_forks(const PathArgs &a, const uint4 *st, const uint32_t *len, const uint64_t *base,
                       const uint32_t *pos_of_node, const uint4 *pstream, uint32_t *colex_at, hipStream_t s);
// cut every cycle at its smallest node (prv[min] = none); *flag = 1 if any was cut
void launch_path_cut(const PathArgs &a, const uint4 *st, uint32_t *prv, uint32_t *flag, hipStream_t s);
// len[start] = path length (len zeroed first); vals[z] = len + k at starts, else 0;
// *n_paths += number of starts
void launch_path_lengths(const PathArgs &a, const uint4 *st, const uint32_t *prv, uint32_t *len, uint32_t *vals,
                         uint32_t *n_paths, hipStream_t s);
// text, node-end bits, colex_at, pos_of_node, puniq (outputs preset: zeros / all ones)
void launch_path_place(const PathArgs &a, const uint4 *st, const uint32_t *prv, const uint64_t *base,
                       uint32_t *colex_at, uint32_t *pos_of_node, uint4 *pstream, uint64_t *puniq, hipStream_t s);
void scan_excl_u32(const uint32_t *in, uint64_t n, uint64_t *out, uint64_t *tmp, hipStream_t s);
void scan_excl_u64(const uint64_t *in, uint64_t n, uint64_t *out, uint64_t *tmp, hipStream_t s);

}  // namespace ntc
