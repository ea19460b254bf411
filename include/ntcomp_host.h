/*
 * ntcomp_host.h -- host-side C ABI of libntcomp_gpu.so: the index producer and file
 * I/O around the GPU hot path, plus the seeded synthetic workload generator used by
 * bench.py and the tests.
 *
 *   ntc_build_index   replaces kbo::build(&[Vec<u8>], BuildOpts{add_revcomp: true, ..})
 *                     (src/main.rs:111-134; tests/fasta_data.rs:56-63): a deterministic
 *                     SBWT subset-matrix + LCS construction.
 *   ntc_index_save /  replace kbo::index::serialize_sbwt (src/main.rs:138) and
 *   ntc_index_load    kbo::index::load_sbwt (src/main.rs:149, :190): <prefix>.sbwt +
 *                     <prefix>.lcs.  NOTE: this round writes this library's own layout
 *                     (DESIGN.md "Index files"); the sbwt 0.3.11 byte layout is not
 *                     available offline and is unpinned.
 */
#ifndef NTCOMP_HOST_H
#define NTCOMP_HOST_H

#include <stdint.h>

#include "ntcomp_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ntc_index_host ntc_index_host;

/* seqs: sequences back to back, seq_offsets[n_seqs+1].  Bytes other than ACGTacgt split
 * a sequence (k-mers containing them are skipped, as in kbo/sbwt).  k in [1,255].
 * n_threads <= 0 picks the hardware concurrency.                                     */
int ntc_build_index(const uint8_t *seqs, const uint64_t *seq_offsets, uint64_t n_seqs,
                    uint32_t k, int add_revcomp, int n_threads, ntc_index_host **out);
/* The same index built on ctx's GPU (build.hip; also kbo::build's stand-in, main.rs:111-134):
 * k-mers, radix sort, dummies, LCS and labels in HBM, then rows + LCS to the host.  Equal
 * to ntc_build_index's output for every input.  Synchronous on ctx's stream; no index
 * needs to be uploaded.  = ntc_build_index_device_ex with default options.            */
int ntc_build_index_device(ntc_ctx *ctx, const uint8_t *seqs, const uint64_t *seq_offsets, uint64_t n_seqs,
                           uint32_t k, int add_revcomp, ntc_index_host **out);
/* Memory bounds of the GPU build: kbo's BuildOpts { mem_gb, temp_dir } (src/cli.rs:56-61,
 * src/main.rs:111-134).  The k-mers are processed in contiguous colex ranges (their last
 * 7 characters) small enough that every pass fits device_budget_bytes; sorted ranges wait in
 * host memory up to host_budget_bytes, past it in unlinked files under temp_dir.  Any input
 * size works (passes never sort 2^32 keys); the index itself must have < 2^32 nodes.   */
typedef struct ntc_build_opts {
    uint64_t device_budget_bytes;  /* 0: 85 % of the device's free memory                          */
    uint64_t host_budget_bytes;    /* 0: no limit (nothing spills)                                  */
    const char *temp_dir;          /* NULL: $TMPDIR, else /tmp                                     */
    uint64_t max_partition_keys;   /* test hook: k-mer occurrences per pass (0: from the budget)    */
} ntc_build_opts;
typedef struct ntc_build_stats {
    uint64_t occurrences;          /* k-mer windows (x2 with reverse complements)                   */
    uint64_t kmers;                /* distinct k-mers                                               */
    uint64_t sources;              /* k-mers without an in-neighbour (each brings k-1 dummies)      */
    uint64_t nodes;                /* index nodes                                                   */
    uint64_t spilled_bytes;        /* partition bytes written under temp_dir                        */
    uint64_t device_budget_bytes;  /* the budget used                                               */
    uint64_t pass_keys;            /* keys per pass                                                 */
    uint64_t peak_device_bytes;    /* the build's largest device allocation total                   */
    uint32_t kmer_partitions, node_partitions, compactions, seq_uploads;
    double seconds, seconds_kmers, seconds_sources, seconds_nodes, seconds_labels;
    double seconds_plan;           /* of seconds_kmers: sequence upload + occurrence histogram      */
    double seconds_sort;           /* every radix sort of the build                                 */
} ntc_build_stats;
int ntc_build_index_device_ex(ntc_ctx *ctx, const uint8_t *seqs, const uint64_t *seq_offsets, uint64_t n_seqs,
                              uint32_t k, int add_revcomp, const ntc_build_opts *opts, ntc_build_stats *stats,
                              ntc_index_host **out);
/* -p/--prefix-precalc (src/cli.rs:46): the colex interval of every p-mer (4^p ranges, first
 * character most significant, [0, 0) when absent), kept with the index and written by the
 * NTC_INDEX_SBWT_RS layout as sbwt's PrefixLookupTable [ext, recalled].  p in [0, min(k, 12)];
 * 0 drops the table.                                                                 */
int ntc_index_set_prefix_precalc(ntc_index_host *ix, uint32_t p);
/* the table's p and range count; ranges (2 x 4^p words: start, end) may be NULL          */
int ntc_index_prefix_table(const ntc_index_host *ix, uint32_t *p, uint64_t *ranges);
void ntc_index_free(ntc_index_host *ix);
/* Borrowed view (valid until ntc_index_free) for ntc_index_upload or inspection. */
int ntc_index_view_of(const ntc_index_host *ix, ntc_index_view *view);
int ntc_index_save(const ntc_index_host *ix, const char *prefix);
int ntc_index_load(const char *prefix, ntc_index_host **out);  /* detects the layout */
/* Save in a chosen layout: NTC_INDEX_OWN (= ntc_index_save) or NTC_INDEX_SBWT_RS, a
 * restatement of sbwt 0.3.11 / kbo 0.5.1 serialisation (write_sbwt_index_variant +
 * LcsArray, main.rs:138) [ext, recalled -- parity unpinned: no reference-written index
 * exists offline]. */
#define NTC_INDEX_OWN 0
#define NTC_INDEX_SBWT_RS 1
int ntc_index_save_as(const ntc_index_host *ix, const char *prefix, int layout);

/* ---- FASTX ingest (CLI) -------------------------------------------------------------- */
/* needletail::parse_fastx_file + SequenceRecord::normalize(true) as src/main.rs:51-62 and
 * :158-163 use them: plain, gzip (BGZF too), bzip2, xz or zstd FASTA/FASTQ
 * (detected from the magic bytes), sequences normalized (ACGTN- kept, lower
 * case upper-cased, U -> T, IUPAC kept, whitespace dropped, anything else -> N), names
 * dropped.  Batches hold up to max_reads reads / about max_bases bases; the buffers are
 * owned by the reader and valid until the next call.  n_reads = 0 at end of input.    */
typedef struct ntc_fastx ntc_fastx;
int ntc_fastx_open(const char *path, ntc_fastx **out);
int ntc_fastx_next_batch(ntc_fastx *fx, uint64_t max_reads, uint64_t max_bases, const uint8_t **bases,
                         const uint64_t **offsets, uint64_t *n_reads);
void ntc_fastx_close(ntc_fastx *fx);
/* The same batch written into caller buffers (e.g. pinned host memory for the H2D copy):
 * bases_capacity bytes, offsets[max_reads + 1].  NTC_ERR_CAPACITY if the bases do not fit. */
int ntc_fastx_next_batch_into(ntc_fastx *fx, uint64_t max_reads, uint64_t max_bases, uint8_t *bases,
                              uint64_t bases_capacity, uint64_t *offsets, uint64_t *n_reads);
/* Plain FASTQ files are memory-mapped and each batch is parsed by this many threads
 * (default ntc_host_threads()); other inputs decode on one producer thread.          */
int ntc_fastx_set_threads(ntc_fastx *fx, int n_threads);
/* CPUs this process may use: NTC_THREADS if set, else min(affinity mask, cgroup v2 CPU
 * quota) -- the thread count of every host pool (FASTX parse, block deflate).         */
int ntc_host_threads(void);
/* decode output (src/main.rs:203-209): ">seq.{first_id + r}\n{read r}\n" for each read;
 * *out is freed with ntc_buffer_free (include/ntcomp_codec.h).                         */
int ntc_fasta_format(const uint8_t *bases, const uint64_t *offsets, uint64_t n_reads, uint64_t first_id,
                     uint8_t **out, uint64_t *out_len);

/* ---- synthetic workload ------------------------------------------- */
/* i.i.d. uniform ACGT genome from SplitMix64(seed). */
int ntc_synth_genome(uint64_t seed, uint64_t length, uint8_t *out);
/* n_strains strains of a collection, each = genome with i.i.d. substitutions at rate
 * snp_per_million / 1e6 (position i of strain s depends only on (seed, s, i)).
 * out = n_strains * glen bytes.  Used for the multi-strain index of bench.py.        */
int ntc_synth_strains(const uint8_t *genome, uint64_t glen, uint64_t seed, uint32_t n_strains,
                      uint32_t snp_per_million, uint8_t *out);
/* Minimizer key of each of n_reads reads of read_len bases (smallest 64-bit hash of its
 * 2-bit w-mers, w <= 32), for read-ordering experiments (bench.py --presort).          */
int ntc_minimizer_keys(const uint8_t *reads, uint64_t n_reads, uint32_t read_len, uint32_t w,
                       int n_threads, uint64_t *keys);
/* n_reads reads of read_len bases from genome; read r depends only on (seed, r): start
 * uniform on [0, glen-read_len], reverse-complemented with probability 1/2, i.i.d.
 * substitutions with probability err_per_million / 1e6.  out = n_reads*read_len bytes.
 * Reads first_read .. first_read+n_reads-1 (so shards regenerate identical data).    */
int ntc_synth_reads(const uint8_t *genome, uint64_t glen, uint64_t seed, uint64_t first_read,
                    uint64_t n_reads, uint32_t read_len, uint32_t err_per_million,
                    int n_threads, uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif
