"""ntcomp command line: `python -m ntcomp_amd build | encode | decode`.

Mirrors the reference CLI (src/cli.rs:27-93, src/main.rs:91-211) with the hot path on
the GPU: FASTX ingest in C++ (needletail parse + normalize(true) restated), encode /
decode through libntcomp_gpu.so, blocks of 65,536 reads (main.rs:152) in the encoded.dat
layout (file header lib.rs:52-67, write_block_to lib.rs:232-252), decode output
">seq.N" (main.rs:203-209).  Block compression runs on a thread pool (ctypes releases the
GIL); blocks are written in order.

Index files: <prefix>.sbwt / <prefix>.lcs in this library's own layout (the sbwt 0.3.11
byte layout is unavailable offline -- DESIGN.md section 8).
"""
import argparse
import concurrent.futures as cf
import os
import sys

import numpy as np

BLOCK_READS = 65536  # main.rs:152


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _read_list(path):
    """--input-list: one path, or tab-separated name and path, per line (main.rs:64-89)."""
    out = []
    with open(path) as f:
        for line in f:
            line = line.rstrip("\n")
            if not line:
                continue
            parts = line.split("\t")
            out.append(parts[1] if len(parts) > 1 else parts[0])
    return out


def cmd_build(args):
    import ntcomp_amd as nt
    files = list(args.seq_files or [])
    if args.input_list:
        files += _read_list(args.input_list)
    if not files:
        raise SystemExit("build: no input files")
    log(f"Building SBWT index from {len(files)} files...")
    seqs = []
    for path in files:
        rd = nt.FastxReader(path)
        for bases, offs in rd:
            for i in range(len(offs) - 1):
                seqs.append(bases[int(offs[i]):int(offs[i + 1])].tobytes())
        rd.close()
    ix = nt.Index.build(seqs, args.kmer_size, add_revcomp=True, threads=args.num_threads)
    log(f"Serializing SBWT index to {args.output_prefix}.sbwt ...")
    log(f"Serializing LCS array to {args.output_prefix}.lcs ...")
    ix.save(args.output_prefix)


def _open_gpus(index, n):
    import ntcomp_amd as nt
    ctxs = []
    for d in range(n):
        c = nt.GpuContext(d)
        c.upload(index)
        ctxs.append(c)
    return ctxs


def cmd_encode(args):
    import ntcomp_amd as nt
    log("Loading SBWT index...")
    index = nt.Index.load(args.index_prefix)
    ctxs = _open_gpus(index, args.gpus)
    out = sys.stdout.buffer
    out.write(nt.file_header())
    log("Encoding fastX data...")
    pool = cf.ThreadPoolExecutor(max_workers=args.threads)
    gpu_pool = cf.ThreadPoolExecutor(max_workers=len(ctxs))
    pending = []  # compressed blocks, in file order

    def flush(wait_all=False):
        while pending and (wait_all or pending[0].done() or len(pending) > 4 * args.threads):
            data = pending.pop(0).result()
            if data is not None:
                out.write(data)

    def compress(recs, nreads):
        try:
            return nt.write_block(recs, nreads)
        except nt.NtcError as e:
            if e.code == 3:  # a stream with no records: write_block_to errs, the
                log("warning: block dropped (no long or no short records; main.rs:170 ignores the error)")
                return None  # reference drops the block
            raise

    carry_recs, carry_counts = [], []  # records of reads not yet in a full block
    rd = nt.FastxReader(args.query_file)
    batch_reads = BLOCK_READS * args.blocks_per_batch
    batches = iter(lambda: rd.batch(max_reads=batch_reads, max_bases=batch_reads * 1024), None)
    # encode batches on the GPUs (one worker per GPU), blocks in order
    jobs = []

    def encode_on(ctx, bases, offs):
        return ctx.encode(bases, offs)

    gi = 0
    for bases, offs in batches:
        jobs.append(gpu_pool.submit(encode_on, ctxs[gi % len(ctxs)], bases, offs))
        gi += 1
        while len(jobs) > len(ctxs) or (jobs and jobs[0].done()):
            _emit(jobs.pop(0).result(), carry_recs, carry_counts, pool, pending, compress)
            flush()
    for j in jobs:
        _emit(j.result(), carry_recs, carry_counts, pool, pending, compress)
        flush()
    if carry_counts:
        counts = np.concatenate(carry_counts)
        recs = np.concatenate(carry_recs) if carry_recs else np.zeros(0, np.uint64)
        pending.append(pool.submit(compress, recs, len(counts)))
    flush(wait_all=True)
    out.flush()
    rd.close()
    for c in ctxs:
        c.close()


def _emit(result, carry_recs, carry_counts, pool, pending, compress):
    recs, roff = result
    counts = np.diff(roff)
    carry_recs.append(recs)
    carry_counts.append(counts)
    total = sum(len(c) for c in carry_counts)
    if total < BLOCK_READS:
        return
    allc = np.concatenate(carry_counts)
    allr = np.concatenate(carry_recs)
    ends = np.concatenate([[0], np.cumsum(allc, dtype=np.uint64)])
    nfull = len(allc) // BLOCK_READS
    for b in range(nfull):
        a0, a1 = int(ends[b * BLOCK_READS]), int(ends[(b + 1) * BLOCK_READS])
        pending.append(pool.submit(compress, allr[a0:a1], BLOCK_READS))
    rest = nfull * BLOCK_READS
    carry_recs.clear()
    carry_counts.clear()
    if rest < len(allc):
        carry_recs.append(allr[int(ends[rest]):])
        carry_counts.append(allc[rest:])


def cmd_decode(args):
    import ntcomp_amd as nt
    index = nt.Index.load(args.index_prefix)
    ctxs = _open_gpus(index, 1)
    ctx = ctxs[0]
    data = np.memmap(args.input_path, dtype=np.uint8, mode="r") if os.path.getsize(args.input_path) else \
        np.zeros(0, dtype=np.uint8)
    out = sys.stdout.buffer
    log("Decoding encoded data...")
    pos = 32  # file header (decode_file_header, main.rs:196-198)
    seq_id = 1
    batch, nbatch = [], 0

    def decode_flush():
        nonlocal seq_id, batch, nbatch
        if not batch:
            return
        recs = np.concatenate(batch)
        bases, offs = ctx.decode(recs)
        out.write(nt.fasta_format(bases, offs, seq_id))
        seq_id += len(offs) - 1
        batch, nbatch = [], 0

    while True:
        try:
            recs, used, _ = nt.read_block(data[pos:])
        except nt.NtcError:
            break  # end of input or a damaged block ends the reference's loop too (main.rs:202)
        pos += used
        batch.append(recs)
        nbatch += 1
        if nbatch >= args.blocks_per_batch:
            decode_flush()
    decode_flush()
    out.flush()
    ctx.close()


def main(argv=None):
    ap = argparse.ArgumentParser(prog="ntcomp", description="Sequencing data compression with SBWT + k-bounded "
                                 "matching statistics; encode/decode hot path on MI355X.")
    sub = ap.add_subparsers(dest="command")
    b = sub.add_parser("build", help="Build the compression dictionary")
    b.add_argument("seq_files", nargs="*", help="Sequence data file(s).")
    b.add_argument("-l", "--input-list", help="File with paths or tab separated name and path on each line.")
    b.add_argument("-o", "--output-prefix", required=True, help="Prefix for output files <prefix>.sbwt and <prefix>.lcs.")
    b.add_argument("-k", dest="kmer_size", type=int, default=31, help="k-mer size.")
    b.add_argument("-p", "--prefix-precalc", type=int, default=8, help="Accepted for compatibility (unused).")
    b.add_argument("-d", "--dedup-batches", action="store_true", help="Accepted for compatibility (unused).")
    b.add_argument("-t", "--threads", dest="num_threads", type=int, default=1)
    b.add_argument("-m", "--mem-gb", type=int, default=4, help="Accepted for compatibility (unused).")
    b.add_argument("--temp-dir", help="Accepted for compatibility (unused; builds in memory).")
    b.add_argument("--verbose", action="store_true")
    e = sub.add_parser("encode", help="Encode fastX data using an SBWT index")
    e.add_argument("query_file", help="Query file with sequence data.")
    e.add_argument("-i", "--index", dest="index_prefix", required=True, help="Prefix for prebuilt <prefix>.sbwt and <prefix>.lcs")
    e.add_argument("--gpus", type=int, default=1, help="GPUs to encode on (batches dealt round-robin).")
    e.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 4), help="block compression threads")
    e.add_argument("--blocks-per-batch", type=int, default=16, help="65,536-read blocks per GPU call")
    d = sub.add_parser("decode", help="Decode data written with Encode")
    d.add_argument("input_path", help="File with encoded fastX data.")
    d.add_argument("-i", "--index", dest="index_prefix", required=True, help="Prefix for prebuilt <prefix>.sbwt and <prefix>.lcs")
    d.add_argument("--blocks-per-batch", type=int, default=16, help="blocks per GPU call")
    args = ap.parse_args(argv)
    if args.command == "build":
        cmd_build(args)
    elif args.command == "encode":
        cmd_encode(args)
    elif args.command == "decode":
        cmd_decode(args)
    else:
        ap.print_help()
    return 0
