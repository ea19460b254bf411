"""ntcomp command line: `python -m ntcomp_amd build | encode | decode`.

Mirrors the reference CLI (src/cli.rs:27-93, src/main.rs:91-211) with the hot path on
the GPU: FASTX ingest in C++ (needletail parse + normalize(true) restated), encode /
decode through libntcomp_gpu.so, blocks of 65,536 reads (main.rs:152) in the encoded.dat
layout (file header lib.rs:52-67, write_block_to lib.rs:232-252), decode output
">seq.N" (main.rs:203-209).  Encode runs the native pipeline (ntc_encode_file,
include/ntcomp_pipeline.h): FASTX batches into pinned buffers, GPU encode + block packer
per context, deflate on the host pool, blocks in file order.  Decode: blocks unzip on a
thread pool (ctypes releases the GIL), batches decode on the GPU contexts, FASTA
formatting on the pool, output in file order.

Index files: <prefix>.sbwt / <prefix>.lcs written by default in a recalled restatement of
the sbwt 0.3.11 / kbo 0.5.1 layout the reference always writes (kbo::index::serialize_sbwt,
main.rs:138), with the -p prefix lookup table (unpinned offline -- DESIGN.md section 8);
--index-format own writes this library's own layout.  encode/decode read either.
"""
import argparse
import sys


BLOCK_READS = 65536  # main.rs:152
# contexts per device (--contexts-per-gpu): encode 2 (one call's H2D of FASTQ text overlaps
# the other's kernels), decode 1 -- as the native CLI (ntcomp_main.cpp)
ENCODE_CONTEXTS_PER_GPU, DECODE_CONTEXTS_PER_GPU = 2, 1


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class _Stats:
    """--stats: seconds spent per pipeline stage (summed over threads) and wall clock."""

    def __init__(self, on):
        import threading
        import time
        self.on, self.time, self.lock = on, time.perf_counter, threading.Lock()
        self.t0 = self.time()
        self.acc = {}

    def wrap(self, name, fn):
        if not self.on:
            return fn

        def run(*a, **k):
            t = self.time()
            try:
                return fn(*a, **k)
            finally:
                with self.lock:
                    self.acc[name] = self.acc.get(name, 0.0) + self.time() - t
        return run

    def report(self, **extra):
        if self.on:
            import json
            d = {k: round(v, 3) for k, v in self.acc.items()}
            try:  # interpreter start -> now, imports included
                import psutil
                import time
                extra["process_s"] = round(time.time() - psutil.Process().create_time(), 3)
            except Exception:
                pass
            log(json.dumps({"stats": d, "wall_s": round(self.time() - self.t0, 3), **extra}))


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
    builder = args.builder
    ctx = None
    if builder in ("auto", "gpu"):
        try:
            ctx = nt.GpuContext(args.device)
            builder = "gpu"
        except Exception as e:  # auto without a usable GPU: the host builder
            if builder == "gpu":
                raise SystemExit(f"build: --builder gpu: {e}")
            builder = "host"
    if builder == "gpu":
        # the same index built on the GPU (build.hip; tests/test_gpu_build.py: equal to the host
        # build).  kbo's BuildOpts (main.rs:111-134; cli.rs:55-60: --temp-dir builds "on temporary
        # disk space instead of in-memory", -m is the memory for that): -m given bounds the device
        # memory of a pass (else 85 % of the free HBM); with --temp-dir, sorted partitions past -m GB
        # of host memory go to files there, without it nothing spills.
        mem = int((args.mem_gb if args.mem_gb is not None else 4) * (1 << 30))
        stats = {}
        try:
            ix = nt.Index.build_gpu(ctx, seqs, args.kmer_size, add_revcomp=True,
                                    device_budget=mem if args.mem_gb is not None else 0,
                                    host_budget=mem if args.temp_dir else 0, temp_dir=args.temp_dir, stats=stats)
        finally:
            ctx.close()
        if args.verbose:
            log("build: " + ", ".join(f"{k}={v:.3f}" if isinstance(v, float) else f"{k}={v}"
                                      for k, v in stats.items()))
    else:
        ix = nt.Index.build(seqs, args.kmer_size, add_revcomp=True, threads=args.num_threads)
    if args.index_format == "sbwt-rs" and args.prefix_precalc:
        ix.set_prefix_precalc(min(args.prefix_precalc, args.kmer_size, 12))
    log(f"Serializing SBWT index to {args.output_prefix}.sbwt ...")
    log(f"Serializing LCS array to {args.output_prefix}.lcs ...")
    ix.save(args.output_prefix, layout=args.index_format)


def _open_gpus(index, devices, st=None, per_gpu=1, decode_only=False):
    """per_gpu contexts per entry of devices; an int n means devices
    0..n-1.  The first context of a device uploads the index, the others on that device share
    it (ntc_index_share): calls alternate over the contexts, so one call's copies and host
    work overlap another's kernels.  decode_only: the upload builds only the walk table
    (ctx option decode_only)."""
    import ntcomp_amd as nt
    ctxs, first = [], {}
    for d in (range(devices) if isinstance(devices, int) else devices):
        for _ in range(max(1, per_gpu)):
            c = (st.wrap("gpu_init", nt.GpuContext) if st else nt.GpuContext)(d)
            if d in first:
                c.share_index(first[d])
            else:
                if decode_only:
                    c.set_option("decode_only", 1)
                (st.wrap("index_upload", c.upload) if st else c.upload)(index)
                first[d] = c
                if st and st.on:
                    st.acc["upload_host_derive"] = (st.acc.get("upload_host_derive", 0.0) +
                                                    c.get_option("upload_host_us") / 1e6)
            ctxs.append(c)
    return ctxs


def _devices(args):
    """--devices 0,0,1 (contexts, several may share a GPU) or --gpus N (devices 0..N-1)."""
    if getattr(args, "devices", None):
        return [int(x) for x in args.devices.split(",") if x.strip() != ""]
    return list(range(args.gpus))


def cmd_encode(args):
    """main.rs:141-181 through the native pipeline (ntc_encode_file): plain FASTQ parsed
    on the GPU (--host-parse: on the host pool, as every other input is), GPU encode +
    block packer per context, deflate on the host pool, blocks written in file order."""
    import ntcomp_amd as nt
    st = _Stats(args.stats)
    log("Loading SBWT index...")
    index = st.wrap("index_load", nt.Index.load)(args.index_prefix)
    ctxs = _open_gpus(index, _devices(args), st, args.contexts_per_gpu)
    log("Encoding fastX data...")
    if args.deflate == "auto":
        args.deflate = "adaptive" if nt.libdeflate_available() else "zlib"
    out = sys.stdout.buffer
    out.flush()
    try:
        res = st.wrap("pipeline", nt.encode_file)(ctxs, args.query_file, out.fileno(), threads=args.threads,
                                                  blocks_per_batch=args.blocks_per_batch, deflate=args.deflate,
                                                  host_parse=args.host_parse)
    except nt.NtcError as e:
        bad = getattr(e, "bad_read", -1)
        raise SystemExit(f"ntcomp encode: {e}" + (f" (read {bad + 1})" if bad is not None and bad >= 0 else ""))
    finally:
        for c in ctxs:
            c.close()
    if res["dropped_blocks"]:
        log(f"warning: {res['dropped_blocks']} block(s) dropped (no long or no short records; "
            "main.rs:170 ignores write_block_to's error, SURVEY App. B.3)")
    if st.on:
        for k in ("parse_s", "gpu_s", "deflate_s", "write_s"):
            st.acc[k[:-2]] = res[k]
    st.report(command="encode", gpus=len(ctxs), threads=res["threads"], reads=res["reads"], blocks=res["blocks"],
              dropped_blocks=res["dropped_blocks"], pipeline_wall_s=round(res["wall_s"], 3), deflate=args.deflate,
              gpu_parsed_batches=res["gpu_parsed"])


def cmd_decode(args):
    """main.rs:183-211 through the native pipeline (ntc_decode_file): blocks inflated and
    stream-decoded on the host pool, inverse-SBWT walk + FASTA formatting per context on the
    GPU, ">seq.N" text written in file order."""
    import ntcomp_amd as nt
    st = _Stats(args.stats)
    index = st.wrap("index_load", nt.Index.load)(args.index_prefix)
    ctxs = _open_gpus(index, _devices(args), st, args.contexts_per_gpu, decode_only=True)
    log("Decoding encoded data...")
    out = sys.stdout.buffer
    out.flush()
    try:
        res = st.wrap("pipeline", nt.decode_file)(ctxs, args.input_path, out.fileno(), threads=args.threads,
                                                  blocks_per_batch=args.blocks_per_batch)
    except nt.NtcError as e:
        raise SystemExit(f"ntcomp decode: {e}")
    finally:
        for c in ctxs:
            c.close()
    if res["dropped_blocks"]:
        # the reference's `while let Ok(..) = decode_block` just ends here (main.rs:202)
        log(f"warning: {res['error']}; {res['dropped_blocks']} block(s) not decoded")
    if st.on:
        for k, name in (("parse_s", "unzip"), ("gpu_s", "gpu"), ("write_s", "write")):
            st.acc[name] = res[k]
    st.report(command="decode", gpus=len(ctxs), threads=res["threads"], reads=res["reads"], blocks=res["blocks"],
              pipeline_wall_s=round(res["wall_s"], 3))


def main(argv=None):
    ap = argparse.ArgumentParser(prog="ntcomp", description="Sequencing data compression with SBWT + k-bounded "
                                 "matching statistics; encode/decode hot path on MI355X.")
    ap.add_argument("-V", "--version", action="version", version="ntcomp 0.1.0")  # Cargo.toml:3, clap's `version`
    sub = ap.add_subparsers(dest="command")
    b = sub.add_parser("build", help="Build the compression dictionary")
    b.add_argument("seq_files", nargs="*", help="Sequence data file(s).")
    b.add_argument("-l", "--input-list", help="File with paths or tab separated name and path on each line.")
    b.add_argument("-o", "--output-prefix", required=True, help="Prefix for output files <prefix>.sbwt and <prefix>.lcs.")
    b.add_argument("-k", dest="kmer_size", type=int, default=31, help="k-mer size.")
    b.add_argument("-p", "--prefix-precalc", type=int, default=8,
                   help="Prefix lookup table length (written with --index-format sbwt-rs).")
    b.add_argument("-d", "--dedup-batches", action="store_true",
                   help="Deduplicate k-mers per batch (the GPU build always deduplicates a full pass in place).")
    b.add_argument("-t", "--threads", dest="num_threads", type=int, default=1)
    b.add_argument("-m", "--mem-gb", type=float, default=None,
                   help="Memory budget in GB (default 4 for --temp-dir): device memory per GPU build pass when given "
                        "(else 85%% of the free HBM), and with --temp-dir the host memory for sorted partitions.")
    b.add_argument("--temp-dir", help="Build on temporary disk space at this path: sorted partitions past -m GB of "
                                      "host memory spill there (without it nothing spills).")
    b.add_argument("--verbose", action="store_true")
    b.add_argument("--builder", choices=["auto", "host", "gpu"], default="auto",
                   help="auto (default): the GPU when one is usable, else the host; host: threaded C++ builder "
                        "(in memory); gpu: k-mer sort, dummies, LCS and labels on the GPU in memory-bounded "
                        "passes (same index)")
    b.add_argument("--device", type=int, default=0, help="GPU for --builder gpu")
    b.add_argument("--index-format", choices=["own", "sbwt-rs"], default="sbwt-rs",
                   help="sbwt-rs (default): a restatement of the sbwt 0.3.11/kbo 0.5.1 files the reference writes "
                        "(parity unpinned); own: this library's layout. encode/decode read either")
    e = sub.add_parser("encode", help="Encode fastX data using an SBWT index")
    e.add_argument("query_file", help="Query file with sequence data.")
    e.add_argument("-i", "--index", dest="index_prefix", required=True, help="Prefix for prebuilt <prefix>.sbwt and <prefix>.lcs")
    e.add_argument("--gpus", type=int, default=1, help="GPUs to encode on (batches dealt round-robin).")
    e.add_argument("--devices", help="comma-separated device list, one context each (e.g. 0,0 shares GPU 0); "
                                     "overrides --gpus")
    e.add_argument("--threads", type=int, default=0,
                   help="host pool for FASTQ parse and deflate (0: CPUs available to the process)")
    e.add_argument("--contexts-per-gpu", type=int, default=ENCODE_CONTEXTS_PER_GPU,
                   help="contexts per device sharing one index copy; calls alternate over them")
    e.add_argument("--blocks-per-batch", type=int, default=4, help="65,536-read blocks per GPU call")
    e.add_argument("--deflate", choices=["auto", "zlib", "libdeflate", "adaptive"], default="auto",
                   help="gzip engine for the block streams, level 6 (the reference's Compression::default()): "
                        "adaptive (auto, when libdeflate.so.0 loads: libdeflate, with streams of >= 7.9 bits of "
                        "entropy per byte stored), libdeflate (~3x faster than zlib) or zlib.  The deflate bytes "
                        "differ, the inflated streams do not; no engine reproduces the reference's zlib-rs bytes")
    e.add_argument("--stats", action="store_true", help="print per-stage seconds to stderr")
    e.add_argument("--host-parse", action="store_true",
                   help="parse a plain FASTQ on the host pool instead of the GPU")
    d = sub.add_parser("decode", help="Decode data written with Encode")
    d.add_argument("input_path", help="File with encoded fastX data.")
    d.add_argument("-i", "--index", dest="index_prefix", required=True, help="Prefix for prebuilt <prefix>.sbwt and <prefix>.lcs")
    d.add_argument("--gpus", type=int, default=1, help="GPUs to decode on (batches dealt round-robin).")
    d.add_argument("--devices", help="comma-separated device list, one context each; overrides --gpus")
    d.add_argument("--threads", type=int, default=0, help="block unzip / format threads (0: CPUs available)")
    d.add_argument("--contexts-per-gpu", type=int, default=DECODE_CONTEXTS_PER_GPU,
                   help="contexts per device sharing one index copy; calls alternate over them")
    d.add_argument("--blocks-per-batch", type=int, default=2, help="blocks per GPU call")
    d.add_argument("--stats", action="store_true", help="print per-stage seconds to stderr")
    args = ap.parse_args(argv)
    if getattr(args, "threads", None) == 0:
        import ntcomp_amd as nt
        args.threads = nt.host_threads()
    if args.command == "build":
        cmd_build(args)
    elif args.command == "encode":
        cmd_encode(args)
    elif args.command == "decode":
        cmd_decode(args)
    else:
        ap.print_help()
    return 0
