#!/usr/bin/env python3
"""End-to-end CLI timing: synthetic FASTQ -> `ntcomp encode` ->
encoded.dat -> `ntcomp decode` -> FASTA, wall clock of each CLI process (index prebuilt
and saved first; the input reads come from the same generator as bench.py)."""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=2_000_000)
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--k", type=int, default=91)
    ap.add_argument("--genome-bp", type=int, default=5_000_000)
    ap.add_argument("--dir", default="/tmp/ntc_e2e")
    ap.add_argument("--gzip", action="store_true", help="gzip the FASTQ (one member, --gzip-level)")
    ap.add_argument("--gzip-level", type=int, default=1)
    ap.add_argument("--bgzf", action="store_true", help="with --gzip: BGZF members (bgzip layout) instead of one member")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--devices", help="CLI --devices list (several contexts may share a GPU)")
    ap.add_argument("--contexts-per-gpu", type=int, default=0, help="CLI --contexts-per-gpu (0: the CLI default)")
    ap.add_argument("--deflate", default="zlib", choices=["zlib", "libdeflate", "adaptive", "auto"])
    ap.add_argument("--keep", action="store_true", help="reuse an existing FASTQ + index in --dir")
    ap.add_argument("--reps", type=int, default=3, help="runs per timing (the best counts)")
    ap.add_argument("--cli", default="native", choices=["native", "python"],
                    help="native: the ntcomp binary (ntcomp_main.cpp); python: python -m ntcomp_amd")
    ap.add_argument("--host-parse", action="store_true", help="CLI --host-parse (FASTQ parsed on the host pool)")
    a = ap.parse_args()
    a.gpus_arg = ["--devices", a.devices] if a.devices else ["--gpus", str(a.gpus)]
    if a.contexts_per_gpu:
        a.gpus_arg += ["--contexts-per-gpu", str(a.contexts_per_gpu)]
    a.enc_arg = ["--host-parse"] if a.host_parse else []
    import numpy as np
    import ntcomp_amd as nt
    os.makedirs(a.dir, exist_ok=True)
    genome = nt.synth_genome(1, a.genome_bp)
    prefix = os.path.join(a.dir, "idx")
    if not (a.keep and os.path.exists(prefix + ".sbwt")):
        ix = nt.Index.build([genome.tobytes()], a.k, threads=16)
        ix.save(prefix)
    L, n = a.read_len, a.reads
    reads = nt.synth_reads(genome, 2, 0, n, L, 10_000, threads=16)
    fq = os.path.join(a.dir, "reads.fq" + (".gz" if a.gzip else ""))
    # FASTQ: @r<i> / read / + / constant quality (vectorised)
    t0 = time.time()
    body = reads.reshape(n, L)
    qual = np.full((n, L), ord("I"), dtype=np.uint8)
    nl = np.full((n, 1), 10, dtype=np.uint8)
    plus = np.frombuffer(b"+\n", dtype=np.uint8)[None, :].repeat(n, 0)
    head = np.frombuffer(b"@r\n", dtype=np.uint8)[None, :].repeat(n, 0)
    rec = np.concatenate([head, body, nl, plus, qual, nl], axis=1).tobytes()
    if a.keep and os.path.exists(fq):
        pass
    elif a.gzip and a.bgzf:
        import struct
        import zlib

        def member(chunk):
            c = zlib.compressobj(1, zlib.DEFLATED, -15)
            body = c.compress(chunk) + c.flush()
            bsize = 18 + len(body) + 8
            return (b"\x1f\x8b\x08\x04" + b"\0" * 4 + b"\x00\xff" + struct.pack("<H", 6) + b"BC" +
                    struct.pack("<HH", 2, bsize - 1) + body + struct.pack("<II", zlib.crc32(chunk), len(chunk)))
        with open(fq, "wb") as f:
            for i in range(0, len(rec), 65280):
                f.write(member(rec[i:i + 65280]))
    elif a.gzip:
        import gzip
        with gzip.open(fq, "wb", compresslevel=a.gzip_level) as f:
            f.write(rec)
    else:
        with open(fq, "wb") as f:
            f.write(rec)
    print(f"fastq {len(rec) / 1e9:.2f} GB written in {time.time() - t0:.1f}s", file=sys.stderr)
    enc, dec = os.path.join(a.dir, "enc.dat"), os.path.join(a.dir, "dec.fa")
    cmd = [os.path.join(REPO, "ntcomp_amd", "ntcomp")] if a.cli == "native" else [sys.executable, "-m", "ntcomp_amd"]

    def stats_line(err):
        for line in reversed(err.decode(errors="replace").splitlines()):
            if line.startswith("{"):
                return json.loads(line)
        return None

    def fresh(dst):
        # the CLI writes a new file: truncating the previous rep's output (1.6 GB of page
        # cache for a decode) is Python's cost, not the CLI's, so it stays outside the clock
        if os.path.exists(dst):
            os.unlink(dst)

    def run_encode(src, dst):
        fresh(dst)
        t0 = time.time()
        with open(dst, "wb") as f:
            r = subprocess.run(cmd + ["encode", "-i", prefix, src, "--stats", "--deflate", a.deflate] + a.gpus_arg + a.enc_arg,
                               stdout=f, stderr=subprocess.PIPE, check=True, cwd=REPO)
        return time.time() - t0, stats_line(r.stderr)

    def run_decode(src, dst):
        fresh(dst)
        t0 = time.time()
        with open(dst, "wb") as f:
            r = subprocess.run(cmd + ["decode", "-i", prefix, src, "--stats"] + a.gpus_arg, stdout=f,
                               stderr=subprocess.PIPE, check=True, cwd=REPO)
        return time.time() - t0, stats_line(r.stderr)

    # fixed cost of one CLI process (interpreter, index load, GPU init + upload, pipeline
    # buffers): encode an empty FASTQ and decode its (header-only) output.  Every timing is
    # the best of --reps runs (process start-up varies by ~0.1 s on a fresh box).
    empty = os.path.join(a.dir, "empty.fq")
    open(empty, "wb").close()
    t_fixed_enc = min(run_encode(empty, os.path.join(a.dir, "empty.dat"))[0] for _ in range(a.reps))
    t_fixed_dec = min(run_decode(os.path.join(a.dir, "empty.dat"), os.path.join(a.dir, "empty.fa"))[0]
                      for _ in range(a.reps))
    runs = [run_encode(fq, enc) for _ in range(a.reps)]
    te, enc_stats = min(runs, key=lambda x: x[0])
    runs = [run_decode(enc, dec) for _ in range(a.reps)]
    td, dec_stats = min(runs, key=lambda x: x[0])
    ok = open(dec, "rb").read().split(b"\n")[1::2]
    same = b"".join(ok) == reads.tobytes()
    bases = n * L
    print(json.dumps({"metric": "end-to-end CLI Mbases/s (process wall clock, incl. index load + upload)",
                      "reads": n, "read_len": L, "k": a.k, "fastq_bytes": len(rec), "gzip": ("bgzf" if a.bgzf else f"one member, level {a.gzip_level}") if a.gzip else False,
                      "input_bytes": os.path.getsize(fq),
                      "encode_s": round(te, 3), "encode_mbases_s": round(bases / te / 1e6, 1),
                      "encoded_bytes": os.path.getsize(enc), "bits_per_base": round(8 * os.path.getsize(enc) / bases, 4),
                      "decode_s": round(td, 3), "decode_mbases_s": round(bases / td / 1e6, 1),
                      "gpus": a.gpus, "devices": a.devices, "contexts_per_gpu": a.contexts_per_gpu, "cli": a.cli,
                      "reps": a.reps,
                      "pipeline_mbases_s": {s: round(bases / st["pipeline_wall_s"] / 1e6, 1)
                                            if st and st.get("pipeline_wall_s") else None
                                            for s, st in (("encode", enc_stats), ("decode", dec_stats))},
                      "fixed_s": {"encode": round(t_fixed_enc, 3), "decode": round(t_fixed_dec, 3)},
                      "streaming_mbases_s": {"encode": round(bases / max(te - t_fixed_enc, 1e-9) / 1e6, 1),
                                             "decode": round(bases / max(td - t_fixed_dec, 1e-9) / 1e6, 1)},
                      "round_trip_exact": same, "deflate": a.deflate,
                      "host": {"cpu": _cpu_model(), "threads": nt.host_threads()},
                      "encode_stages": enc_stats, "decode_stages": dec_stats}))


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


if __name__ == "__main__":
    main()
