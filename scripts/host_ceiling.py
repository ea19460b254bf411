#!/usr/bin/env python3
"""Host ceiling of the native file pipelines (SURVEY §8(e) "Bound: per-GPU throughput x G
until host ingest and codec saturate"): ntc_encode_file / ntc_decode_file (pipeline.cpp) with
their GPU stage replaced by a memo of its first output per batch shape
(tests/san/gpu_stub.cpp, -DNTC_STUB_MEMO, tests/san/Makefile `host_ceiling`), so what is
timed is the host side alone: the FASTQ text into pinned buffers (plain), the parallel
inflate (single-member gzip, pgzip.cpp), deflate of the four streams per block and the
encoded.dat writes (encode); block inflate and the FASTA writes (decode).  One JSON line per
(input, threads, contexts): the best of --reps timed runs after one warm run.

  python scripts/host_ceiling.py [--reads 4000000] [--threads 4,8,16] [--ctx 2] [--out DIR]

Runs on the CPU (no GPU needed); on a GPU box it measures that box's host share.
"""
import argparse
import gzip
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

import ntcomp_amd as nt  # noqa: E402


def run(binary, args):
    r = subprocess.run([binary, *map(str, args)], capture_output=True, text=True, timeout=1200)
    out = dict(x.split("=", 1) for x in r.stdout.split() if "=" in x)
    if r.returncode != 0 or out.get("rc") != "0":
        raise RuntimeError(f"{args}: rc={r.returncode} {r.stdout} {r.stderr[-2000:]}")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=4_000_000)
    ap.add_argument("--len", type=int, default=150)
    ap.add_argument("--threads", default="4,8,16")
    ap.add_argument("--ctx", default="2")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--gzip-level", type=int, default=6)
    ap.add_argument("--out", default="/tmp/ntc_ceiling")
    ap.add_argument("--kinds", default="plain,gz,decode")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "tests", "san"), "host_ceiling"])
    binary = os.path.join(REPO, "tests", "san", "host_ceiling")
    # the C91 workload's shape (bench.py): 5 Mbp genome, k = 91, 1 % substitutions
    genome = nt.synth_genome(1, 5_000_000)
    ix = nt.Index.build([genome.tobytes()], 91, threads=8)
    ix.save(os.path.join(a.out, "idx"))
    fq = os.path.join(a.out, "r.fq")
    n, L = a.reads, a.len
    if not os.path.exists(fq) or os.path.getsize(fq) != n * (2 * L + 7):
        t = time.time()
        with open(fq, "wb") as f:
            for c0 in range(0, n, 500_000):
                m = min(500_000, n - c0)
                reads = nt.synth_reads(genome, 7 + c0, 0, m, L, 10_000).reshape(m, L)
                rec = np.empty((m, 2 * L + 7), dtype=np.uint8)
                rec[:, 0:2] = np.frombuffer(b"@r", np.uint8)
                rec[:, 2] = ord("\n")
                rec[:, 3:3 + L] = reads
                rec[:, 3 + L:6 + L] = np.frombuffer(b"\n+\n", np.uint8)
                rec[:, 6 + L:6 + 2 * L] = ord("I")
                rec[:, 2 * L + 6] = ord("\n")
                f.write(rec.tobytes())
        print(f"# wrote {fq} in {time.time() - t:.1f} s", file=sys.stderr)
    kinds = a.kinds.split(",")
    gz = os.path.join(a.out, "r.fq.gz")
    if "gz" in kinds and not os.path.exists(gz):
        with open(fq, "rb") as f, open(gz, "wb") as g:
            g.write(gzip.compress(f.read(), a.gzip_level))
    dat = os.path.join(a.out, "e.dat")
    cpus = len(os.sched_getaffinity(0))
    for T in [int(x) for x in a.threads.split(",")]:
        for C in [int(x) for x in a.ctx.split(",")]:
            base = {"reads": n, "read_len": L, "threads": T, "contexts": C, "cpus_available": cpus}
            for kind in kinds:
                if kind == "decode":
                    if not os.path.exists(dat):
                        run(binary, ["encode", os.path.join(a.out, "idx"), fq, dat, T, 0, C, 2, 0, 0])
                    got = run(binary, ["decode", os.path.join(a.out, "idx"), dat, os.path.join(a.out, "o.fa"), T, 0, C,
                                       2, 0, a.reps])
                else:
                    got = run(binary, ["encode", os.path.join(a.out, "idx"), fq if kind == "plain" else gz,
                                       os.path.join(a.out, "x.dat"), T, 0, C, 2, 0, a.reps])
                print(json.dumps({**base, "pipeline": "decode" if kind == "decode" else "encode",
                                  "input": {"plain": "plain FASTQ", "gz": f"single-member gzip -{a.gzip_level}",
                                            "decode": "encoded.dat"}[kind],
                                  "wall_s": float(got["wall"]), "host_gbases_s": float(got["gbases_s"]),
                                  "bases": int(got["bases"]),
                                  "thread_s": {x: float(got[x + "_s"]) for x in ("parse", "gpu", "deflate", "write", "alloc")},
                                  "first_batch_s": float(got["first_batch_s"]),
                                  "reader_done_s": float(got["reader_done_s"])}), flush=True)


if __name__ == "__main__":
    main()
