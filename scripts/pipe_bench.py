#!/usr/bin/env python3
"""ntc_encode_file / ntc_decode_file timeline on the e2e_bench.py files (no CLI process
around it): per-stage thread-seconds and when the reader / GPU finished, for sizing the host
pipeline."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/tmp/ntc_e2e")
    ap.add_argument("--deflate", default="libdeflate")
    ap.add_argument("--bpb", type=int, nargs="+", default=[16])
    ap.add_argument("--threads", type=int, nargs="+", default=[0])
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--mode", default="encode", choices=["encode", "decode"])
    ap.add_argument("--batch-bases", type=int, nargs="+", default=[0], help="encode: pinned batch buffer (0: default)")
    ap.add_argument("--contexts", type=int, nargs="+", default=[1], help="contexts on device 0 (calls alternate)")
    ap.add_argument("--parse", nargs="+", default=["gpu"], choices=["gpu", "host"],
                    help="encode: plain FASTQ parsed on the GPU or the host pool")
    a = ap.parse_args()
    import ntcomp_amd as nt
    ix = nt.Index.load(os.path.join(a.dir, "idx"))
    pool = [nt.GpuContext(0).upload(ix)]
    for _ in range(max(a.contexts) - 1):  # further contexts share the first one's index
        pool.append(nt.GpuContext(0).share_index(pool[0]))
    fq = os.path.join(a.dir, "reads.fq")
    for bpb, bb, nc, pa in [(x, y, z, w) for x in a.bpb for y in a.batch_bases for z in a.contexts for w in a.parse]:
        ctxs = pool[:nc]
        for th in a.threads:
            for rep in range(a.reps):
                t0 = time.time()
                if a.mode == "encode":
                    with open(os.path.join(a.dir, "pipe.dat"), "wb") as f:
                        st = nt.encode_file(ctxs, fq, f.fileno(), threads=th, blocks_per_batch=bpb,
                                            batch_bases=bb, deflate=a.deflate, host_parse=pa == "host")
                else:
                    with open(os.path.join(a.dir, "pipe.fa"), "wb") as f:
                        st = nt.decode_file(ctxs, os.path.join(a.dir, "enc.dat"), f.fileno(), threads=th,
                                            blocks_per_batch=bpb)
                w = time.time() - t0
                st.pop("error")
                print(json.dumps({"mode": a.mode, "parse": pa, "bpb": bpb, "batch_bases": bb, "contexts": nc, "threads": th, "rep": rep,
                                  "wall": round(w, 3),
                                  "gbases_s": round(st["bases"] / w / 1e9, 3),
                                  **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in st.items()}}),
                      flush=True)
    for c in pool:
        c.close()


if __name__ == "__main__":
    main()
