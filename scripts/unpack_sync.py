#!/usr/bin/env python3
"""Why is the GPU unpacker slow?  C91 blocks from the GPU packer -> per stream: the code
statistics, and (Rice streams) how often k_unpack_streams's speculative chains run through
the next segment before meeting a later one's, or meet none within 8 segments (which sends
the whole stream to one thread);
then ntc_unpack_streams wall time for a 2-block and a 16-block call.

usage: unpack_sync.py [--reads N] [--out JSON]
"""
import argparse
import bisect
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ntcomp_amd as nt  # noqa: E402

THREADS = 1024


def rice_sim(bits, p, n):
    """k_unpack_streams phases A/B on one Rice stream: segments whose successor's chain is
    not met within the next segment, and how many segments on the chains do meet."""
    nbits = len(bits)
    ones = np.flatnonzero(bits)

    def code(pos):
        i = bisect.bisect_left(ones, pos)
        if i >= len(ones):
            return None
        e = int(ones[i]) + 1 + p
        return e - pos if e <= nbits else None

    S = ((nbits + THREADS - 1) // THREADS + 63) & ~63
    segs = [(t * S, min(t * S + S, nbits)) for t in range(THREADS) if t * S < nbits]
    marks, ends = [], []
    for a, b in segs:
        pos, m = a, set()
        while pos < b:
            c = code(pos)
            if c is None:
                break
            m.add(pos)
            pos += c
        marks.append(m)
        ends.append(pos)
    later, fail, dist = 0, 0, []
    for t in range(len(segs) - 1):
        q, u, steps = ends[t], t + 1, 0
        met = None
        while q < nbits and q < segs[t][1] + 8 * S:
            while u < len(segs) and q >= segs[u][1]:
                u += 1
            if u >= len(segs):
                break
            if q in marks[u] and q >= segs[u][0]:
                met = u
                break
            c = code(q)
            if c is None:
                break
            q += c
            steps += 1
        if met is None and q < nbits:
            fail += 1
        elif met is not None and met > t + 1:
            later += 1
        dist.append(steps)
    return {"segments": len(segs), "seg_bits": S, "met_a_later_segment": later, "not_met_within_8": fail,
            "codes_to_meet_mean": round(float(np.mean(dist)), 2) if dist else None,
            "codes_to_meet_max": int(max(dist)) if dist else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=16 * 65536)
    ap.add_argument("--out", default="gpurun_out/unpack_sync.json")
    ap.add_argument("--no-sim", action="store_true", help="only the timings (e.g. under rocprofv3)")
    a = ap.parse_args()
    genome = nt.synth_genome(1, 5_000_000)
    ix = nt.Index.build([genome.tobytes()], 91, threads=16)
    ctx = nt.GpuContext(0)
    ctx.upload(ix)
    n, L = a.reads, 150
    reads = nt.synth_reads(genome, 2, 0, n, L, 10_000, threads=16)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    metas, payload = ctx.encode_pack(reads, offs)
    eng = "libdeflate" if nt.libdeflate_available() else "zlib"
    blocks = [nt.read_block_streams(nt.deflate_block(m, payload, eng))[:2] for m in metas]
    res = {"reads": n, "blocks": len(blocks), "streams": []}
    m0, p0 = blocks[0]
    for s in range(4):
        sm = m0.stream[s]
        raw = np.frombuffer(p0, dtype=np.uint8)[sm.offset:sm.offset + 8 * sm.encoded_size]
        bits = np.unpackbits(raw)
        e = {"stream": s + 1, "coder": "rice" if s in (1, 2) else "minimal binary", "param": int(sm.param),
             "values": int(sm.num_u64), "bits": int(len(bits)),
             "bits_per_value": round(len(bits) / max(1, sm.num_u64), 2)}
        if s in (1, 2) and not a.no_sim:
            t0 = time.time()
            e.update(rice_sim(bits, int(sm.param), int(sm.num_u64)))
            e["sim_s"] = round(time.time() - t0, 1)
        else:
            l = int(sm.param).bit_length() - 1
            e["l"] = l
            e["limit"] = (2 << l) - int(sm.param)
        res["streams"].append(e)
        print(json.dumps(e), flush=True)
    for nb in (2, len(blocks)):
        um, up = nt.concat_streams(blocks[:nb])
        ctx.unpack(um, up, nb)
        ts = []
        for _ in range(10):
            ctx.synchronize()
            t0 = time.perf_counter()
            ctx.unpack(um, up, nb)
            ts.append(time.perf_counter() - t0)
        res[f"unpack_ms_{nb}_blocks"] = round(1e3 * float(np.median(ts)), 3)
        print(nb, "blocks:", res[f"unpack_ms_{nb}_blocks"], "ms", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
