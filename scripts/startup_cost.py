#!/usr/bin/env python3
"""Process start and exit around the native CLI (DESIGN.md "End-to-end"): wall clock of
`ntcomp` printing its usage (dynamic loading + static initialisers, no GPU call), and of
`ntcomp encode` on a one-read FASTQ against the process_s it reports itself (from main)."""
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
BIN = os.path.join(REPO, "ntcomp_amd", "ntcomp")


def wall(cmd, **kw):
    t = time.time()
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, **kw)
    return time.time() - t, r


def main():
    import numpy as np
    import ntcomp_amd as nt
    d = "/tmp/ntc_startup"
    os.makedirs(d, exist_ok=True)
    g = nt.synth_genome(3, 200_000)
    nt.Index.build([g.tobytes()], 31).save(os.path.join(d, "idx"))
    with open(os.path.join(d, "one.fq"), "wb") as f:
        f.write(b"@r\n" + g[1000:1150].tobytes() + b"\n+\n" + b"F" * 150 + b"\n")
    out = {"usage_s": [], "encode_wall_s": [], "encode_process_s": []}
    for _ in range(5):
        out["usage_s"].append(round(wall([BIN])[0], 4))
    for _ in range(5):
        w, r = wall([BIN, "encode", "-i", os.path.join(d, "idx"), os.path.join(d, "one.fq"), "--stats"])
        st = json.loads([x for x in r.stderr.decode().splitlines() if x.startswith("{")][-1])
        out["encode_wall_s"].append(round(w, 4))
        out["encode_process_s"].append(st["process_s"])
        out["encode_stats"] = st["stats"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
