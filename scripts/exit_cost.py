#!/usr/bin/env python3
"""Exit cost of the native CLI on a 10 M-read encode (DESIGN.md "End-to-end"): wall clock
around the process against the process_s it reports from main.  (Round 4 compared leaving
the contexts to the exit with freeing them first, an env hook since removed: 0.10-0.13 s
against 0.05-0.08 s after main, profiles/round4/cli_exit_cost_r04.jsonl.)  Uses
/tmp/ntc_e2e from scripts/e2e_bench.py.  Prints one JSON line per run."""
import json
import os
import subprocess
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "ntcomp_amd", "ntcomp")
d = "/tmp/ntc_e2e"
for mode in ("default",) * 4:
    env = dict(os.environ)
    if mode == "teardown":
        env["NTC_EXIT_TEARDOWN"] = "1"
    t = time.time()
    with open(os.path.join(d, "x.dat"), "wb") as f:
        r = subprocess.run([BIN, "encode", "-i", os.path.join(d, "idx"), os.path.join(d, "reads.fq"), "--stats"],
                           stdout=f, stderr=subprocess.PIPE, env=env)
    w = time.time() - t
    lines = [json.loads(x) for x in r.stderr.decode().splitlines() if x.startswith("{")]
    st = [x for x in lines if "process_s" in x][-1]
    td = [x["teardown_s"] for x in lines if "teardown_s" in x]
    print(json.dumps({"mode": mode, "wall_s": round(w, 4), "process_s": st["process_s"],
                      "teardown_s": td[0] if td else None, "pipeline_wall_s": st["pipeline_wall_s"]}), flush=True)
