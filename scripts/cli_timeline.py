#!/usr/bin/env python3
"""Where a native CLI process's wall clock goes: the loader (exec -> main), main's own
process_s, the context teardown and _exit (-> the parent's waitpid), from NTC_INIT_TRACE's
wall-clock stamps.  One JSON line per run.

  python scripts/cli_timeline.py encode|decode IDX INPUT [--reps 3] [-- extra CLI args]"""
import json
import os
import re
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "ntcomp_amd", "ntcomp")


def main():
    args = sys.argv[1:]
    extra = []
    if "--" in args:
        i = args.index("--")
        args, extra = args[:i], args[i + 1:]
    reps = 3
    if "--reps" in args:
        i = args.index("--reps")
        reps = int(args[i + 1])
        args = args[:i] + args[i + 2:]
    cmd, idx, inp = args[:3]
    env = dict(os.environ, NTC_INIT_TRACE="1")
    for _ in range(reps):
        # a fresh output file, as scripts/e2e_bench.py does: truncating the previous run's
        # output makes ext4 (auto_da_alloc) start its writeback at the last close
        if os.path.exists("/tmp/ntc_cli_timeline.out"):
            os.unlink("/tmp/ntc_cli_timeline.out")
        t0 = time.time()
        with open("/tmp/ntc_cli_timeline.out", "wb") as f:
            r = subprocess.run([BIN, cmd, "-i", idx, inp, "--stats", *extra], stdout=f, stderr=subprocess.PIPE, env=env)
        t1 = time.time()
        err = r.stderr.decode(errors="replace")
        m0 = re.search(r"\[init\] main at ([0-9.]+)", err)
        m1 = re.search(r"_exit at ([0-9.]+)", err)
        m2 = re.search(r"contexts freed in ([0-9.]+) ms", err)
        st = [json.loads(x) for x in err.splitlines() if x.startswith("{") and "process_s" in x]
        print(json.dumps({"cmd": cmd, "input": os.path.basename(inp), "rc": r.returncode, "wall_s": round(t1 - t0, 4),
                          "loader_s": round(float(m0.group(1)) - t0, 4) if m0 else None,
                          "process_s": st[-1]["process_s"] if st else None,
                          "pipeline_wall_s": st[-1].get("pipeline_wall_s") if st else None,
                          "ctx_free_ms": float(m2.group(1)) if m2 else None,
                          "exit_s": round(t1 - float(m1.group(1)), 4) if m1 else None}), flush=True)


if __name__ == "__main__":
    main()
