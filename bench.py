#!/usr/bin/env python3
"""ntcomp encode/decode throughput on MI355X -- BASELINE.json's metric:
"encode Mbases/sec at k=91, 150bp reads, 1/2/4/8 MI355X; bit-exact vs CPU".

Launch: `python bench.py --gpus N` (N > 1 without RANK in the environment starts a
torch.distributed.run child with N ranks before anything touches the GPU), or the driver's
`python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`.  One process
per GPU; reads shard over ranks with the index replicated and no data-path collective
(main.rs:152,162-173): torch.distributed (gloo) only carries the barriers,
the max-over-ranks of the timed region and the per-rank parity verdicts.

Workload:
  C91   per GPU 10M (N = 1) or 25M (N > 1: 8 x 25M = C91x8's 200M) synthetic 150 bp reads
        (uniform starts, 50 % reverse complemented, 1 % i.i.d. substitutions) against the
        SBWT (k = 91, + reverse complements) of a 5 Mbp synthetic genome.
  D91   decode of C91's records back to bases (lib.rs:254-318).
  S91   (N = 1) the same reads drawn from an 11-genome collection: the 5 Mbp genome plus 10
        strains at 1 % substitutions (reference-based compression of a strain collection,
        README.md:2): 70 M nodes, a fragmented path cover.
A step = one pass of the hot path over the rank's whole shard, in device calls of at most
--batch-reads reads (10M), inputs already resident in HBM.  C91 and D91 keep --inflight (2)
calls in flight on as many contexts of the rank's GPU (each with its own index copy,
stream and output buffers; a context takes a call only after its previous one is
finalized), so the next call's kernels fill the current one's drain; S91 runs one call at
a time.  The top-level line is C91 encode; "decode" and "strains" carry D91 and S91 with
their own rooflines and parity.

roofline: bytes past L2 per launch of the dominant kernel (k_ms4 / k_dec_rec), from the
rocprofv3 PMC passes of THIS device build (profiles/pmc_traffic.json, keyed by the device
source hash; scaled per read or per base to the launch), / the kernel's live HIP-event
time, against 8 TB/s.  Each read request is counted at its own size (32/64/128 B:
TCC_EA0_RDREQ_{32B,64B,128B}), writes at theirs (TCC_EA0_WRREQ, _64B), so random 64 B
lines are not double-counted.  `line_rate` puts the request rate past L2 (reads and
writes) against the random-line roof measured by scripts/randbw.hip.
roofline.algorithmic: the bytes THIS design must move per launch -- encode: the distinct
128 B lines a read's lanes touch (the emulator's line trace of encode_core.h,
profiles/algorithmic_lines.json, scripts/trace_lines.py --json) x reads; decode: one 128 B
walk-table line per 112 bases of each long record, plus 8 B per record in and 1 B per base
out -- over the kernel time (algorithmic frac), and traffic / algorithmic bytes (waste:
1.0 = every line fetched once per read).  Encode also gives the lines counted distinct per
lane step (step_lines_per_read: a line a read touches again in a later step counted again,
as an L2 that keeps nothing across a lane's steps would fetch it) and the traffic against
those (waste_vs_step_lines < 1: L2 kept some lines across steps).
cpu_baseline: the faithful C oracle (oracle/ntcomp_oracle.c, test infrastructure) on one
pinned host core, rank 0 at N = 1, on a bounded sample; it is also the parity checker.  The
reference encoder is single-threaded (main.rs:162-173), so one core is the faithful figure;
"all_cores" times the same sample read-sharded over every CPU the process may use, and the
host's CPU model and counts are reported beside it.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

METRIC = "encode Mbases/sec at k=91, 150bp reads, 1/2/4/8 MI355X; bit-exact vs CPU"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md "HBM": 8 TB/s spec
PMC_JSON = os.path.join(REPO, "profiles", "pmc_traffic.json")
RANDBW_JSONL = os.path.join(REPO, "profiles", "round1", "randbw.jsonl")
ALG_JSON = os.path.join(REPO, "profiles", "algorithmic_lines.json")
WALK_SPAN = 112  # characters per walk-table entry (encode_core.h kWalkSpan): one 128 B line each


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--configs", default=None,
                    help="comma list of encode,decode,strains,c31 (default: all four at N=1, encode,decode at N>1)")
    ap.add_argument("--mode", choices=["encode", "decode"], default=None, help="(legacy) = --configs <mode>")
    ap.add_argument("--k", type=int, default=91)
    ap.add_argument("--reads-per-gpu", type=int, default=None, help="default 10M at N=1, 25M at N>1 (C91x8)")
    ap.add_argument("--batch-reads", type=int, default=0,
                    help="reads per device call (0: the rank's whole shard in one call; the library sizes "
                         "its workspace by need)")
    ap.add_argument("--inflight", type=int, default=2,
                    help="device calls in flight per GPU: contexts on the rank's GPU (each with its own index "
                         "copy, stream and output buffers) take the calls in turn; a context is reused only after "
                         "its previous call is finalized (status + that launch's kernel time)")
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--err-ppm", type=int, default=10_000)
    ap.add_argument("--genome-bp", type=int, default=5_000_000)
    ap.add_argument("--strains", type=int, default=10)
    ap.add_argument("--strain-snp-ppm", type=int, default=10_000)
    ap.add_argument("--strain-reads", type=int, default=10_000_000)
    ap.add_argument("--strain-inflight", type=int, default=1, help="S91 device calls in flight (contexts)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU only: ranks, shards, oracle samples and the gathers, no GPU calls")
    ap.add_argument("--opt", action="append", default=[], help="ctx option key=value (A/B)")
    ap.add_argument("--presort", action="store_true",
                    help="experiment: reorder each batch's reads by minimizer on the host before upload")
    ap.add_argument("--pmc-json", default=PMC_JSON)
    args = ap.parse_args(argv)
    if args.mode and not args.configs:
        args.configs = args.mode
    return args


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args):
    """`bench.py --gpus N` outside torch.distributed.run: start it as a CHILD process (this
    process has not touched the GPU or imported torch) and exit with its code."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[launcher] {args.gpus} ranks: {' '.join(cmd[1:6])} ...")
    return subprocess.call(cmd, env=env)


# ---- counters ----------------------------------------------------------------------
def load_pmc(path, want_hash):
    """-> (workloads dict or None, note)"""
    try:
        with open(path) as f:
            pj = json.load(f)
    except (OSError, ValueError):
        return None, f"no {os.path.relpath(path, REPO)}"
    if pj.get("device_source_hash") != want_hash:
        return None, (f"{os.path.relpath(path, REPO)} is from device build {pj.get('device_source_hash')}, "
                      f"this build is {want_hash}: counters not applied")
    return pj.get("workloads", {}), "ok"


def random_line_roof(working_set=None):
    """Random 128 B line requests per second past L2 (scripts/randbw.hip): the best rate over
    buffers >= 32 MB, or, for a kernel whose random loads go to one structure of working_set
    bytes (k_dec_rec: the walk table), the rate measured on the largest buffer not larger
    than it (the rate falls with the buffer: 66 G/s at 32 MB, 55 at 512 MB, 51 at 4 GB)."""
    try:
        roofs = [r for r in (json.loads(l) for l in open(RANDBW_JSONL))
                 if r.get("test") == "random_8B_loads" and r["buffer_bytes"] >= (32 << 20)]
        if working_set:
            fit = [r for r in roofs if r["buffer_bytes"] <= working_set]
            if fit:
                return max(fit, key=lambda r: r["buffer_bytes"])["g_lines_per_s"]
        return max(r["g_lines_per_s"] for r in roofs)
    except (OSError, ValueError, KeyError):
        return None


def launch_ms(kms, units, ref):
    """kernel ms of a launch of `ref` units from launches of different sizes (a shard's last
    batch is smaller): (mean, min) of time per unit x ref, launches in timed() order"""
    per = [t / u for t, u in zip(kms, units * (len(kms) // len(units)))]
    return sum(kms) / sum(units * (len(kms) // len(units))) * ref, min(per) * ref


def roofline(kname, kernel_ms, kernel_ms_min, units, unit_name, pmc, pmc_note, wl_key, extra=None, working_set=None):
    """Roofline of one dominant kernel: PMC bytes past L2 per unit (read or base) x units per
    launch / live kernel time."""
    r = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": None, "traffic": None,
         "kernel": kname, "kernel_ms": round(kernel_ms, 4), "kernel_ms_min": round(kernel_ms_min, 4),
         "units_per_launch": int(units), "unit_kind": unit_name}
    kd = ((pmc or {}).get(wl_key) or {}).get("kernels", {}).get(kname) if pmc is not None else None
    if kd:
        per = (pmc[wl_key].get("units_per_launch") or 0)
        scale = units / per if per else 1.0
        rd, wr = kd["read_bytes"] * scale, kd["write_bytes"] * scale
        traffic = rd + wr
        r.update(achieved=round(traffic / (kernel_ms / 1e3) / 1e9, 1), traffic=int(traffic),
                 read_bytes=int(rd), write_bytes=int(wr))
        r["frac"] = round(r["achieved"] / HBM_PEAK_GBPS, 4)
        r["bytes_per_" + unit_name] = round(traffic / units, 2)
        if kd.get("dram_read_bytes") is not None:
            r["dram_read_bytes"] = int(kd["dram_read_bytes"] * scale)
        roof = random_line_roof(working_set)
        rq, wq = kd.get("rdreq", 0) * scale, (kd.get("wrreq") or 0) * scale
        if roof and rq:
            # the random READ lines against the random-read roof (scripts/randbw.hip) of the
            # kernel's random working set; the writes are streamed (coalesced output), not
            # random lines, so they are reported beside it, not counted against it
            rate = rq / (kernel_ms / 1e3) / 1e9
            r["line_rate"] = {"read_requests_per_launch": int(rq), "write_requests_per_launch": int(wq),
                              "read_requests_per_" + unit_name: round(rq / units, 3),
                              "write_requests_per_" + unit_name: round(wq / units, 3),
                              "g_read_requests_per_s": round(rate, 2), "roof_g_requests_per_s": roof,
                              "roof_working_set_bytes": working_set, "frac": round(rate / roof, 4)}
        r["pmc_profile_kernel_ms"] = round(kd.get("avg_ns", 0) / 1e6 * scale, 4)
    r["note"] = ("achieved = bytes past L2 per launch (rocprofv3 PMC of this device build, each request at its "
                 "own 32/64/128 B size, plus writes; " + pmc_note + ") / live HIP-event kernel time of isolated "
                 "launches (one call in flight, after the timed region)")
    if extra:
        r.update(extra)
    return r


def load_alg(path):
    try:
        with open(path) as f:
            return json.load(f).get("workloads", {})
    except (OSError, ValueError):
        return {}


def algorithmic(bytes_per_launch, units, unit_name, kernel_ms, traffic, source):
    """the design's own bytes per launch against the kernel time and the counter traffic"""
    gbs = bytes_per_launch / (kernel_ms / 1e3) / 1e9
    return {"bytes_per_launch": int(bytes_per_launch), "bytes_per_" + unit_name: round(bytes_per_launch / units, 2),
            "achieved": round(gbs, 1), "peak": HBM_PEAK_GBPS, "frac": round(gbs / HBM_PEAK_GBPS, 4),
            "waste": round(traffic / bytes_per_launch, 3) if traffic else None, "source": source}


def alg_encode(alg, wl, units, kernel_ms, traffic):
    w = alg.get(wl)
    if not w:
        return None
    per = w["k_ms4_lines_per_read"] * 128
    r = algorithmic(per * units, units, "read", kernel_ms, traffic,
                    f"{w['k_ms4_lines_per_read']} distinct 128 B lines per read (emulator trace of "
                    f"{w['reads']} reads, encode_core.h {w['encode_core_sha256']}) x reads")
    step = w.get("k_ms4_step_lines_per_read")
    if step:  # the same lines counted distinct per lane step: no L2 reuse across a lane's steps
        r["step_lines_per_read"] = step
        r["waste_vs_step_lines"] = round(traffic / (step * 128 * units), 3) if traffic else None
    return r


def alg_decode(recs, bases, kernel_ms, traffic):
    """k_dec_rec: ceil(L / 112) walk lines per long record + records in + ASCII out"""
    import numpy as np
    flags = recs >> np.uint64(56)
    long_ = (flags & np.uint64(2)) == 0
    L = ((recs[long_] >> np.uint64(32)) & np.uint64(0xFFFFFF)).astype(np.int64)
    walk = int(((L + WALK_SPAN - 1) // WALK_SPAN).sum())
    b = 128 * walk + 8 * len(recs) + bases
    return algorithmic(b, bases, "base", kernel_ms, traffic,
                       f"{walk} walk-table lines (ceil(L/{WALK_SPAN}) per long record) x 128 B + 8 B per record "
                       f"+ 1 B per base")


def io_floor(in_bytes, out_bytes, call_ms):
    """The path's own I/O -- its input read once and its output written once (encode: 1 B
    of ASCII per base in, 8 B per record out; decode: 8 B per record in, 1 B per base out)
    -- over the whole call's device time (every kernel), against 8 TB/s: the efficiency a
    perfect kernel would reach 1.0 on, beside the counter-based frac."""
    b = in_bytes + out_bytes
    gbs = b / (call_ms / 1e3) / 1e9
    return {"bytes_per_call": int(b), "in_bytes": int(in_bytes), "out_bytes": int(out_bytes),
            "call_ms": round(call_ms, 4), "achieved": round(gbs, 1), "peak": HBM_PEAK_GBPS,
            "frac": round(gbs / HBM_PEAK_GBPS, 4)}


def aggregate_roofline(per_rank, world):
    """N > 1: every rank's dominant-kernel bytes past L2 summed, over the slowest rank's
    kernel time, against N x 8 TB/s (BASELINE's 1/2/4/8-GPU fractions)."""
    rs = [x for x in per_rank if x and x.get("traffic")]
    if len(rs) != world:
        return None
    tot = sum(x["traffic"] for x in rs)
    tmax = max(x["kernel_ms"] for x in rs)
    gbs = tot / (tmax / 1e3) / 1e9
    return {"ranks": world, "traffic": int(tot), "kernel_ms_max": round(tmax, 4), "achieved": round(gbs, 1),
            "peak": HBM_PEAK_GBPS * world, "unit": "GB/s", "frac": round(gbs / (HBM_PEAK_GBPS * world), 4)}


def _opt(ctx, key):
    """a context option, None when the library predates it (A/B runs against older builds)"""
    try:
        return ctx.get_option(key)
    except Exception:
        return None


def _gb(v):
    return None if v is None else round(v / 1e9, 2)


# ---- workload ----------------------------------------------------------------------
def minimizer_order(nt, reads, n, L, threads):
    """(experiment) read order grouped by minimizer: smallest hashed 20-mer, strand as read"""
    import numpy as np
    return np.argsort(nt.minimizer_keys(reads, n, L, 20, threads), kind="stable")


class Shard:
    """One rank's reads of one workload, in device batches."""

    def __init__(self, nt, ctx, text, first, n, L, err, batch, threads, dry, presort=False, n_out=1):
        import numpy as np
        self.L, self.n, self.first = L, n, first
        self.batches = []
        batch = batch or n
        off = 0
        while off < n:
            nb = min(batch, n - off)
            reads = nt.synth_reads(text, 2, first + off, nb, L, err, threads=threads)
            if presort:
                reads = reads.reshape(nb, L)[minimizer_order(nt, reads, nb, L, threads)].ravel()
            b = {"first": first + off, "n": nb, "reads": reads, "bases": nb * L}
            if not dry:
                offs = np.arange(0, nb * L + 1, L, dtype=np.uint64)
                cap = nb * L // 4 + 64
                b.update(d_bases=ctx.alloc(reads.nbytes), d_offs=ctx.alloc(offs.nbytes), cap=cap,
                         out=[{"d_recs": ctx.alloc(cap * 8), "d_roffs": ctx.alloc(offs.nbytes)} for _ in range(n_out)])
                ctx.h2d(b["d_bases"], reads)
                ctx.h2d(b["d_offs"], offs)
            self.batches.append(b)
            off += nb
        self.bases = n * L

    def free(self, ctx):
        for b in self.batches:
            for o in [b] + b.get("out", []):
                for key in ("d_bases", "d_offs", "d_recs", "d_roffs", "d_out", "d_ooffs"):
                    if o.get(key):
                        ctx.free(o[key])
                        o[key] = None


class Pipe:
    """Device calls of one kind kept in flight over the contexts of one GPU (--inflight):
    call i goes to context i % n with that context's output buffers, and a context takes a
    new call only after its previous one is finalized -- status checked and the launch's
    dominant-kernel time (HIP events on that context's stream) recorded.  With two
    contexts the next call's kernels fill the drain of the current one."""

    def __init__(self, ctxs, kind):
        self.ctxs, self.kind = ctxs, kind
        self.pending = [None] * len(ctxs)
        self.i = 0
        self.kms = []  # the dominant kernel's ms per call
        self.tms = []  # the whole call's device ms (every kernel of it)

    def issue(self, sh, b, check=False):
        c = self.i % len(self.ctxs)
        self.i += 1
        self.finish(c)
        ctx, o = self.ctxs[c], b["out"][c]
        if self.kind == "encode":
            ctx.encode_device(b["d_bases"], b["d_offs"], b["n"], sh.L, o["d_recs"], b["cap"], o["d_roffs"])
        else:
            if not o.get("d_out"):
                o["d_out"], o["d_ooffs"] = ctx.alloc(b["bases"] + 64), ctx.alloc((b["n"] + 1) * 8)
            ctx.decode_device(o["d_recs"], b["n_recs"], o["d_out"], b["bases"] + 64, o["d_ooffs"], b["n"] + 1)
        self.pending[c] = (b, check)

    def finish(self, c):
        if self.pending[c] is None:
            return
        b, check = self.pending[c]
        self.pending[c] = None
        ctx = self.ctxs[c]
        if self.kind == "encode":
            got = ctx.encode_status()
            if check:
                b["n_recs"] = got
            elif got != b["n_recs"]:
                raise RuntimeError(f"record count changed between passes: {got} vs {b['n_recs']}")
        elif ctx.decode_status() != (b["n"], b["bases"]):
            raise RuntimeError(f"decode status {ctx.decode_status()} != {(b['n'], b['bases'])}")
        t = ctx.timing()
        self.kms.append(t["main_ms"])
        self.tms.append(t["total_ms"])

    def drain(self):
        for k in range(len(self.ctxs)):
            self.finish((self.i + k) % len(self.ctxs))


def encode_all_outputs(ctxs, sh):
    """every context's output buffers hold every batch's records (for decode and checks)"""
    for c, ctx in enumerate(ctxs):
        for b in sh.batches:
            o = b["out"][c]
            ctx.encode_device(b["d_bases"], b["d_offs"], b["n"], sh.L, o["d_recs"], b["cap"], o["d_roffs"])
            got = ctx.encode_status()
            if b.get("n_recs") is not None and got != b["n_recs"]:
                raise RuntimeError(f"context {c}: {got} records, expected {b['n_recs']}")
            b["n_recs"] = got


def timed(pipe, sh, steps, warmup, barrier, sync, dist):
    """W untimed steps, then K steps between barrier + sync; a step = one call per batch of
    the shard through the pipe.  -> (max over ranks of the elapsed time, dominant-kernel ms per
    call); the whole calls' device ms stay in pipe.tms"""
    from ntcomp_amd import shard as shard_mod
    for _ in range(warmup):
        for b in sh.batches:
            pipe.issue(sh, b)
    pipe.drain()
    barrier()
    sync()
    pipe.kms, pipe.tms = [], []
    t0 = time.perf_counter()
    for _ in range(steps):
        for b in sh.batches:
            pipe.issue(sh, b)
    pipe.drain()
    sync()
    el = time.perf_counter() - t0
    barrier()
    return shard_mod.max_over_ranks(el, dist), list(pipe.kms)


def records_of(ctx, b, a_read, b_read):
    import numpy as np
    o = b["out"][0]
    ro = ctx.d2h(np.zeros(b["n"] + 1, dtype=np.uint64), o["d_roffs"])
    lo, hi = int(ro[a_read]), int(ro[b_read])
    recs = ctx.d2h(np.zeros(hi - lo, dtype=np.uint64), o["d_recs"] + 8 * lo) if hi > lo else np.zeros(0, np.uint64)
    return recs, ro


def check_shard(ctx, orc, sh, seconds, full_decode, pin, dry):
    """Bit-exactness of GPU records vs the oracle on a bounded sample of every batch (timed:
    the CPU baseline), and of the decoded bases vs the reads over the whole shard."""
    import numpy as np
    L = sh.L
    res = {"encode_ok": True, "reads_checked": 0, "cpu_encode_s": 0.0, "decode_ok": None, "cpu_decode_s": 0.0,
           "cpu_decode_bases": 0}
    old = os.sched_getaffinity(0)
    core = sorted(old)[-1]
    if pin:
        os.sched_setaffinity(0, {core})
    try:
        per_batch = seconds / max(1, len(sh.batches))
        for b in sh.batches:
            chunk, done, spent = min(2000, b["n"]), 0, 0.0
            while spent < per_batch and done + chunk <= b["n"]:
                sl = b["reads"][done * L:(done + chunk) * L]
                o = np.arange(0, chunk * L + 1, L, dtype=np.uint64)
                t1 = time.perf_counter()
                exp, eoff = orc.encode(sl, o)
                spent += time.perf_counter() - t1
                if not dry:
                    got, ro = records_of(ctx, b, done, done + chunk)
                    res["encode_ok"] &= bool(np.array_equal(got, exp))
                    if res["cpu_decode_s"] < seconds / 4:
                        t1 = time.perf_counter()
                        out, _ = orc.decode(exp)
                        res["cpu_decode_s"] += time.perf_counter() - t1
                        res["cpu_decode_bases"] += len(out)
                        res["encode_ok"] &= bool(np.array_equal(out, sl))
                done += chunk
            res["reads_checked"] += done
            res.setdefault("spans", []).append(done)
            res["cpu_encode_s"] += spent
            o = b["out"][0] if b.get("out") else {}
            if full_decode and not dry and o.get("d_out"):
                out = ctx.d2h(np.zeros(b["bases"], dtype=np.uint8), o["d_out"])
                oo = ctx.d2h(np.zeros(b["n"] + 1, dtype=np.uint64), o["d_ooffs"])
                ok = bool(np.array_equal(out, b["reads"])) and bool(
                    np.array_equal(oo, np.arange(0, b["bases"] + 1, L, dtype=np.uint64)))
                res["decode_ok"] = ok if res["decode_ok"] is None else (res["decode_ok"] and ok)
    finally:
        if pin:
            os.sched_setaffinity(0, old)
    res["core"] = core
    return res


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_all_cores(orc, sh, spans, threads):
    """The same oracle sample as the one-core baseline, read-sharded over `threads` host
    threads (the C oracle is reentrant and ctypes releases the GIL, so they run in
    parallel): wall-clock Mbases/s."""
    import concurrent.futures as cf

    import numpy as np
    L = sh.L
    reads = np.concatenate([b["reads"][:d * L] for b, d in zip(sh.batches, spans) if d])
    n = len(reads) // L
    cuts = [n * i // threads for i in range(threads + 1)]

    def work(i):
        a, b = cuts[i], cuts[i + 1]
        if b > a:
            orc.encode(reads[a * L:b * L], np.arange(0, (b - a) * L + 1, L, dtype=np.uint64))

    with cf.ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        list(ex.map(work, range(threads)))
        el = time.perf_counter() - t0
    return n * L / el / 1e6, n


def main():
    args = parse_args()
    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(spawn_ranks(args))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    configs = (args.configs or ("encode,decode,strains,c31" if world == 1 else "encode,decode")).split(",")
    reads_per_gpu = args.reads_per_gpu or (10_000_000 if world == 1 else 25_000_000)

    import numpy as np
    import torch  # before ntcomp_amd: one HIP runtime per process

    dist = None
    if world > 1:
        import torch.distributed as dist
        # gloo's native "[Gloo] Rank i is connected to ..." lines go to fd 1; stdout must carry
        # rank 0's JSON line alone, so the native side writes to stderr while the group forms
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")  # barriers, max over ranks, parity verdicts
            dist.barrier()
        finally:
            os.dup2(saved, 1)
            os.close(saved)
    device = 0
    if not args.dry_run:
        ndev = torch.cuda.device_count()  # a box with fewer GPUs than ranks (rehearsal): ranks share
        device = local % ndev if ndev else local
        torch.cuda.set_device(device)

    import ntcomp_amd as nt
    from ntcomp_amd import shard as shard_mod
    from oracle_lib import OracleIndex  # the checker / CPU baseline (test infrastructure)

    def barrier():
        if dist is not None:
            dist.barrier()

    ctx = None

    def sync():
        for c in ctxs:
            c.synchronize()
        torch.cuda.synchronize()

    def gather(obj):
        if dist is None:
            return [obj]
        out = [None] * world
        dist.all_gather_object(out, obj)
        return out

    nthreads = max(1, min(16, (os.cpu_count() or 8) // max(1, world)))
    pmc, pmc_note = load_pmc(args.pmc_json, nt.device_source_hash())
    alg = load_alg(ALG_JSON)
    # counters exist for the profiled workloads only (scripts/profile_bench.sh: the defaults)
    default_wl = (args.read_len, args.err_ppm, args.genome_bp, args.strains, args.strain_snp_ppm) == \
        (150, 10_000, 5_000_000, 10, 10_000)
    if not default_wl and pmc is not None:
        pmc, pmc_note = None, "counters are profiled for the default workloads only"
    if not default_wl:
        alg = {}  # so are the line traces
    L, k = args.read_len, args.k
    first, n = shard_mod.read_range(rank, world, reads_per_gpu)
    line = {}
    t_start = time.time()

    ctxs = []

    build_info = {}

    def setup_index(texts, label, n_ctx, kk=None):
        nonlocal ctx
        kk = kk or k
        if not args.dry_run and ctx is None:
            for _ in range(max(1, args.inflight)):
                c = nt.GpuContext(device)
                for kv in args.opt:
                    key, val = kv.split("=")
                    c.set_option(key, int(val))
                ctxs.append(c)
            ctx = ctxs[0]
        t0 = time.time()
        seqs = [t.tobytes() for t in texts]
        # the GPU builder (build.hip; equal to the host builder, tests/test_gpu_build.py), the
        # host one for --dry-run
        bst = {}
        index = nt.Index.build(seqs, kk, threads=nthreads) if args.dry_run else \
            nt.Index.build_gpu(ctx, seqs, kk, stats=bst)
        build_info[label] = {"builder": "host" if args.dry_run else "gpu", "seconds": round(time.time() - t0, 3)}
        if bst:
            build_info[label].update({x: bst[x] for x in ("kmer_partitions", "node_partitions", "occurrences",
                                                          "peak_device_bytes")})
        log(f"[rank {rank}] {label} index k={kk} n={index.n} built in {time.time() - t0:.1f}s ({build_info[label]['builder']})")
        if not args.dry_run:
            t0 = time.time()
            for c in ctxs[:n_ctx]:
                c.upload(index)
            log(f"[rank {rank}] upload {time.time() - t0:.1f}s, {ctx.get_option('n_paths')} paths, SCAN filter "
                f"{'on' if ctx.get_option('filter') else 'off'} (density {ctx.get_option('filter_density_ppm') / 1e4:.1f} %)")
        return index

    genome = nt.synth_genome(1, args.genome_bp)
    base_cfg = {"k": k, "read_len": L, "genome_bp": args.genome_bp, "err_ppm": args.err_ppm,
                "reads_per_gpu": n, "batch_reads": min(args.batch_reads or n, n)}

    def c_block(kk, want_enc, want_dec, label, cpu_secs):
        """C{kk} encode (+ D{kk} decode) of this rank's shard: the timed lines, rooflines
        (dominant kernel per launch; at N > 1 also summed over ranks), I/O floor, parity on an
        oracle sample (every rank) and, on rank 0, the oracle on one pinned core."""
        index = setup_index([genome], label, len(ctxs) or max(1, args.inflight), kk)
        sh = Shard(nt, ctx, genome, first, n, L, args.err_ppm, args.batch_reads, nthreads, args.dry_run,
                   args.presort, n_out=len(ctxs))
        log(f"[rank {rank}] {label}{kk}: reads {first}..{first + n} in {len(sh.batches)} batch(es)")
        orc = OracleIndex(index.n, kk, index.rows, index.C, index.lcs)
        n_recs = None
        if not args.dry_run:
            encode_all_outputs(ctxs, sh)
            n_recs = sum(b["n_recs"] for b in sh.batches)
        enc = dec = None
        iso = {}  # isolated launches (one context, one call at a time): the roofline's denominator --
        # with calls in flight, a launch shares the GPU with the other context's kernels
        n_iso = max(3, len(sh.batches))
        if want_enc and not args.dry_run:
            enc = timed(Pipe(ctxs, "encode"), sh, args.steps, args.warmup, barrier, sync, dist)
            ip = Pipe(ctxs[:1], "encode")
            iso["encode"] = (timed(ip, sh, n_iso, 0, barrier, sync, dist)[1], list(ip.tms))
            encode_all_outputs(ctxs, sh)  # the timed calls alternate contexts: refresh every output
        if want_dec and not args.dry_run:
            dec = timed(Pipe(ctxs, "decode"), sh, args.steps, args.warmup, barrier, sync, dist)
            ip = Pipe(ctxs[:1], "decode")
            iso["decode"] = (timed(ip, sh, n_iso, 0, barrier, sync, dist)[1], list(ip.tms))
        pin = rank == 0
        secs = 0 if args.no_cpu else (cpu_secs if rank == 0 else 2.0)
        chk = check_shard(ctx, orc, sh, secs, dec is not None, pin, args.dry_run) if secs > 0 else None
        verdicts = gather({"rank": rank, "first": first, "n": n, "check": chk})
        units_all = sh.bases * world * args.steps
        par = {"ranks": world, "encode_bit_exact_all_ranks": all(v["check"]["encode_ok"] for v in verdicts)
               if chk else None,
               "reads_checked_per_rank": [v["check"]["reads_checked"] for v in verdicts] if chk else None,
               "shards": [[v["first"], v["n"]] for v in verdicts]}
        cpu = None
        if chk and rank == 0 and not args.no_cpu:
            cv = chk["reads_checked"] * L / chk["cpu_encode_s"] / 1e6
            avail = nt.host_threads()
            cpu = {"value": round(cv, 3), "unit": "Mbases/s", "cores": 1, "kind": "port",
                   "sample": f"{chk['reads_checked']} reads ({chk['reads_checked'] * L} bases) from the start of "
                             f"each batch, faithful C oracle (oracle/ntcomp_oracle.c) on one pinned core "
                             f"({chk['core']}) of {os.cpu_count()}" +
                             (f"; rank 0 of {world}, while the other ranks check their own samples" if world > 1
                              else ""),
                   "cpu_model": cpu_model(), "logical_cpus": os.cpu_count(), "cpus_available": avail,
                   "cpus_available_note": "min(affinity mask, cgroup v2 CPU quota): the CPUs this process may use"}
            if world == 1:
                av, an = cpu_all_cores(orc, sh, chk["spans"], avail)
                cpu["all_cores"] = {"value": round(av, 3), "unit": "Mbases/s", "cores": avail, "kind": "port",
                                    "sample": f"the same {an} reads, read-sharded over {avail} threads of the "
                                              f"reentrant C oracle (wall clock)"}
        wl_c = (f"C{kk}: {n} x {L}bp synthetic reads per GPU ({args.err_ppm / 1e4:g}% subst, 50% revcomp) vs SBWT "
                f"of a {args.genome_bp / 1e6:g} Mbp synthetic genome (+revcomp), k={kk}"
                + (f"; {world} GPUs x {n} = {world * n} reads" if world > 1 else ""))
        cfg = dict(base_cfg, k=kk, workload=wl_c, index_nodes=index.n, records_per_gpu=n_recs,
                   suffix_table_u=None if args.dry_run else ctx.get_option("tab_u"),
                   workspace_gb_per_context=None if args.dry_run else _gb(_opt(ctx, "workspace_bytes")),
                   spill_reruns=None if args.dry_run else _opt(ctx, "spill_reruns"),
                   index_build=build_info.get(label),
                   parallelism=f"reads sharded over {world} GPU(s), index replicated, no collective",
                   inflight=len(ctxs) or None)
        out = {}
        if enc is not None:
            el, kms = enc
            b0 = sh.batches[0]
            units = [b["n"] for b in sh.batches]
            kavg, kmin = launch_ms(iso["encode"][0], units, b0["n"])
            call_ms = launch_ms(iso["encode"][1], units, b0["n"])[0]
            kin = launch_ms(kms, units, b0["n"])[0]
            rl = roofline("k_ms4", kavg, kmin, b0["n"], "read", pmc, pmc_note, f"C{kk}",
                          {"kernel_ms_inflight": round(kin, 4), "isolated_launches": len(iso["encode"][0]),
                           "reference_work_avoided": round(
                              b0["bases"] * (1 + 2 * 64) / (kavg / 1e3) / 1e9 / HBM_PEAK_GBPS, 3),
                           "reference_work_note": "SURVEY 8(d) B_enc (1 B + two 64 B rank lines per base) / "
                                                  "kernel time / peak: the reference algorithm's bytes this "
                                                  "kernel's suffix table and path runs avoid; not a roofline"})
            rl["io_floor"] = io_floor(b0["bases"], 8 * n_recs * b0["n"] / n, call_ms)
            rl["algorithmic"] = alg_encode(alg, f"C{kk}", b0["n"], kavg, rl.get("traffic"))
            if world > 1:
                rl["aggregate"] = aggregate_roofline(gather({"traffic": rl.get("traffic"), "kernel_ms": kavg}), world)
            metric = METRIC if kk == 91 else METRIC.replace("k=91", f"k={kk}")
            out.update({"metric": metric, "value": round(units_all / el / 1e6, 2), "unit": "Mbases/s",
                        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                        "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
                        "scaling": "weak", "vs_baseline": None, "dtype": "u32",
                        "data": "synthetic (seeded; reads regenerate per shard)", "config": cfg,
                        "roofline": rl, "cpu_baseline": cpu, "parity": par,
                        "kernel_ms_per_step": round(sum(kms) / args.steps, 3)})
            if cpu:
                cpu["speedup_gpu_vs_cpu"] = round(out["value"] / cpu["value"], 1)
                if "all_cores" in cpu:
                    cpu["all_cores"]["speedup_gpu_vs_cpu"] = round(out["value"] / cpu["all_cores"]["value"], 1)
        if dec is not None:
            el, kms = dec
            b0 = sh.batches[0]
            units = [b["bases"] for b in sh.batches]
            kavg, kmin = launch_ms(iso["decode"][0], units, b0["bases"])
            call_ms = launch_ms(iso["decode"][1], units, b0["bases"])[0]
            kin = launch_ms(kms, units, b0["bases"])[0]
            dcpu = None
            if chk and chk["cpu_decode_s"] > 0 and rank == 0:
                dcpu = {"value": round(chk["cpu_decode_bases"] / chk["cpu_decode_s"] / 1e6, 3), "unit": "Mbases/s",
                        "cores": 1, "kind": "port",
                        "sample": f"oracle decode of {chk['cpu_decode_bases']} bases of oracle records, one pinned core"}
            drl = roofline("k_dec_rec", kavg, kmin, b0["bases"], "base", pmc, pmc_note, f"D{kk}",
                           {"kernel_ms_inflight": round(kin, 4), "isolated_launches": len(iso["decode"][0])},
                           working_set=index.n * 32)
            drl["io_floor"] = io_floor(8 * n_recs * b0["n"] / n, b0["bases"], call_ms)
            drl["algorithmic"] = alg_decode(records_of(ctx, b0, 0, b0["n"])[0], b0["bases"], kavg, drl.get("traffic"))
            if world > 1:
                drl["aggregate"] = aggregate_roofline(gather({"traffic": drl.get("traffic"), "kernel_ms": kavg}),
                                                      world)
            d = {"metric": f"decode Mbases/sec at k={kk}, 150bp reads (output bases), MI355X; bit-exact vs CPU",
                 "value": round(units_all / el / 1e6, 2), "unit": "Mbases/s",
                 "ms_per_step": round(el / args.steps * 1e3, 3),
                 "config": {"workload": f"D{kk}: decode of the C{kk} records ({n_recs} records, {n} reads per GPU) "
                                        f"-> bases via the inverse-SBWT walk, k={kk}"},
                 "roofline": drl, "cpu_baseline": dcpu,
                 "parity": {"round_trip_exact_all_ranks": all(v["check"]["decode_ok"] for v in verdicts)
                            if chk else None, "bases_checked_per_rank": n * L if chk else None},
                 "kernel_ms_per_step": round(sum(kms) / args.steps, 3)}
            if dcpu:
                d["cpu_baseline"]["speedup_gpu_vs_cpu"] = round(d["value"] / dcpu["value"], 1)
            if out:
                out["decode"] = d
            else:
                out.update({"metric": d["metric"], "value": d["value"], "unit": "Mbases/s", "n_gpus": world,
                            "steps": args.steps, "warmup": args.warmup, "ms_per_step": d["ms_per_step"],
                            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
                            "data": "synthetic (seeded; reads regenerate per shard)",
                            "config": dict(cfg, workload=d["config"]["workload"]), "roofline": d["roofline"],
                            "cpu_baseline": d["cpu_baseline"], "parity": dict(par, **d["parity"])})
        if args.dry_run:
            out.update({"metric": METRIC, "value": None, "unit": "Mbases/s", "n_gpus": world, "dry_run": True,
                        "config": cfg, "parity": par})
        if not args.dry_run:
            sh.free(ctx)
        return out

    # ---- C91 encode / D91 decode -------------------------------------------------
    if "encode" in configs or "decode" in configs:
        line.update(c_block(k, "encode" in configs, "decode" in configs, "C",
                            args.cpu_seconds if world == 1 else args.cpu_seconds / 2))
    # ---- C31: BASELINE configs[1], the same reads at k = 31 -----------------------------
    if "c31" in configs:
        c31 = c_block(31, True, False, "C31_", 4.0)
        if line:
            line["c31"] = c31
        else:
            line.update(c31)

    # ---- S91: strain collection ------------------------------------------------------
    if "strains" in configs:
        strains = nt.synth_strains(genome, 3, args.strains, args.strain_snp_ppm)
        texts = [genome] + [strains[i] for i in range(args.strains)]
        # S91 calls in flight (--strain-inflight): round 5 measured two 3 % slower than one (k_ms4
        # at 0.89 of the line rate then, two persistent grids only competing); round 6, with the
        # linked cover, 131.3-133.9 against 130.7-132.4 Gbases/s (3 runs each, one box,
        # profiles/round6/ab_strain_inflight/): within the noise, one stays the default
        n_s = max(1, min(args.strain_inflight, len(ctxs) or 1))
        index = setup_index(texts, "S", n_s)
        sctx = ctxs[:n_s]
        coll = np.concatenate(texts)
        ns = args.strain_reads if world == 1 else min(args.strain_reads, n)
        fs, ns = shard_mod.read_range(rank, world, ns)
        sh = Shard(nt, ctx, coll, fs, ns, L, args.err_ppm, args.batch_reads, nthreads, args.dry_run,
                   args.presort, n_out=len(sctx))
        orc = OracleIndex(index.n, k, index.rows, index.C, index.lcs)
        s = {"config": {"workload": f"S{k}: {ns} x {L}bp reads ({args.err_ppm / 1e4:g}% subst, 50% revcomp) drawn "
                                    f"from a collection of the {args.genome_bp / 1e6:g} Mbp genome + {args.strains} "
                                    f"strains at {args.strain_snp_ppm / 1e4:g}% substitutions, SBWT k={k} (+revcomp)",
                        "index_nodes": index.n}}
        if not args.dry_run:
            encode_all_outputs(sctx, sh)
            s["config"]["records_per_gpu"] = sum(b["n_recs"] for b in sh.batches)
            s["config"]["suffix_table_u"] = ctx.get_option("tab_u")
            s["config"]["n_paths"] = ctx.get_option("n_paths")
            s["config"]["scan_filter"] = bool(ctx.get_option("filter"))
            s["config"]["joint_runs"] = bool(ctx.get_option("joint"))
            s["config"]["entry_slots_per_read"] = 4 + (_opt(ctx, "ent_slots") or 0)
            s["config"]["index_build"] = build_info.get("S")
            pe = Pipe(sctx, "encode")
            el, kms = timed(pe, sh, args.steps, args.warmup, barrier, sync, dist)
            s["config"]["workspace_gb_per_context"] = _gb(_opt(ctx, "workspace_bytes"))
            s["config"]["spill_reruns"] = _opt(ctx, "spill_reruns")
            b0 = sh.batches[0]
            units = [b["n"] for b in sh.batches]
            kavg, kmin = launch_ms(kms, units, b0["n"])
            srecs = s["config"]["records_per_gpu"]
            srl = roofline("k_ms4", kavg, kmin, b0["n"], "read", pmc, pmc_note, f"S{k}")
            srl["io_floor"] = io_floor(b0["bases"], 8 * srecs * b0["n"] / ns, launch_ms(pe.tms, units, b0["n"])[0])
            srl["algorithmic"] = alg_encode(alg, f"S{k}", b0["n"], kavg, srl.get("traffic"))
            s.update(value=round(sh.bases * world * args.steps / el / 1e6, 2), unit="Mbases/s",
                     ms_per_step=round(el / args.steps * 1e3, 3), roofline=srl)
            pd = Pipe(sctx, "decode")
            el, kms = timed(pd, sh, args.steps, args.warmup, barrier, sync, dist)
            units = [b["bases"] for b in sh.batches]
            kavg, kmin = launch_ms(kms, units, b0["bases"])
            sdrl = roofline("k_dec_rec", kavg, kmin, b0["bases"], "base", pmc, pmc_note, f"SD{k}",
                            working_set=index.n * 32)
            sdrl["io_floor"] = io_floor(8 * srecs * b0["n"] / ns, b0["bases"], launch_ms(pd.tms, units, b0["bases"])[0])
            sdrl["algorithmic"] = alg_decode(records_of(ctx, b0, 0, b0["n"])[0], b0["bases"], kavg, sdrl.get("traffic"))
            s["decode"] = {"value": round(sh.bases * world * args.steps / el / 1e6, 2), "unit": "Mbases/s",
                           "ms_per_step": round(el / args.steps * 1e3, 3), "roofline": sdrl}
        secs = 0 if args.no_cpu else 3.0
        chk = check_shard(ctx, orc, sh, secs, not args.dry_run, False, args.dry_run) if secs > 0 else None
        vs = gather(chk)
        s["parity"] = {"encode_bit_exact_all_ranks": all(v["encode_ok"] for v in vs) if chk else None,
                       "reads_checked_per_rank": [v["reads_checked"] for v in vs] if chk else None,
                       "round_trip_exact_all_ranks": all(v["decode_ok"] for v in vs) if chk and not args.dry_run
                       else None}
        if not args.dry_run:
            sh.free(ctx)
        if line:
            line["strains"] = s
        else:
            line.update({"metric": METRIC, "value": s.get("value"), "unit": "Mbases/s", "n_gpus": world,
                         "steps": args.steps, "warmup": args.warmup, "ms_per_step": s.get("ms_per_step"),
                         "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
                         "data": "synthetic (seeded)", "config": dict(base_cfg, **s["config"]),
                         "roofline": s.get("roofline"), "cpu_baseline": None, "parity": s["parity"],
                         "decode": s.get("decode")})

    if rank == 0:
        line["wall_s"] = round(time.time() - t_start, 1)
        print(json.dumps(line), flush=True)
    for c in ctxs:
        c.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
