"""bench.py's multi-GPU launch on CPU (--dry-run stops at the GPU boundary): `bench.py
--gpus 2` outside torch.distributed.run starts a 2-rank child job itself, each rank takes its
shard (weak scaling, data independent of the sharding, main.rs:152,162-173), checks an
oracle sample of its own reads, and rank 0 prints one line carrying every rank's verdict."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                       timeout=600, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout  # stdout: the JSON line alone
    return json.loads(lines[0]), p.stderr


def test_bench_spawns_ranks_without_torchrun():
    line, err = _run(["--gpus", "2", "--dry-run", "--configs", "encode", "--reads-per-gpu", "4000",
                      "--batch-reads", "1500", "--genome-bp", "200000"])
    assert "[launcher] 2 ranks" in err
    assert line["n_gpus"] == 2 and line["dry_run"] is True
    par = line["parity"]
    assert par["ranks"] == 2 and par["shards"] == [[0, 4000], [4000, 4000]]
    assert par["encode_bit_exact_all_ranks"] is True
    assert all(c > 0 for c in par["reads_checked_per_rank"])
    assert "[rank 1] C91: reads 4000..8000 in 3 batch(es)" in err


def test_bench_default_sizing_is_c91x8_per_gpu_at_n_gt_1():
    sys.path.insert(0, REPO)
    import bench
    a = bench.parse_args(["--gpus", "8"])
    assert a.reads_per_gpu is None  # resolved per world size in main(): 25M at N > 1, 10M at N = 1
    src = open(os.path.join(REPO, "bench.py")).read()
    assert "10_000_000 if world == 1 else 25_000_000" in src
