"""world_size-2 gloo run of the sharded encode path on CPU: each rank
generates its own read range (data independent of the sharding), encodes it (kernel
algorithm via the test-only emulator, checked against the oracle), and the union over
ranks equals the single-process result; the timed region's max-over-ranks is a gloo
all-reduce.  No collective touches the data path -- the gathers below are test-only."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import ntcomp_amd as nt
from ntcomp_amd import shard

K, GENOME, PER_RANK, L = 31, 60_000, 300, 150


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _work(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from emu_lib import emu_encode
    from oracle_lib import OracleIndex
    genome = nt.synth_genome(7, GENOME)
    ix = nt.Index.build([genome.tobytes()], K, threads=1)
    first, n = shard.read_range(rank, world, PER_RANK)
    reads = nt.synth_reads(genome, 2, first, n, L, 10_000)
    offs = np.arange(0, n * L + 1, L, dtype=np.uint64)
    recs, roff = emu_encode(ix.n, K, ix.rows, ix.C, ix.lcs, reads, offs)
    exp, eoff = OracleIndex(ix.n, K, ix.rows, ix.C, ix.lcs).encode(reads, offs)
    ok = bool(np.array_equal(recs, exp) and np.array_equal(roff, eoff))
    dist.barrier()
    t = shard.max_over_ranks(1.0 + rank, dist)
    np.savez(os.path.join(outdir, f"r{rank}.npz"), reads=reads, recs=recs, roff=roff, ok=ok, t=t, first=first)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_encode_equals_unsharded(tmp_path, world):
    mp.start_processes(_work, args=(world, _free_port(), str(tmp_path)), nprocs=world, start_method="spawn")
    parts = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    assert all(bool(p["ok"]) for p in parts), "a rank's records differ from the oracle"
    assert all(float(p["t"]) == float(world) for p in parts), "max over ranks"
    assert [int(p["first"]) for p in parts] == [r * PER_RANK for r in range(world)]
    # data depends on the read index only: the union equals one unsharded generation
    genome = nt.synth_genome(7, GENOME)
    allreads = nt.synth_reads(genome, 2, 0, world * PER_RANK, L, 10_000)
    assert np.array_equal(np.concatenate([p["reads"] for p in parts]), allreads)
    from emu_lib import emu_encode
    ix = nt.Index.build([genome.tobytes()], K, threads=1)
    offs = np.arange(0, world * PER_RANK * L + 1, L, dtype=np.uint64)
    recs, roff = emu_encode(ix.n, K, ix.rows, ix.C, ix.lcs, allreads, offs)
    assert np.array_equal(np.concatenate([p["recs"] for p in parts]), recs)


def test_split_range_covers_every_read_once():
    for n in (0, 1, 7, 100, 1001):
        for world in (1, 2, 3, 8):
            got = [shard.split_range(r, world, n) for r in range(world)]
            assert sum(c for _, c in got) == n
            pos = 0
            for f, c in got:
                assert f == pos
                pos += c
    with pytest.raises(ValueError):
        shard.read_range(2, 2, 10)
