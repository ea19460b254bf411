"""Multi-GPU sharding of the encode/decode path.

Reads are independent (the reference encodes them one by one, src/main.rs:162-173), so
a job splits into contiguous read ranges, one per rank, with the index replicated on
every GPU and no data-path collective.  torch.distributed only provides the barrier
around the timed region and the max of the per-rank times (one process per GPU; backend
"nccl" = RCCL on a GPU node, "gloo" in the CPU tests).
"""


def read_range(rank, world, reads_per_rank):
    """Weak scaling: rank r owns reads [r * reads_per_rank, (r + 1) * reads_per_rank)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world of {world}")
    first = rank * reads_per_rank
    return first, reads_per_rank


def split_range(rank, world, n_reads):
    """Strong scaling: n_reads split into world contiguous ranges differing by <= 1 read."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world of {world}")
    base, extra = divmod(n_reads, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def max_over_ranks(value, dist=None):
    """The job's time is its slowest rank's (one all-reduce of a float, not on the data path)."""
    if dist is None:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
