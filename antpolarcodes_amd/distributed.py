"""Multi-GPU sharding: independent codewords, no data-path collective.

Frames are split into contiguous shards, one per rank (= one GPU, one process);
each rank owns its own decoder plan and decodes its shard.  Only host-side
bookkeeping crosses ranks (timing max, frame / error counts), through
torch.distributed on the host (gloo) -- RCCL is never needed on the data path.
"""
import os


def world():
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_bounds(total, world_size, rank):
    """Contiguous shard [lo, hi) of `total` frames for `rank`; the remainder goes to
    the last rank."""
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError("bad rank / world size")
    base = total // world_size
    lo = base * rank
    hi = total if rank == world_size - 1 else lo + base
    return lo, hi


def reduce_stats(stats, group=None):
    """Combine per-rank host statistics: times by max, counts by sum.
    `stats` maps name -> (value, "max"|"sum").  Returns name -> global value."""
    import torch
    import torch.distributed as dist
    out = {}
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return {k: v for k, (v, _) in stats.items()}
    for k, (v, how) in sorted(stats.items()):
        t = torch.tensor([float(v)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX if how == "max" else dist.ReduceOp.SUM, group=group)
        out[k] = float(t.item())
    return out
