"""Multi-GPU plumbing of the hot path: pairs shard with no exchange; the only
collective is one SUM all-reduce of the engine's flat u64 accumulator block (Stats x4,
FilterResult, polyX, insert-size histogram), plus a host-side union of the adapter-string maps
(FilterResult::merge semantics, reference src/filterresult.cpp:85-99).

One process per GPU; backend "nccl" is RCCL over xGMI on the GPU box, "gloo" in the CPU tests.
"""
import torch
import torch.distributed as dist


def shard(rank, world, pairs_per_rank):
    """Weak scaling: rank r owns the global pair indices [r*n, (r+1)*n)."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return rank * pairs_per_rank, pairs_per_rank


def reduce_accumulator(acc):
    """Sum the accumulator block over all ranks in place.  The engine's counters are u64; they
    travel as int64, whose two's-complement addition wraps exactly like u64 addition."""
    if acc.dtype != torch.int64:
        raise TypeError("accumulator must be an int64 view of the u64 block")
    if dist.is_initialized():  # (a world of one still runs the collective: bench.py --pg)
        dist.all_reduce(acc, op=dist.ReduceOp.SUM)
    return acc


def merge_adapter_counts(counts):
    """Union of per-rank adapter-string -> count dicts (FilterResult::merge)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return dict(counts)
    parts = [None] * dist.get_world_size()
    dist.all_gather_object(parts, dict(counts))
    out = {}
    for part in parts:
        for k, v in part.items():
            out[k] = out.get(k, 0) + v
    return out
