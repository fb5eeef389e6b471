"""Multi-GPU sharding of the trace space (one process per GPU).

Traces are independent, so a node-wide run partitions trace
ids: rank r of a world of N, at step s with B traces per rank, owns
[(s*N + r)*B, (s*N + r + 1)*B).  Philox counters are keyed by the global
trace id, so results are identical for any N.  The only exchange is the
merge of the per-rank stats buffers: one all-reduce SUM over the u64
counters/histograms (RCCL over xGMI with the "nccl" backend; gloo in the CPU
tests) plus a 2-word MAX for the latency extrema (stored as [~min, max]).
"""
from __future__ import annotations

from . import native


def shard_begin(rank: int, world: int, step: int, batch: int) -> int:
    return (step * world + rank) * batch


def merge_stats(stats, group=None):
    """In-place merge of an int64 torch tensor laid out as isim stats words."""
    import torch.distributed as dist
    lo, hi = native.ST_NOT_MIN_LATENCY, native.ST_MAX_LATENCY + 1
    # The extrema words are u64 ([~min, max]); flipping the sign bit maps
    # unsigned order onto int64 order, so a signed MAX merges them.
    flip = -(1 << 63)
    ext = stats[lo:hi] ^ flip
    dist.all_reduce(stats, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(ext, op=dist.ReduceOp.MAX, group=group)
    stats[lo:hi] = ext ^ flip
    return stats
