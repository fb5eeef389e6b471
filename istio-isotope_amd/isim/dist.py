"""Multi-GPU sharding of the trace space and the stats merge.

Traces are independent, so a node-wide run partitions trace
ids: rank r of a world of N, at step s with B traces per rank, owns
[(s*N + r)*B, (s*N + r + 1)*B).  Philox counters are keyed by the global
trace id, so results are identical for any N.  The only exchange is the
merge of the per-rank stats buffers: SUM over the u64 counters/histograms
plus MAX over the latency extrema (stored as [~min, max]).

Two implementations of the merge:
  * ``Multi`` — libisim's own RCCL communicator (include/isim.h isim_multi_*,
    csrc/multi.hip): what a Go host calls through cgo; bench.py uses it.
  * ``merge_stats`` — the same merge through torch.distributed (RCCL with the
    "nccl" backend, gloo in the CPU tests).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

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


def stats_merge(handler, dst: np.ndarray, src: np.ndarray) -> np.ndarray:
    """dst += src under the merge rules, in libisim (isim_stats_merge)."""
    assert dst.dtype == np.uint64 and src.dtype == np.uint64 and dst.flags.c_contiguous
    assert dst.size >= handler.stats_words and src.size >= handler.stats_words
    src = np.ascontiguousarray(src)
    native.check(native.load().isim_stats_merge(handler._h, dst.ctypes.data, src.ctypes.data))
    return dst


def des_table_merge(handler, dst: np.ndarray, src: np.ndarray) -> np.ndarray:
    """dst += src for DES tables (ISIM_DES_MAX_WAIT by MAX), isim_des_table_merge."""
    assert dst.dtype == np.uint64 and src.dtype == np.uint64 and dst.flags.c_contiguous
    words = int(handler.info.n_reachable) * native.DES_ROW_WORDS
    assert dst.size >= words and src.size >= words
    src = np.ascontiguousarray(src)
    native.check(native.load().isim_des_table_merge(handler._h, dst.ctypes.data, src.ctypes.data))
    return dst


def _ptrs(xs: Optional[Sequence[int]], n: int):
    arr = (C.c_void_p * n)()
    if xs is None:
        return None
    for i, x in enumerate(xs):
        arr[i] = x or None
    return arr


class Multi:
    """An RCCL communicator of libisim with one or more local devices."""

    def __init__(self, handle: C.c_void_p):
        self._m = handle
        n, loc, first = C.c_int(), C.c_int(), C.c_int()
        native.check(native.load().isim_multi_info(self._m, C.byref(n), C.byref(loc), C.byref(first)))
        self.n_ranks, self.n_local, self.first_rank = n.value, loc.value, first.value

    @staticmethod
    def precheck(device: int) -> None:
        """isim_multi_precheck: RCCL loads and `device` can be selected (local, no communication)."""
        native.check(native.load().isim_multi_precheck(device))

    @staticmethod
    def get_id() -> bytes:
        mid = native.MultiId()
        native.check(native.load().isim_multi_get_id(C.byref(mid)))
        return bytes(C.string_at(C.addressof(mid), 128))

    @classmethod
    def init_rank(cls, id_bytes: bytes, n_ranks: int, rank: int, device: int) -> "Multi":
        mid = native.MultiId()
        C.memmove(C.addressof(mid), bytes(id_bytes), 128)
        out = C.c_void_p()
        native.check(native.load().isim_multi_init_rank(C.byref(mid), n_ranks, rank, device, C.byref(out)))
        return cls(out)

    @classmethod
    def init_all(cls, devices: Sequence[int]) -> "Multi":
        arr = (C.c_int * len(devices))(*devices)
        out = C.c_void_p()
        native.check(native.load().isim_multi_init_all(arr, len(devices), C.byref(out)))
        return cls(out)

    def close(self):
        if self._m is not None and self._m.value and native._lib is not None:
            native._lib.isim_multi_free(self._m)
        self._m = None

    def __del__(self):
        self.close()

    def abort(self):
        """isim_multi_abort: peers' collectives on this communicator fail (ECOMM) instead of waiting."""
        if self._m is not None and self._m.value:
            native.check(native.load().isim_multi_abort(self._m))

    def allreduce_stats(self, handler, d_stats: Sequence[int], streams: Optional[Sequence[int]] = None):
        """In-place merge of the local devices' stats buffers (device pointers)."""
        native.check(native.load().isim_stats_allreduce_device(
            handler._h, self._m, _ptrs(d_stats, self.n_local), _ptrs(streams, self.n_local)))

    def allreduce_des_table(self, handler, d_tables: Sequence[int], streams: Optional[Sequence[int]] = None):
        native.check(native.load().isim_des_table_allreduce_device(
            handler._h, self._m, _ptrs(d_tables, self.n_local), _ptrs(streams, self.n_local)))

    def serve(self, handler, trace_begin: int, n_per_rank: int, records: bool = True):
        """Synchronous sharded batch (isim_serve_multi): (local records or None, merged stats)."""
        from .sim import REC_DTYPE
        stats = handler.new_stats()
        recs = np.zeros(self.n_local * n_per_rank, REC_DTYPE) if records else None
        native.check(native.load().isim_serve_multi(
            handler._h, self._m, trace_begin, n_per_rank,
            recs.ctypes.data if records and n_per_rank else None, stats.ctypes.data))
        return recs, stats
