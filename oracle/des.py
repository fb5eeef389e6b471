"""ctypes driver for the DES oracle ``des_oracle.c`` (test infrastructure only):
the sequential event-driven restatement of isim DES semantics v1 (DESIGN.md
§10) that the GPU DES is checked against, and the cpu_baseline of
``bench.py --config c5`` (kind "port").
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from .executor import OracleGraph, _Graph, _Params, check_acyclic, lib
from .executor_py import SimGraph, SimParams

DES_ROW = 72  # isim.h ISIM_DES_ROW_WORDS


class _Des(C.Structure):
    _fields_ = [("mean_interarrival_ns", C.c_uint64), ("replicas", C.c_void_p)]


def _bind():
    L = lib()
    if not getattr(L, "_des_bound", False):
        L.isim_oracle_des_run.argtypes = [C.POINTER(_Graph), C.POINTER(_Params), C.POINTER(_Des), C.c_uint64,
                                          C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
        L.isim_oracle_des_run.restype = C.c_int
        L.isim_oracle_des_stats_words.argtypes = [C.c_int32, C.c_int32]
        L.isim_oracle_des_stats_words.restype = C.c_uint64
        L.isim_oracle_des_exp_q24.argtypes = [C.c_uint32]
        L.isim_oracle_des_exp_q24.restype = C.c_uint64
        L.isim_oracle_des_ln_table.argtypes = [C.c_void_p]
        L._des_bound = True
    return L


def ln_table() -> np.ndarray:
    out = np.zeros(257, np.int64)
    _bind().isim_oracle_des_ln_table(out.ctypes.data)
    return out


def exp_q24(u: int) -> int:
    return int(_bind().isim_oracle_des_exp_q24(u & 0xFFFFFFFF))


def exp_q24_py(u: int) -> int:
    """Pure-Python restatement of the same fixed-point inverse CDF."""
    tab = [round(math.log1p(i / 256.0) * 16777216.0) for i in range(257)]
    w = (u >> 8) + 1
    e = w.bit_length() - 1
    f = (w << (24 - e)) & 0xFFFFFF
    idx, rem = f >> 16, f & 0xFFFF
    lnm = tab[idx] + (((tab[idx + 1] - tab[idx]) * rem) >> 16)
    return 24 * 11629080 - (e * 11629080 + lnm)


def run(sg: SimGraph, params: SimParams, entry: int, trace_begin: int, n_traces: int, mean_interarrival_ns: int,
        records: bool = True, og: OracleGraph = None):
    """Returns (records [n,2] u64 or None, stats u64 (oracle layout), des rows [n_services][72])."""
    check_acyclic(sg, entry)
    og = og or OracleGraph(sg, params)
    L = _bind()
    reps = np.array([max(1, s.num_replicas) for s in sg.g.services] or [1], np.int32)
    d = _Des(int(mean_interarrival_ns), reps.ctypes.data)
    stats = np.zeros(L.isim_oracle_des_stats_words(og.n_services, og.n_sites), np.uint64)
    des = np.zeros((max(1, og.n_services), DES_ROW), np.uint64)
    recs = np.zeros((n_traces, 2), np.uint64) if records else None
    p = _Params(params.seed & ((1 << 64) - 1), params.error_mode, entry)
    rc = L.isim_oracle_des_run(C.byref(og.g), C.byref(p), C.byref(d), trace_begin, n_traces,
                               recs.ctypes.data if records else None, stats.ctypes.data, des.ctypes.data)
    if rc != 0:
        raise MemoryError("DES oracle run failed")
    return recs, stats, des[:og.n_services]
