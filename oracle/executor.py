"""ctypes driver for the C oracle ``isim_oracle.c`` (test infrastructure only).

Packs an ``executor_py.SimGraph`` into the oracle's plain arrays and runs
``isim_oracle_run`` over a trace range with OpenMP.  Also the ``cpu_baseline``
leg of bench.py (kind "port": the Go reference cannot be built here).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from .executor_py import MODE_A, SimGraph, SimParams, N_LOG2, N_PROM

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

ST_HDR = 8
ST_PROM = ST_HDR
ST_LOG2 = ST_PROM + 2 * N_PROM
ST_SVC = ST_LOG2 + 2 * N_LOG2
SVC_DUR_WORDS = 2 * N_PROM + 2


class _Cmd(C.Structure):
    _fields_ = [("kind", C.c_int32), ("site", C.c_int32), ("k", C.c_int32),
                ("sub_off", C.c_int32), ("sub_len", C.c_int32), ("pad", C.c_int32),
                ("sleep_ns", C.c_int64)]


class _Graph(C.Structure):
    _fields_ = [("n_services", C.c_int32), ("n_sites", C.c_int32),
                ("thr", C.c_void_p), ("step_off", C.c_void_p), ("step_len", C.c_void_p),
                ("cmds", C.c_void_p), ("site_callee", C.c_void_p), ("site_prob", C.c_void_p),
                ("site_hop", C.c_void_p)]


class _Params(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("error_mode", C.c_int32), ("entry", C.c_int32)]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = C.CDLL(_LIB_PATH)
        _lib.isim_oracle_run.argtypes = [C.POINTER(_Graph), C.POINTER(_Params), C.c_uint64,
                                         C.c_uint64, C.c_void_p, C.c_void_p, C.c_int]
        _lib.isim_oracle_run.restype = C.c_int
        _lib.isim_oracle_stats_words.argtypes = [C.c_int32, C.c_int32]
        _lib.isim_oracle_stats_words.restype = C.c_uint64
        _lib.isim_oracle_philox.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    return _lib


class CycleError(Exception):
    pass


def check_acyclic(sg: SimGraph, entry: int) -> None:
    """EXT (F12): a cycle reachable from the entry would recurse forever in
    the reference; the oracle refuses it like the product does (ECYCLE)."""
    WHITE, GREY, BLACK = 0, 1, 2
    color = [WHITE] * len(sg.g.services)
    callees = [[] for _ in sg.g.services]
    for caller, callee, _, _ in sg.sites:
        callees[caller].append(callee)
    stack = [(entry, iter(callees[entry]))]
    color[entry] = GREY
    while stack:
        node, it = stack[-1]
        nxt = next(it, None)
        if nxt is None:
            color[node] = BLACK
            stack.pop()
        elif color[nxt] == GREY:
            raise CycleError(f"call cycle through service {sg.g.services[nxt].name!r}")
        elif color[nxt] == WHITE:
            color[nxt] = GREY
            stack.append((nxt, iter(callees[nxt])))


class OracleGraph:
    def __init__(self, sg: SimGraph, params: SimParams):
        self.sg = sg
        n = len(sg.g.services)
        cmds = []
        step_off = np.zeros(n, np.int32)
        step_len = np.zeros(n, np.int32)
        # top-level steps of each service are contiguous; concurrent
        # sub-commands are appended after all top-level steps.
        pending = []
        for s in range(n):
            step_off[s] = len(cmds)
            step_len[s] = len(sg.steps[s])
            for st in sg.steps[s]:
                if st[0] == "sleep":
                    cmds.append([0, 0, 0, 0, 0, st[1]])
                elif st[0] == "call":
                    cmds.append([1, st[1], st[2], 0, 0, 0])
                else:
                    cmds.append([2, 0, 0, 0, len(st[1]), 0])
                    pending.append((len(cmds) - 1, st[1]))
        for idx, subs in pending:
            cmds[idx][3] = len(cmds)
            for x in subs:
                if x[0] == "sleep":
                    cmds.append([0, 0, 0, 0, 0, x[1]])
                else:
                    cmds.append([1, x[1], x[2], 0, 0, 0])
        arr = (_Cmd * max(1, len(cmds)))()
        for i, c in enumerate(cmds):
            arr[i].kind, arr[i].site, arr[i].k, arr[i].sub_off, arr[i].sub_len = c[:5]
            arr[i].sleep_ns = c[5]
        self.cmds = arr
        self.thr = np.array(sg.thr, np.uint64)
        self.step_off, self.step_len = step_off, step_len
        m = len(sg.sites)
        self.site_callee = np.array([x[1] for x in sg.sites] or [0], np.int32)
        self.site_prob = np.array([x[3] for x in sg.sites] or [0], np.int32)
        hops = [sg.hop_cost(i, params) for i in range(m)]
        if any(h >= (1 << 63) for h in hops):
            raise OverflowError("hop cost overflows int64")
        self.site_hop = np.array(hops or [0], np.uint64)
        self.g = _Graph(n, m, self.thr.ctypes.data, step_off.ctypes.data, step_len.ctypes.data,
                        C.addressof(arr), self.site_callee.ctypes.data, self.site_prob.ctypes.data,
                        self.site_hop.ctypes.data)
        self.n_services, self.n_sites = n, m


def run(sg: SimGraph, params: SimParams, entry: int, trace_begin: int, n_traces: int,
        records: bool = True, n_threads: int = 0, og: OracleGraph = None):
    """Returns (records ndarray [n,2] u64 or None, stats ndarray u64)."""
    check_acyclic(sg, entry)
    og = og or OracleGraph(sg, params)
    L = lib()
    words = L.isim_oracle_stats_words(og.n_services, og.n_sites)
    stats = np.zeros(words, np.uint64)
    recs = np.zeros((n_traces, 2), np.uint64) if records else None
    p = _Params(params.seed & ((1 << 64) - 1), params.error_mode, entry)
    rc = L.isim_oracle_run(C.byref(og.g), C.byref(p), trace_begin, n_traces,
                           recs.ctypes.data if records else None, stats.ctypes.data, n_threads)
    if rc != 0:
        raise MemoryError("oracle run failed")
    return recs, stats


def split_stats(stats: np.ndarray, n_services: int, n_sites: int) -> dict:
    return {
        "n_traces": int(stats[0]), "sum_latency": int(stats[1]), "sum_hops": int(stats[2]),
        "sum_err_hops": int(stats[3]), "n_500": int(stats[4]),
        "min_latency": int(stats[5]), "max_latency": int(stats[6]),
        "lat_prom": stats[ST_PROM:ST_PROM + 2 * N_PROM].reshape(2, N_PROM),
        "lat_log2": stats[ST_LOG2:ST_LOG2 + 2 * N_LOG2].reshape(2, N_LOG2),
        "svc_calls": stats[ST_SVC:ST_SVC + n_services],
        "svc_errs": stats[ST_SVC + n_services:ST_SVC + 2 * n_services],
        "site_calls": stats[ST_SVC + 2 * n_services:ST_SVC + 2 * n_services + n_sites],
        # [n_services][68]: duration buckets [code][33] then sums [code] (ns)
        "svc_dur": stats[ST_SVC + 2 * n_services + n_sites:
                         ST_SVC + 2 * n_services + n_sites + SVC_DUR_WORDS * n_services].reshape(n_services,
                                                                                               SVC_DUR_WORDS),
    }


def philox(ctr, key):
    L = lib()
    c = np.array(ctr, np.uint32)
    k = np.array(key, np.uint32)
    out = np.zeros(4, np.uint32)
    L.isim_oracle_philox(c.ctypes.data, k.ctypes.data, out.ctypes.data)
    return tuple(int(x) for x in out)


__all__ = ["run", "split_stats", "OracleGraph", "check_acyclic", "CycleError", "philox",
           "MODE_A", "build"]
