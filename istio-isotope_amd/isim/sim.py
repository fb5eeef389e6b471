"""Handler API: the simulated counterpart of isotope's srv.Handler.

    handler_from_service_graph_yaml(path, name, params)
        ~ srv.HandlerFromServiceGraphYAML(path, serviceName)   srv/graph.go:34-60
    Handler.serve(trace_begin, n_traces)
        ~ n_traces independent Handler.ServeHTTP requests        srv/handler.go:37-79
          (virtual time, on the GPU through libisim's walk kernel)
    Handler.serve_device(...)  — device pointers + HIP stream, no host sync
    Handler.fold(stats)        — per-service / per-call-site counters
                                 (prometheus.Record*, srv/prometheus/handler.go:87-106)
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import native
from .graph import ServiceGraph

REC_DTYPE = np.dtype([("latency_ns", "<u8"), ("hops", "<u4"), ("status_err", "<u4")])


@dataclass
class SimParams:
    """isim_params: hop-cost model + RNG seed + error mode."""
    seed: int = 0x15070BE
    hop_base_ns: int = 250_000
    req_ps_per_byte: int = 80
    resp_ps_per_byte: int = 80
    error_mode: int = native.MODE_A
    max_depth: int = 0
    flags: int = 0

    def to_c(self) -> native.Params:
        return native.Params(self.seed & ((1 << 64) - 1), self.hop_base_ns, self.req_ps_per_byte,
                             self.resp_ps_per_byte, self.error_mode, self.max_depth, self.flags, 0)


class Handler:
    def __init__(self, graph: ServiceGraph, service_name: Optional[str] = None,
                 params: Optional[SimParams] = None):
        self.graph = graph  # keeps the native graph alive
        self.params = params or SimParams()
        lib = native.load()
        out = C.c_void_p()
        p = self.params.to_c()
        name = service_name.encode("utf-8") if service_name is not None else None
        native.check(lib.isim_handler_create(graph.handle, name, C.byref(p), C.byref(out)))
        self._h = out
        info = native.HandlerInfo()
        native.check(lib.isim_handler_info_get(self._h, C.byref(info)))
        self.info = info
        self.slot_site = np.zeros(max(1, info.n_slots), np.int32)
        self.slot_callee = np.zeros(max(1, info.n_slots), np.int32)
        native.check(lib.isim_handler_slots(self._h, self.slot_site.ctypes.data,
                                            self.slot_callee.ctypes.data))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and native._lib is not None:
            native._lib.isim_handler_free(h)
            self._h = None

    def launch_info(self, device: int = 0) -> dict:
        li = native.LaunchInfo()
        native.check(native.load().isim_handler_launch_info(self._h, device, C.byref(li)))
        return {k: getattr(li, k) for k, _ in native.LaunchInfo._fields_}

    @property
    def stats_words(self) -> int:
        return int(self.info.stats_words)

    def new_stats(self) -> np.ndarray:
        return np.zeros(self.stats_words, np.uint64)

    def serve(self, trace_begin: int, n_traces: int, device: int = 0, records: bool = True):
        """Synchronous: returns (records structured array or None, stats u64 array)."""
        stats = self.new_stats()
        recs = np.zeros(n_traces, REC_DTYPE) if records else None
        native.check(native.load().isim_serve(
            self._h, device, trace_begin, n_traces,
            recs.ctypes.data if records and n_traces else None, stats.ctypes.data))
        return recs, stats

    def serve_device(self, trace_begin: int, n_traces: int, d_records: int, d_stats: int,
                     stream: int = 0) -> None:
        """Asynchronous on the current HIP device; pointers are device addresses."""
        native.check(native.load().isim_serve_device(
            self._h, trace_begin, n_traces, d_records or None, d_stats, stream or None))

    def fold(self, stats: np.ndarray) -> dict:
        n, m = self.info.n_services, self.info.n_sites
        svc_calls = np.zeros(max(1, n), np.uint64)
        svc_errs = np.zeros(max(1, n), np.uint64)
        site_calls = np.zeros(max(1, m), np.uint64)
        stats = np.ascontiguousarray(stats, dtype=np.uint64)
        native.check(native.load().isim_stats_fold(self._h, stats.ctypes.data, svc_calls.ctypes.data,
                                                   svc_errs.ctypes.data, site_calls.ctypes.data))
        d = decode_stats(stats)
        d["svc_calls"] = svc_calls[:n]
        d["svc_errs"] = svc_errs[:n]
        d["site_calls"] = site_calls[:m]
        dur = np.zeros((max(1, n), native.SVC_DUR_WORDS), np.uint64)
        rc = native.load().isim_stats_fold_durations(self._h, stats.ctypes.data, dur.ctypes.data)
        # per service: [code][33] duration bucket counts, then [code] sums (ns);
        # absent when a dynamic walk was created with FLAG_NO_SVC_DUR
        d["svc_dur"] = dur[:n] if rc == 0 else None
        return d


def decode_stats(stats: np.ndarray) -> dict:
    s = stats
    return {
        "n_traces": int(s[native.ST_N_TRACES]),
        "sum_latency": int(s[native.ST_SUM_LATENCY]),
        "sum_hops": int(s[native.ST_SUM_HOPS]),
        "sum_err_hops": int(s[native.ST_SUM_ERR_HOPS]),
        "n_500": int(s[native.ST_N_500]),
        "min_latency": int(~np.uint64(s[native.ST_NOT_MIN_LATENCY])) if s[native.ST_N_TRACES] else 0,
        "max_latency": int(s[native.ST_MAX_LATENCY]),
        "lat_prom": s[native.ST_PROM:native.ST_PROM + 2 * native.N_PROM].reshape(2, native.N_PROM),
        "lat_log2": s[native.ST_LOG2:native.ST_LOG2 + 2 * native.N_LOG2].reshape(2, native.N_LOG2),
    }


def handler_from_service_graph_yaml(path: str, service_name: Optional[str] = None,
                                    params: Optional[SimParams] = None) -> Handler:
    """srv.HandlerFromServiceGraphYAML (srv/graph.go:34-60); service_name None
    picks the first isEntrypoint service (the client's target)."""
    return Handler(ServiceGraph.from_yaml_file(path), service_name, params)
