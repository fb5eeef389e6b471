"""Per-replica worker-pool DES (BASELINE config 5).

    d = DesHandler(handler, mean_interarrival_ns=6_000_000)
    recs, stats, table = d.serve(trace_begin, n_traces, device=0)
    rows = d.fold(table)      # [n_services][DES_ROW_WORDS]

The simulated counterpart of isotope under load: the client (Fortio's
open-loop mode) issues requests at exponential gaps; each replica of a
service (numReplicas, convert/pkg/graph/svc/service.go:30-31) is a FIFO queue
in front of one worker.  Statuses/hops/counters are the static walk's;
latencies and per-service durations include queueing.  Runs on the GPU
through libisim (isim_serve_des*); graphs outside the DES class raise
IsimError(EINVAL) with the reason.

Rows are 32-bit by default (times relative to each trace's arrival); a
device batch with a latency of 2^31 ns or more is not accumulated and is
counted in stats[ST_DES_RETRY] — rerun it with ``wide=True``.  ``serve``
does that itself.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import native
from .sim import REC_DTYPE, Handler


class DesHandler:
    def __init__(self, handler: Handler, mean_interarrival_ns: int):
        self.handler = handler
        self.params = native.DesParams(int(mean_interarrival_ns), 0, 0)
        info = native.DesInfo()
        native.check(native.load().isim_des_info_get(handler._h, C.byref(info)))
        self.info = info

    def last_batch(self) -> dict:
        """isim_des_last_batch: the item engine's last batch on this handler
        (passes over the rounds, host synchronisations, executed invocations)."""
        st = native.DesBatchStats()
        native.check(native.load().isim_des_last_batch(self.handler._h, C.byref(st)))
        return {"passes": int(st.passes), "syncs": int(st.syncs), "items": int(st.items)}

    @property
    def table_words(self) -> int:
        return int(self.info.table_rows) * native.DES_ROW_WORDS

    def new_table(self) -> np.ndarray:
        return np.zeros(max(1, self.table_words), np.uint64)

    def workspace_bytes(self, n_traces: int) -> int:
        out = C.c_uint64()
        native.check(native.load().isim_des_workspace_bytes(self.handler._h, n_traces, C.byref(out)))
        return int(out.value)

    def serve(self, trace_begin: int, n_traces: int, device: int = 0, records: bool = True, wide: bool = False):
        """Synchronous: (records or None, stats, DES table)."""
        stats = self.handler.new_stats()
        table = self.new_table()
        recs = np.zeros(n_traces, REC_DTYPE) if records else None
        p = native.DesParams(self.params.mean_interarrival_ns, native.DES_FLAG_WIDE if wide else 0, 0)
        native.check(native.load().isim_serve_des(
            self.handler._h, device, C.byref(p), trace_begin, n_traces,
            recs.ctypes.data if records and n_traces else None, stats.ctypes.data, table.ctypes.data))
        return recs, stats, table

    def serve_device(self, trace_begin: int, n_traces: int, d_records: int, d_stats: int, d_table: int,
                     d_workspace: int, workspace_bytes: int, stream: int = 0, wide: bool = False) -> None:
        p = self.params
        if wide:
            p = native.DesParams(p.mean_interarrival_ns, native.DES_FLAG_WIDE, 0)
        native.check(native.load().isim_serve_des_device(
            self.handler._h, C.byref(p), trace_begin, n_traces, d_records or None, d_stats, d_table,
            d_workspace, workspace_bytes, stream or None))

    def fold(self, table: np.ndarray) -> np.ndarray:
        n = self.handler.info.n_services
        out = np.zeros((max(1, n), native.DES_ROW_WORDS), np.uint64)
        table = np.ascontiguousarray(table, dtype=np.uint64)
        native.check(native.load().isim_des_fold(self.handler._h, table.ctypes.data, out.ctypes.data))
        return out[:n]
