"""Pure-Python restatement of the isotope script executor in virtual time
(oracle — test infrastructure only; small cases).

Mirrors the reference recursion one request at a time:
  Handler.ServeHTTP              isotope/service/pkg/srv/handler.go:37-79
  execute (type switch)          isotope/service/pkg/srv/executable.go:43-76
  executeSleepCommand            executable.go:78-82      -> virtual t += max(d, 0)
  shouldSkipRequest              executable.go:84-90      -> Philox probability draw
  executeRequestCommand          executable.go:94-144     -> H + T(callee); 500 swallowed (mode A)
  executeConcurrentCommand       executable.go:148-179    -> max over children, OR of errors
  prometheus.Record*             srv/prometheus/handler.go:87-106 -> stats
with the EXT rules of "isim semantics v1" (DESIGN.md §2): hop-cost model,
Philox draw schedule, error-rate injection at the respond point, error mode B.

The call of a service name resolves to the FIRST service of that name, as
extractService does (isotope/service/pkg/srv/graph.go:97-109).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

from . import graph_ref as gr
from .gounits import error_threshold
from .philox import err_draw, prob_draw

MODE_A, MODE_B = 0, 1

# service_request_duration_seconds buckets (srv/prometheus/handler.go:26-31) in ns.
PROM_EDGES_NS = [int(ms * 1_000_000) for ms in (
    7, 8, 9, 10, 11, 12, 14, 16, 18, 20, 25, 30, 35, 40, 45, 50, 60, 70, 80, 90,
    100, 120, 140, 160, 180, 200, 250, 300, 350, 400, 450, 500)]
N_PROM = len(PROM_EDGES_NS) + 1   # + the +Inf bucket
N_LOG2 = 64


def prom_bucket(t_ns: int) -> int:
    for i, e in enumerate(PROM_EDGES_NS):
        if t_ns <= e:
            return i
    return len(PROM_EDGES_NS)


def log2_bucket(t_ns: int) -> int:
    return 0 if t_ns == 0 else t_ns.bit_length()


@dataclass
class SimParams:
    seed: int = 0x15070BE
    hop_base_ns: int = 250_000
    req_ps_per_byte: int = 80
    resp_ps_per_byte: int = 80
    error_mode: int = MODE_A


class SimGraph:
    """Resolved view of a ServiceGraph for execution: name->first index,
    error thresholds, call-site ids (document order) and static call
    indices k within each script."""

    def __init__(self, g: gr.ServiceGraph):
        self.g = g
        self.index = {}
        for i, s in enumerate(g.services):
            self.index.setdefault(s.name, i)
        self.thr = [error_threshold(s.error_rate) for s in g.services]
        self.resp = [s.response_size for s in g.services]
        # per service: list of steps; each call gets (site_id, k)
        self.sites = []          # site id -> (caller svc, callee svc, size, prob)
        self.steps = []
        for si, s in enumerate(g.services):
            k = 0
            steps = []
            for c in s.script:
                if isinstance(c, gr.ConcurrentCommand):
                    sub = []
                    for x in c.commands:
                        if isinstance(x, gr.RequestCommand):
                            sub.append(("call", self._site(si, x), k))
                            k += 1
                        else:
                            sub.append(("sleep", x.ns))
                    steps.append(("conc", sub))
                elif isinstance(c, gr.RequestCommand):
                    steps.append(("call", self._site(si, c), k))
                    k += 1
                else:
                    steps.append(("sleep", c.ns))
            self.steps.append(steps)

    def _site(self, caller, c: gr.RequestCommand) -> int:
        self.sites.append((caller, self.index[c.service], c.size, c.probability))
        return len(self.sites) - 1

    def entry(self, name: Optional[str] = None) -> int:
        if name is not None:
            if name not in self.index:
                raise KeyError(name)
            return self.index[name]
        for i, s in enumerate(self.g.services):
            if s.is_entrypoint:
                return i
        raise ValueError("no service has isEntrypoint: true")

    def hop_cost(self, site: int, p: SimParams) -> int:
        _, callee, size, _ = self.sites[site]
        return p.hop_base_ns + (size * p.req_ps_per_byte + self.resp[callee] * p.resp_ps_per_byte) // 1000


class Stats:
    def __init__(self, sg: SimGraph):
        n = len(sg.g.services)
        self.svc_calls = [0] * n
        self.svc_errs = [0] * n
        self.site_calls = [0] * len(sg.sites)
        # RecordResponseSent (prometheus/handler.go:101-106): per service, the
        # invocation's own duration on the duration buckets [code][33] + sums
        self.svc_dur = [[[0] * N_PROM for _ in range(2)] for _ in range(n)]
        self.svc_dur_sum = [[0, 0] for _ in range(n)]
        # optional per-event log, in the order the reference process would
        # record them: ("recv", svc) / ("sent", caller, site) / ("resp", svc, T, err)
        self.events = None
        self.lat_prom = [[0] * N_PROM for _ in range(2)]
        self.lat_log2 = [[0] * N_LOG2 for _ in range(2)]
        self.n_traces = 0
        self.sum_latency = 0
        self.sum_hops = 0
        self.sum_err_hops = 0
        self.n_500 = 0
        self.min_latency = (1 << 64) - 1
        self.max_latency = 0


class _Trace:
    __slots__ = ("t", "next_hop", "err_hops")

    def __init__(self, t):
        self.t = t
        self.next_hop = 0
        self.err_hops = 0


def _skip(sg, p, tr, hop, k, q) -> bool:
    """shouldSkipRequest, executable.go:84-90: p==0 never skips; else skip iff
    Intn(100) < 100-p.  EXT: Intn(100) := draw % 100 (q==100 never skips)."""
    if q == 0 or q >= 100:
        return False
    return prob_draw(p.seed, tr.t, hop, k) % 100 < 100 - q


def _invoke(sg: SimGraph, p: SimParams, st: Stats, tr: _Trace, s: int):
    """Handler.ServeHTTP for one request to service s -> (T, status500)."""
    hop = tr.next_hop
    tr.next_hop += 1
    st.svc_calls[s] += 1                      # RecordRequestReceived (handler.go:43)
    if st.events is not None:
        st.events.append(("recv", s))
    thr = sg.thr[s]
    T = 0
    failed = False
    for step in sg.steps[s]:                  # handler.go:66-76
        kind = step[0]
        if kind == "sleep":
            T += max(step[1], 0)
        elif kind == "call":
            _, site, k = step
            q = sg.sites[site][3]
            if _skip(sg, p, tr, hop, k, q):
                continue
            tc, e = _invoke(sg, p, st, tr, sg.sites[site][1])
            st.site_calls[site] += 1          # RecordRequestSent (executable.go:124-129)
            if st.events is not None:
                st.events.append(("sent", s, site))
            T += sg.hop_cost(site, p) + tc
            if p.error_mode == MODE_B and e:
                failed = True
                break
        else:                                 # concurrent: all children run, max, OR
            m = 0
            cerr = False
            for sub in step[1]:
                if sub[0] == "sleep":
                    m = max(m, max(sub[1], 0))
                    continue
                _, site, k = sub
                q = sg.sites[site][3]
                if _skip(sg, p, tr, hop, k, q):
                    continue
                tc, e = _invoke(sg, p, st, tr, sg.sites[site][1])
                st.site_calls[site] += 1
                if st.events is not None:
                    st.events.append(("sent", s, site))
                m = max(m, sg.hop_cost(site, p) + tc)
                if p.error_mode == MODE_B and e:
                    cerr = True
            T += m
            if cerr:
                failed = True
                break
    if failed:
        err = True
    else:                                     # EXT: errorRate at the respond point
        err = thr >= (1 << 32) or (thr > 0 and err_draw(p.seed, tr.t, hop) < thr)
    if err:
        st.svc_errs[s] += 1
        tr.err_hops += 1
    st.svc_dur[s][int(err)][prom_bucket(T)] += 1   # handler.go:56-58
    if st.events is not None:
        st.events.append(("resp", s, T, int(err)))
    st.svc_dur_sum[s][int(err)] += T
    return T, err


def run(sg: SimGraph, p: SimParams, entry: int, trace_begin: int, n_traces: int, events: bool = False):
    """Simulate traces [trace_begin, trace_begin + n_traces). Returns
    (records, stats); a record is (latency_ns, hops, status500, err_hops).
    events=True also logs every Record* call into stats.events."""
    st = Stats(sg)
    if events:
        st.events = []
    recs = []
    for i in range(n_traces):
        tr = _Trace(trace_begin + i)
        T, e = _invoke(sg, p, st, tr, entry)
        recs.append((T, tr.next_hop, int(e), tr.err_hops))
        st.n_traces += 1
        st.sum_latency += T
        st.sum_hops += tr.next_hop
        st.sum_err_hops += tr.err_hops
        st.n_500 += int(e)
        st.min_latency = min(st.min_latency, T)
        st.max_latency = max(st.max_latency, T)
        st.lat_prom[int(e)][prom_bucket(T)] += 1
        st.lat_log2[int(e)][log2_bucket(T)] += 1
    return recs, st
