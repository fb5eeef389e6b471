"""Per-service Prometheus metrics of a simulated run, rendered as each
isotope pod's `/metrics` endpoint would serve them.

The reference records, in every service process (isotope/service/pkg/srv/
prometheus/handler.go):

    service_incoming_requests_total                      counter     :37-41, RecordRequestReceived :87-89
    service_outgoing_requests_total{destination_service} counter     :43-47, RecordRequestSent :93-97
    service_outgoing_request_size{destination_service}   histogram   :49-54 (sizeBuckets)
    service_request_duration_seconds{code}               histogram   :56-61 (durationBuckets), RecordResponseSent :101-106
    service_response_size{code}                          histogram   :63-68 (sizeBuckets)

isim produces the same quantities from one stats buffer (`Handler.fold`):
incoming requests and 500s per service, executed calls per call site, and
per-service invocation-duration histograms.  Request and response sizes are
static per call site / per service, so their histograms follow from the
counters.  Rendering follows the Prometheus text format as client_golang's
promhttp writes it (families sorted by name, children by label value,
cumulative `le` buckets, `+Inf`, `_sum`, `_count`; every number through Go's
`strconv.FormatFloat(v, 'g', -1, 64)`).

Differences, by construction: the Go/process collectors of the default
registry are not emitted (they describe the Go process, not the service);
`service_request_duration_seconds_sum` is the exact ns sum / 1e9 rather than a
float64 running sum in arrival order.
"""
from __future__ import annotations

import math
from decimal import Decimal
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import native
from .graph import ConcurrentCommand, RequestCommand

# prometheus/handler.go:26-35
DURATION_BUCKETS = (0.007, 0.008, 0.009, 0.01, 0.011, 0.012, 0.014, 0.016, 0.018, 0.02, 0.025,
                    0.03, 0.035, 0.04, 0.045, 0.05, 0.06, 0.07, 0.08, 0.09, 0.1, 0.12, 0.14,
                    0.16, 0.18, 0.2, 0.25, 0.3, 0.35, 0.4, 0.45, 0.5)
SIZE_BUCKETS = (1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9)

HELP = {
    "service_incoming_requests_total": "Number of requests sent to this service.",
    "service_outgoing_requests_total": "Number of requests sent from this service.",
    "service_outgoing_request_size": "Size in bytes of requests sent from this service.",
    "service_request_duration_seconds": "Duration in seconds it took to serve requests to this service.",
    "service_response_size": "Size in bytes of responses sent from this service.",
}
CODES = ("200", "500")


def go_float(f: float) -> str:
    """strconv.FormatFloat(f, 'g', -1, 64) as expfmt's writeFloat uses it."""
    f = float(f)
    if f == 1:
        return "1"
    if f == 0:
        return "0"
    if f == -1:
        return "-1"
    if math.isnan(f):
        return "NaN"
    if math.isinf(f):
        return "+Inf" if f > 0 else "-Inf"
    sign = "-" if f < 0 else ""
    # shortest round-trip digits (Python's repr and Go's shortest agree)
    t = Decimal(repr(abs(f))).normalize().as_tuple()
    digs = "".join(str(d) for d in t.digits)
    nd = len(digs)
    dp = nd + t.exponent  # decimal point position
    x = dp - 1
    if x < -4 or x >= 6:  # shortest: eprec = 6 (strconv/ftoa.go %g rule)
        mant = digs[0] + ("." + digs[1:] if nd > 1 else "")
        return f"{sign}{mant}e{'-' if x < 0 else '+'}{abs(x):02d}"
    if dp <= 0:
        return f"{sign}0.{'0' * -dp}{digs}"
    if dp >= nd:
        return f"{sign}{digs}{'0' * (dp - nd)}"
    return f"{sign}{digs[:dp]}.{digs[dp:]}"


def _bucket_index(v: float, edges) -> int:
    for i, e in enumerate(edges):
        if v <= e:
            return i
    return len(edges)


def call_sites(graph) -> List[Tuple[int, str, int]]:
    """(caller index, callee name, size) per call command in document order
    (services -> steps -> concurrent sub-commands) — the site ids of
    isim_handler_slots / fold()["site_calls"]."""
    out = []
    for i, s in enumerate(graph.services):
        for step in s.script:
            if isinstance(step, RequestCommand):
                out.append((i, step.service, step.size))
            elif isinstance(step, ConcurrentCommand):
                for c in step.commands:
                    if isinstance(c, RequestCommand):
                        out.append((i, c.service, c.size))
    return out


class Histogram:
    """One histogram child: non-cumulative counts per bucket (+Inf last) and a sum."""

    def __init__(self, edges):
        self.edges = edges
        self.counts = [0] * (len(edges) + 1)
        self.sum = 0.0

    def observe_n(self, value: float, n: int):
        if n:
            self.counts[_bucket_index(value, self.edges)] += n
            self.sum += float(value) * n

    @property
    def count(self) -> int:
        return sum(self.counts)


class ServiceMetrics:
    """The isotope metric families of one service's process."""

    def __init__(self, name: str):
        self.name = name
        self.incoming = 0
        self.outgoing: Dict[str, int] = {}
        self.outgoing_size: Dict[str, Histogram] = {}
        self.duration: Dict[str, Histogram] = {}
        self.response_size: Dict[str, Histogram] = {}

    def exposition(self) -> str:
        """Text format 0.0.4, as promhttp renders this service's registry."""
        out: List[str] = []

        def head(name, typ):
            out.append(f"# HELP {name} {HELP[name]}")
            out.append(f"# TYPE {name} {typ}")

        def hist(name, label, children: Dict[str, Histogram]):
            if not children:
                return
            head(name, "histogram")
            for lv in sorted(children):
                h = children[lv]
                lab = f'{label}="{lv}"'
                cum = 0
                for e, c in zip(h.edges, h.counts):
                    cum += c
                    out.append(f'{name}_bucket{{{lab},le="{go_float(e)}"}} {go_float(cum)}')
                out.append(f'{name}_bucket{{{lab},le="+Inf"}} {go_float(h.count)}')
                out.append(f"{name}_sum{{{lab}}} {go_float(h.sum)}")
                out.append(f"{name}_count{{{lab}}} {go_float(h.count)}")

        head("service_incoming_requests_total", "counter")
        out.append(f"service_incoming_requests_total {go_float(self.incoming)}")
        hist("service_outgoing_request_size", "destination_service", self.outgoing_size)
        if self.outgoing:
            head("service_outgoing_requests_total", "counter")
            for d in sorted(self.outgoing):
                out.append(f'service_outgoing_requests_total{{destination_service="{d}"}} '
                           f'{go_float(self.outgoing[d])}')
        hist("service_request_duration_seconds", "code", self.duration)
        hist("service_response_size", "code", self.response_size)
        return "\n".join(out) + "\n"


def service_metrics(handler, folded: Optional[dict] = None, stats: Optional[np.ndarray] = None
                    ) -> Dict[str, ServiceMetrics]:
    """Per-service metric families from a folded stats buffer (`Handler.fold`)."""
    if folded is None:
        folded = handler.fold(stats)
    graph = handler.graph
    svcs = graph.services
    res: Dict[str, ServiceMetrics] = {}
    for s in svcs:
        res.setdefault(s.name, ServiceMetrics(s.name))   # duplicate names: first wins (extractService)
    first = {}
    for i, s in enumerate(svcs):
        first.setdefault(s.name, i)
    calls = folded["svc_calls"]
    errs = folded["svc_errs"]
    dur = folded.get("svc_dur")
    for i, s in enumerate(svcs):
        if first[s.name] != i:
            continue
        m = res[s.name]
        m.incoming = int(calls[i])
        n5 = int(errs[i])
        n2 = int(calls[i]) - n5
        for code, n in zip(CODES, (n2, n5)):
            if n:
                h = m.response_size.setdefault(code, Histogram(SIZE_BUCKETS))
                h.observe_n(s.response_size, n)
        if dur is not None:
            row = dur[i]
            for ci, code in enumerate(CODES):
                counts = [int(x) for x in row[ci * native.N_PROM:(ci + 1) * native.N_PROM]]
                if sum(counts):
                    h = Histogram(DURATION_BUCKETS)
                    h.counts = counts
                    h.sum = int(row[2 * native.N_PROM + ci]) / 1e9
                    m.duration[code] = h
    site_calls = folded["site_calls"]
    for site, (caller, callee, size) in enumerate(call_sites(graph)):
        n = int(site_calls[site])
        if not n:
            continue
        m = res[svcs[caller].name]
        m.outgoing[callee] = m.outgoing.get(callee, 0) + n
        m.outgoing_size.setdefault(callee, Histogram(SIZE_BUCKETS)).observe_n(size, n)
    return res


def exposition(handler, folded: dict, service: str) -> str:
    """`/metrics` text of one service's pod."""
    return service_metrics(handler, folded)[service].exposition()
