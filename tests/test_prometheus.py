"""Per-service Prometheus exposition (isim.prometheus) on CPU: Go float
formatting, and the families folded from a stats buffer equal a registry fed
one Record* call at a time (the reference's own recording pattern,
srv/prometheus/handler.go:87-106) by the event log of the pure-Python
oracle."""
import json
import os

import pytest

import isim
from isim import prometheus as P
from isim.yamljson import yaml_to_json
from conftest import TOPOLOGIES
from oracle import executor as oc
from oracle import executor_py as ex
from oracle import graph_ref as gr


@pytest.mark.parametrize("v,s", [
    (1, "1"), (0, "0"), (0.007, "0.007"), (0.5, "0.5"), (1e6, "1e+06"), (1e5, "100000"), (1e9, "1e+09"),
    (4194304, "4.194304e+06"), (123456.7, "123456.7"), (1234567.0, "1.234567e+06"), (0.0025, "0.0025"),
    (1e-05, "1e-05"), (0.0001, "0.0001"), (10, "10"), (999999, "999999"), (3.0e-3, "0.003"),
    (float("inf"), "+Inf"), (-2.5, "-2.5"), (12.0, "12"), (0.1 + 0.2, "0.30000000000000004")])
def test_go_float(v, s):
    # strconv.FormatFloat(v, 'g', -1, 64)
    assert P.go_float(v) == s


GRAPHS = {
    "canonical": (yaml_to_json(open(os.path.join(TOPOLOGIES, "canonical.yaml"), "rb").read()), 0),
    "mixed": (json.dumps({"defaults": {"requestSize": "1 KB", "responseSize": 2000000},
                          "services": [
        {"name": "front", "isEntrypoint": True, "errorRate": 0.05,
         "script": [{"sleep": "3ms"}, {"call": {"service": "mid", "probability": 60}},
                    [{"call": "leaf"}, {"call": {"service": "mid", "size": 5}}, {"sleep": "6ms"}],
                    {"call": {"service": "leaf", "size": 20000000}}]},
        {"name": "mid", "errorRate": 0.2, "responseSize": 7,
         "script": [{"sleep": "4ms"}, {"call": {"service": "leaf", "probability": 50}}]},
        {"name": "leaf", "errorRate": 0.1, "script": [{"sleep": "2ms"}]},
        {"name": "idle"}]}), 0),
    "mode_b": (None, 1),
}
GRAPHS["mode_b"] = (GRAPHS["mixed"][0], 1)


def _registry_from_events(sg, events, graph):
    """Feed Record* calls one by one, like each pod's client_golang registry."""
    reg = {s.name: P.ServiceMetrics(s.name) for s in graph.services}
    sums = {}
    for ev in events:
        if ev[0] == "recv":
            reg[graph.services[ev[1]].name].incoming += 1
        elif ev[0] == "sent":
            _, caller, site = ev
            _, callee, size, _ = sg.sites[site]
            m = reg[graph.services[caller].name]
            dest = graph.services[callee].name
            m.outgoing[dest] = m.outgoing.get(dest, 0) + 1
            m.outgoing_size.setdefault(dest, P.Histogram(P.SIZE_BUCKETS)).observe_n(size, 1)
        else:
            _, s, T, err = ev
            svc = graph.services[s]
            code = P.CODES[err]
            m = reg[svc.name]
            # time.Duration.Seconds() against the float64 edges, as Observe does
            sec = float(T // 10 ** 9) + float(T % 10 ** 9) / 1e9
            m.duration.setdefault(code, P.Histogram(P.DURATION_BUCKETS)).observe_n(sec, 1)
            sums[(svc.name, code)] = sums.get((svc.name, code), 0) + T
            m.response_size.setdefault(code, P.Histogram(P.SIZE_BUCKETS)).observe_n(svc.response_size, 1)
    for (name, code), ns in sums.items():
        reg[name].duration[code].sum = ns / 1e9
    return reg


@pytest.mark.parametrize("name", sorted(GRAPHS))
def test_exposition_matches_event_registry(name):
    text, mode = GRAPHS[name]
    graph = isim.ServiceGraph.from_json(text)
    h = isim.Handler(graph, None, isim.SimParams(error_mode=mode))
    sg = ex.SimGraph(gr.unmarshal_service_graph(text))
    p = ex.SimParams(error_mode=mode)
    _, st = ex.run(sg, p, sg.entry(None), 1000, 300, events=True)
    _, cst = oc.run(sg, p, sg.entry(None), 1000, 300)
    folded = oc.split_stats(cst, len(sg.g.services), len(sg.sites))
    got = P.service_metrics(h, folded)
    want = _registry_from_events(sg, st.events, graph)
    for s in graph.services:
        assert got[s.name].exposition() == want[s.name].exposition(), s.name


def test_exposition_text_canonical():
    text = GRAPHS["canonical"][0]
    graph = isim.ServiceGraph.from_json(text)
    h = isim.Handler(graph)
    sg = ex.SimGraph(gr.unmarshal_service_graph(text))
    _, cst = oc.run(sg, ex.SimParams(), sg.entry(None), 0, 3)
    folded = oc.split_stats(cst, len(sg.g.services), len(sg.sites))
    d = P.exposition(h, folded, "d")
    lines = d.splitlines()
    assert lines[0] == "# HELP service_incoming_requests_total Number of requests sent to this service."
    assert lines[1] == "# TYPE service_incoming_requests_total counter"
    assert lines[2] == "service_incoming_requests_total 3"
    # d calls a, c (concurrently) then b; 1 KiB requests
    assert 'service_outgoing_requests_total{destination_service="a"} 3' in lines
    assert 'service_outgoing_request_size_bucket{destination_service="b",le="1000"} 0' in lines
    assert 'service_outgoing_request_size_bucket{destination_service="b",le="10000"} 3' in lines
    assert 'service_outgoing_request_size_sum{destination_service="b"} 3072' in lines
    # d lasts 4 hops of 250163 ns = 1.000652 ms: first duration bucket
    assert 'service_request_duration_seconds_bucket{code="200",le="0.007"} 3' in lines
    assert 'service_request_duration_seconds_sum{code="200"} 0.003001956' in lines
    assert 'service_request_duration_seconds_count{code="200"} 3' in lines
    assert 'service_response_size_bucket{code="200",le="1000"} 0' in lines
    assert 'service_response_size_bucket{code="200",le="10000"} 3' in lines
    names = [l.split()[2] for l in lines if l.startswith("# TYPE")]
    assert names == sorted(names)
    # a leaf with no calls has no outgoing families
    a = P.exposition(h, folded, "a")
    assert "service_outgoing" not in a and "service_incoming_requests_total 6" in a
