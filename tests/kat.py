"""Executor known-answer tests (tests/golden/executor_kat.json, SURVEY
Appendix B + the hand-derived abort / default-script / 500-payload cases):
loading, and the assertions shared by the oracle test (test_oracle.py) and
the HIP-path test (test_kat_gpu.py).  Every expected number in the JSON was
derived by hand from the reference's own graphs and code, not from either
implementation."""
from __future__ import annotations

import json
import os

from conftest import GOLDEN, TOPOLOGIES

KAT = json.load(open(os.path.join(GOLDEN, "executor_kat.json")))
CASES = KAT["cases"]


def case_id(c) -> str:
    return f"{c['graph']}-{c['entry']}-{c['hop_ns']}-{c.get('mode', 'A')}-{c.get('req_ps', 0)}-{c.get('resp_ps', 0)}"


def graph_json(name: str) -> str:
    from isim.generators import tree_topology
    from isim.yamljson import obj_to_json, yaml_to_json
    if name.startswith("topology:"):
        return yaml_to_json(open(os.path.join(TOPOLOGIES, name.split(":", 1)[1]), "rb").read())
    if name.startswith("tree:"):
        _, shape, kind = name.split(":")
        lv, br = map(int, shape.split("x"))
        return obj_to_json(tree_topology(lv, br, sequential=(kind == "sequential")))
    return KAT["graphs"][name]


def params(case):
    """(hop_base_ns, req_ps_per_byte, resp_ps_per_byte, error_mode)."""
    return case["hop_ns"], case.get("req_ps", 0), case.get("resp_ps", 0), 1 if case.get("mode", "A") == "B" else 0


def check_record(case, latency: int, hops: int, is500: int, err_hops: int):
    assert latency == case["latency"], (latency, case["latency"])
    assert hops == case["hops"], (hops, case["hops"])
    if "status" in case:
        assert is500 == (case["status"] == 500), (is500, case["status"])
        assert err_hops == case["err_hops"], (err_hops, case["err_hops"])


class _H:
    def __init__(self, graph):
        self.graph = graph


def check_folded(case, names, folded: dict, n: int, graph=None):
    """Per-service calls / 500s (RecordRequestReceived, RecordResponseSent
    codes) and, when `graph` (an isim.ServiceGraph) is given, the request /
    response size histograms of the rendered Prometheus families — n traces,
    each contributing the case's per-trace numbers."""
    calls = {nm: int(c) for nm, c in zip(names, folded["svc_calls"]) if c}
    if "calls" in case:
        assert calls == {k: v * n for k, v in case["calls"].items()}, calls
    else:
        assert set(calls.values()) == {case["calls_each"] * n} and len(calls) == case["hops"]
    if "errs" in case:
        errs = {nm: int(c) for nm, c in zip(names, folded["svc_errs"]) if c}
        assert errs == {k: v * n for k, v in case["errs"].items()}, errs
    if graph is None:
        return
    from isim.prometheus import service_metrics
    m = service_metrics(_H(graph), folded)
    for svc, codes in case.get("response_size", {}).items():
        got = {code: (h.count, h.sum) for code, h in m[svc].response_size.items()}
        assert got == {code: (c * n, float(s * n)) for code, (c, s) in codes.items()}, (svc, got)
    for svc, dests in case.get("request_size", {}).items():
        got = {d: (h.count, h.sum) for d, h in m[svc].outgoing_size.items()}
        assert got == {d: (c * n, float(s * n)) for d, (c, s) in dests.items()}, (svc, got)
