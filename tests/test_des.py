"""DES (BASELINE config 5) on the CPU: the fixed-point
exponential, the DES v1 graph class, and the two oracles against each other
and against the static walk.  The GPU parity tests are in test_des_gpu.py."""
import json
import os
import re

import numpy as np
import pytest

import isim
from isim.generators import config2_topology, mesh_topology, realistic_topology, tree_topology
from isim.yamljson import obj_to_json, yaml_to_json
from oracle import des as od
from oracle import des_levels as dl
from oracle import executor as oc
from oracle import graph_ref as gr
from oracle.executor_py import SimGraph

from conftest import TOPOLOGIES
from parity import oracle_params

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "istio-isotope_amd", "csrc")


def test_ln_table_is_libm():
    text = open(os.path.join(CSRC, "des_ln_table.inc")).read()
    vals = [int(x) for x in re.findall(r"-?\d+", text.split("\n", 1)[1])]
    assert vals == od.ln_table().tolist()


def test_exp_q24_c_vs_python():
    rng = np.random.default_rng(1)
    us = [0, 1, 255, 256, 0xFF, 0xFFFFFF00, 0xFFFFFFFF, 0x80000000] + rng.integers(0, 1 << 32, 2000).tolist()
    for u in us:
        assert od.exp_q24(u) == od.exp_q24_py(int(u))
    assert od.exp_q24(0xFFFFFFFF) == 0                       # w = 2^24: -ln 1
    assert od.exp_q24(0) == 24 * 11629080                    # w = 1: 24 ln 2


def test_exp_q24_is_exponential():
    # E[-ln U] = 1 and E[(-ln U)^2] = 2 over a stratified grid of u
    u = (np.arange(1 << 16, dtype=np.uint64) << np.uint64(16)) + np.uint64(0x8000)
    e = np.array([od.exp_q24(int(x)) for x in u], np.float64) / (1 << 24)
    assert abs(e.mean() - 1.0) < 2e-3 and abs((e * e).mean() - 2.0) < 2e-2
    # the fixed-point table error itself is tiny: compare with libm at the bucket centres
    exact = -np.log(((u >> np.uint64(8)) + np.uint64(1)).astype(np.float64) / (1 << 24))
    assert np.max(np.abs(e - exact)) < 2e-5


def test_piecewise_duration_bucket():
    # des.hip des_prom_bucket: the 32 Prometheus duration edges are six
    # arithmetic runs of whole milliseconds; its closed form (restated here)
    # equals the first-edge->=t search for every t (the GPU tables are
    # checked bit-exact against the oracle in test_des_gpu.py)
    from isim.prometheus import DURATION_BUCKETS
    edges = [round(e * 1000) for e in DURATION_BUCKETS]

    def search(t):
        return next((i for i, e in enumerate(edges) if t <= e * 1_000_000), 32)

    def closed(t):
        if t > 500_000_000:
            return 32
        m = (t + 999_999) // 1_000_000
        lo, base, d = next(r for r in ((12, 7, 0, 1), (20, 12, 5, 2), (50, 20, 9, 5), (100, 50, 15, 10),
                                       (200, 100, 20, 20), (10 ** 9, 200, 25, 50)) if m <= r[0])[1:]
        n = max(0, m - lo)
        return base + (((n + d - 1) * -(-65536 // d)) >> 16)

    rng = np.random.default_rng(5)
    ts = [max(0, e * 1_000_000 + dd) for e in range(0, 505) for dd in (-1, 0, 1, 499_999, 999_999)]
    ts += rng.integers(0, 600_000_000, 20000).tolist()
    assert all(search(t) == closed(t) for t in ts)


def canonical_concurrent(sleep="300us"):
    """example-topologies/canonical.yaml with every service's calls in one
    concurrent step (a and b are then invoked twice per trace: a DAG)."""
    j = yaml_to_json(open(os.path.join(TOPOLOGIES, "canonical.yaml"), "rb").read())
    doc = json.loads(j)
    for s in doc["services"]:
        calls = []
        for st in s.get("script", []):
            calls += st if isinstance(st, list) else [st]
        s["script"] = [{"sleep": sleep}] + ([calls] if calls else [])
    return doc


def _handler(doc, **kw):
    return isim.Handler(isim.ServiceGraph.from_json(obj_to_json(doc) if isinstance(doc, dict) else doc),
                        None, isim.SimParams(**kw))


def _rejects(h, needle):
    with pytest.raises(isim.IsimError) as e:
        isim.DesHandler(h, 1_000_000)
    assert e.value.code == isim.native.EINVAL and needle in str(e.value), str(e.value)


def test_des_class():
    isim.DesHandler(_handler(config2_topology()), 1_000_000)  # sequential calls: step begins
    # probabilistic calls: the item engine (mode A) over the tree's potential invocations
    dm = isim.DesHandler(_handler(mesh_topology(800, 4)), 1_000_000)
    assert dm.info.items == 1 and dm.info.n_positions == 40 and dm.info.n_fused == 0
    # mode B: the same engine, its walks drawing the errors (a failed step ends the script)
    db = isim.DesHandler(_handler(mesh_topology(800, 4), error_mode=isim.MODE_B), 1_000_000)
    assert db.info.items == 1 and db.info.n_positions == 40
    # a call step after one that can fail: dynamic in mode B only
    seq = tree_topology(2, 3, sequential=True)
    for sv in seq["services"]:
        sv["errorRate"] = 0.1
    assert isim.DesHandler(_handler(seq), 1_000_000).info.items == 0
    assert isim.DesHandler(_handler(seq, error_mode=isim.MODE_B), 1_000_000).info.items == 1
    # more than 65,535 potential invocations: a wide tree (round 5) — a chain of
    # 17 services each calling the next twice: 2^17 - 1 positions
    def chain(conc):
        call = {"call": {"service": None, "probability": 50}}
        out = []
        for i in range(17):
            c = [json.loads(json.dumps(call).replace("null", f'"s{i + 1}"')) for _ in range(2)] if i < 16 else []
            out.append({"name": f"s{i}", "isEntrypoint": i == 0, "script": ([c] if conc else c) if c else []})
        return {"services": out}
    dw = isim.DesHandler(_handler(chain(True)), 1_000_000)
    assert dw.info.items == 1 and dw.info.n_positions == (1 << 17) - 1
    # sequential: every call step after the previous one's subtree — 131,071 rounds
    _rejects(_handler(chain(False)), "rounds")
    doc = tree_topology(3, 3)
    doc["services"][-1]["numReplicas"] = 65
    isim.DesHandler(_handler(doc), 1_000_000)  # no sleeps: never queues, replicas do not matter
    doc["services"][-1]["script"] = [{"sleep": "1ms"}]
    isim.DesHandler(_handler(doc), 1_000_000)  # > 64 replicas: the sort path's segmented scan
    doc["services"][-1]["numReplicas"] = 70000
    _rejects(_handler(doc), "more than 65536 replicas")
    d = isim.DesHandler(_handler(realistic_topology(200, concurrent=True, sleep_ms=(1, 5))), 5_000_000)
    assert (d.info.n_positions, d.info.table_rows) == (200, 200)
    assert d.info.items == 0
    assert d.info.cyclic == 0 and 0 < d.info.n_fused < 200  # the tree's leaves finish in their queue pass
    assert d.info.n_levels >= 2 and d.info.max_width >= 1
    assert d.workspace_bytes(1000) >= 200 * 1000 * 8 + 1000 * 12
    # DAG graphs (a service at several positions) and replicated callers take the sort path
    canon = json.loads(yaml_to_json(open(os.path.join(TOPOLOGIES, "canonical.yaml"), "rb").read()))
    # b is called inside d's first call step (through c) and in its second:
    # without sleeps b never queues (one start op per position) ...
    isim.DesHandler(_handler(canon), 1_000_000)
    # ... with a hold, b's queue waits for its own finish: a cyclic schedule,
    # run as passes to its fixed point
    assert isim.DesHandler(_handler(canon), 1_000_000).info.cyclic == 0  # zero holds: per-position starts
    canon["services"][1]["script"] = [{"sleep": "1ms"}]
    assert isim.DesHandler(_handler(canon), 1_000_000).info.cyclic == 1
    dc = isim.DesHandler(_handler(canonical_concurrent()), 1_000_000)
    assert dc.info.n_positions == 6
    assert dc.workspace_bytes(1000) > 6 * 1000 * 8 + 2 * 1000 * 24  # a and b: 2 positions each
    doc = tree_topology(3, 3)
    doc["services"][1]["numReplicas"] = 3
    isim.DesHandler(_handler(doc), 1_000_000)
    # the DES rejects bad parameters
    with pytest.raises(isim.IsimError):
        isim.DesHandler(d.handler, 0).serve(0, 1)


def _binary_dag(depth):
    """s_i calls s_{i+1} twice, in two sequential call steps: 2^(depth+1) - 1
    invocations per trace, and every step begin waits for the previous step's
    whole subtree, so the DES schedule chains every position."""
    svcs = [{"name": f"s{i}", "script": [{"call": f"s{i + 1}"}, {"call": f"s{i + 1}"}]} for i in range(depth)]
    svcs.append({"name": f"s{depth}", "errorRate": 1.0})
    svcs[0]["isEntrypoint"] = True
    return {"services": svcs}


def test_des_plan_lazy_and_round_limit():
    # a walk handler never builds the DES plan (it unrolls the whole tree):
    # 2^23 invocations per trace compile in about a second
    import time
    t0 = time.perf_counter()
    h = _handler(_binary_dag(22), hop_base_ns=1, req_ps_per_byte=0, resp_ps_per_byte=0)
    assert h.info.hops_upper == (1 << 23) - 1 and time.perf_counter() - t0 < 20
    # the plan of a short chain is built in linear time (topological longest
    # path) and its schedule is one round per link of the chain
    d = isim.DesHandler(_handler(_binary_dag(10)), 1_000_000)
    assert d.info.n_positions == (1 << 11) - 1
    # past kDesMaxRounds rounds the graph is outside the DES class
    t0 = time.perf_counter()
    _rejects(_handler(_binary_dag(16)), "rounds")
    assert time.perf_counter() - t0 < 20


def _oracle_case(doc, **kw):
    j = obj_to_json(doc)
    h = isim.Handler(isim.ServiceGraph.from_json(j), None, isim.SimParams(**kw))
    sg = SimGraph(gr.unmarshal_service_graph(j))
    return h, sg, oracle_params(h.params)


def _canonical_doc():
    return json.loads(yaml_to_json(open(os.path.join(TOPOLOGIES, "canonical.yaml"), "rb").read()))


def _prob_canonical():
    doc = _canonical_doc()
    for sv in doc["services"]:
        for st in sv.get("script", []):
            for c in (st if isinstance(st, list) else [st]):
                if "call" in c:
                    c["call"] = {"service": c["call"] if isinstance(c["call"], str) else c["call"]["service"],
                                 "probability": 50}
    return doc


@pytest.mark.parametrize("mode", [isim.MODE_A, isim.MODE_B])
@pytest.mark.parametrize("doc", [tree_topology(3, 3), tree_topology(4, 4),
                                 realistic_topology(300, concurrent=True, error_rate=(0.0, 0.3)),
                                 _canonical_doc(), tree_topology(3, 4, sequential=True),
                                 realistic_topology(300, error_rate=(0.0, 0.3))],
                         ids=["tree3x3", "tree4x4", "realistic300", "canonical", "tree3x4seq",
                              "realistic300seq"])
def test_event_oracle_without_holds_is_the_static_walk(doc, mode):
    # no sleeps -> no worker is ever held -> no queueing: the DES must
    # reproduce the static walk trace by trace (latency, hops, status)
    doc = json.loads(json.dumps(doc))
    doc.setdefault("defaults", {})["errorRate"] = 0.2
    h, sg, op = _oracle_case(doc, error_mode=mode)
    if not h.info.static_walk:
        pytest.skip("mode B aborts make this graph a dynamic walk (outside the DES)")
    n = 700
    rs, ss = oc.run(sg, op, sg.entry(), 5, n)
    rd, sd, des = od.run(sg, op, sg.entry(), 5, n, 1_000_000)
    assert np.array_equal(rs, rd)
    o = oc.split_stats(ss, len(sg.g.services), len(sg.sites))
    assert np.array_equal(ss[:o["svc_dur"].size and len(sd)], sd)
    assert des[:, od.DES_ROW - 3].sum() == 0  # no waits
    # durations: the static walk's per-service table
    assert np.array_equal(des[:, :68], o["svc_dur"])


@pytest.mark.parametrize("doc", [realistic_topology(300, concurrent=True, error_rate=(0.0, 0.3), probability=60),
                                 realistic_topology(300, error_rate=(0.0, 0.3), probability=75),
                                 mesh_topology(800, 4), _prob_canonical()],
                         ids=["realistic300p60", "realistic300seq_p75", "mesh800", "canonical_p50"])
def test_event_oracle_probabilistic_without_holds_is_the_walk(doc):
    """Probabilistic calls (mode A): the event oracle's pre-walk fixes the
    executed calls and hop ids (executable.go:84-90, semantics v1 §2.3); with
    no holds nothing queues, so every trace must equal the walk oracle's
    (latency, hops, status, err_hops) and the per-service durations its table."""
    doc = json.loads(json.dumps(doc))
    doc.setdefault("defaults", {})["errorRate"] = 0.2
    h, sg, op = _oracle_case(doc)
    assert not h.info.static_walk
    n = 700
    rs, ss = oc.run(sg, op, sg.entry(), (1 << 32) - 300, n)
    rd, sd, des = od.run(sg, op, sg.entry(), (1 << 32) - 300, n, 1_000_000)
    assert np.array_equal(rs, rd)
    o = oc.split_stats(ss, len(sg.g.services), len(sg.sites))
    assert np.array_equal(ss[:len(sd)], sd)
    assert des[:, od.DES_ROW - 3].sum() == 0
    assert np.array_equal(des[:, :68], o["svc_dur"])
    assert 0 < int(ss[2]) < n * int(h.info.hops_upper)  # some calls were skipped


@pytest.mark.parametrize("prob", [40, 80])
def test_event_oracle_probabilistic_tree_spaced_arrivals(prob):
    """A probabilistic tree with sleeps (holds) whose traces never overlap
    (mean gap far above any latency): every service is invoked at most once
    per trace, so no invocation ever waits and the latencies are the walk's."""
    doc = realistic_topology(200, concurrent=True, sleep_ms=(1, 5), error_rate=(0.0, 0.1), probability=prob)
    h, sg, op = _oracle_case(doc)
    n = 300
    rs, _ = oc.run(sg, op, sg.entry(), 77, n)
    rd, _, des = od.run(sg, op, sg.entry(), 77, n, 1 << 40)
    assert np.array_equal(rs, rd)
    assert des[:, od.DES_ROW - 3].sum() == 0


@pytest.mark.parametrize("mean", [400_000, 3_000_000, 20_000_000])
@pytest.mark.parametrize("case", ["realistic", "tree_reps"])
def test_level_restatement_matches_event_oracle(case, mean):
    if case == "realistic":
        doc = realistic_topology(250, concurrent=True, sleep_ms=(1, 5), error_rate=(0.0, 0.02))
    else:
        doc = tree_topology(3, 4)
        for s in doc["services"]:
            s["script"] = [{"sleep": "2ms"}] + s.get("script", []) + [{"sleep": "500us"}]
        for s in doc["services"][5:]:
            s["numReplicas"] = 3  # leaves
    h, sg, op = _oracle_case(doc)
    n = 1500
    rd, sd, des = od.run(sg, op, sg.entry(), 11, n, mean)
    lat, wsum, wmax, pos = dl.run(sg, op, sg.entry(), 11, n, mean)
    assert np.array_equal(rd[:, 0].astype(np.int64), lat)
    for i, q in enumerate(pos):
        assert des[q["svc"], 69] == wsum[i] and des[q["svc"], 70] == wmax[i], (i, q["svc"])
    if mean == 400_000:
        assert wsum.sum() > 0  # the load actually queues
