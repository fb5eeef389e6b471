"""Graph encoders: json.Marshal(graph.ServiceGraph) and the graphviz DOT text
(SURVEY.md §8f row 3).  CPU only.

Pinned by the reference's own vectors (tests/golden/go_vectors.json):
  graphviz_graph   graphviz/graphviz_test.go:28-168 (ServiceGraphToGraph)
  service_marshal  graph/svc/marshal_test.go:24-37  (Service MarshalJSON)
  bytes_size / pct_string / duration (already pinned in test_loader.py)
and by DOT fixtures rendered from the reference's own template text
(tests/golden/make_dot_fixtures.py).  Round trips: unmarshal(marshal(g)) == g.
"""
import glob
import json
import os

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import isim
from oracle import graph_ref as gr
from oracle import marshal_ref as mr

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
VEC = json.load(open(os.path.join(GOLDEN, "go_vectors.json")))
TOPOS = sorted(glob.glob(os.path.join(GOLDEN, "topologies", "*.yaml")))


def test_oracle_graphviz_struct_vector():
    v = VEC["graphviz_graph"]
    g = gr.unmarshal_service_graph(v["input"])
    assert mr.service_graph_to_graph(g) == v["expected"]


def test_service_marshal_vector():
    for doc, want in VEC["service_marshal"]["cases"]:
        g = isim.ServiceGraph.from_json(doc)
        out = g.marshal_json()
        assert out == b'{"services":[' + want.encode() + b"]}"
        assert mr.marshal_service_graph(gr.unmarshal_service_graph(doc)) == out


@pytest.mark.parametrize("path", TOPOS + ["graphviz_test"], ids=lambda p: os.path.basename(p))
def test_dot_matches_reference_template(path):
    if path == "graphviz_test":
        j, name = VEC["graphviz_graph"]["input"], "graphviz_test"
    else:
        j, name = isim.yaml_to_json(open(path, "rb").read()), os.path.basename(path)[:-5]
    want = open(os.path.join(GOLDEN, "dot", name + ".dot")).read()
    assert isim.ServiceGraph.from_json(j).to_dot() == want


@pytest.mark.parametrize("path", TOPOS, ids=os.path.basename)
def test_marshal_json_topologies(path):
    j = isim.yaml_to_json(open(path, "rb").read())
    g = isim.ServiceGraph.from_json(j)
    out = g.marshal_json()
    assert out == mr.marshal_service_graph(gr.unmarshal_service_graph(j))
    # round trip: decoding Go's own encoding gives back the same graph
    assert isim.ServiceGraph.from_json(out).canonical() == g.canonical()


def test_marshal_null_and_empty():
    assert isim.ServiceGraph.from_json(b"{}").marshal_json() == b'{"services":null}'
    assert isim.ServiceGraph.from_json(b'{"services":null}').marshal_json() == b'{"services":null}'
    assert isim.ServiceGraph.from_json(b'{"services":[]}').marshal_json() == b'{"services":[]}'
    assert isim.ServiceGraph.from_json(b'{"services":[]}').to_dot() == open(
        os.path.join(GOLDEN, "dot", "empty.dot")).read()


def test_marshal_escapes_and_formats():
    NAME = "a<b>&\"q\"\\\u2028\u00e9\t"
    doc = {"defaults": {"type": "grpc", "numReplicas": 0, "errorRate": 1e-7, "responseSize": "1.5MiB"},
           "services": [
               {"name": NAME, "errorRate": "0.0003%", "script": [
                   {"sleep": "1h2m3.5s"}, {"sleep": "1500us"}, {"sleep": "1500ns"}, {"sleep": "-3ns"}, {"sleep": "0s"},
                   {"call": {"service": "z", "size": "1023.9", "probability": 42}}]},
               {"name": "z", "isEntrypoint": True, "type": "http", "errorRate": 1, "numRbacPolicies": 7,
                "responseSize": 1 << 40, "script": [[{"call": NAME}, {"sleep": "10ms"}]]},
               {"name": "y"}]}
    # NAME calls z and z calls NAME: the loader accepts cycles (validation.go does not check)
    j = json.dumps(doc)
    g = isim.ServiceGraph.from_json(j)
    out = g.marshal_json()
    assert out == mr.marshal_service_graph(gr.unmarshal_service_graph(j))
    assert b"\\u003cb\\u003e\\u0026\\\"q\\\"\\\\\\u2028\xc3\xa9\\t" in out
    assert b'"errorRate":1e-7' in out and b'"errorRate":0.0000029999999999999997' in out and b'"sleep":"1h2m3.5s"' in out and b'"sleep":"1.5ms"' in out
    assert "1.5µs".encode() in out and b'"size":"1023B"' in out
    assert b'"type":"grpc"' in out and b'"responseSize":"1.5MiB"' in out and b'"responseSize":"1TiB"' in out
    # no round-trip check here: omitempty drops numReplicas 0, which decodes
    # back as defaultDefaults' 1 (unmarshal.go:64-70) -- Go behaves the same


@pytest.mark.parametrize("f,want", [(0.0001, b"0.0001"), (1e-6, b"0.000001"), (9.99e-7, b"9.99e-7"),
                                    (0.5, b"0.5"), (1.0, b"1"), (1e-10, b"1e-10"), (0.1 + 0.2, b"0.30000000000000004"),
                                    (1e21, b"1e+21"), (123456789012345680000.0, b"123456789012345680000")])
def test_go_json_float(f, want):
    assert mr.go_json_float(f) == want


_names = st.text(alphabet=st.characters(min_codepoint=1, max_codepoint=0x2030, blacklist_categories=("Cs",)),
                 min_size=1, max_size=6)


@st.composite
def graphs(draw):
    n = draw(st.integers(1, 5))
    names = draw(st.lists(_names, min_size=n, max_size=n, unique=True))
    svcs = []
    for i, nm in enumerate(names):
        script = []
        for _ in range(draw(st.integers(0, 4))):
            k = draw(st.integers(0, 2))
            if k == 0:
                script.append({"sleep": "%dns" % draw(st.integers(0, 10 ** 13))})
            elif k == 1:
                script.append({"call": {"service": draw(st.sampled_from(names)),
                                        "size": draw(st.integers(0, 1 << 45)),
                                        "probability": draw(st.integers(0, 100))}})
            else:
                script.append([{"call": draw(st.sampled_from(names))},
                               {"sleep": "%dus" % draw(st.integers(0, 10 ** 7))}])
        svcs.append({"name": nm, "errorRate": draw(st.floats(0, 1)), "isEntrypoint": draw(st.booleans()),
                     "responseSize": draw(st.integers(0, 1 << 50)), "numReplicas": draw(st.integers(1, 9)),
                     "type": draw(st.sampled_from(["http", "grpc"])), "script": script})
    return json.dumps({"services": svcs})


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(graphs())
def test_marshal_and_dot_vs_oracle(j):
    g = isim.ServiceGraph.from_json(j)
    og = gr.unmarshal_service_graph(j)
    out = g.marshal_json()
    assert out == mr.marshal_service_graph(og)
    g2 = isim.ServiceGraph.from_json(out)
    # sizes go through BytesSize ("%.4g"): exact only when 4 significant
    # binary-unit digits suffice; everything else must round-trip exactly
    c1, c2 = g.canonical(), g2.canonical()
    for s1, s2 in zip(c1["services"], c2["services"]):
        assert (s1["name"], s1["type"], s1["numReplicas"], s1["isEntrypoint"], s1["errorRateBits"]) == \
               (s2["name"], s2["type"], s2["numReplicas"], s2["isEntrypoint"], s2["errorRateBits"])
    d = g.to_dot()
    assert d.startswith("digraph {\n") and d.endswith("\n}\n")
    assert d.count("[label=<") == len(og.services)
