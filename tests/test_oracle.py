"""The oracle itself, pinned against the reference's own test vectors
(tests/golden/go_vectors.json), the Random123 Philox KATs and the Appendix B
executor KATs; plus the pure-Python vs C executor cross-check."""
import json
import os

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import kat
from conftest import GOLDEN
from oracle import executor as oc
from oracle import executor_py as ex
from oracle import gounits as gu
from oracle import graph_ref as gr
from oracle import philox

VEC = json.load(open(os.path.join(GOLDEN, "go_vectors.json")))
PHX = json.load(open(os.path.join(GOLDEN, "philox_kat.json")))


@pytest.mark.parametrize("x,want,err", VEC["size_from_int64"]["cases"])
def test_size_from_int64(x, want, err):
    if err:
        with pytest.raises(gu.NegativeSizeError):
            gu.size_from_int64(x)
    else:
        assert gu.size_from_int64(x) == want


@pytest.mark.parametrize("s,want,err", VEC["size_from_string"]["cases"])
def test_size_from_string(s, want, err):
    assert gu.size_from_string(s) == want


@pytest.mark.parametrize("f,want,err", VEC["pct_from_float"]["cases"])
def test_pct_from_float(f, want, err):
    if err:
        with pytest.raises(gu.OutOfRangeError):
            gu.pct_from_float(f)
    else:
        assert gu.pct_from_float(f) == want


@pytest.mark.parametrize("s,want,err", VEC["pct_from_string"]["cases"])
def test_pct_from_string(s, want, err):
    if err:
        with pytest.raises(getattr(gu, err)):
            gu.pct_from_string(s)
    else:
        assert gu.pct_from_string(s) == want


def test_pct_out_of_range_value():
    # percentage_test.go:58: "110%" -> OutOfRangeError{1.1}
    with pytest.raises(gu.OutOfRangeError) as e:
        gu.pct_from_string("110%")
    assert e.value.f == 1.1


@pytest.mark.parametrize("p,want", VEC["pct_string"]["cases"])
def test_pct_string(p, want):
    assert gu.pct_string(p) == want


@pytest.mark.parametrize("n,want", VEC["bytes_size"]["cases"])
def test_bytes_size(n, want):
    assert gu.bytes_size(float(n)) == want


@pytest.mark.parametrize("s,want", VEC["duration"]["parse"])
def test_parse_duration(s, want):
    assert gu.parse_duration(s) == want


@pytest.mark.parametrize("d,want", VEC["duration"]["string"])
def test_duration_string(d, want):
    assert gu.duration_string(d) == want


@pytest.mark.parametrize("s,want", [
    ("1h2m3.5s", 3723500000000), ("1.5us", 1500), ("1.5µs", 1500), ("1.5μs", 1500), ("-2m", -120000000000),
    ("+3ns", 3), ("0", 0), (".5s", 500000000), ("1.s", 1000000000), ("2562047h47m16.854775807s", (1 << 63) - 1)])
def test_parse_duration_more(s, want):
    assert gu.parse_duration(s) == want


@pytest.mark.parametrize("s", ["", "1", "h", "1x", ".s", "-", "9223372036854775808ns", "2562048h", "1.2.3s"])
def test_parse_duration_errors(s):
    with pytest.raises(gu.DurationError):
        gu.parse_duration(s)


def test_ram_in_bytes_edges():
    assert gu.ram_in_bytes("1.5k") == 1536
    assert gu.ram_in_bytes("5 ") == 5
    assert gu.ram_in_bytes("3P") == 3 << 50
    assert gu.ram_in_bytes("100000000P") == gu.INT64_MIN   # Go float->int64 overflow
    for bad in ["", "k", "-1", "1 2", "1kk", "1.k", " 1", "1e3", "1.2.3"]:
        with pytest.raises((gu.InvalidSizeError, gu.ParseFloatError)):
            gu.ram_in_bytes(bad)


def test_request_command_vectors():
    for key, dflt in (("default_size_0", 0), ("default_size_512", 512)):
        for raw, name, size in VEC["request_command"][key]:
            c = gr.unmarshal_request(gr.loads(raw), gr.RequestCommand(size=dflt))
            assert (c.service, c.size, c.probability) == (name, size, 0)


def test_script_vectors():
    for raw, want in VEC["script"]["cases"]:
        got = [gr._cmd_canon(c) for c in gr.parse_commands(gr.loads(raw), gr.RequestCommand())]
        assert got == want


def test_service_vectors():
    for raw, want, err in VEC["service"]["cases"]:
        if err:
            with pytest.raises(gr.ErrEmptyName):
                gr.unmarshal_service(gr.loads(raw), gr.Service(), gr.RequestCommand())
        else:
            s = gr.unmarshal_service(gr.loads(raw), gr.Service(), gr.RequestCommand())
            assert (s.name, s.type, s.num_replicas) == (want["name"], want["type"], want["numReplicas"])


def _canon_services(want):
    import struct
    out = []
    for s in want:
        s = dict(s)
        s["errorRateBits"] = struct.unpack("<Q", struct.pack("<d", s.pop("errorRate")))[0]
        out.append(s)
    return out


def test_service_graph_vectors():
    v = VEC["service_graph"]
    for key in ("one_service", "defaults_and_many_services"):
        g = gr.unmarshal_service_graph(v[key]["json"])
        assert gr.canonical(g)["services"] == _canon_services(v[key]["services"])
    with pytest.raises(gr.ErrRequestToUndefinedService) as e:
        gr.unmarshal_service_graph(v["undefined_service"]["json"])
    assert str(e.value) == v["undefined_service"]["message"]
    with pytest.raises(gr.ErrNestedConcurrentCommand):
        gr.unmarshal_service_graph(v["nested_concurrent"]["json"])


@pytest.mark.parametrize("case", PHX["cases"])
def test_philox_kat(case):
    ctr = [int(x, 16) for x in case["ctr"]]
    key = [int(x, 16) for x in case["key"]]
    want = tuple(int(x, 16) for x in case["out"])
    assert philox.philox4x32_10(ctr, key) == want
    assert oc.philox(ctr, key) == want


@pytest.mark.parametrize("case", kat.CASES, ids=kat.case_id)
def test_executor_kat(case):
    import isim
    j = kat.graph_json(case["graph"])
    g = gr.unmarshal_service_graph(j)
    sg = ex.SimGraph(g)
    hop, req, resp, mode = kat.params(case)
    p = ex.SimParams(seed=1, hop_base_ns=hop, req_ps_per_byte=req, resp_ps_per_byte=resp, error_mode=mode)
    e = sg.entry(case["entry"])
    recs, st = ex.run(sg, p, e, 0, 1)
    kat.check_record(case, *recs[0][:2], recs[0][2], recs[0][3])
    crec, cst = oc.run(sg, p, e, 0, 3)
    for r in crec:
        kat.check_record(case, int(r[0]), int(r[1]) & 0xFFFFFFFF, int(r[1]) >> 63, (int(r[1]) >> 32) & 0x7FFFFFFF)
    names = [s.name for s in g.services]
    kat.check_folded(case, names, {"svc_calls": st.svc_calls, "svc_errs": st.svc_errs, "site_calls": st.site_calls}, 1,
                     isim.ServiceGraph.from_json(j))
    kat.check_folded(case, names, oc.split_stats(cst, len(g.services), len(sg.sites)), 3)


# ---- pure-Python executor vs C executor on random small graphs -------------
@st.composite
def random_graph(draw):
    n = draw(st.integers(1, 7))
    services = []
    for i in range(n):
        steps = []
        for _ in range(draw(st.integers(0, 4))):
            kind = draw(st.sampled_from(["sleep", "call", "conc"]))
            if kind == "sleep":
                steps.append({"sleep": f"{draw(st.integers(-2, 40))}ms"})
            elif kind == "call" and i + 1 < n:
                steps.append({"call": {"service": f"s{draw(st.integers(i + 1, n - 1))}",
                                       "size": draw(st.integers(0, 5000)),
                                       "probability": draw(st.sampled_from([0, 0, 1, 30, 50, 99, 100]))}})
            elif kind == "conc" and i + 1 < n:
                sub = []
                for _ in range(draw(st.integers(0, 3))):
                    if draw(st.booleans()):
                        sub.append({"call": f"s{draw(st.integers(i + 1, n - 1))}"})
                    else:
                        sub.append({"sleep": f"{draw(st.integers(0, 9))}ms"})
                steps.append(sub)
        svc = {"name": f"s{i}", "script": steps,
               "errorRate": draw(st.sampled_from([0, 0.001, 0.1, 0.5, 1.0])),
               "responseSize": draw(st.integers(0, 100000))}
        services.append(svc)
    services[0]["isEntrypoint"] = True
    return json.dumps({"defaults": {"requestSize": 100}, "services": services})


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(random_graph(), st.sampled_from([0, 1]), st.integers(0, 2 ** 64 - 1), st.integers(0, 2 ** 40))
def test_python_vs_c_executor(j, mode, seed, begin):
    sg = ex.SimGraph(gr.unmarshal_service_graph(j))
    p = ex.SimParams(seed=seed, error_mode=mode)
    recs, st_ = ex.run(sg, p, 0, begin, 40)
    crec, cst = oc.run(sg, p, 0, begin, 40)
    assert [r[0] for r in recs] == [int(x) for x in crec[:, 0]]
    assert [r[1] | ((r[2] << 31 | r[3]) << 32) for r in recs] == [int(x) for x in crec[:, 1]]
    cs = oc.split_stats(cst, len(sg.g.services), len(sg.sites))
    assert list(cs["svc_calls"]) == st_.svc_calls
    assert list(cs["svc_errs"]) == st_.svc_errs
    assert list(cs["site_calls"]) == st_.site_calls
    dur = cs["svc_dur"]
    assert dur[:, :2 * ex.N_PROM].reshape(-1, 2, ex.N_PROM).tolist() == st_.svc_dur
    assert dur[:, 2 * ex.N_PROM:].tolist() == st_.svc_dur_sum
    # the entry's own duration histogram is the end-to-end latency histogram
    assert dur[0, :2 * ex.N_PROM].reshape(2, ex.N_PROM).tolist() == cs["lat_prom"].tolist()
    assert int(dur[0, 2 * ex.N_PROM:].sum()) == cs["sum_latency"]
    # one observation per invocation, split by code as the 500 counters
    assert dur[:, ex.N_PROM:2 * ex.N_PROM].sum(axis=1).tolist() == list(cs["svc_errs"])
    assert dur[:, :2 * ex.N_PROM].sum(axis=1).tolist() == list(cs["svc_calls"])
    assert cs["lat_prom"].tolist() == st_.lat_prom and cs["lat_log2"].tolist() == st_.lat_log2
    assert (cs["sum_latency"], cs["sum_hops"], cs["n_500"]) == (st_.sum_latency, st_.sum_hops, st_.n_500)


def test_oracle_cycle_rejected():
    sg = ex.SimGraph(gr.unmarshal_service_graph(
        '{"services":[{"name":"a","isEntrypoint":true,"script":[{"call":"b"}]},{"name":"b","script":[{"call":"a"}]}]}'))
    with pytest.raises(oc.CycleError):
        oc.run(sg, ex.SimParams(), 0, 0, 1)


def test_prom_buckets():
    edges = ex.PROM_EDGES_NS
    assert ex.prom_bucket(0) == 0 and ex.prom_bucket(edges[0]) == 0 and ex.prom_bucket(edges[0] + 1) == 1
    assert ex.prom_bucket(edges[-1]) == 31 and ex.prom_bucket(edges[-1] + 1) == 32
    assert ex.log2_bucket(0) == 0 and ex.log2_bucket(1) == 1 and ex.log2_bucket(2 ** 62) == 63
    assert np.all(np.diff(edges) > 0)
