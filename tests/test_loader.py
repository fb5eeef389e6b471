"""The product's C++ graph loader (isim_graph_unmarshal_json through the C
ABI) against the reference's Go test vectors and against the oracle's
restatement of (*ServiceGraph).UnmarshalJSON — on every reference topology,
hand-written edge cases and hypothesis-generated documents.  CPU only."""
import glob
import json
import os
import struct

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import isim
from conftest import GOLDEN, TOPOLOGIES
from oracle import gounits as gu
from oracle import graph_ref as gr

VEC = json.load(open(os.path.join(GOLDEN, "go_vectors.json")))

# Go error message prefix -> oracle exception class
KINDS = [
    ("cannot call undefined service", gr.ErrRequestToUndefinedService),
    ("concurrent commands may not be nested", gr.ErrNestedConcurrentCommand),
    ("services must have a name", gr.ErrEmptyName),
    ("unknown command:", gr.UnknownCommandKeyError),
    ("multiple keys for command", gr.MultipleKeysInCommandMapError),
    ("math: invalid probability", gr.InvalidProbabilityError),
    ("unknown service type:", gr.InvalidServiceTypeStringError),
    ("invalid percentage as string", gu.InvalidPercentageStringError),
    ("percentage ", gu.OutOfRangeError),
    ("invalid size:", gu.InvalidSizeError),
    ("strconv.ParseFloat", gu.ParseFloatError),
    ("time: ", gu.DurationError),
    ("json: cannot unmarshal", gr.UnmarshalTypeError),
]


def product_kind(msg: str):
    for prefix, cls in KINDS:
        if msg.startswith(prefix):
            return cls
    if msg.endswith("must be non-negative"):
        return gu.NegativeSizeError
    return "syntax"


def load_both(doc: str):
    """(product canonical | error kind, oracle canonical | error kind)."""
    try:
        p = isim.ServiceGraph.from_json(doc).canonical()
    except isim.GraphError as e:
        p = product_kind(str(e))
    try:
        o = gr.canonical(gr.unmarshal_service_graph(doc))
    except (json.JSONDecodeError, ValueError) as e:
        o = type(e) if isinstance(e, gu.GoError) else "syntax"
    except gu.GoError as e:
        o = type(e)
    return p, o


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(TOPOLOGIES, "*.yaml"))),
                         ids=lambda p: os.path.basename(p))
def test_reference_topologies(path):
    doc = isim.yaml_to_json(open(path, "rb").read())
    p, o = load_both(doc)
    assert isinstance(p, dict) and p == o


def _canon(want):
    out = []
    for s in want:
        s = dict(s)
        s["errorRateBits"] = struct.unpack("<Q", struct.pack("<d", s.pop("errorRate")))[0]
        out.append(s)
    return out


def test_go_service_graph_vectors():
    v = VEC["service_graph"]
    for key in ("one_service", "defaults_and_many_services"):
        g = isim.ServiceGraph.from_json(v[key]["json"])
        assert g.canonical()["services"] == _canon(v[key]["services"])
    for key in ("undefined_service", "nested_concurrent"):
        with pytest.raises(isim.GraphError) as e:
            isim.ServiceGraph.from_json(v[key]["json"])
        assert str(e.value) == v[key]["message"]


def test_go_service_vectors():
    for raw, want, err in VEC["service"]["cases"]:
        doc = '{"services": [' + raw + "]}"
        if err:
            with pytest.raises(isim.GraphError, match="services must have a name"):
                isim.ServiceGraph.from_json(doc)
        else:
            s = isim.ServiceGraph.from_json(doc).services[0]
            assert (s.name, s.type, s.num_replicas) == (want["name"], want["type"], want["numReplicas"])


def test_go_request_command_vectors():
    for key, dflt in (("default_size_0", 0), ("default_size_512", 512)):
        for raw, name, size in VEC["request_command"][key]:
            doc = ('{"defaults": {"requestSize": %d}, "services": [{"name": "%s"}, {"name": "x", "script": [{"call": %s}]}]}'
                   % (dflt, name, raw))
            c = isim.ServiceGraph.from_json(doc).services[1].script[0]
            assert (c.service, c.size, c.probability) == (name, size, 0)


def test_go_script_vectors():
    for raw, want in VEC["script"]["cases"]:
        doc = '{"services": [{"name": "A"}, {"name": "B"}, {"name": "x", "script": ' + raw + "}]}"
        assert isim.ServiceGraph.from_json(doc).canonical()["services"][2]["script"] == want


@pytest.mark.parametrize("s,want,err", VEC["size_from_string"]["cases"])
def test_size_from_string(s, want, err):
    assert isim.size_from_string(s) == want


@pytest.mark.parametrize("s,want,err", VEC["pct_from_string"]["cases"])
def test_pct_from_string(s, want, err):
    if err:
        with pytest.raises(isim.GraphError):
            isim.percentage_from_string(s)
    else:
        assert isim.percentage_from_string(s) == want


@pytest.mark.parametrize("s", ["100ms", "1s", "10ms", "1h2m3.5s", "1.5µs", "1.5μs", "-2m", ".5s", "0",
                               "2562047h47m16.854775807s", "1.0000000000000000001h", "3.999999999999ns"])
def test_duration_matches_oracle(s):
    assert isim.duration_parse(s) == gu.parse_duration(s)


@pytest.mark.parametrize("s", ["", "1", "h", "1x", ".s", "9223372036854775808ns", "2562048h"])
def test_duration_errors(s):
    with pytest.raises(isim.GraphError):
        isim.duration_parse(s)


@pytest.mark.parametrize("s", ["0", "10k", "1.5k", "5 ", "3P", "100000000P", "9223372036854775807",
                               "1e3", "1.2.3", "", "k", "10 KiB", "7b", "7ib"])
def test_size_matches_oracle(s):
    try:
        want = gu.size_from_string(s)
    except gu.GoError:
        with pytest.raises(isim.GraphError):
            isim.size_from_string(s)
        return
    assert isim.size_from_string(s) == want


EDGE_DOCS = [
    '{"services": null}',
    'null',
    '[]',
    '{"services": [null]}',
    '{"services": [{"name": "a", "script": null}]}',
    '{"defaults": {"script": [{"call": "a"}]}, "services": [{"name": "a"}]}',        # F11 size 0... and self call
    '{"defaults": {"requestSize": 7, "script": [{"call": "b"}]}, "services": [{"name": "a"}, {"name": "b", "script": []}]}',
    '{"default": {"requestSize": 7}, "services": [{"name": "a", "script": [{"call": "a"}]}]}',  # F10
    '{"services": [{"NAME": "a", "IsEntryPoint": true, "errorrate": "5%"}]}',        # case-insensitive fields
    '{"services": [{"name": "a", "type": "HTTP"}]}',
    '{"services": [{"name": "a", "type": null}]}',
    '{"services": [{"name": "a", "numReplicas": "3"}]}',
    '{"services": [{"name": "a", "numReplicas": 2.0}]}',
    '{"services": [{"name": "a", "numReplicas": 4294967296}]}',
    '{"services": [{"name": "a", "responseSize": -1}]}',
    '{"services": [{"name": "a", "responseSize": 1.5}]}',
    '{"services": [{"name": "a", "responseSize": null}]}',
    '{"services": [{"name": "a", "responseSize": "1 GB"}]}',
    '{"services": [{"name": "a", "errorRate": 1.0000001}]}',
    '{"services": [{"name": "a", "errorRate": "50%%"}]}',
    '{"services": [{"name": "a", "errorRate": "x%"}]}',
    '{"services": [{"name": "a", "errorRate": "0x1p-3%"}]}',
    '{"services": [{"name": "a", "errorRate": "inf%"}]}',
    '{"services": [{"name": "a", "errorRate": true}]}',
    '{"services": [{"name": "a", "script": [{"sleep": "1s", "call": "a"}]}]}',
    '{"services": [{"name": "a", "script": [{}]}]}',
    '{"services": [{"name": "a", "script": [null]}]}',
    '{"services": [{"name": "a", "script": ["a"]}]}',
    '{"services": [{"name": "a", "script": [{"Sleep": "1s"}]}]}',
    '{"services": [{"name": "a", "script": [{"sleep": 5}]}]}',
    '{"services": [{"name": "a", "script": [{"sleep": null}]}]}',
    '{"services": [{"name": "a", "script": [{"call": null}]}]}',
    '{"services": [{"name": "a", "script": [{"call": 5}]}]}',
    '{"services": [{"name": "a", "script": [{"call": {"service": "a", "probability": 101}}]}]}',
    '{"services": [{"name": "a", "script": [{"call": {"service": "a", "probability": -1}}]}]}',
    '{"services": [{"name": "a", "script": [{"call": {"service": "a", "probability": 50.5}}]}]}',
    '{"services": [{"name": "a", "script": [{"call": {"Service": "a", "SIZE": "2k", "extra": 1}}]}]}',
    '{"services": [{"name": "a", "script": [[]]}]}',
    '{"services": [{"name": "a", "script": [[[]]]}]}',
    '{"services": [{"name": "a"}, {"name": "a", "errorRate": 0.5}]}',
    '{"services": [{"name": "a", "numReplicas": "x", "script": [{"bogus": 1}]}]}',
    '{"services": [{"name": 5}]}',
    '{"services": {"name": "a"}}',
    '{"services": [{"name": "a"}], "services": [{"name": "b"}]}',
    '{"services": [{"name": "a", "isEntrypoint": "yes"}]}',
    '{"services": [{"name": "a\\u00e9\\ud83d\\ude00", "script": [{"sleep": "1\\u00b5s"}]}]}',
    '{"services": [{"name": "a"}]',
    '{"services": [{"name": "a"}]} x',
    '{"services": [{"name": "a", "errorRate": 01}]}',
    '{"services": [{"name": "a", "errorRate": -0}]}',
    '{"services": [{"name": "a", "errorRate": 1e-400}]}',
    '{"services": [{"name": "a", "errorRate": 1E0}]}',
]


@pytest.mark.parametrize("doc", EDGE_DOCS)
def test_edge_documents(doc):
    p, o = load_both(doc)
    assert p == o, (p, o)


# ---- hypothesis: random documents over the schema's vocabulary ------------
_names = st.sampled_from(["a", "b", "c", "A", ""])
_sizes = st.one_of(st.integers(-5, 10 ** 6), st.sampled_from(["1 KB", "10k", "1.5M", "x", "2 GiB", "-1"]),
                   st.none(), st.floats(0, 10, allow_nan=False))
_durs = st.one_of(st.sampled_from(["1ms", "10ms", "1.5s", "-3ms", "100us", "1h", "bad", "0", ""]), st.none(),
                  st.integers(0, 5))
_pcts = st.one_of(st.floats(-0.5, 1.5, allow_nan=False), st.sampled_from(["5%", "100%", "110%", "1", "x%"]),
                  st.none())


def _call():
    return st.one_of(_names, st.fixed_dictionaries({}, optional={
        "service": _names, "size": _sizes, "probability": st.one_of(st.integers(-2, 102), st.none())}))


def _cmd(depth=0):
    leaf = st.one_of(st.builds(lambda d: {"sleep": d}, _durs), st.builds(lambda c: {"call": c}, _call()))
    if depth >= 2:
        return leaf
    return st.one_of(leaf, st.lists(_cmd(depth + 1), max_size=3))


_service = st.fixed_dictionaries({"name": _names}, optional={
    "type": st.sampled_from(["http", "grpc", "tcp"]), "numReplicas": st.integers(0, 5),
    "isEntrypoint": st.booleans(), "errorRate": _pcts, "responseSize": _sizes,
    "script": st.lists(_cmd(), max_size=4), "numRbacPolicies": st.integers(0, 3)})
_doc = st.fixed_dictionaries({"services": st.lists(_service, max_size=4)}, optional={
    "defaults": st.fixed_dictionaries({}, optional={
        "requestSize": _sizes, "responseSize": _sizes, "errorRate": _pcts, "numReplicas": st.integers(0, 4),
        "type": st.sampled_from(["http", "grpc"]), "script": st.lists(_cmd(), max_size=3)})})


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(_doc)
def test_random_documents(doc):
    p, o = load_both(json.dumps(doc))
    assert p == o, (p, o)
