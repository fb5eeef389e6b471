"""The C ABI boundary on CPU: the library loads, exports exactly what
include/isim.h declares, and the host-side (no GPU) entry points behave:
handler compilation, static analysis and error codes."""
import ctypes as C
import json
import os
import re
import subprocess

import pytest

import isim
from isim import native
from conftest import ROOT, TOPOLOGIES

HEADER = os.path.join(ROOT, "include", "isim.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"ISIM_API\s+[^;(]*?\b(isim_\w+)\s*\(", src)))


def test_header_declarations_are_bound():
    assert set(declared_functions()) == set(native.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = native.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", native.LIB_PATH], capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l and l.split()[-1].startswith("isim_")}
    assert exported == set(declared_functions())


def test_abi_version():
    assert native.load().isim_abi_version() == native.ABI_VERSION == 10


def _handler(doc, entry=None, **kw):
    return isim.Handler(isim.ServiceGraph.from_json(json.dumps(doc) if isinstance(doc, dict) else doc), entry,
                        isim.SimParams(**kw))


def test_handler_info_canonical():
    h = isim.handler_from_service_graph_yaml(os.path.join(TOPOLOGIES, "canonical.yaml"))
    i = h.info
    assert (i.n_services, i.n_sites, i.n_slots, i.max_depth) == (4, 5, 5, 3)
    assert i.static_walk == 1 and i.hops_upper == 6
    # H = 250us + (1024*80 + 1024*80)/1000 ns = 250163 ns per call; d: [a || c(a, b)], b
    assert i.max_latency_ns == 250163 * 4
    assert i.stats_words == native.ST_SITES + 2 * 5


def test_mode_b_makes_canonical_dynamic():
    # with errors possible, d's concurrent step can fail (mode B) and is
    # followed by `call b`, so a failure would skip a step
    doc = json.loads(isim.yaml_to_json(open(os.path.join(TOPOLOGIES, "canonical.yaml"), "rb").read()))
    assert _handler(doc, error_mode=isim.MODE_B).info.static_walk == 1   # no errorRate: nothing fails
    doc["defaults"]["errorRate"] = 0.1
    assert _handler(doc, error_mode=isim.MODE_B).info.static_walk == 0
    assert _handler(doc, error_mode=isim.MODE_A).info.static_walk == 1
    doc = {"services": [{"name": "a", "isEntrypoint": True, "script": [{"call": "b"}]}, {"name": "b", "errorRate": 0.5}]}
    assert _handler(doc, error_mode=isim.MODE_B).info.static_walk == 1   # failing step is the last


def test_probability_makes_walk_dynamic():
    doc = {"services": [{"name": "a", "isEntrypoint": True, "script": [{"call": {"service": "b", "probability": 50}}]},
                        {"name": "b"}]}
    assert _handler(doc).info.static_walk == 0
    doc["services"][0]["script"][0]["call"]["probability"] = 100   # 100 never skips
    assert _handler(doc).info.static_walk == 1


def test_time_bits():
    small = {"services": [{"name": "a", "isEntrypoint": True, "script": [{"sleep": "4s"}]}]}
    big = {"services": [{"name": "a", "isEntrypoint": True, "script": [{"sleep": "5s"}]}]}
    assert _handler(small).info.time_bits == 32 and _handler(big).info.time_bits == 64


def test_error_codes():
    cyc = {"services": [{"name": "a", "isEntrypoint": True, "script": [{"call": "b"}]},
                        {"name": "b", "script": [{"call": "a"}]}]}
    with pytest.raises(isim.IsimError) as e:
        _handler(cyc)
    assert e.value.status == "ECYCLE"
    chain = {"services": [{"name": f"s{i}", "script": [{"call": f"s{i + 1}"}] if i < 70 else []} for i in range(71)]}
    chain["services"][0]["isEntrypoint"] = True
    with pytest.raises(isim.IsimError) as e:
        _handler(chain)
    assert e.value.status == "EDEPTH"
    with pytest.raises(isim.IsimError) as e:
        _handler(chain, "s10", max_depth=30)
    assert e.value.status == "EDEPTH"
    assert _handler(chain, "s10").info.max_depth == 61
    noentry = {"services": [{"name": "a"}]}
    with pytest.raises(isim.IsimError) as e:
        _handler(noentry)
    assert e.value.status == "EINVAL"
    with pytest.raises(isim.IsimError) as e:
        _handler(noentry, "zz")
    assert e.value.status == "ENOTFOUND"
    huge = {"services": [{"name": "a", "isEntrypoint": True, "script": [{"sleep": "2000000h"}, {"sleep": "2000000h"},
                                                                        {"sleep": "2000000h"}]}]}
    with pytest.raises(isim.IsimError) as e:
        _handler(huge)
    assert e.value.status == "ERANGE"


def test_cycle_not_reachable_is_fine():
    doc = {"services": [{"name": "e", "isEntrypoint": True}, {"name": "a", "script": [{"call": "b"}]},
                        {"name": "b", "script": [{"call": "a"}]}]}
    assert _handler(doc).info.n_slots == 0


def test_duplicate_names_resolve_to_first():
    # extractService picks the first service of a name (srv/graph.go:97-109)
    doc = {"services": [{"name": "e", "isEntrypoint": True, "script": [{"call": "a"}]},
                        {"name": "a", "script": [{"sleep": "1ms"}]}, {"name": "a", "script": [{"sleep": "9ms"}]}]}
    h = _handler(doc, hop_base_ns=0, req_ps_per_byte=0, resp_ps_per_byte=0)
    assert h.info.max_latency_ns == 1_000_000


def test_stats_fold_host_only():
    h = isim.handler_from_service_graph_yaml(os.path.join(TOPOLOGIES, "canonical.yaml"))
    import numpy as np
    st = h.new_stats()
    st[native.ST_N_TRACES] = 10
    st[native.ST_N_500] = 2
    st[native.ST_SITES:native.ST_SITES + 5] = [10, 10, 10, 10, 10]      # calls per slot
    st[native.ST_SITES + 5:native.ST_SITES + 10] = [1, 0, 0, 3, 0]      # callee 500s
    f = h.fold(st)
    g = h.graph.services
    names = [s.name for s in g]
    assert dict(zip(names, f["svc_calls"].tolist())) == {"a": 20, "b": 20, "c": 10, "d": 10}
    assert int(f["svc_errs"][names.index("d")]) == 2
    assert f["site_calls"].tolist() == [10, 10, 10, 10, 10]


def test_stats_fold_durations_static_derivation():
    # static walk: every invocation of a service lasts T(s); the fold splits
    # calls by code from the counters (no device table)
    h = isim.handler_from_service_graph_yaml(os.path.join(TOPOLOGIES, "canonical.yaml"))
    import numpy as np
    assert h.info.svc_dur_rows == 0 and h.info.n_reachable == 4
    st = h.new_stats()
    st[native.ST_N_TRACES] = 10
    st[native.ST_N_500] = 2
    st[native.ST_SITES:native.ST_SITES + 5] = 10
    st[native.ST_SITES + 5:native.ST_SITES + 10] = [1, 0, 0, 3, 0]
    f = h.fold(st)
    names = [s.name for s in h.graph.services]
    dur = f["svc_dur"]
    d = dur[names.index("d")]
    b = int(np.nonzero(d[:native.N_PROM])[0][0])
    # d's T = 4 hops of 250163 ns (1.0007 ms) -> the first bucket (<= 7 ms)
    assert b == 0 and int(d[b]) == 8 and int(d[native.N_PROM + b]) == 2
    assert int(d[2 * native.N_PROM]) == 8 * 250163 * 4 and int(d[2 * native.N_PROM + 1]) == 2 * 250163 * 4
    assert dur[:, :2 * native.N_PROM].sum(axis=1).tolist() == f["svc_calls"].tolist()


def test_dynamic_walk_has_duration_table():
    doc = {"services": [{"name": "a", "isEntrypoint": True, "script": [{"call": {"service": "b", "probability": 50}}]},
                        {"name": "b"}, {"name": "unreachable"}]}
    h = _handler(doc)
    assert h.info.static_walk == 0 and h.info.svc_dur_rows == 2 and h.info.n_reachable == 2
    assert h.stats_words == native.ST_SITES + 2 * 1 + 2 * native.SVC_DUR_WORDS
    off = _handler(doc, flags=native.FLAG_NO_SVC_DUR)
    assert off.info.svc_dur_rows == 0 and off.stats_words == native.ST_SITES + 2
    assert off.fold(off.new_stats())["svc_dur"] is None


def test_des_last_batch_zero_before_any_batch():
    """isim_des_last_batch (round 5) is host state: zero before the handler
    served an item-engine batch; the DES class check itself needs no GPU."""
    from isim.generators import config3p_topology
    from isim.yamljson import obj_to_json
    h = isim.Handler(isim.ServiceGraph.from_json(obj_to_json(config3p_topology(50, n=200))), None, isim.SimParams())
    d = isim.DesHandler(h, 1_000_000)
    assert d.info.items == 1
    assert d.last_batch() == {"passes": 0, "syncs": 0, "items": 0}


def test_debug_spin_limit_hook():
    """The look-back timeout hook: process-wide, read at
    each DES launch; the default is 2^26 polls.  The GPU side of the error
    path is tests/test_des_items_gpu.py::test_lookback_timeout_fails_loudly."""
    lib = native.load()
    assert lib.isim_debug_spin_limit() == 1 << 26
    try:
        lib.isim_debug_set_spin_limit(0)
        assert lib.isim_debug_spin_limit() == 0
        lib.isim_debug_set_spin_limit(12345)
        assert lib.isim_debug_spin_limit() == 12345
    finally:
        lib.isim_debug_set_spin_limit(1 << 26)
    assert lib.isim_debug_spin_limit() == 1 << 26
