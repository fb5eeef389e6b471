"""CPU check of the DES item engine's algorithm: the C++
restatement in tests/cpp/des_items_check.cpp runs the product's own plan
(build_des_plan over the lane tree walk's positions) and pre-walk with the
engine's rounds, queue order and fixed-point passes in plain loops; its
records, stats and DES table must equal the event-driven oracle's
(oracle/des_oracle.c) bit for bit.  The HIP kernels are checked against the
same oracle by tests/test_des_items_gpu.py."""
import os
import shutil
import subprocess

import numpy as np
import pytest

import isim
from isim.yamljson import obj_to_json
from oracle import des as od
from oracle import executor as oc
from oracle import graph_ref as gr
from oracle.executor_py import SimGraph

from parity import assert_records_equal, assert_stats_equal, oracle_params
from test_des_items_gpu import CASES, MODE_B_CASES

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "istio-isotope_amd", "csrc")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    out = str(tmp_path_factory.mktemp("dic") / "des_items_check")
    srcs = [os.path.join(ROOT, "tests", "cpp", "des_items_check.cpp")] + \
        [os.path.join(CSRC, f) for f in ("json.cpp", "gounits.cpp", "graph.cpp", "program.cpp", "des_plan.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"), "-I", CSRC, *srcs,
                    "-o", out], check=True)
    return out


def _check(checker, tmp_path, doc, mean, begin, n, mode=isim.MODE_A):
    j = obj_to_json(doc)
    (tmp_path / "g.json").write_text(j)
    h = isim.Handler(isim.ServiceGraph.from_json(j), None,
                     isim.SimParams(flags=isim.native.FLAG_DYNAMIC, error_mode=mode))
    d = isim.DesHandler(h, mean)
    assert d.info.items == 1
    p = h.params
    prefix = str(tmp_path / "out")
    r = subprocess.run([checker, str(tmp_path / "g.json"), str(p.seed), str(p.hop_base_ns), str(p.req_ps_per_byte),
                        str(p.resp_ps_per_byte), str(mean), str(begin), str(n), prefix,
                        "1" if mode == isim.MODE_B else "0"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr + r.stdout
    rec = np.fromfile(prefix + ".rec", np.uint64).reshape(n, 2)
    st = np.fromfile(prefix + ".stats", np.uint64)
    tab = np.fromfile(prefix + ".table", np.uint64)
    sg = SimGraph(gr.unmarshal_service_graph(j))
    op = oracle_params(h.params)
    orec, ost, odes = od.run(sg, op, sg.entry(), begin, n, mean)
    recs = np.zeros(n, isim.REC_DTYPE)
    recs["latency_ns"] = rec[:, 0]
    recs["hops"] = (rec[:, 1] & 0xFFFFFFFF).astype(np.uint32)
    recs["status_err"] = (rec[:, 1] >> np.uint64(32)).astype(np.uint32)
    assert_records_equal(recs, orec)
    stats = np.zeros(h.info.stats_words, np.uint64)
    stats[:st.size] = st
    ns, nsite = len(sg.g.services), len(sg.sites)
    o = oc.split_stats(np.concatenate([ost, np.zeros(68 * ns, np.uint64)]), ns, nsite)
    f = h.fold(stats)
    f["svc_dur"] = None
    assert_stats_equal(f, o)
    rows = d.fold(tab)
    bad = np.argwhere(rows != odes)
    assert bad.size == 0, f"DES table differs at {bad[:4].tolist()}"
    return r.stdout


@pytest.mark.parametrize("mean", [300_000, 3_000_000])
@pytest.mark.parametrize("name", sorted(CASES))
def test_restatement_matches_event_oracle(checker, tmp_path, name, mean):
    out = _check(checker, tmp_path, CASES[name](), mean, 1000, 1500)
    if name in ("canonical_p50", "mesh_des"):
        assert "cyclic 1" in out  # the fixed-point passes are exercised
    _check(checker, tmp_path, CASES[name](), mean, (1 << 32) - 300, 601)


@pytest.mark.parametrize("mean", [300_000, 3_000_000])
@pytest.mark.parametrize("name", sorted(MODE_B_CASES))
def test_restatement_mode_b(checker, tmp_path, name, mean):
    """Mode B: the walks draw errors, a failed call step ends its script (no
    later step, sleep or call), the worker hold stays the service's sleep
    total; the oracle's walk records where each script
    stops and its simulation responds there."""
    _check(checker, tmp_path, MODE_B_CASES[name](), mean, 1000, 1500, isim.MODE_B)
    _check(checker, tmp_path, MODE_B_CASES[name](), mean, (1 << 32) - 300, 601, isim.MODE_B)
