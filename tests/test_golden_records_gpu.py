"""The committed per-trace record fixtures (tests/golden/records/, made once
by the C oracle) reproduced by every HIP kernel kind
through the C ABI, bit for bit: records and stats of the walks (draw stream,
mode-B ancestor marking, close list and bit stack, static interpreter, lane tree walk, wave
walk) and records, stats and DES tables of the per-replica DES (32-bit rows
with the automatic wide retry, and 64-bit rows).  Unlike the parity tests
these compare with stored outputs, so no oracle runs here."""
import numpy as np
import pytest

import golden_records as gr
import isim
from oracle import executor as oc
from parity import assert_records_equal, assert_stats_equal

pytestmark = pytest.mark.gpu

N = isim.native
KERNELS = {
    "default": 0,
    "stream_walk": N.FLAG_WALK_ALL,
    "bitstack": N.FLAG_WALK_ALL | N.FLAG_BIT_STACK,
    "closelist": N.FLAG_WALK_ALL | N.FLAG_CLOSE_LIST,
    "interp": N.FLAG_NO_STREAM,
    "dynamic": N.FLAG_DYNAMIC,
    "dynamic_wave": N.FLAG_DYNAMIC | N.FLAG_WAVE_WALK,
}


def _handler(case, flags=0):
    p = case["params"]
    g = isim.ServiceGraph.from_json(case["graph"])
    return g, isim.Handler(g, case["entry"], isim.SimParams(seed=p["seed"], hop_base_ns=p["hop_base_ns"],
                                                            req_ps_per_byte=p["req_ps_per_byte"],
                                                            resp_ps_per_byte=p["resp_ps_per_byte"],
                                                            error_mode=p["error_mode"], flags=flags))


def _expected_stats(case, fx, des=False):
    sg = gr.oracle_graph(case)[0]  # the loader restatement: service and call-site counts
    ns, nsite = len(sg.g.services), len(sg.sites)
    st = fx["stats"]
    if des:
        st = np.concatenate([st, np.zeros(68 * ns, np.uint64)])
    return oc.split_stats(st, ns, nsite)


@pytest.mark.parametrize("kernel", list(KERNELS))
@pytest.mark.parametrize("case", gr.WALK_CASES, ids=gr.case_id)
def test_walk_matches_fixture(gpu, case, kernel):
    if kernel in ("bitstack", "closelist") and case["params"]["error_mode"] == 0:
        pytest.skip("the bit stack and the close list are mode-B kernels")
    fx = gr.load(case)
    _, h = _handler(case, KERNELS[kernel])
    recs, stats = h.serve(case["begin"], case["n"])
    assert_records_equal(recs, fx["records"])
    assert_stats_equal(h.fold(stats), _expected_stats(case, fx))


@pytest.mark.parametrize("wide", [False, True])
@pytest.mark.parametrize("case", gr.DES_CASES, ids=gr.case_id)
def test_des_matches_fixture(gpu, case, wide):
    fx = gr.load(case)
    _, h = _handler(case)
    d = isim.DesHandler(h, case["des_mean_ns"])
    recs, stats, table = d.serve(case["begin"], case["n"], wide=wide)
    assert_records_equal(recs, fx["records"])
    f = h.fold(stats)
    f["svc_dur"] = None
    assert_stats_equal(f, _expected_stats(case, fx, des=True))
    rows = d.fold(table)
    assert np.array_equal(rows, fx["des"]), np.argwhere(rows != fx["des"])[:4].tolist()
