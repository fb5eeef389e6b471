"""The executor known-answer tests on the HIP path (through the C ABI).

Every case of tests/golden/executor_kat.json — SURVEY Appendix B on the
reference's own graphs (isotope/convert/pkg/graphviz/graphviz_test.go:111-168,
example-topologies/canonical.yaml, convert/pkg/graph/unmarshal_test.go:82-126,
the create_tree_topology.py trees) plus the hand-derived abort, default-script
(F11) and 500-payload cases (executable.go:107-120,148-179, handler.go:59,66-76)
— is run on every kernel kind that can take it, and the per-trace record, the
per-service calls / 500s, the request / response size histograms and the
entry's duration histogram are asserted equal to the HAND-DERIVED numbers
(not to the oracle).  All these graphs are deterministic (errorRate 0 or 1),
so every trace of a batch must carry the same record."""
import numpy as np
import pytest

import isim
import kat

pytestmark = pytest.mark.gpu

N = isim.native
KERNELS = {
    "stream": 0,                                   # draw-free graphs: one walk + record fill
    "stream_walk": N.FLAG_WALK_ALL,                # kinds 4 (mode A) / 8 (mode B ancestor marking)
    "closelist": N.FLAG_WALK_ALL | N.FLAG_CLOSE_LIST,  # mode B: kind 6 (the close list)
    "bitstack": N.FLAG_WALK_ALL | N.FLAG_BIT_STACK,  # mode B: kind 5
    "interp": N.FLAG_NO_STREAM,                    # static interpreter, kinds 0/1
    "dynamic": N.FLAG_DYNAMIC,                     # general path: the lane tree walk, kind 7
    "dynamic_nodur": N.FLAG_DYNAMIC | N.FLAG_NO_SVC_DUR,
    "dynamic_wave": N.FLAG_DYNAMIC | N.FLAG_WAVE_WALK,  # the wave walk, kinds 2/3 (per-lane time)
}


@pytest.mark.parametrize("kernel", list(KERNELS))
@pytest.mark.parametrize("case", kat.CASES, ids=kat.case_id)
def test_kat_hip(gpu, case, kernel):
    hop, req, resp, mode = kat.params(case)
    flags = KERNELS[kernel]
    if kernel in ("bitstack", "closelist") and mode == 0:
        pytest.skip("the bit stack and the close list are mode-B kernels")
    j = kat.graph_json(case["graph"])
    g = isim.ServiceGraph.from_json(j)
    h = isim.Handler(g, case["entry"], isim.SimParams(seed=1, hop_base_ns=hop, req_ps_per_byte=req,
                                                      resp_ps_per_byte=resp, error_mode=mode, flags=flags))
    kind = h.launch_info(0)["kernel_kind"]
    if kernel == "dynamic_wave":
        assert kind in (2, 3)
    elif kernel.startswith("dynamic"):
        # the lane tree walk (u32 or u64 time); kind 3 only when a position's own time reaches 2^32 ns
        assert kind == 7 or (h.info.time_bits == 64 and kind == 3)
    elif kernel == "interp":
        assert kind in (0, 1) or not h.info.static_walk
    elif kernel == "stream_walk" and mode == 1 and h.info.static_walk:
        assert kind == 8
    elif kernel == "closelist" and h.info.static_walk:
        assert kind == 6
    n = 3000
    begin = (1 << 32) - 1500  # the batch straddles trace id 2^32
    recs, stats = h.serve(begin, n)
    for f in ("latency_ns", "hops", "status_err"):
        assert np.all(recs[f] == recs[f][0]), f
    r = recs[0]
    kat.check_record(case, int(r["latency_ns"]), int(r["hops"]), int(r["status_err"]) >> 31,
                     int(r["status_err"]) & 0x7FFFFFFF)
    f = h.fold(stats)
    names = [s.name for s in g.services]
    kat.check_folded(case, names, f, n, g)
    assert f["n_traces"] == n and f["sum_latency"] == n * case["latency"] and f["sum_hops"] == n * case["hops"]
    assert f["min_latency"] == f["max_latency"] == case["latency"]
    # the entry's RecordResponseSent duration histogram: n observations of the latency
    if f["svc_dur"] is not None:
        from oracle.executor_py import prom_bucket
        code = 1 if case.get("status", 200) == 500 else 0
        row = f["svc_dur"][names.index(case["entry"])]
        assert int(row[code * N.N_PROM + prom_bucket(case["latency"])]) == n
        assert int(row[2 * N.N_PROM + code]) == n * case["latency"]
