"""GPU parity of the DES item engine: dynamic walks —
probabilistic calls (shouldSkipRequest, executable.go:84-90), and mode-B
aborts (a failed call step ends its script, handler.go:66-75) — under
per-replica worker-pool contention, through the C ABI, against the
sequential event-driven C oracle (oracle/des_oracle.c: its pre-walk fixes the
executed calls and hop ids) — records, stats and the per-service DES table,
bit-exact; and, for static graphs forced onto the item engine
(ISIM_FLAG_DYNAMIC), against the level-synchronous static engine at sizes the
oracle would take long on."""
import json

import numpy as np
import pytest

import isim
from isim import native
from isim.generators import mesh_des_topology, realistic_topology, tree_topology
from isim.yamljson import obj_to_json

from parity import assert_records_equal
from test_des import _prob_canonical
from test_des_gpu import DesCase, _sleepy_tree

pytestmark = pytest.mark.gpu


def _with_prob(doc, p):
    doc = json.loads(json.dumps(doc))
    for sv in doc["services"]:
        for st in sv.get("script", []):
            for c in (st if isinstance(st, list) else [st]):
                if "call" in c:
                    name = c["call"] if isinstance(c["call"], str) else c["call"]["service"]
                    c["call"] = {"service": name, "probability": p}
    return doc


def _sleepy(doc, pre="400us", post="100us"):
    doc = json.loads(json.dumps(doc))
    for s in doc["services"]:
        s["script"] = [{"sleep": pre}] + s.get("script", []) + [{"sleep": post}]
    return doc


def _zero_hold_min():
    """A sleep-free (zero-hold) service `z` called in the entry's second call
    step, after a probabilistic call: its arrivals leave trace order whenever
    a trace that ran `b` reaches `z` after a later one that skipped it; each
    invocation of `z` must start at its own arrival (des_oracle.c), not at
    the latest arrival before it (the sort-free rounds)."""
    return {"services": [
        {"name": "a", "isEntrypoint": True,
         "script": [{"sleep": "300us"}, {"call": {"service": "b", "probability": 50}}, {"call": "z"}]},
        {"name": "b", "script": [{"sleep": "1ms"}]},
        {"name": "z"},
    ]}


def _zero_hold_mix():
    """Zero-hold services as leaves and as callers (`w` calls `b`), a
    replicated entry, and `b` reached from three positions."""
    return {"services": [
        {"name": "a", "isEntrypoint": True, "numReplicas": 2,
         "script": [{"sleep": "200us"}, {"call": {"service": "b", "probability": 50}}, {"call": "z"},
                    [{"call": {"service": "c", "probability": 60}}, {"call": "w"}], {"call": "z"},
                    {"sleep": "50us"}]},
        {"name": "b", "script": [{"sleep": "700us"}]},
        {"name": "c", "script": [{"sleep": "300us"}, {"call": {"service": "b", "probability": 50}}]},
        {"name": "w", "script": [{"call": {"service": "b", "probability": 40}}, {"call": "z"}]},
        {"name": "z"},
    ]}


CASES = {
    "zero_hold_min": _zero_hold_min,
    "zero_hold_mix": _zero_hold_mix,
    "real300p60": lambda: realistic_topology(300, concurrent=True, sleep_ms=(1, 5), error_rate=(0.0, 0.3),
                                             probability=60),
    "real300seq_p75": lambda: realistic_topology(300, sleep_ms=(1, 5), error_rate=(0.0, 0.3), probability=75),
    # a latency bound past 2^32 ns: the pre-walk keeps u64 time (Program::tree_t64)
    "real300seq_t64": lambda: realistic_topology(300, sleep_ms=(20, 40), error_rate=(0.0, 0.3), probability=75),
    "mesh_des": lambda: mesh_des_topology(4000, 6, 3, 40),
    "canonical_p50": lambda: _sleepy(_prob_canonical()),
    "tree_reps_p70": lambda: _with_prob(_sleepy_tree(3, 4, reps_leaves=3), 70),
    "seq_tree_p50": lambda: _with_prob(_sleepy(tree_topology(3, 3, sequential=True)), 50),
    # ~54 calls of one trace reach `z` at the same instant: runs of equal queue
    # keys longer than k_tiefix's insertion-sort bound (its heapsort)
    "fanout_ties": lambda: {"services": [
        {"name": "a", "isEntrypoint": True,
         "script": [{"sleep": "100us"}, [{"call": {"service": "z", "probability": 90}}] * 60]},
        {"name": "z", "script": [{"sleep": "10us"}]}]},
}


def _err(doc, rate):
    doc = json.loads(json.dumps(doc))
    for i, s in enumerate(doc["services"]):
        s["errorRate"] = rate if not isinstance(rate, list) else rate[i % len(rate)]
    return doc


# mode B (EXT): a callee's 500 fails its call step and ends the caller's
# script (handler.go:66-75 with the 500 propagated); a call step or sleep
# after a step that can fail makes the walk dynamic even without
# probabilities, so these run on the item engine
MODE_B_CASES = {
    # sequential steps with sleeps between and after: aborts skip both
    "seq_tree_abort": lambda: _err(_sleepy(tree_topology(3, 3, sequential=True)), [0.15, 0.0, 0.3]),
    # concurrent steps: the step waits for every callee, then the script ends
    "conc_tree_abort": lambda: _err(_sleepy_tree(3, 4, reps_leaves=2), [0.2, 0.0, 0.05]),
    "canonical_p50_b": lambda: _err(_sleepy(_prob_canonical()), 0.1),
    "zero_hold_mix_b": lambda: _err(_zero_hold_mix(), [0.0, 0.3, 0.2, 0.5, 0.25]),
    "real300p60_b": CASES["real300p60"],
    "real300seq_b": CASES["real300seq_p75"],
    "real300seq_t64_b": CASES["real300seq_t64"],
    # rare errors: most traces run every step, a few abort deep in the tree
    "real300seq_lo_b": lambda: realistic_topology(300, sleep_ms=(1, 5), error_rate=(0.0, 0.004), probability=75),
    "mesh_des_b": lambda: _err(mesh_des_topology(4000, 6, 3, 40), [0.0, 0.02, 0.1]),
}


@pytest.mark.parametrize("mean", [300_000, 3_000_000])
@pytest.mark.parametrize("name", sorted(CASES))
def test_items_match_event_oracle(gpu, name, mean):
    c = DesCase(CASES[name](), mean)
    assert c.d.info.items == 1
    recs, _, rows = c.compare(1000, 3000)
    assert 0 < int(recs["hops"].sum()) < 3000 * int(c.h.info.hops_upper) or c.h.info.hops_upper == 1
    c.compare((1 << 32) - 500, 1001)


@pytest.mark.parametrize("mean", [300_000, 3_000_000])
@pytest.mark.parametrize("name", sorted(MODE_B_CASES))
def test_items_mode_b(gpu, name, mean):
    c = DesCase(MODE_B_CASES[name](), mean, error_mode=isim.MODE_B)
    assert c.d.info.items == 1
    recs, _, _ = c.compare(1000, 3000)
    assert int((recs["status_err"] >> 31).sum()) > 0  # some trace's entry responded 500
    c.compare((1 << 32) - 500, 1001)


def test_items_tie_runs_out_of_order(gpu):
    # arrivals 1 ns apart on average: many traces start at the same instant, so
    # z's sorted round holds runs of equal keys from many traces in the
    # round's position-major list order — far from (trace, hop) order, past
    # k_tiefix's insertion-sort budget: its heapsort
    c = DesCase(CASES["fanout_ties"](), 1)
    c.compare(0, 3000)
    c.compare((1 << 32) - 500, 1001)


@pytest.mark.parametrize("n", [1, 2, 63, 257])
def test_items_ragged(gpu, n):
    DesCase(CASES["real300p60"](), 1_000_000).compare(55, n)


def test_items_contention(gpu):
    # arrivals far faster than the services: long queues, every wait recorded
    c = DesCase(CASES["mesh_des"](), 50_000)
    _, _, rows = c.compare(0, 4000)
    assert int(rows[:, isim.native.DES_ROW_WORDS - 2].max()) > 500_000  # some wait above 0.5 ms (sleeps are 50-250 us)


def _static_pair(doc, mean):
    j = obj_to_json(doc)
    g = isim.ServiceGraph.from_json(j)
    hs = isim.Handler(g, None, isim.SimParams())
    hd = isim.Handler(g, None, isim.SimParams(flags=native.FLAG_DYNAMIC))
    ds, dd = isim.DesHandler(hs, mean), isim.DesHandler(hd, mean)
    assert ds.info.items == 0 and dd.info.items == 1
    return hs, hd, ds, dd


@pytest.mark.parametrize("case", ["realistic", "tree_reps", "sequential"])
def test_items_equal_static_engine(gpu, case):
    if case == "realistic":
        doc = realistic_topology(400, concurrent=True, sleep_ms=(1, 5), error_rate=(0.0, 0.05))
    elif case == "tree_reps":
        doc = _sleepy_tree(3, 5, reps_leaves=4)
    else:
        doc = _sleepy(tree_topology(3, 4, sequential=True))
    hs, hd, ds, dd = _static_pair(doc, 700_000)
    n = 150_000
    rs, ss, ts = ds.serve(12345, n, wide=True)
    rd, sd, td = dd.serve(12345, n)
    assert np.array_equal(rs, rd)
    fs, fd = hs.fold(ss), hd.fold(sd)
    for k in ("n_traces", "sum_latency", "sum_hops", "sum_err_hops", "n_500", "max_latency", "min_latency"):
        assert fs[k] == fd[k], k
    for k in ("lat_prom", "lat_log2", "svc_calls", "svc_errs", "site_calls"):
        assert np.array_equal(np.asarray(fs[k], np.uint64), np.asarray(fd[k], np.uint64)), k
    assert np.array_equal(ds.fold(ts), dd.fold(td))


def test_items_device_entry_accumulates(gpu):
    import torch
    c = DesCase(CASES["real300p60"](), 1_000_000)
    n = 5000
    ws = torch.zeros(c.d.workspace_bytes(n) + 8, dtype=torch.uint8, device="cuda")
    stats = torch.zeros(len(c.h.new_stats()), dtype=torch.int64, device="cuda")
    table = torch.zeros(max(1, c.d.table_words), dtype=torch.int64, device="cuda")
    rec = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for b in (0, n):
        c.d.serve_device(b, n, rec.data_ptr(), stats.data_ptr(), table.data_ptr(), ws.data_ptr(), ws.numel(), s)
    torch.cuda.synchronize()
    _, st, tab = c.d.serve(0, 2 * n, device=0, records=False)
    # two batches of n from time 0 each vs one of 2n: counts add up the same
    got = stats.cpu().numpy().view(np.uint64)
    assert int(got[native.ST_N_TRACES]) == 2 * n
    assert int(got[native.ST_SUM_HOPS]) == int(c.h.fold(got)["sum_hops"])
    tabn = table.cpu().numpy().view(np.uint64).reshape(-1, native.DES_ROW_WORDS)
    assert int(tabn[:, native.DES_ROW_WORDS - 4].sum()) == int(got[native.ST_SUM_HOPS])
    # the second batch's records are the oracle's for its trace ids
    from oracle import des as od
    orec, _, _ = od.run(c.sg, c.op, c.sg.entry(), n, n, c.mean, og=c.og)
    r = rec.cpu().numpy().view(isim.REC_DTYPE)
    assert_records_equal(r, orec)


@pytest.mark.parametrize("name", ["real300p60", "tree_reps_p70", "canonical_p50"])
def test_items_two_sort_queue_path(gpu, name):
    # the fallback queue path (replica | arrival, then the row: two stable
    # sorts), taken when row | replica | arrival does not fit one 64-bit key
    DesCase(CASES[name](), 500_000, flags=native.FLAG_DES_TWO_SORTS).compare(31, 2500)


def test_items_c5p_bench_batch_sparse_load(gpu):
    """c5p exactly as bench.py builds it, at its bench batch (2^19 traces),
    under a sparse load (mean gap 17 s against ~35 ms latencies): the
    executed calls, hop counts and statuses of every trace are the lane tree
    walk's (isim_serve on the same graph: queueing changes no skip and no
    error), no latency is below the walk's (queueing only adds), and the
    traces that do not overlap another — all but the ~0.2 % whose
    exponential gap is shorter than a latency — equal it.  Size-independent
    properties at the full size, where the event oracle is too slow to run."""
    import bench
    j, _ = bench.build_graph("c5p")
    h = isim.Handler(isim.ServiceGraph.from_json(j), None, isim.SimParams())
    n = bench.BENCH_BATCH["c5p"]
    d = isim.DesHandler(h, 1 << 34)
    assert d.info.items == 1
    recs, stats, table = d.serve(1 << 31, n, device=0)
    wrec, wstats = h.serve(1 << 31, n, device=0)
    assert np.array_equal(recs["hops"], wrec["hops"])
    assert np.array_equal(recs["status_err"], wrec["status_err"])
    assert np.all(recs["latency_ns"] >= wrec["latency_ns"])
    same = np.count_nonzero(recs["latency_ns"] == wrec["latency_ns"])
    assert same >= 0.99 * n, same
    rows = d.fold(table)
    assert int(rows[:, native.DES_ROW_WORDS - 4].sum()) == int(recs["hops"].sum())
    # the executed-call counters are the walk's too
    fd, fw = h.fold(stats), h.fold(wstats)
    assert np.array_equal(np.asarray(fd["site_calls"]), np.asarray(fw["site_calls"]))
    assert np.array_equal(np.asarray(fd["svc_errs"]), np.asarray(fw["svc_errs"]))


@pytest.mark.parametrize("mean", [50_000, 400_000])
def test_items_kept_queue_order(gpu, mean):
    """A cyclic schedule's quiet passes reuse a sort round's previous sorted
    order when it still sorts the new arrivals (k_ordchk / k_pairs1o); under
    heavy and light contention, at a size where some kept orders hold and
    some fail, everything equals the run that sorts every round
    (ISIM_FLAG_DES_SORT_ALL) and, at a smaller size, the oracle."""
    c = DesCase(CASES["mesh_des"](), mean)
    assert c.d.info.items == 1 and c.d.info.cyclic == 1
    recs, _, _ = c.compare(7, 1500)
    # isim_des_last_batch: a cyclic schedule's quiet passes and the recording one
    rep = c.d.last_batch()
    assert rep["passes"] >= 2 and rep["syncs"] >= rep["passes"] and rep["items"] == int(recs["hops"].sum())
    n = 40_000
    got = c.d.serve(1 << 20, n, device=0)
    ref = DesCase(CASES["mesh_des"](), mean, flags=native.FLAG_DES_SORT_ALL).d.serve(1 << 20, n, device=0)
    assert np.array_equal(got[0], ref[0])
    assert np.array_equal(np.asarray(got[1]), np.asarray(ref[1]))
    assert np.array_equal(np.asarray(got[2]), np.asarray(ref[2]))


def _bench_case(cfg, flags=0):
    import bench
    j, _ = bench.build_graph(cfg)
    mean = 150_000 if cfg == "c4d" else 6_000_000  # bench.py's default gaps
    return DesCase(j, mean, flags=flags), bench.BENCH_BATCH[cfg]


def test_items_c5p_bench_graph_and_load(gpu):
    """c5p exactly as bench.py builds it (config 3's 10k
    graph at probability 50) at the bench's own mean gap of 6 ms: 20,000
    traces bit-exact against des_oracle.c — records, stats and the DES table
    (the oracle runs ~3 s)."""
    c, _ = _bench_case("c5p")
    assert c.d.info.items == 1
    _, _, rows = c.compare(1000, 20_000)
    assert int(rows[:, native.DES_SUM_WAIT].sum()) > 0  # contended


def test_items_c4d_bench_graph_and_load(gpu):
    """c4d exactly as bench.py builds it (config 4's 100k
    mesh with sleeps, a cyclic schedule) at the bench's own mean gap of
    150 us: 20,000 traces bit-exact against des_oracle.c, and a second window
    whose trace ids cross 2^32."""
    c, _ = _bench_case("c4d")
    assert c.d.info.items == 1 and c.d.info.cyclic == 1
    _, _, rows = c.compare(0, 20_000)
    assert int(rows[:, native.DES_SUM_WAIT].sum()) > 0
    c.compare((1 << 32) - 7000, 14_000)


def test_items_c4d_bench_batch(gpu):
    """c4d at its bench batch (2^23 traces per step, mean gap 150 us), where the
    event oracle would take minutes: the executed calls, hops and statuses of
    every trace are the lane tree walk's (isim_serve on the same graph:
    queueing changes no skip and no error), no latency is below the walk's
    (queueing only adds), the DES table counts every executed invocation once,
    and the call counters equal the walk's (executable.go:84-105,
    svc/service.go:30-31)."""
    c, n = _bench_case("c4d")
    recs, stats, table = c.d.serve(1 << 23, n, device=0)
    wrec, wstats = c.h.serve(1 << 23, n, device=0)
    assert np.array_equal(recs["hops"], wrec["hops"])
    assert np.array_equal(recs["status_err"], wrec["status_err"])
    assert np.all(recs["latency_ns"] >= wrec["latency_ns"])
    rows = c.d.fold(table)
    assert int(rows[:, native.DES_ROW_WORDS - 4].sum()) == int(recs["hops"].sum())
    assert int(rows[:, native.DES_SUM_WAIT].sum()) > 0
    fd, fw = c.h.fold(stats), c.h.fold(wstats)
    assert np.array_equal(np.asarray(fd["site_calls"]), np.asarray(fw["site_calls"]))
    assert np.array_equal(np.asarray(fd["svc_calls"]), np.asarray(fw["svc_calls"]))
    assert np.array_equal(np.asarray(fd["svc_errs"]), np.asarray(fw["svc_errs"]))
    assert fd["n_traces"] == n and fd["sum_hops"] == fw["sum_hops"]


def test_items_c3s_u64_walk(gpu):
    """c3s (config 3's 10k graph in the generator's
    sequential shape at probability 50; a ~30 s latency bound, the lane tree
    walk's u64 time) is in the item engine's DES class: 4,000 traces at the
    config-5 load bit-exact against des_oracle.c."""
    import bench
    j, _ = bench.build_graph("c3s")
    c = DesCase(j, 6_000_000)
    assert c.d.info.items == 1 and c.h.info.time_bits == 64
    c.compare(1 << 20, 4000)


@pytest.mark.parametrize("name", ["real300p60", "canonical_p50", "mesh_des"])
def test_items_wide_tree(gpu, name):
    """The item engine over a wide tree (ISIM_FLAG_TREE_WIDE: 16-byte nodes,
    32-bit frames in the pre-walk; positions past 16 bits in the records and
    the renumbering sort), modes A and B, against the oracle."""
    W = native.FLAG_TREE_WIDE
    DesCase(CASES[name](), 300_000, flags=W).compare(1000, 3000)
    DesCase(MODE_B_CASES["seq_tree_abort"](), 300_000, error_mode=isim.MODE_B, flags=W).compare(9, 2000)


@pytest.mark.parametrize("case", ["c5p", "c4d", "mesh_heavy"])
def test_items_qscan_equals_scan_by_key(gpu, case):
    """The one-pass queue kernel (k_qscan: a segmented prefix max of
    a_i - i*h with a decoupled look-back across thousands of tiles) against
    the independent path it replaced (rocPRIM's scan by key over max-plus
    maps, then k_qout; ISIM_FLAG_DES_SCAN_BY_KEY) at sizes where the rounds
    span thousands of tiles and queue segments span many of them: records,
    statistics and the DES table identical.  c5p at its bench batch and gap,
    c4d at 2^21 of its bench gap (cyclic, kept orders), and the mesh under
    heavy contention (waits far above the holds: long carries)."""
    def handler(flags):
        if case == "mesh_heavy":
            return DesCase(CASES["mesh_des"](), 20_000, flags=flags).d, 300_000
        c, n = _bench_case(case, flags)
        return c.d, (n if case == "c5p" else 1 << 21)

    d, n = handler(0)
    got = d.serve(1 << 22, n, device=0)
    ref = handler(native.FLAG_DES_SCAN_BY_KEY)[0].serve(1 << 22, n, device=0)
    assert np.array_equal(got[0], ref[0])
    assert np.array_equal(np.asarray(got[1]), np.asarray(ref[1]))
    assert np.array_equal(np.asarray(got[2]), np.asarray(ref[2]))
    rows = d.fold(got[2])
    assert int(rows[:, native.DES_SUM_WAIT].sum()) > 0


def test_items_c4w_graph(gpu):
    """the DES item engine on c4w's own graph (the
    100,000-service realistic graph at probability 30: a wide tree whose
    pre-walk runs the 16-byte-node lane walk), 20,000 traces at the config-5
    load against des_oracle.c — records, stats and the DES table
    (create_realistic_topology.py:28-76, executable.go:84-179,
    svc/service.go:30-31)."""
    import bench
    j, _ = bench.build_graph("c4w")
    c = DesCase(j, 6_000_000)
    assert c.d.info.items == 1 and c.h.launch_info(0)["tree_wide"] == 1
    _, _, rows = c.compare((1 << 32) - 10_000, 20_000)
    assert int(rows[:, native.DES_COUNT].sum()) > 20_000


@pytest.fixture
def spin_limit_zero():
    lib = native.load()
    lib.isim_debug_set_spin_limit(0)
    try:
        yield
    finally:
        lib.isim_debug_set_spin_limit(1 << 26)


def test_lookback_timeout_fails_loudly(gpu, spin_limit_zero):
    """VERDICT r5 item 3 / ADVICE r5: a decoupled look-back that gives up
    (forced here: isim_debug_set_spin_limit(0) makes every look-back fail at
    once) fails the batch — ISIM_EHIP with the reason, no record written, no
    trace counted, the fault marked in ISIM_ST_DES_RETRY's high half (the
    item engine's other statistics of a failed batch are undefined, isim.h) —
    instead of returning ISIM_OK with wrong queue starts.
    The item engine's k_qscan (des_items.hip) through both the device entry
    and isim_serve_des, then the static engine's chained queue pass (des.hip)
    whose async entry flags the fault in ISIM_ST_DES_RETRY's high half."""
    import torch
    c = DesCase(CASES["mesh_des"](), 20_000)
    n = 300_000
    with pytest.raises(native.IsimError) as ei:
        c.d.serve(0, n, device=0)
    assert ei.value.code == native.EHIP and "look-back" in str(ei.value)
    ws = torch.zeros(c.d.workspace_bytes(n) + 8, dtype=torch.uint8, device="cuda")
    stats = torch.zeros(len(c.h.new_stats()), dtype=torch.int64, device="cuda")
    table = torch.zeros(max(1, c.d.table_words), dtype=torch.int64, device="cuda")
    rec = torch.full((n * 2,), -1, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    with pytest.raises(native.IsimError):
        c.d.serve_device(0, n, rec.data_ptr(), stats.data_ptr(), table.data_ptr(), ws.data_ptr(), ws.numel(), s)
    torch.cuda.synchronize()
    got = stats.cpu().numpy().view(np.uint64)
    assert int(got[native.ST_DES_RETRY]) == 1 << 32 and int(got[native.ST_N_TRACES]) == 0
    assert int(got[native.ST_SUM_HOPS]) == 0 and int(got[native.ST_SUM_LATENCY]) == 0
    assert bool((rec == -1).all())
    # the static (level-synchronous) engine: the chained pass's look-back
    doc = realistic_topology(400, concurrent=True, sleep_ms=(1, 5), error_rate=(0.0, 0.05))
    hs = isim.Handler(isim.ServiceGraph.from_json(obj_to_json(doc)), None, isim.SimParams())
    ds = isim.DesHandler(hs, 700_000)
    assert ds.info.items == 0
    with pytest.raises(native.IsimError) as ei:
        ds.serve(0, 1 << 18, device=0)
    assert ei.value.code == native.EHIP and "look-back" in str(ei.value)


def test_lookback_limit_restored_runs_clean(gpu):
    """After the hook is reset the same batches run and match the oracle."""
    assert native.load().isim_debug_spin_limit() == 1 << 26
    DesCase(CASES["mesh_des"](), 20_000).compare(0, 2000)
