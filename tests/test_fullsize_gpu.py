"""Full-size GPU runs (BASELINE-scale batches) checked through size-independent
properties, plus bit-exact windows sampled across the trace range and
recomputed by the CPU oracle.  The bench's own batches (bench.BENCH_BATCH:
config 3 at 2^24 traces per launch in modes A and B, config 4 at 2^26) are
checked at exactly those sizes, two consecutive launches into one stats
buffer as bench.time_walk runs them, with oracle windows at the first and
last traces of each launch and across every internal launch split
(isim_launch_info.max_launch_traces).  Reference behaviour:
isotope/service/pkg/srv/executable.go:84-144 (skips, calls, error handling)."""
import numpy as np
import pytest

import bench
import isim
from isim.generators import config2_topology, config3_topology, mesh_topology, realistic_topology
from isim.yamljson import obj_to_json

from parity import Case, assert_records_equal, with_defaults

pytestmark = pytest.mark.gpu


def _device_run(case: Case, begin: int, n: int, launches: int = 1, raw: bool = False):
    """`launches` consecutive isim_serve_device calls of n traces each (trace
    ids begin + i*n), records into one device buffer, ONE stats buffer
    accumulated across them (bench.time_walk's pattern); raw: the stats
    words themselves instead of their fold."""
    import torch
    h = case.handler
    dev = torch.device("cuda", 0)
    stats = torch.zeros(h.stats_words, dtype=torch.int64, device=dev)
    recs = torch.empty((n * launches, 2), dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev)
    for i in range(launches):
        h.serve_device(begin + i * n, n, recs[i * n:].data_ptr(), stats.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    r = recs.cpu().numpy().view(np.uint64)
    del recs
    rec = np.zeros(n * launches, isim.REC_DTYPE)
    rec["latency_ns"] = r[:, 0]
    rec["hops"] = (r[:, 1] & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    rec["status_err"] = (r[:, 1] >> np.uint64(32)).astype(np.uint32)
    st = stats.cpu().numpy().view(np.uint64)
    return rec, (st if raw else h.fold(st))


def _check_window(case: Case, rec, begin, s0, width):
    orec, _ = case.cpu(begin + int(s0), width)
    assert_records_equal(rec[s0:s0 + width], orec)


def _sampled_windows(case: Case, rec, begin, n, windows=8, width=256, seed=0):
    rng = np.random.default_rng(seed)
    starts = sorted(set([0, n - width] + list(rng.integers(0, n - width, windows))))
    for s0 in starts:
        _check_window(case, rec, begin, s0, width)


def _launch_edge_windows(case: Case, rec, begin, n, launches, width=256):
    """Oracle windows at the first and last `width` traces of every launch and
    straddling every internal split of a launch (the library splits a batch
    into launches of at most max_launch_traces traces so that no u32 LDS
    counter can wrap: api.hip launch_walk, Program::tree_mult)."""
    m = int(case.handler.launch_info(0)["max_launch_traces"])
    assert m >= 1
    edges = set()
    for i in range(launches):
        lo = i * n
        edges.update([lo, lo + n - width])
        for cut in range(lo + m, lo + n, m):  # internal splits of launch i (a window inside the records)
            edges.add(min(cut - width // 2, launches * n - width))
    for s0 in sorted(edges):
        _check_window(case, rec, begin, s0, width)
    return m


def _common_properties(f, rec, n):
    assert f["n_traces"] == n
    assert f["sum_hops"] == int(rec["hops"].astype(np.uint64).sum())
    assert f["sum_latency"] == int(rec["latency_ns"].astype(np.uint64).sum())
    err = (rec["status_err"] & 0x7FFFFFFF).astype(np.uint64)
    st500 = (rec["status_err"] >> 31).astype(np.uint64)
    assert f["sum_err_hops"] == int(err.sum())
    assert f["n_500"] == int(st500.sum())
    assert int(f["lat_prom"].sum()) == n and int(f["lat_log2"].sum()) == n
    assert int(f["lat_prom"][1].sum()) == f["n_500"]
    assert f["min_latency"] == int(rec["latency_ns"].min()) and f["max_latency"] == int(rec["latency_ns"].max())
    # every 500 response is one invocation's: services' 500s add up to err_hops
    assert int(f["svc_errs"].sum()) == f["sum_err_hops"]
    assert int(f["svc_calls"].sum()) == f["sum_hops"]


def test_config3_full_batch(gpu):
    """BASELINE config 3 graph, 2^22 traces at a trace offset beyond 2^32;
    mode A (the bench batch itself: test_config3_bench_batch)."""
    c = Case(obj_to_json(config3_topology()))
    n, begin = 1 << 22, (1 << 32) - (1 << 21)
    rec, f = _device_run(c, begin, n)
    info = c.handler.info
    _common_properties(f, rec, n)
    # static walk: every trace visits every service once, same latency
    assert np.all(rec["hops"] == 10000)
    assert np.all(rec["latency_ns"] == info.max_latency_ns)
    assert np.all(f["svc_calls"] == n)
    # per-service error frequencies match errorRate (binomial, 6 sigma)
    p = np.array([s.error_rate for s in c.graph.services])
    e = f["svc_errs"].astype(np.float64)
    sigma = np.sqrt(n * p * (1 - p)) + 1.0
    assert np.all(np.abs(e - n * p) < 6 * sigma)
    _sampled_windows(c, rec, begin, n)


def config3_informative():
    """Config 3's graph (same generator seed: same tree and sleeps) with
    errorRate U[0, 1e-4]: about 0.5 error draws per trace, so in mode B the
    entry answers 200 or 500 in comparable proportions (config 3's own
    U[0, 1%] makes every trace a 500)."""
    return obj_to_json(realistic_topology(10_000, "multitier", 42, concurrent=True, sleep_ms=(1, 5),
                                          error_rate=(0.0, 1e-4)))


@pytest.mark.parametrize("informative", [True, False])
def test_config3_mode_b_full_batch(gpu, informative):
    c = Case(config3_informative() if informative else obj_to_json(config3_topology()), None,
             isim.SimParams(error_mode=isim.MODE_B))
    n = 1 << 21
    rec, f = _device_run(c, 123, n)
    _common_properties(f, rec, n)
    # mode B: any invocation's 500 fails its caller's step, up to the entry;
    # so the entry answers 500 exactly when the trace drew some error
    st500 = (rec["status_err"] >> 31).astype(bool)
    errh = rec["status_err"] & 0x7FFFFFFF
    assert np.array_equal(st500, errh > 0)
    frac = f["n_500"] / n
    if informative:
        assert 0.2 < frac < 0.8, frac
    else:
        assert frac > 0.99
    _sampled_windows(c, rec, 123, n, windows=8 if informative else 4)


def test_config2_full_batch(gpu):
    """BASELINE config 2 (tree 4x8, sequential) with a 0.1% errorRate."""
    c = Case(with_defaults(obj_to_json(config2_topology()), errorRate=0.001))
    n = 1 << 23
    rec, f = _device_run(c, 0, n)
    _common_properties(f, rec, n)
    assert np.all(rec["hops"] == 585) and np.all(rec["latency_ns"] == c.handler.info.max_latency_ns)
    _sampled_windows(c, rec, 0, n)


def test_config4_mesh_full_batch(gpu):
    """BASELINE config 4 graph (100k-service mesh, probability 30): dynamic
    walk; hop counts vary per trace."""
    c = Case(with_defaults(obj_to_json(mesh_topology()), errorRate=0.01))
    assert not c.handler.info.static_walk
    n = 1 << 21
    rec, f = _device_run(c, 7, n)
    _common_properties(f, rec, n)
    hops = rec["hops"].astype(np.float64)
    # E[hops] = sum_k 0.9^k over 8 layers (3 calls at probability 30 each)
    expected = sum(0.9 ** k for k in range(8))
    assert abs(hops.mean() - expected) < 0.05
    _sampled_windows(c, rec, 7, n)


def test_config3_bench_batch(gpu):
    """config 3 exactly as bench.py times it: bench.build_graph("c3"), the
    bench's params (mode A, every trace walked), BENCH_BATCH["c3"] = 2^24
    traces per launch, two consecutive launches into one stats buffer, trace
    ids from just below 2^32 (the bench's shard_begin ids cross it at step
    256)."""
    j, _ = bench.build_graph("c3")
    c = Case(j, None, isim.SimParams(flags=isim.native.FLAG_WALK_ALL))
    n, L = bench.BENCH_BATCH["c3"], 2
    assert n == 1 << 24
    begin = (1 << 32) - n - 1000
    rec, f = _device_run(c, begin, n, L)
    _common_properties(f, rec, n * L)
    assert np.all(rec["hops"] == 10000)
    assert np.all(rec["latency_ns"] == c.handler.info.max_latency_ns)
    assert np.all(f["svc_calls"] == n * L)
    # executed calls per site = traces (static walk); callee 500s per site sum to the services' 500s
    assert np.all(f["site_calls"] == n * L)
    _launch_edge_windows(c, rec, begin, n, L)
    _sampled_windows(c, rec, begin, n * L, windows=6, seed=3)
    # the full stats (per service, per site, svc_dur) of an oracle-sized window through the same handler
    c.compare(begin + 3 * n // 2, 1 << 14)


def test_config3_bench_batch_mode_b(gpu):
    """config 3's graph in mode B with the informative errorRate
    (bench.mode_b_legs "mode_b_informative"), sparse ancestor marking (kind
    8), 2^24 traces per launch, two launches into one stats buffer."""
    c = Case(config3_informative(), None, isim.SimParams(error_mode=isim.MODE_B, flags=isim.native.FLAG_WALK_ALL))
    assert c.handler.launch_info(0)["kernel_kind"] == 8
    n, L = bench.BENCH_BATCH["c3"], 2
    begin = 5 * n
    rec, f = _device_run(c, begin, n, L)
    _common_properties(f, rec, n * L)
    st500 = (rec["status_err"] >> 31).astype(bool)
    assert np.array_equal(st500, (rec["status_err"] & 0x7FFFFFFF) > 0)
    assert 0.2 < f["n_500"] / (n * L) < 0.8
    _launch_edge_windows(c, rec, begin, n, L)
    _sampled_windows(c, rec, begin, n * L, windows=4, seed=4)
    c.compare(begin + 3 * n // 2, 1 << 14)


def test_config4_bench_batch(gpu):
    """config 4 exactly as bench.py times it: bench.build_graph("c4") (no
    errorRate: every draw is a probability skip), per-service duration rows
    on, BENCH_BATCH["c4"] = 2^26 traces per launch (1 GiB of records), two
    launches into one stats buffer; oracle windows at every launch edge and
    internal split; the duration table's counts and sums checked against the
    records and the slot counters."""
    j, _ = bench.build_graph("c4")
    c = Case(j, None, isim.SimParams(flags=isim.native.FLAG_WALK_ALL))
    li = c.handler.launch_info(0)
    assert li["kernel_kind"] == 7
    n, L = bench.BENCH_BATCH["c4"], 2
    assert n == 1 << 26
    begin = 11
    rec, f = _device_run(c, begin, n, L)
    N = n * L
    _common_properties(f, rec, N)
    hops = rec["hops"].astype(np.float64)
    expected = sum(0.9 ** k for k in range(8))
    assert abs(hops.mean() - expected) < 0.01
    assert f["n_500"] == 0 and f["sum_err_hops"] == 0
    # duration table: every row's code-200 bucket counts = the service's invocations
    dur = np.asarray(f["svc_dur"], np.uint64)
    assert np.array_equal(dur[:, :isim.native.N_PROM].sum(axis=1), np.asarray(f["svc_calls"], np.uint64))
    assert int(dur[:, isim.native.N_PROM:2 * isim.native.N_PROM].sum()) == 0
    entry = c.handler.info.entry
    assert int(dur[entry, 2 * isim.native.N_PROM]) == f["sum_latency"]
    m = _launch_edge_windows(c, rec, begin, n, L)
    _sampled_windows(c, rec, begin, N, windows=8, seed=5)
    # the full stats of one oracle-sized window through the same kernel (1 launch, svc_dur included)
    c.compare(begin + 3 * n // 2, 1 << 16)
    print(f"max_launch_traces={m}")


def test_tree_guarded_counters_overflow(gpu):
    """The lane tree walk keeps per-slot calls and 500s as two 16-bit fields of
    one LDS word, each moved to the stats in steps of 2^15 when it reaches
    2^15 (tree.hip TreeSink::move, with the duration buckets and leaf sums
    derived from them).  A tiny dynamic graph at 2^25 traces per launch
    makes every workgroup cross 2^15 many times at several sites, calls and
    500s (errorRate 0.7), leaf and calling callees: the full stats must equal
    the oracle's over the whole launch, and sampled record windows too."""
    doc = {"defaults": {"requestSize": 64, "responseSize": 256},
           "services": [
               {"name": "front", "isEntrypoint": True, "errorRate": 0.1,
                "script": [{"call": "mid"}, [{"call": {"service": "leaf", "probability": 90}}, {"call": "leaf"}]]},
               {"name": "mid", "errorRate": 0.7, "script": [{"sleep": "1ms"}, {"call": {"service": "leaf",
                                                                                    "probability": 60}}]},
               {"name": "leaf", "errorRate": 0.7, "script": [{"sleep": "2ms"}]}]}
    import json as _json
    c = Case(_json.dumps(doc))
    assert c.handler.launch_info(0)["kernel_kind"] == 7
    n = 1 << 25
    rec, f = _device_run(c, 3, n)
    _, ost = c.cpu(3, n, records=False)
    from oracle import executor as oc
    from parity import assert_stats_equal
    assert_stats_equal(f, oc.split_stats(ost, len(c.sg.g.services), len(c.sg.sites)))
    _sampled_windows(c, rec, 3, n, windows=4)
    assert int(f["site_calls"].max()) > 1 << 24


@pytest.mark.parametrize("prob", [50])
def test_config3p_bench_batch(gpu, prob):
    """c3p exactly as bench.py times it: config 3's 10k
    graph with probability `prob` on every call — a dynamic walk over a
    10,000-position tree (frames beyond the register stack spill, most
    duration rows by global atomics) on the lane tree walk, not kinds 2/3 —
    BENCH_BATCH["c3p"] traces per launch, two launches into one stats
    buffer; oracle windows at every launch edge and split, sampled windows,
    and the full stats (per service, per site, svc_dur) of a window."""
    j, _ = bench.build_graph("c3p", prob)
    c = Case(j, None, isim.SimParams(flags=isim.native.FLAG_WALK_ALL))
    assert c.handler.launch_info(0)["kernel_kind"] == 7
    n, L = bench.BENCH_BATCH["c3p"], 2
    begin = (1 << 32) - n // 2
    rec, f = _device_run(c, begin, n, L)
    _common_properties(f, rec, n * L)
    hops = rec["hops"].astype(np.float64)
    assert 1 < hops.mean() < 10000 and hops.min() >= 1
    _launch_edge_windows(c, rec, begin, n, L, width=128)
    _sampled_windows(c, rec, begin, n * L, windows=4, width=128, seed=9)
    c.compare(begin + n - 2048, 4096)


def test_config3s_bench_batch(gpu):
    """c3s exactly as bench.py times it: config 3's 10k
    graph in the generator's sequential shape at probability 50, whose ~30 s
    latency bound needs u64 time — on the lane tree walk (kind 7), not the
    wave interpreter — BENCH_BATCH["c3s"] traces per launch, two launches
    into one stats buffer; oracle windows at every launch edge and split,
    sampled windows, and the full stats of a window."""
    j, _ = bench.build_graph("c3s", 50)
    c = Case(j, None, isim.SimParams(flags=isim.native.FLAG_WALK_ALL))
    assert c.handler.info.time_bits == 64 and c.handler.info.max_latency_ns >= 1 << 32
    assert c.handler.launch_info(0)["kernel_kind"] == 7
    n, L = bench.BENCH_BATCH["c3s"], 2
    begin = (1 << 33) - n // 2
    rec, f = _device_run(c, begin, n, L)
    _common_properties(f, rec, n * L)
    _launch_edge_windows(c, rec, begin, n, L, width=128)
    _sampled_windows(c, rec, begin, n * L, windows=4, width=128, seed=11)
    c.compare(begin + n - 2048, 4096)


def test_config4w_bench_batch(gpu):
    """c4w exactly as bench.py times it —
    bench.build_graph("c4w") (create_realistic_topology.py:28-76's multitier
    graph at 100,000 services, probability 30 on every call, errorRate U[0,1%])
    on the WIDE lane tree walk (kind 7, 16-byte nodes, 100,000 positions and
    call sites), BENCH_BATCH["c4w"] = 2^22 traces per launch, two launches into
    one stats buffer with trace ids crossing 2^32; oracle windows at every
    launch edge and internal split, sampled windows, and the full stats
    (per service, per site, svc_dur) of a window (executable.go:84-179)."""
    j, _ = bench.build_graph("c4w")
    c = Case(j, None, isim.SimParams(flags=isim.native.FLAG_WALK_ALL))
    li = c.handler.launch_info(0)
    assert li["kernel_kind"] == 7 and li["tree_wide"] == 1
    n, L = bench.BENCH_BATCH["c4w"], 2
    assert n == 1 << 22
    begin = (1 << 32) - n - n // 3  # the second launch crosses 2^32
    rec, f = _device_run(c, begin, n, L)
    _common_properties(f, rec, n * L)
    assert rec["hops"].min() >= 1 and f["n_500"] > 0
    _launch_edge_windows(c, rec, begin, n, L, width=128)
    _sampled_windows(c, rec, begin, n * L, windows=4, width=128, seed=13)
    c.compare(begin + n - 2048, 4096)


@pytest.mark.parametrize("informative", [True, False])
def test_mode_b_marking_equals_close_list(gpu, informative):
    """mode B by sparse ancestor marking (kind 8: +1 at
    every erring invocation, -1 at the LCA of consecutive ones, subtree sums
    per launch) against the independent close-list kernel (kind 6: every
    calling invocation's subtree tested) on config 3's graph (~50 erring
    invocations per trace at U[0,1%], ~0.5 at U[0,1e-4]), 2^22 traces of one
    launch from a trace id crossing 2^32: records and every statistic equal
    (executable.go:131-143, handler.go:66-75 with the 500 propagated)."""
    j = config3_informative() if informative else obj_to_json(config3_topology())
    n, begin = 1 << 22, (1 << 32) - (1 << 21)
    out = []
    for flags in (0, isim.native.FLAG_CLOSE_LIST):
        c = Case(j, None, isim.SimParams(error_mode=isim.MODE_B, flags=isim.native.FLAG_WALK_ALL | flags))
        assert c.handler.launch_info(0)["kernel_kind"] == (6 if flags else 8)
        out.append(_device_run(c, begin, n, raw=True))
    (r8, s8), (r6, s6) = out
    assert np.array_equal(r8, r6)
    # every stats word: header, histograms, per-site calls and per-site callee 500s
    bad = np.nonzero(s8 != s6)[0]
    assert bad.size == 0, f"stats words differ at {bad[:8].tolist()}"
    assert int(s8[isim.native.ST_N_500]) > 0


def test_cdag_bench_batch(gpu):
    """cdag exactly as bench.py times it (round 6): bench.build_graph("cdag"),
    a layered DAG of shared callees whose unrolled tree would have 8^9 = 134M
    positions, on the lane walk over the site graph (kind 7, tree_wide 2),
    BENCH_BATCH["cdag"] = 2^22 traces per launch, two launches into one stats
    buffer from trace ids crossing 2^32; oracle windows at every launch edge
    and internal split, sampled windows, and the full stats of a window
    (executable.go:84-179, validation.go:28-57)."""
    j, _ = bench.build_graph("cdag", 10)
    c = Case(j, None, isim.SimParams(flags=isim.native.FLAG_WALK_ALL))
    li = c.handler.launch_info(0)
    assert li["kernel_kind"] == 7 and li["tree_wide"] == 2
    n, L = bench.BENCH_BATCH["cdag"], 2
    begin = (1 << 32) - n - 12345
    rec, f = _device_run(c, begin, n, L)
    _common_properties(f, rec, n * L)
    assert rec["hops"].min() >= 1 and f["n_500"] > 0
    _launch_edge_windows(c, rec, begin, n, L, width=128)
    _sampled_windows(c, rec, begin, n * L, windows=4, width=128, seed=17)
    c.compare(begin + n - 2048, 4096)
