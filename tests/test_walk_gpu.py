"""GPU parity: the HIP walk kernel (through the C ABI) against the CPU oracle,
bit-exact per-trace records and stats, on seeded inputs."""
import glob
import json
import os

import numpy as np
import pytest

import isim
from isim.generators import config2_topology, config3_topology, mesh_topology, realistic_topology, tree_topology
from isim.yamljson import obj_to_json, yaml_to_json

from conftest import TOPOLOGIES
from parity import Case, with_defaults

pytestmark = pytest.mark.gpu

FIXTURES = sorted(glob.glob(os.path.join(TOPOLOGIES, "*.yaml")))


def _fixture_json(path, error_rate=None):
    j = yaml_to_json(open(path, "rb").read())
    if error_rate is not None:
        j = with_defaults(j, errorRate=error_rate)
    return j


KERNELS = {"stream": 0, "interp": isim.native.FLAG_NO_STREAM, "bitstack": isim.native.FLAG_BIT_STACK,
           "closelist": isim.native.FLAG_CLOSE_LIST,
           # the general path on every graph: the lane tree walk (kind 7) and the wave walk (kinds 2/3)
           "tree": isim.native.FLAG_DYNAMIC,
           "wave": isim.native.FLAG_DYNAMIC | isim.native.FLAG_WAVE_WALK}
STREAM_KINDS = (4, 5, 6, 8)


def dynamic_kind(handler, flags):
    """Kernel kind a dynamic walk takes: 7 (the lane tree walk, u32 or — a
    latency bound of 2^32 ns or more — u64 time) unless the wave walk is
    asked for: then 2/3 by the time width."""
    if flags & isim.native.FLAG_WAVE_WALK:
        return 2 + int(handler.info.time_bits == 64)
    return 7


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
@pytest.mark.parametrize("mode", [isim.MODE_A, isim.MODE_B])
@pytest.mark.parametrize("kernel", list(KERNELS))
def test_reference_topologies(gpu, path, mode, kernel):
    c = Case(_fixture_json(path, error_rate=0.05), None, isim.SimParams(error_mode=mode, flags=KERNELS[kernel]))
    kind = c.handler.launch_info(0)["kernel_kind"]
    tb64 = c.handler.info.time_bits == 64
    if not c.handler.info.static_walk:
        assert kind == dynamic_kind(c.handler, KERNELS[kernel])
    elif c.handler.info.static_walk:
        if kernel == "interp":
            assert kind == int(tb64)
        elif mode == isim.MODE_A:
            assert kind == 4
        elif kernel == "stream":
            assert kind == 8  # mode B: sparse ancestor marking
        elif kernel == "closelist":
            assert kind == 6
        else:
            assert kind == (5 if c.handler.info.max_depth <= 32 else 4)
    c.compare(0, 3000)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 4097])
@pytest.mark.parametrize("kernel", list(KERNELS))
def test_ragged_batches(gpu, n, kernel):
    c = Case(_fixture_json(os.path.join(TOPOLOGIES, "canonical.yaml"), 0.3), None,
             isim.SimParams(flags=KERNELS[kernel]))
    c.compare(777, n)


def test_zero_traces(gpu):
    c = Case(_fixture_json(os.path.join(TOPOLOGIES, "canonical.yaml"), 0.3))
    recs, stats = c.gpu(0, 0)
    assert stats.sum() == 0


@pytest.mark.parametrize("kernel", list(KERNELS))
def test_trace_ids_cross_2_32(gpu, kernel):
    c = Case(_fixture_json(os.path.join(TOPOLOGIES, "canonical.yaml"), 0.3), None,
             isim.SimParams(flags=KERNELS[kernel]))
    c.compare((1 << 32) - 1000, 2000)


@pytest.mark.parametrize("kernel", list(KERNELS))
def test_error_always_and_never(gpu, kernel):
    j = json.dumps({"services": [
        {"name": "e", "isEntrypoint": True, "script": [{"call": "a"}, [{"call": "b"}, {"call": "a"}]]},
        {"name": "a", "errorRate": 1.0},
        {"name": "b", "errorRate": "0%", "script": [{"call": "a"}, {"sleep": "1ms"}]}]})
    for mode in (isim.MODE_A, isim.MODE_B):
        Case(j, None, isim.SimParams(error_mode=mode, flags=KERNELS[kernel])).compare(0, 500)


def test_probability_and_mode_b_abort(gpu):
    # sequential calls after fallible calls: mode B aborts change the walk per lane
    j = json.dumps({"defaults": {"errorRate": 0.2, "requestSize": "1 KB", "responseSize": 300},
                    "services": [
        {"name": "e", "isEntrypoint": True, "script": [
            {"call": {"service": "a", "probability": 50}}, {"sleep": "3ms"},
            [{"call": "b"}, {"call": {"service": "c", "probability": 70}}, {"sleep": "2ms"}],
            {"call": "d"}, {"sleep": "1ms"}]},
        {"name": "a", "script": [{"call": {"service": "c", "probability": 20}}, {"call": "d"}]},
        {"name": "b", "script": [{"sleep": "500us"}, {"call": "d"}, {"call": "c"}]},
        {"name": "c", "script": [{"call": {"service": "d", "probability": 99}}, {"sleep": "1.5ms"}]},
        {"name": "d", "script": [{"sleep": "250us"}]}]})
    for mode in (isim.MODE_A, isim.MODE_B):
        c = Case(j, None, isim.SimParams(error_mode=mode, seed=99))
        assert not c.handler.info.static_walk
        c.compare(5, 20000)


@pytest.mark.parametrize("mode", [isim.MODE_A, isim.MODE_B])
def test_tree_walk_lane_refill(gpu, mode):
    """Kind 7 hands a lane its next trace as soon as one responds: the config-4
    graph over more traces than the resident waves' first batches (every lane
    walks many traces of different lengths), bit-exact against the oracle —
    per-trace state (Philox caches, the frame stack) must not leak between a
    lane's traces."""
    c = Case(with_defaults(obj_to_json(mesh_topology()), errorRate=0.01), None, isim.SimParams(error_mode=mode))
    li = c.handler.launch_info(0)
    assert li["kernel_kind"] == 7
    n = 3 * li["max_blocks"] * li["wg_threads"] + 777  # three batches of 64 per wave, and a ragged one
    c.compare((1 << 32) - 5000, n)


def test_large_latency_u64(gpu):
    # latency bound above 2^32 ns forces the 64-bit per-lane time kernel
    j = json.dumps({"services": [
        {"name": "e", "isEntrypoint": True, "errorRate": 0.5,
         "script": [{"sleep": "3s"}, {"call": {"service": "a", "probability": 40}}, {"sleep": "2h"}]},
        {"name": "a", "errorRate": 0.5, "script": [{"sleep": "1h"}, {"call": "b"}]},
        {"name": "b", "script": [{"sleep": "-5s"}, {"sleep": "100ns"}]}]})
    c = Case(j)
    assert c.handler.info.time_bits == 64
    c.compare(0, 5000)


@pytest.mark.parametrize("kernel", list(KERNELS))
def test_tree_sequential_config2(gpu, kernel):
    j = obj_to_json(config2_topology())
    c = Case(with_defaults(j, errorRate=0.01), None, isim.SimParams(flags=KERNELS[kernel]))
    c.compare(0, 2048)


@pytest.mark.parametrize("kernel", list(KERNELS))
def test_realistic_config3(gpu, kernel):
    j = obj_to_json(config3_topology())
    for mode in (isim.MODE_A, isim.MODE_B):
        Case(j, None, isim.SimParams(error_mode=mode, flags=KERNELS[kernel])).compare(1 << 20, 1024)


@pytest.mark.parametrize("kernel", list(KERNELS))
def test_config3_mode_b_informative(gpu, kernel):
    """Mode B on config 3's graph with errorRate U[0, 1e-4]: the entry's status
    is 200 in some traces and 500 in others (20-80 %), so the close-list
    kernel's subtree tests decide real outcomes at 10k-service scale."""
    from test_fullsize_gpu import config3_informative
    c = Case(config3_informative(), None, isim.SimParams(error_mode=isim.MODE_B, flags=KERNELS[kernel]))
    recs, _ = c.compare(1 << 30, 4096)
    frac = float((recs["status_err"] >> 31).mean())
    assert 0.2 < frac < 0.8, frac


def test_realistic_sequential_probability(gpu):
    d = realistic_topology(2000, "multitier", seed=3, concurrent=False, sleep_ms=(1, 5), error_rate=(0, 0.05))
    for i, s in enumerate(d["services"]):
        if i % 3 == 0:
            s["script"] = [({"call": {"service": c["call"], "probability": 60}} if isinstance(c, dict) and "call" in c else c)
                           for c in s["script"]]
    j = obj_to_json(d)
    for mode in (isim.MODE_A, isim.MODE_B):
        c = Case(j, None, isim.SimParams(error_mode=mode))
        # a ~6.5 s latency bound: the lane tree walk with u64 time (round 5), no longer kinds 2/3
        assert c.handler.info.time_bits == 64 and c.handler.launch_info(0)["kernel_kind"] == 7
        c.compare(0, 2000)


def test_mesh_config4(gpu):
    j = obj_to_json(mesh_topology(n_services=8000, layers=8, fanout=3, probability=30, seed=11))
    c = Case(with_defaults(j, errorRate=0.02))
    c.compare(0, 20000)


def _chain(n, fan=2):
    """svc-0 -> svc-1 -> ... -> svc-(n-1), each link also calling `fan` leaves."""
    svcs = []
    for i in range(n):
        calls = [[{"call": f"c{i + 1}"}] + [{"call": f"l{i}-{j}"} for j in range(fan)]] if i + 1 < n else []
        svcs.append({"name": f"c{i}", "script": [{"sleep": "1us"}] + calls, "errorRate": 0.02})
        svcs += [{"name": f"l{i}-{j}", "errorRate": 0.03} for j in range(fan)]
    svcs[0]["isEntrypoint"] = True
    return json.dumps({"services": svcs})


@pytest.mark.parametrize("depth,kind", [(31, 5), (32, 5), (33, 4), (64, 4)])
def test_mode_b_stack_depths(gpu, depth, kind):
    # the bit-stack kernel (kind 5) holds 32 stack positions; deeper graphs take kind 4
    c = Case(_chain(depth), None, isim.SimParams(error_mode=isim.MODE_B, flags=isim.native.FLAG_BIT_STACK))
    assert c.handler.info.max_depth == depth
    assert c.handler.launch_info(0)["kernel_kind"] == kind
    c.compare(5, 3000)


@pytest.mark.parametrize("kind", [6, 8])
@pytest.mark.parametrize("depth", [1, 2, 31, 33, 64])
@pytest.mark.parametrize("fan", [0, 2, 40])
def test_mode_b_close_list_depths(gpu, depth, fan, kind):
    # the close-list kernel (kind 6) and sparse ancestor marking (kind 8) have
    # no depth limit; chains whose subtrees end inside, at and across the
    # 32-record chunk boundaries (kind 6), LCAs at every depth (kind 8)
    flags = isim.native.FLAG_CLOSE_LIST if kind == 6 else 0
    c = Case(_chain(depth, fan), None, isim.SimParams(error_mode=isim.MODE_B, flags=flags))
    assert c.handler.info.max_depth == depth
    assert c.handler.launch_info(0)["kernel_kind"] == kind
    c.compare(5, 3000)
    c.compare((1 << 32) - 700, 1500)


# ---- batch queues: past the first wave-stride, waves claim batches from
# per-XCD queues (walk.hip); each launch re-arms its queue set on exit

@pytest.mark.parametrize("kernel", list(KERNELS))
def test_batch_queue_claims(gpu, kernel):
    # more batches than resident waves (stream: 128 traces per batch,
    # interpreter: 64), so most batches are claimed from the queues
    c = Case(_fixture_json(os.path.join(TOPOLOGIES, "canonical.yaml"), 0.3), None,
             isim.SimParams(flags=KERNELS[kernel]))
    li = c.handler.launch_info(0)
    per = 128 if li["kernel_kind"] in STREAM_KINDS else 64
    n = 3 * li["max_blocks"] * li["wg_threads"] // 64 * per + 4097
    c.compare(11, n)


@pytest.mark.parametrize("kernel", list(KERNELS))
def test_batch_queue_rearms(gpu, kernel):
    import torch
    c = Case(_fixture_json(os.path.join(TOPOLOGIES, "canonical.yaml"), 0.3), None,
             isim.SimParams(flags=KERNELS[kernel]))
    li = c.handler.launch_info(0)
    per = 128 if li["kernel_kind"] in STREAM_KINDS else 64
    n = 2 * li["max_blocks"] * li["wg_threads"] // 64 * per + 999
    _, one = c.gpu(0, n, records=False)
    dev = torch.device("cuda", 0)
    st = torch.zeros(c.handler.stats_words, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    k = 300  # more launches than queue sets (kWorkSlots): every set is reused
    for _ in range(k):
        c.handler.serve_device(0, n, 0, st.data_ptr(), s)
    torch.cuda.synchronize()
    got = st.cpu().numpy().view(np.uint64)
    f1, fk = c.handler.fold(one), c.handler.fold(got)
    assert fk["n_traces"] == k * n and f1["n_traces"] == n
    assert fk["sum_latency"] == k * f1["sum_latency"] and fk["n_500"] == k * f1["n_500"]
    assert np.array_equal(fk["site_calls"], k * f1["site_calls"])


# ---- draw-free static walks: one walk, then a record fill + n x statistics

@pytest.mark.parametrize("mode", [isim.MODE_A, isim.MODE_B])
@pytest.mark.parametrize("n", [1, 1000, 1 << 20])
def test_draw_free_fill(gpu, mode, n):
    doc = config2_topology()
    for i, s in enumerate(doc["services"]):
        s["errorRate"] = 1 if i % 7 == 3 else 0  # deterministic 500s: statuses and error counts
    j = json.dumps(doc)
    fill = Case(j, None, isim.SimParams(error_mode=mode))
    walk = isim.Handler(isim.ServiceGraph.from_json(j), None,
                        isim.SimParams(error_mode=mode, flags=isim.native.FLAG_WALK_ALL))
    r1, s1 = fill.gpu(3, n)
    r2, s2 = walk.serve(3, n)
    assert np.array_equal(r1, r2) and np.array_equal(s1, s2)
    if n <= 1000:
        fill.compare(3, n)


def test_site_counter_beyond_u32(gpu):
    """Per-workgroup LDS site counters are u32: a binary DAG chain whose leaf
    is called 2^22 times per trace pushes one workgroup's leaf-error counter
    (2,048 traces x 2^22) past 2^32, so the library must split the launch
    (api.hip launch_walk: 1,023 traces per launch here).  Expected numbers are
    analytic: every trace makes 2^23 - 1 invocations, 2^22 of them the
    errorRate-1 leaf."""
    depth = 22
    svcs = [{"name": f"s{i}", "script": [{"call": f"s{i + 1}"}, {"call": f"s{i + 1}"}]} for i in range(depth)]
    svcs.append({"name": f"s{depth}", "errorRate": 1.0})
    svcs[0]["isEntrypoint"] = True
    h = isim.Handler(isim.ServiceGraph.from_json(json.dumps({"services": svcs})), None,
                     isim.SimParams(hop_base_ns=1, req_ps_per_byte=0, resp_ps_per_byte=0,
                                    flags=isim.native.FLAG_WALK_ALL))
    assert h.launch_info(0)["kernel_kind"] == 4 and h.launch_info(0)["lds_counters"] == 1
    n = 4200
    recs, stats = h.serve(0, n)
    inv, leaf = (1 << (depth + 1)) - 1, 1 << depth
    assert np.all(recs["hops"] == inv) and np.all(recs["latency_ns"] == inv - 1)
    assert np.all(recs["status_err"] == leaf)  # entry 200 (mode A), 2^22 erring leaves
    f = h.fold(stats)
    assert int(f["svc_calls"][depth]) == n * leaf and int(f["svc_errs"][depth]) == n * leaf
    assert n * leaf > 1 << 32
    assert int(f["svc_errs"][:depth].sum()) == 0 and int(f["svc_calls"][0]) == n


def test_tree_row_counter_split(gpu):
    """ADVICE round 2 (kind 7): a service whose per-service duration row keeps
    an LDS bucket table (its duration varies: it calls a 10 ms service with
    probability 50) is reached from 1,600 positions through four callers (one
    concurrent step of 400 calls each, probability 99), so
    one workgroup's u32 bucket counter of that row can take 1,600 counts per
    trace, more than any one call site (400).  The launch split must follow
    the row (Program::tree_mult takes the row's positions):
    max_launch_traces = (2^32 - 1) // 1600.  A batch is then bit-exact
    against the oracle."""
    svcs = [{"name": "e", "isEntrypoint": True, "script": [{"call": f"m{i}"} for i in range(4)]}]
    for i in range(4):
        # one concurrent step of 400 calls (the latency bound stays below 2^32 ns: kind 7)
        svcs.append({"name": f"m{i}", "script": [[{"call": {"service": "x", "probability": 99}}] * 400]})
    svcs.append({"name": "x", "script": [{"call": {"service": "y", "probability": 50}}]})
    svcs.append({"name": "y", "script": [{"sleep": "10ms"}]})
    c = Case(json.dumps({"services": svcs}), None, isim.SimParams())
    info = c.handler.launch_info(0)
    assert info["kernel_kind"] == 7 and info["lds_counters"] == 1
    assert info["max_launch_traces"] == 0xFFFFFFFF // 1600
    c.compare(5, 300)


def _prob_chain(depth, p=90):
    """A chain of `depth` calling services, every call probabilistic: a
    dynamic walk whose frames go deeper than the 16 register frames of the
    lane tree walk (the spill areas)."""
    doc = json.loads(_chain(depth, 1))
    for s in doc["services"]:
        for st in s.get("script", []):
            for c in (st if isinstance(st, list) else [st]):
                if "call" in c:
                    c["call"] = {"service": c["call"], "probability": p}
    return json.dumps(doc)


def test_tree_spill_two_streams(gpu):
    """a spilling lane tree walk (call depth 40 > 16 register
    frames) launched on two streams at once, many launches each, must give
    every launch its own frames: each stream's accumulated stats and its last
    records equal the sequential walk's (and the oracle's, on a window)."""
    import torch
    c = Case(_prob_chain(40), None, isim.SimParams())
    li = c.handler.launch_info(0)
    assert li["kernel_kind"] == 7 and c.handler.info.max_depth == 40
    n = li["max_blocks"] * li["wg_threads"] + 777  # every lane of the grid walks (and spills)
    begins = (1 << 20, (1 << 32) - 5000)
    ref = [c.gpu(b, n) for b in begins]
    c.compare(begins[1], 3000)
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(dev) for _ in begins]
    st = [torch.zeros(c.handler.stats_words, dtype=torch.int64, device=dev) for _ in begins]
    rec = [torch.zeros(n * 16, dtype=torch.uint8, device=dev) for _ in begins]
    k = 6
    torch.cuda.synchronize()
    for _ in range(k):
        for i, b in enumerate(begins):
            c.handler.serve_device(b, n, rec[i].data_ptr(), st[i].data_ptr(), streams[i].cuda_stream)
    torch.cuda.synchronize()
    for i in range(len(begins)):
        r = rec[i].cpu().numpy().view(isim.REC_DTYPE)
        assert np.array_equal(r, ref[i][0])
        fk, f1 = c.handler.fold(st[i].cpu().numpy().view(np.uint64)), c.handler.fold(ref[i][1])
        assert fk["n_traces"] == k * n and fk["sum_latency"] == k * f1["sum_latency"]
        assert fk["sum_hops"] == k * f1["sum_hops"] and fk["n_500"] == k * f1["n_500"]
        assert np.array_equal(fk["site_calls"], k * f1["site_calls"])


def test_tree_graph_capture(gpu):
    """isim_serve_device is graph-capturable after the first
    call on a device (isim.h), except for a spilling lane tree walk, whose
    spill area a graph would pin while eager launches on other streams take
    the same area: that capture returns ISIM_EINVAL.  A non-spilling dynamic
    walk captured on one stream and replayed alongside eager launches of the
    same handler on a second stream gives each its own, correct results."""
    import torch
    dev = torch.device("cuda", 0)
    deep = Case(_prob_chain(40), None, isim.SimParams())
    deep.gpu(0, 1000)  # the first call prepares the device
    st = torch.zeros(deep.handler.stats_words, dtype=torch.int64, device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        with pytest.raises(isim.IsimError) as ei:
            deep.handler.serve_device(0, 1000, 0, st.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert ei.value.code == isim.native.EINVAL and "captured" in str(ei.value)

    c = Case(_prob_chain(8), None, isim.SimParams())
    assert c.handler.launch_info(0)["kernel_kind"] == 7
    n, b1, b2 = 50_000, 1 << 30, 77
    ref1, ref2 = c.gpu(b1, n), c.gpu(b2, n)
    rec1 = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    st1 = torch.zeros(c.handler.stats_words, dtype=torch.int64, device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        c.handler.serve_device(b1, n, rec1.data_ptr(), st1.data_ptr(), torch.cuda.current_stream().cuda_stream)
    other = torch.cuda.Stream(dev)
    rec2 = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    st2 = torch.zeros(c.handler.stats_words, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    k = 4
    for _ in range(k):
        g.replay()
        c.handler.serve_device(b2, n, rec2.data_ptr(), st2.data_ptr(), other.cuda_stream)
    torch.cuda.synchronize()
    for rec, stt, ref in ((rec1, st1, ref1), (rec2, st2, ref2)):
        assert np.array_equal(rec.cpu().numpy().view(isim.REC_DTYPE), ref[0])
        fk, f1 = c.handler.fold(stt.cpu().numpy().view(np.uint64)), c.handler.fold(ref[1])
        assert fk["n_traces"] == k * n and fk["sum_latency"] == k * f1["sum_latency"]
        assert np.array_equal(fk["site_calls"], k * f1["site_calls"])


@pytest.mark.parametrize("mode", [isim.MODE_A, isim.MODE_B])
def test_tree_u64_time(gpu, mode):
    """The lane tree walk with u64 time (Program::tree_t64): a chain of 1.5 s
    sleeps with probabilistic concurrent calls, whose traces exceed 2^32 ns,
    bit-exact against the oracle — records (both latency words), stats and
    the per-service duration rows (durations past 2^32 ns go to their
    row's sum in HBM) — on the kernel kind 7, next to the wave interpreter
    (kind 3) on the same graph."""
    svcs = [{"name": f"s{i}", "errorRate": 0.1,
             "script": [{"sleep": "1500ms"}] + ([[{"call": {"service": f"s{i + 1}", "probability": 90}},
                                                  {"call": f"s{i + 1}"}]] if i < 3 else [])} for i in range(4)]
    svcs[0]["isEntrypoint"] = True
    j = json.dumps({"services": svcs})
    c = Case(j, None, isim.SimParams(error_mode=mode))
    assert c.handler.info.time_bits == 64 and c.handler.launch_info(0)["kernel_kind"] == 7
    recs, _ = c.compare((1 << 32) - 1000, 3000)
    assert int(recs["latency_ns"].max()) > 1 << 32
    w = Case(j, None, isim.SimParams(error_mode=mode, flags=isim.native.FLAG_WAVE_WALK))
    assert w.handler.launch_info(0)["kernel_kind"] == 3
    w.compare(7, 1000)


# ---- wide trees (round 5): past 65,535 positions, call sites or rows, or
# per-slot counters that do not fit in LDS — 16-byte nodes, 32-bit frames,
# the hottest call sites counted in LDS, the rest by global atomics (tree.hip
# WideSink; isim_launch_info.tree_wide)
@pytest.mark.parametrize("mode", [isim.MODE_A, isim.MODE_B])
def test_tree_wide_forced(gpu, mode):
    """Every tree shape in the wide format (ISIM_FLAG_TREE_WIDE): a mesh,
    a deep concurrent realistic graph, a 40-deep chain (spilled frames), u64
    time — bit-exact against the oracle on windows across 2^32."""
    docs = [with_defaults(obj_to_json(mesh_topology(1200, 6, seed=3)), errorRate=0.05),
            obj_to_json(realistic_topology(400, concurrent=True, sleep_ms=(1, 5), error_rate=(0.0, 0.2),
                                           probability=70)),
            _prob_chain(40),
            obj_to_json(realistic_topology(300, sleep_ms=(20, 40), error_rate=(0.0, 0.1), probability=75))]
    for j in docs:
        c = Case(j, None, isim.SimParams(error_mode=mode, flags=isim.native.FLAG_TREE_WIDE))
        li = c.handler.launch_info(0)
        assert li["kernel_kind"] == 7 and li["tree_wide"] == 1
        c.compare(1000, 3000)
        c.compare((1 << 32) - 700, 1400)


def test_tree_wide_by_size(gpu):
    """70,000 services with probabilistic calls: 70,000 positions and call
    sites, past the 8-byte nodes — the wide kernel without forcing."""
    j = obj_to_json(realistic_topology(70000, concurrent=True, sleep_ms=(1, 3), error_rate=(0.0, 0.01),
                                       probability=40))
    c = Case(j, None, isim.SimParams())
    li = c.handler.launch_info(0)
    assert li["kernel_kind"] == 7 and li["tree_wide"] == 1
    c.compare(77, 2000)


def test_tree_wide_equals_narrow(gpu):
    """2^24 traces of one graph on the 8-byte kernel and forced wide: equal
    records and statistics word for word — at that size a workgroup counts
    more than 2^15 calls at the hot sites, so the wide sink's guarded LDS
    fields move 2^15 events (and their leaf durations) to HBM mid-launch."""
    j = obj_to_json(realistic_topology(400, concurrent=True, sleep_ms=(1, 5), error_rate=(0.0, 0.2), probability=70))
    n = 1 << 24
    narrow = Case(j, None, isim.SimParams())
    assert narrow.handler.launch_info(0)["tree_wide"] == 0
    r1, s1 = narrow.gpu(12345, n)
    wide = Case(j, None, isim.SimParams(flags=isim.native.FLAG_TREE_WIDE))
    assert wide.handler.launch_info(0)["tree_wide"] == 1
    r2, s2 = wide.gpu(12345, n)
    assert np.array_equal(r1, r2)
    assert np.array_equal(s1, s2)


# ---- the site graph (round 6, Program::tree_dag): kind 7 over one node per
# call site for DAGs whose unrolled tree would pass 2^24 positions
# (validation.go:28-57 accepts any DAG; before round 6 such walks ran on the
# wave interpreter, kinds 2/3, 17-18x slower)

@pytest.mark.parametrize("mode", [isim.MODE_A, isim.MODE_B])
def test_tree_dag_forced(gpu, mode):
    """Every dynamic walk over the site graph (ISIM_FLAG_TREE_DAG): a mesh, a
    deep concurrent realistic graph, a 40-deep chain (spilled frames), u64
    time, a shared-callee DAG — bit-exact against the oracle on windows
    across 2^32 (executable.go:84-179, handler.go:37-79)."""
    from test_tree_walk import layered_dag
    docs = [with_defaults(obj_to_json(mesh_topology(1200, 6, seed=3)), errorRate=0.05),
            obj_to_json(realistic_topology(400, concurrent=True, sleep_ms=(1, 5), error_rate=(0.0, 0.2),
                                           probability=70)),
            _prob_chain(40),
            obj_to_json(realistic_topology(300, sleep_ms=(20, 40), error_rate=(0.0, 0.1), probability=75)),
            layered_dag(5, 4, prob=40)]
    for j in docs:
        c = Case(j, None, isim.SimParams(error_mode=mode, flags=isim.native.FLAG_TREE_DAG))
        li = c.handler.launch_info(0)
        assert li["kernel_kind"] == 7 and li["tree_wide"] == 2
        c.compare(1000, 3000)
        c.compare((1 << 32) - 700, 1400)


@pytest.mark.parametrize("mode", [isim.MODE_A, isim.MODE_B])
def test_tree_dag_by_size(gpu, mode):
    """A DAG of 72 services whose unrolled tree has 8^9 = 134M positions
    (every service of a layer calls every one of the next at probability 10):
    the site graph without forcing (u32 time: concurrent fan-out) —
    bit-exact against the oracle,
    and at 2^20 traces record for record equal to the wave interpreter (kinds
    2/3, ISIM_FLAG_WAVE_WALK), the path such walks took before.  The DES
    rejects it (no unrolled tree to schedule)."""
    from test_tree_walk import layered_dag
    j = layered_dag()
    c = Case(j, None, isim.SimParams(error_mode=mode))
    li = c.handler.launch_info(0)
    assert li["kernel_kind"] == 7 and li["tree_wide"] == 2
    c.compare(5, 3000)
    c.compare((1 << 32) - 1500, 3000)
    n = 1 << 20
    r1, s1 = c.gpu(1 << 33, n)
    w = isim.Handler(isim.ServiceGraph.from_json(j), None,
                     isim.SimParams(error_mode=mode, flags=isim.native.FLAG_WAVE_WALK))
    assert w.launch_info(0)["kernel_kind"] in (2, 3)
    r2, s2 = w.serve(1 << 33, n)
    assert np.array_equal(r1, r2)
    f1, f2 = c.handler.fold(s1), w.fold(s2)
    for k in ("n_traces", "sum_latency", "sum_hops", "sum_err_hops", "n_500"):
        assert f1[k] == f2[k], k
    for k in ("site_calls", "svc_calls", "svc_errs"):
        assert np.array_equal(np.asarray(f1[k]), np.asarray(f2[k])), k
    with pytest.raises(isim.IsimError) as ei:
        isim.DesHandler(c.handler, 1_000_000)
    assert ei.value.code == isim.native.EINVAL and "site graph" in str(ei.value)
