"""GPU parity of the DES (BASELINE config 5): the HIP
level-synchronous DES through the C ABI against the sequential event-driven
C oracle — per-trace records, stats, and the per-service DES table, bit-exact."""
import json

import numpy as np
import pytest

import isim
from isim.generators import config3_topology, realistic_topology, tree_topology
from isim.yamljson import obj_to_json
from oracle import des as od
from oracle import executor as oc
from oracle import graph_ref as gr
from oracle.executor_py import SimGraph

from parity import assert_records_equal, assert_stats_equal, oracle_params

pytestmark = pytest.mark.gpu


class DesCase:
    def __init__(self, doc, mean_ns, **kw):
        self.json = obj_to_json(doc) if isinstance(doc, dict) else doc
        self.h = isim.Handler(isim.ServiceGraph.from_json(self.json), None, isim.SimParams(**kw))
        self.d = isim.DesHandler(self.h, mean_ns)
        self.sg = SimGraph(gr.unmarshal_service_graph(self.json))
        self.op = oracle_params(self.h.params)
        self.og = oc.OracleGraph(self.sg, self.op)
        self.mean = mean_ns

    def compare(self, begin, n, records=True):
        recs, stats, table = self.d.serve(begin, n, device=0, records=records)
        orec, ost, odes = od.run(self.sg, self.op, self.sg.entry(), begin, n, self.mean, records=records, og=self.og)
        if records:
            assert_records_equal(recs, orec)
        ns, nsite = len(self.sg.g.services), len(self.sg.sites)
        o = oc.split_stats(np.concatenate([ost, np.zeros(68 * ns, np.uint64)]), ns, nsite)
        f = self.h.fold(stats)
        f["svc_dur"] = None
        assert_stats_equal(f, o)
        rows = self.d.fold(table)
        bad = np.argwhere(rows != odes)
        assert bad.size == 0, f"DES table differs at (service, word) {bad[:4].tolist()}: " \
                              f"gpu {rows[tuple(bad[0])]} oracle {odes[tuple(bad[0])]}"
        return recs, stats, rows


def _sleepy_tree(levels, branches, reps_leaves=1, post=True):
    doc = tree_topology(levels, branches)
    for s in doc["services"]:
        s["script"] = [{"sleep": "2ms"}] + s.get("script", []) + ([{"sleep": "300us"}] if post else [])
    if reps_leaves > 1:
        for s in doc["services"]:
            if not any(isinstance(x, list) for x in s["script"]):
                s["numReplicas"] = reps_leaves
    return doc


@pytest.mark.parametrize("mean", [300_000, 2_500_000, 40_000_000])
@pytest.mark.parametrize("mode", [isim.MODE_A, isim.MODE_B])
def test_realistic_loads(gpu, mean, mode):
    c = DesCase(realistic_topology(400, concurrent=True, sleep_ms=(1, 5), error_rate=(0.0, 0.05)), mean,
                error_mode=mode)
    recs, _, rows = c.compare(3, 5000)
    if mean == 300_000:
        assert rows[:, isim.native.DES_SUM_WAIT].sum() > 0


@pytest.mark.parametrize("n", [1, 2, 1023, 8191, 8192, 8193, 20000])
def test_ragged_batches(gpu, n):
    DesCase(_sleepy_tree(3, 3), 1_000_000, ).compare(1 << 33, n)  # trace ids past 2^32


@pytest.mark.parametrize("reps", [2, 5, 64])
def test_leaf_replicas(gpu, reps):
    DesCase(_sleepy_tree(3, 4, reps), 700_000).compare(0, 12000)


def test_error_rate_extremes(gpu):
    # mode B static walks have no step after a step that can fail: no post-call sleeps
    doc = _sleepy_tree(4, 3, post=False)
    for i, s in enumerate(doc["services"]):
        s["errorRate"] = [0, 1, 0.5][i % 3]
    DesCase(doc, 1_500_000, error_mode=isim.MODE_B).compare(0, 3000)
    DesCase(doc, 1_500_000, error_mode=isim.MODE_A).compare(0, 3000)
    doc = _sleepy_tree(4, 3)
    for i, s in enumerate(doc["services"]):
        s["errorRate"] = [0, 1, 0.5][i % 3]
    DesCase(doc, 1_500_000, error_mode=isim.MODE_A).compare(0, 3000)
    # a failing call step followed by a sleep is not a static walk: the item engine (mode-B aborts)
    c = DesCase(doc, 1_500_000, error_mode=isim.MODE_B)
    assert c.d.info.items == 1
    c.compare(0, 3000)


def test_zero_traces(gpu):
    c = DesCase(_sleepy_tree(2, 2), 1_000_000)
    recs, stats, table = c.d.serve(0, 0)
    assert stats.sum() == 0 and table.sum() == 0


def test_config5_slice(gpu):
    # the config-5 graph (BASELINE config 3's 10k services), a batch the oracle finishes quickly
    c = DesCase(config3_topology(), 6_000_000)
    c.compare(0, 256)


def test_config5_bench_scale(gpu):
    """The config-5 graph on a batch that crosses the chained look-back of the
    narrow queue pass (chunks of 4,096 traces) and the arrival scan's blocks
    (8,192 traces) several times, with a ragged tail: 20,000 traces, bit-exact
    against the event-driven DES oracle (about 30 s of oracle time)."""
    c = DesCase(config3_topology(), 6_000_000)
    recs, _, rows = c.compare(1000, 20_000)
    assert int(rows[:, isim.native.DES_SUM_WAIT].sum()) > 0  # the queues are contended


def test_config5_bench_batch_prefix(gpu):
    """The bench's own batch (2^20 traces per step, bench.py --config c5):
    on the config-5 graph every service has one position fed by one caller,
    so arrivals stay in trace order and a trace never waits for a later one —
    the first 20,000 records of the 2^20 batch equal the 20,000-trace batch
    that test_config5_bench_scale pins to the event-driven oracle."""
    c = DesCase(config3_topology(), 6_000_000)
    full, stats, table = c.d.serve(1000, 1 << 20)
    pre, _, _ = c.d.serve(1000, 20_000)
    rows = c.d.fold(table)
    assert np.array_equal(full[:20_000], pre)
    f = c.h.fold(stats)
    assert f["n_traces"] == 1 << 20 and f["sum_hops"] == (1 << 20) * 10_000
    assert int(full["latency_ns"].astype(np.uint64).sum()) == f["sum_latency"]
    assert int(rows[:, isim.native.DES_SUM_WAIT].sum()) > 0


@pytest.mark.parametrize("wide", [False, True])
def test_device_entry_accumulates(gpu, wide):
    import torch
    c = DesCase(_sleepy_tree(3, 3), 3_000_000)  # latencies well below 2^31 ns
    n = 5000
    dev = torch.device("cuda", 0)
    rec = torch.zeros(n * 2, dtype=torch.int64, device=dev)
    st = torch.zeros(c.h.stats_words, dtype=torch.int64, device=dev)
    tab = torch.zeros(max(1, c.d.table_words), dtype=torch.int64, device=dev)
    wsb = c.d.workspace_bytes(n)
    ws = torch.empty(wsb // 8 + 1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for half in (0, 1):  # two batches accumulate into the same stats/table
        c.d.serve_device(half * n, n, rec.data_ptr(), st.data_ptr(), tab.data_ptr(), ws.data_ptr(), wsb, s,
                         wide=wide)
    torch.cuda.synchronize()
    _, s0, t0 = c.d.serve(0, n, records=False)
    _, s1, t1 = c.d.serve(n, n, records=False)
    stg = st.cpu().numpy().view(np.uint64)
    assert int(stg[0]) == 2 * n
    assert int(stg[isim.native.ST_SUM_LATENCY]) == int(s0[1]) + int(s1[1])
    W = isim.native.DES_ROW_WORDS
    tg = tab.cpu().numpy().view(np.uint64)[:t0.size].reshape(-1, W)
    want = (t0 + t1).reshape(-1, W)
    mw = isim.native.DES_MAX_WAIT  # the longest wait merges with max
    want[:, mw] = np.maximum(t0.reshape(-1, W)[:, mw], t1.reshape(-1, W)[:, mw])
    assert np.array_equal(tg, want)


# ---- the sort path: DAG graphs (a service at several positions per trace)
# and replicated callers (arrivals out of trace order)

def _dag(levels=4, width=5, fan=2, seed=3, reps=1):
    import random
    rnd = random.Random(seed)
    svcs = []
    for l in range(levels):
        for j in range(width if l else 1):
            calls = []
            if l + 1 < levels:
                calls = [{"call": f"n{l + 1}-{c}"} for c in sorted(rnd.sample(range(width), fan))]
            script = [{"sleep": f"{rnd.randint(100, 900)}us"}] + ([calls] if calls else []) + \
                     ([{"sleep": "50us"}] if l % 2 else [])
            svcs.append({"name": f"n{l}-{j}", "script": script, "errorRate": 0.01,
                         "numReplicas": reps if l and rnd.random() < 0.5 else 1})
    svcs[0]["isEntrypoint"] = True
    return {"services": svcs}


@pytest.mark.parametrize("mean", [200_000, 2_000_000])
def test_canonical_dag(gpu, mean):
    from test_des import canonical_concurrent
    DesCase(canonical_concurrent(), mean, error_mode=isim.MODE_A).compare(0, 9000)


@pytest.mark.parametrize("reps", [1, 3])
@pytest.mark.parametrize("mean", [150_000, 1_500_000])
def test_random_dags(gpu, reps, mean):
    DesCase(_dag(reps=reps), mean).compare(7, 10000)


def test_replicated_callers(gpu):
    doc = _sleepy_tree(4, 3)
    for i, s in enumerate(doc["services"]):
        s["numReplicas"] = 1 + i % 4  # internal services too
    DesCase(doc, 600_000).compare(0, 12000)


def test_dag_mode_b(gpu):
    doc = _dag(levels=5, width=6, fan=3, reps=2)
    for s in doc["services"]:
        s["script"] = [x for x in s["script"] if not (isinstance(x, dict) and x.get("sleep") == "50us")]
        s["errorRate"] = 0.05
    DesCase(doc, 400_000, error_mode=isim.MODE_B).compare(0, 6000)


# ---- calls after calls (step begins)

def _sleepy(doc, pre="400us", post="100us"):
    for s in doc["services"]:
        s["script"] = [{"sleep": pre}] + s.get("script", []) + ([{"sleep": post}] if post else [])
    return doc


@pytest.mark.parametrize("mean", [300_000, 3_000_000])
def test_sequential_tree(gpu, mean):
    DesCase(_sleepy(tree_topology(3, 4, sequential=True)), mean).compare(0, 8000)


def test_sequential_realistic(gpu):
    # the reference generator's default: one call step per child (mode A: in
    # mode B a 500 would abort the later steps, not a static walk)
    doc = realistic_topology(150, sleep_ms=(1, 3), error_rate=(0.0, 0.05))
    DesCase(doc, 2_000_000).compare(3, 6000)


def test_mixed_steps_and_replicas(gpu):
    doc = tree_topology(4, 3)
    for i, s in enumerate(doc["services"]):
        calls = [c for st in s.get("script", []) for c in (st if isinstance(st, list) else [st])]
        if len(calls) == 3:  # [a || b], sleep, c
            s["script"] = [{"sleep": "200us"}, [calls[0], calls[1], {"sleep": "50us"}], {"sleep": "70us"}, calls[2]]
        else:
            s["script"] = [{"sleep": f"{100 + 37 * i}us"}]
        s["numReplicas"] = 1 + i % 3
        s["errorRate"] = 0.02
    DesCase(doc, 500_000).compare(0, 7000)


# ---- row widths: 32-bit rows relative to each trace's
# arrival, 64-bit rows on request or when a latency reaches 2^31 ns

def test_narrow_equals_wide(gpu):
    c = DesCase(realistic_topology(300, concurrent=True, sleep_ms=(1, 5), error_rate=(0.0, 0.05)), 900_000)
    r1, s1, t1 = c.d.serve(5, 6000)
    r2, s2, t2 = c.d.serve(5, 6000, wide=True)
    assert np.array_equal(r1, r2) and np.array_equal(s1, s2) and np.array_equal(t1, t2)
    assert s1[isim.native.ST_DES_RETRY] == 0


def _overloaded():
    # 5 ms of service per trace every ~100 us: the queue grows ~5 ms per
    # trace, so late traces wait for tens of seconds (> 2^31 ns)
    doc = tree_topology(2, 2)
    for s in doc["services"]:
        s["script"] = [{"sleep": "5ms"}] + s.get("script", [])
    return doc


def test_overflow_retries_wide(gpu):
    import torch
    c = DesCase(_overloaded(), 100_000)
    n = 3000
    recs, stats, rows = c.compare(0, n)  # the synchronous entry reruns the batch with 64-bit rows
    assert int(stats[isim.native.ST_MAX_LATENCY]) >= 1 << 31 and stats[isim.native.ST_DES_RETRY] == 0
    # the device entry drops the batch and counts it
    dev = torch.device("cuda", 0)
    st = torch.zeros(c.h.stats_words, dtype=torch.int64, device=dev)
    tab = torch.zeros(max(1, c.d.table_words), dtype=torch.int64, device=dev)
    rec = torch.full((2 * n,), -1, dtype=torch.int64, device=dev)
    wsb = c.d.workspace_bytes(n)
    ws = torch.empty(wsb // 8 + 1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    c.d.serve_device(0, n, rec.data_ptr(), st.data_ptr(), tab.data_ptr(), ws.data_ptr(), wsb, s)
    torch.cuda.synchronize()
    got = st.cpu().numpy().view(np.uint64)
    assert got[isim.native.ST_DES_RETRY] == 1
    got[isim.native.ST_DES_RETRY] = 0
    assert got.sum() == 0 and tab.sum().item() == 0 and (rec == -1).all().item()
    # wide rows on the same buffers: the oracle's numbers
    c.d.serve_device(0, n, rec.data_ptr(), st.data_ptr(), tab.data_ptr(), ws.data_ptr(), wsb, s, wide=True)
    torch.cuda.synchronize()
    got = st.cpu().numpy().view(np.uint64).copy()
    assert got[isim.native.ST_DES_RETRY] == 1  # the earlier drop stays counted
    got[isim.native.ST_DES_RETRY] = 0
    assert np.array_equal(got, stats)
    assert np.array_equal(c.d.fold(tab.cpu().numpy().view(np.uint64)), rows)


# ---- zero-hold services (no sleeps): start = arrival, one op per position

def _fixture_doc(name):
    import os
    from isim.yamljson import yaml_to_json
    from conftest import TOPOLOGIES
    return json.loads(yaml_to_json(open(os.path.join(TOPOLOGIES, name), "rb").read()))


@pytest.mark.parametrize("name", ["canonical.yaml", "canonical-2-replicas.yaml", "10-svc_1000-end.yaml",
                                  "chain-3-services.yaml", "tree-111-services.yaml", "1-service.yaml"])
def test_reference_topologies_as_written(gpu, name):
    # the reference's example graphs have no sleeps: nothing queues, the
    # cyclic canonical schedule and 100-replica services are in the class
    doc = _fixture_doc(name)
    doc.setdefault("defaults", {})["errorRate"] = 0.1
    DesCase(doc, 200_000).compare(0, 4000)


@pytest.mark.parametrize("mean", [150_000, 1_000_000])
def test_canonical_zero_hold_cycle_with_queues(gpu, mean):
    # b (no sleep) is called inside d's first step (through c) and in its
    # second; a, c and d hold their workers
    doc = _fixture_doc("canonical.yaml")
    for s in doc["services"]:
        if s["name"] != "b":
            s["script"] = [{"sleep": "300us"}] + s.get("script", [])
    doc["services"][0]["numReplicas"] = 2
    DesCase(doc, mean).compare(0, 6000)


# ---- replicated services on the sort path: one segmented scan over the
# replicas' queues (any replica count)

@pytest.mark.parametrize("reps", [65, 300])
def test_many_replicas_with_holds(gpu, reps):
    doc = _sleepy_tree(3, 3)
    doc["services"][2]["numReplicas"] = reps  # a middle service
    doc["services"][-1]["numReplicas"] = reps  # a leaf
    DesCase(doc, 30_000).compare(0, 9000)


def test_replicated_dag_segmented(gpu):
    # several positions per service and replicas: sort path, segmented by replica
    DesCase(_dag(levels=4, width=4, fan=2, reps=7), 120_000).compare(3, 8000)


# ---- random graphs: every DES feature at once (call steps after call
# steps, concurrent sleeps, replicas up to 70, zero-hold services, shared
# callees), against the event-driven oracle

def _random_graph(seed):
    import random
    rnd = random.Random(seed)
    layers = [rnd.randint(1, 3) for _ in range(rnd.randint(2, 4))]
    layers[0] = 1
    names = [[f"s{l}_{j}" for j in range(w)] for l, w in enumerate(layers)]
    svcs = []
    for l, row in enumerate(names):
        for name in row:
            script = []
            if rnd.random() < 0.7:
                script.append({"sleep": f"{rnd.randint(0, 400)}us"})
            if l + 1 < len(names):
                callees = rnd.sample(names[l + 1], rnd.randint(1, len(names[l + 1])))
                while callees:
                    take = callees[:rnd.randint(1, len(callees))]
                    callees = callees[len(take):]
                    step = [{"call": c} for c in take]
                    if rnd.random() < 0.4:
                        step.append({"sleep": f"{rnd.randint(1, 200)}us"})
                    script.append(step if len(step) > 1 or rnd.random() < 0.5 else step[0])
                    if rnd.random() < 0.4:
                        script.append({"sleep": f"{rnd.randint(1, 150)}us"})
            if rnd.random() < 0.25:  # a zero-hold service
                script = [c for c in script if not (isinstance(c, dict) and "sleep" in c)]
                script = [[x for x in c if "sleep" not in x] if isinstance(c, list) else c for c in script]
                script = [c for c in script if c != []]
            reps = rnd.choice([1, 1, 1, 2, 3, 5, 70])
            svcs.append({"name": name, "script": script, "numReplicas": reps,
                         "errorRate": rnd.choice([0, 0.01, 0.05, 0.3])})
    svcs[0]["isEntrypoint"] = True
    return {"services": svcs}


@pytest.mark.parametrize("seed", range(40))
def test_random_graphs(gpu, seed):
    doc = _random_graph(seed)
    mode = isim.MODE_B if seed % 3 == 0 else isim.MODE_A
    mean = [60_000, 300_000, 2_000_000][seed % 3]
    try:
        c = DesCase(doc, mean, error_mode=mode)
    except isim.IsimError as e:  # outside the class: a dynamic walk without the lane tree walk's tree
        assert e.code == isim.native.EINVAL and "unrolled tree" in str(e)
        pytest.skip(str(e)[:80])
    c.compare(seed, 3000)


# ---- cyclic schedules: passes to the fixed point

@pytest.mark.parametrize("mean", [120_000, 400_000, 3_000_000])
def test_canonical_with_holds(gpu, mean):
    # b (with a sleep) is called inside d's first step (through c) and in
    # its second: b's queue depends on its own finishes
    doc = _fixture_doc("canonical.yaml")
    for s in doc["services"]:
        s["script"] = [{"sleep": "250us"}] + s.get("script", [])
    DesCase(doc, mean).compare(0, 5000)


def test_cyclic_mode_b_and_wide(gpu):
    doc = _fixture_doc("canonical.yaml")
    for s in doc["services"]:
        s["script"] = [{"sleep": "150us"}] + s.get("script", [])
        s["errorRate"] = 0.05
    c = DesCase(doc, 300_000, error_mode=isim.MODE_A)
    c.compare(7, 3000)
    r1, s1, t1 = c.d.serve(7, 3000)
    r2, s2, t2 = c.d.serve(7, 3000, wide=True)
    assert np.array_equal(r1, r2) and np.array_equal(s1, s2) and np.array_equal(t1, t2)



# ---- round 3: callers record their callees' durations (kDesFlagParentDur:
# the first kDesDurKids = 8 non-fused callees), finishes without the start
# row (kDesFlagNoStart: every callee's hop cost >= the call step's longest
# sleep), 32-bit queue keys per 64-trace group
def _wide_fanout(n_mid=12, conc_sleep_every=2, err=0.02):
    svcs = [{"name": "r", "isEntrypoint": True, "errorRate": err,
             "script": [{"sleep": "1ms"}, [{"call": f"c{i}"} for i in range(n_mid)]]}]
    for i in range(n_mid):
        step = [{"call": f"l{i}_{j}"} for j in range(3)]
        if i % conc_sleep_every == 0:
            step.append({"sleep": "5ms"})  # longer than the hop cost: the finish needs the start row
        svcs.append({"name": f"c{i}", "errorRate": err, "script": [{"sleep": "2ms"}, step]})
        for j in range(3):
            svcs.append({"name": f"l{i}_{j}", "errorRate": err, "script": [{"sleep": "1ms"}]})
    return {"services": svcs}


@pytest.mark.parametrize("mode", [isim.MODE_A, isim.MODE_B])
@pytest.mark.parametrize("mean", [400_000, 3_000_000])
def test_caller_recorded_durations(gpu, mode, mean):
    # 12 non-leaf callees of the entry: 8 recorded by the entry's finish
    # block, 4 by their own; half the callers need their start row
    DesCase(_wide_fanout(), mean, error_mode=mode).compare(5, 9000)


def test_group_bases_long_gaps(gpu):
    # 64-trace groups spanning ~1.3 s of arrivals (20 ms mean gap): the
    # group-relative rows and keys near their 32-bit range, ragged batch
    DesCase(_wide_fanout(6, 1, 0.05), 20_000_000).compare(1 << 32, 4099)


@pytest.mark.parametrize("mean", [500_000, 3_000_000])
def test_single_service_with_hold(gpu, mean):
    # the entry is a fused leaf (its queue pass records its durations;
    # des_finalize must not add them again), ragged batch
    doc = {"services": [{"name": "a", "isEntrypoint": True, "errorRate": 0.2, "script": [{"sleep": "1ms"}]}]}
    DesCase(doc, mean).compare(7, 3001)
