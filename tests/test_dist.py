"""Multi-process path on CPU (gloo, world_size 2): trace sharding and the
stats merge (isim.dist: torch.distributed across ranks, libisim's
isim_stats_merge across steps), with the C oracle producing each rank's
shard.  The merged buffer must equal one process over the union.  The same
with the HIP walk producing the shards: tests/test_multi_gpu.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _graph_json():
    from isim.generators import realistic_topology
    from isim.yamljson import obj_to_json
    return obj_to_json(realistic_topology(300, "multitier", seed=5, concurrent=True, sleep_ms=(1, 5),
                                          error_rate=(0, 0.2)))


def _oracle_stats(begin, n):
    from oracle import executor as oc
    from oracle import graph_ref as gr
    from oracle.executor_py import SimGraph, SimParams
    sg = SimGraph(gr.unmarshal_service_graph(_graph_json()))
    _, st = oc.run(sg, SimParams(), sg.entry(), begin, n, records=False, n_threads=1)
    return st


def _to_isim_layout(st):
    # oracle layout keeps min at word 5; isim keeps ~min
    out = st.astype(np.uint64).copy()
    out[5] = ~out[5]
    return out.view(np.int64)


def _worker(rank, world, port, steps, batch, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "istio-isotope_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from isim.dist import merge_stats, shard_begin, stats_merge
    h = _handler()
    acc = None
    for s in range(steps):
        st = _to_isim_layout(_oracle_stats(shard_begin(rank, world, s, batch), batch)).view(np.uint64)
        st = st[:h.stats_words]  # the oracle appends per-service duration rows
        # the per-rank accumulation across steps uses libisim's host merge
        acc = st.copy() if acc is None else stats_merge(h, acc, st)
    t = torch.from_numpy(acc.view(np.int64).copy())
    merge_stats(t)
    if rank == 0:
        q.put(t.numpy().copy())
    dist.destroy_process_group()


def _handler():
    import isim
    return isim.Handler(isim.ServiceGraph.from_json(_graph_json()))


def test_stats_merge_host_equals_union():
    """isim_stats_merge (the product's host merge) of oracle shards equals the
    oracle run over the union: SUM everywhere, MAX on [~min, max]."""
    from isim.dist import stats_merge
    h = _handler()
    w = h.stats_words  # the oracle appends per-service duration rows
    a = _to_isim_layout(_oracle_stats(0, 200)).view(np.uint64)[:w].copy()
    b = _to_isim_layout(_oracle_stats(200, 300)).view(np.uint64)[:w]
    union = _to_isim_layout(_oracle_stats(0, 500)).view(np.uint64)[:w]
    assert np.array_equal(stats_merge(h, a, b), union)
    # merging an all-zero buffer (an idle rank) changes nothing
    assert np.array_equal(stats_merge(h, a, np.zeros_like(a)), union)


def test_des_table_merge_rules():
    import isim
    from isim.dist import des_table_merge
    h = _handler()
    rows = int(h.info.n_reachable)
    rng = np.random.default_rng(3)
    a = rng.integers(0, 1 << 40, rows * isim.native.DES_ROW_WORDS, dtype=np.uint64)
    b = rng.integers(0, 1 << 40, rows * isim.native.DES_ROW_WORDS, dtype=np.uint64)
    want = (a + b).reshape(rows, -1)
    want[:, isim.native.DES_MAX_WAIT] = np.maximum(a.reshape(rows, -1)[:, isim.native.DES_MAX_WAIT],
                                                   b.reshape(rows, -1)[:, isim.native.DES_MAX_WAIT])
    assert np.array_equal(des_table_merge(h, a.copy(), b).reshape(rows, -1), want)


@pytest.mark.parametrize("world", [2])
def test_sharded_merge_equals_single_process(world):
    steps, batch = 2, 150
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, steps, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    merged = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    single = _to_isim_layout(_oracle_stats(0, steps * world * batch))[:merged.size]
    assert np.array_equal(merged.view(np.uint64), single.view(np.uint64))


def test_shard_ranges_partition():
    from isim.dist import shard_begin
    world, steps, batch = 4, 3, 10
    ids = sorted(i for s in range(steps) for r in range(world)
                 for i in range(shard_begin(r, world, s, batch), shard_begin(r, world, s, batch) + batch))
    assert ids == list(range(world * steps * batch))


def _make_multi_worker(rank, world, port, scenario, q, arrived):
    """bench.make_multi's collective choice with a stand-in for isim.dist.Multi
    (no RCCL on a CPU): every rank must come out with the same decision."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "istio-isotope_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import isim.dist

    class FakeMulti:
        closed = False

        @staticmethod
        def precheck(local):
            if scenario == "precheck_fails_on_1" and rank == 1:
                raise RuntimeError("hipSetDevice")

        @staticmethod
        def get_id():
            if scenario == "id_fails_on_1" and rank == 1:
                raise RuntimeError("no RCCL here")
            return bytes(128)

        @staticmethod
        def init_rank(mid, w, r, local):
            # ncclCommInitRank is collective: a rank returns only once every
            # rank has entered it, or (libisim's non-blocking creation) with
            # ECOMM after ISIM_MULTI_TIMEOUT_S, modelled here as 3 s
            if scenario == "init_fails_on_0" and r == 0:  # entered, then failed: the peer got its comm
                arrived[r].set()
                raise RuntimeError("ncclCommInitRank")
            if scenario == "init_local_fails_on_0" and r == 0:
                raise RuntimeError("local failure before entering ncclCommInitRank")
            arrived[r].set()
            if not all(e.wait(timeout=3.0) for e in arrived):
                raise RuntimeError("ISIM_ECOMM: no answer from the peer ranks within ISIM_MULTI_TIMEOUT_S")
            return FakeMulti()

        def close(self):
            FakeMulti.closed = True

    isim.dist.Multi = FakeMulti
    multi, label = bench.make_multi(rank, world, rank)
    q.put((rank, multi is not None, label, FakeMulti.closed))
    dist.destroy_process_group()


@pytest.mark.parametrize("scenario", ["ok", "id_fails_on_1", "precheck_fails_on_1", "init_fails_on_0",
                                      "init_local_fails_on_0"])
def test_make_multi_is_collective(scenario):
    """ADVICE rounds 2-3: a local failure on one rank (loading RCCL, selecting
    the device, drawing the id, or creating the communicator) sends EVERY rank
    to the torch.distributed merge, and a rank that did create a communicator
    frees it.  init_local_fails_on_0: rank 0 fails before it enters the
    collective creation; rank 1 waits inside it until the (modelled) timeout,
    then both agree on the fallback."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    arrived = [ctx.Event() for _ in range(world)]
    procs = [ctx.Process(target=_make_multi_worker, args=(r, world, port, scenario, q, arrived)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    uses = {g[1] for g in got}
    assert len(uses) == 1, got  # one decision for all ranks
    if scenario == "ok":
        assert uses == {True} and all("libisim RCCL" in g[2] for g in got)
    else:
        assert uses == {False} and all(g[2].startswith("torch.distributed") for g in got)
    if scenario == "init_fails_on_0":
        assert got[1][3]  # rank 1 had a communicator: closed
