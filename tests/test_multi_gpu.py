"""Multi-device entry points of the C ABI on the GPU (include/isim.h
isim_multi_*, csrc/multi.hip): libisim's own RCCL communicator, the sharded
isim_serve_multi and the device all-reduce of stats and DES tables.  The
box has one GPU, so RCCL runs with one rank (the results must equal
isim_serve bit for bit); the N > 1 data path — shards walked by the HIP
kernel in separate processes, merged across ranks — runs as two processes
on cuda:0 with the gloo backend and is checked against one process over the
union of the shards."""
import os
import socket

import numpy as np
import pytest

import isim
from isim.dist import Multi, shard_begin, stats_merge
from isim.generators import mesh_topology, realistic_topology
from isim.yamljson import obj_to_json

pytestmark = pytest.mark.gpu


def _json(kind):
    if kind == "static":
        return obj_to_json(realistic_topology(2000, "multitier", 11, concurrent=True, sleep_ms=(1, 5),
                                              error_rate=(0.0, 0.02)))
    return obj_to_json(mesh_topology(4000, 5))  # probabilistic calls: the dynamic kernel


def _handler(kind, mode=isim.MODE_A):
    return isim.Handler(isim.ServiceGraph.from_json(_json(kind)), None, isim.SimParams(error_mode=mode))


@pytest.mark.parametrize("kind", ["static", "dynamic"])
@pytest.mark.parametrize("init", ["all", "rank"])
def test_serve_multi_one_rank_equals_serve(gpu, kind, init):
    h = _handler(kind)
    m = Multi.init_all([0]) if init == "all" else Multi.init_rank(Multi.get_id(), 1, 0, 0)
    assert (m.n_ranks, m.n_local, m.first_rank) == (1, 1, 0)
    recs, stats = m.serve(h, 12345, 5000)
    r1, s1 = h.serve(12345, 5000)
    assert np.array_equal(recs, r1) and np.array_equal(stats, s1)
    assert h.fold(stats)["n_traces"] == 5000
    m.close()


def test_allreduce_device_one_rank_is_identity(gpu):
    import torch
    h = _handler("static")
    m = Multi.init_all([0])
    dev = torch.device("cuda", 0)
    st = torch.zeros(h.stats_words, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    h.serve_device(0, 3000, 0, st.data_ptr(), stream.cuda_stream)
    before = st.clone()
    m.allreduce_stats(h, [st.data_ptr()], [stream.cuda_stream])
    torch.cuda.synchronize()
    assert torch.equal(st, before)
    # the DES table's MAX-word staging (gather, SUM + MAX, scatter) is the identity on one rank
    rows = int(h.info.n_reachable)
    tab = torch.randint(0, 1 << 40, (rows * isim.native.DES_ROW_WORDS,), dtype=torch.int64, device=dev)
    tb = tab.clone()
    m.allreduce_des_table(h, [tab.data_ptr()], None)
    torch.cuda.synchronize()
    assert torch.equal(tab, tb)
    m.close()


def test_multi_rejects_bad_arguments(gpu):
    with pytest.raises(isim.IsimError):
        Multi.init_rank(Multi.get_id(), 1, 1, 0)  # rank out of range
    with pytest.raises(isim.IsimError):
        Multi.init_all([])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, kind, batch, steps, q):
    import sys
    import torch
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "istio-isotope_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import isim as I
    from isim.dist import merge_stats, shard_begin as sb, stats_merge as sm
    h = I.Handler(I.ServiceGraph.from_json(_json(kind)))
    acc, recs = None, []
    for s in range(steps):
        r, st = h.serve(sb(rank, world, s, batch), batch, device=0)  # the HIP walk on cuda:0
        recs.append(r)
        acc = st if acc is None else sm(h, acc, st)
    t = torch.from_numpy(acc.view(np.int64).copy())
    merge_stats(t)  # across ranks (gloo here; RCCL in bench.py / isim_multi on a node)
    q.put((rank, t.numpy().copy(), recs))
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["static", "dynamic"])
def test_two_ranks_product_shards_merge_to_union(gpu, kind):
    import torch.multiprocessing as mp
    world, batch, steps = 2, 3000, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, batch, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    h = _handler(kind)
    urec, ust = h.serve(0, world * steps * batch)
    for rank, merged, recs in got:
        assert np.array_equal(merged.view(np.uint64), ust), rank
        for s, r in enumerate(recs):
            b = shard_begin(rank, world, s, batch)
            assert np.array_equal(r, urec[b:b + batch]), (rank, s)
    # and the host merge of the two ranks' merged-per-step buffers is the same rule
    assert np.array_equal(stats_merge(h, np.zeros_like(ust), ust), ust)


def test_precheck(gpu):
    """isim_multi_precheck: the local steps a rank agrees on before the
    collective creation (RCCL loads, the device can be selected)."""
    Multi.precheck(0)
    with pytest.raises(isim.IsimError):
        Multi.precheck(4096)  # no such device: EHIP, no communication attempted


_LONE_RANK = r"""
import os, sys, time
sys.path[:0] = [os.environ["ISIM_ROOT"], os.path.join(os.environ["ISIM_ROOT"], "istio-isotope_amd")]
import isim
from isim import native
from isim.dist import Multi
os.environ["ISIM_MULTI_TIMEOUT_S"] = "5"
t0 = time.time()
try:
    Multi.init_rank(Multi.get_id(), 2, 0, 0)   # rank 1 never comes
    print("CREATED")
except isim.IsimError as e:
    print("ERR", e.code, round(time.time() - t0, 1), e)
"""


def test_init_rank_times_out_without_peer(gpu):
    """a rank whose peer never enters ncclCommInitRank (it
    failed locally first) must not wait forever: libisim creates the
    communicator non-blocking and gives up after ISIM_MULTI_TIMEOUT_S with
    ISIM_ECOMM.  Run in a child process under a hard limit."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ISIM_ROOT=root)
    out = subprocess.run([sys.executable, "-c", _LONE_RANK], env=env, capture_output=True, text=True, timeout=90)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith(("ERR", "CREATED"))]
    assert line, out.stdout + out.stderr
    parts = line[0].split()
    assert parts[0] == "ERR" and int(parts[1]) == isim.ECOMM, line[0]
    assert 4.0 <= float(parts[2]) < 60.0, line[0]


def _abort_worker(rank, world, port, q):
    import torch  # noqa: F401  (RCCL from torch's bundle, as in bench.py)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ISIM_MULTI_TIMEOUT_S="60")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    obj = [Multi.get_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    m = Multi.init_rank(obj[0], world, rank, rank)
    dist.barrier()
    h = _handler("static")
    try:
        if rank == 0:
            m.abort()  # a local failure before the collective
            q.put((rank, "aborted"))
        else:
            m.serve(h, 0, 4096)
            q.put((rank, "no error"))
    except isim.IsimError as e:
        q.put((rank, e.code))
    m.close()
    dist.destroy_process_group()


def test_peer_abort_returns_ecomm(gpu):
    """rank 0 aborts the communicator before the stats
    all-reduce; rank 1, which walked its shard and entered the collective,
    returns ISIM_ECOMM (polled wait) instead of hanging.  Needs two GPUs
    (RCCL refuses two ranks on one device); skipped on the one-GPU box."""
    import torch
    import torch.multiprocessing as mp
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_abort_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert got[0] == "aborted" and got[1] == isim.ECOMM, got
