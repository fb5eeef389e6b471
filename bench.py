#!/usr/bin/env python3
"""Benchmark: simulated isotope request traces per second (node), 10k-service
realistic topology (BASELINE.json config 3), MI355X.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

One step = one launch of the walk kernel (isim_serve_device) over a batch of
`--batch` traces per rank, trace ids sharded globally (rank r, step s owns
[(s*N + r)*B, (s*N + r + 1)*B)), per-trace 16-byte records written to HBM,
per-site counters and latency histograms accumulated on device.  Weak
scaling: per-GPU work is fixed.  After the K timed steps the per-rank stats
buffers are merged with one RCCL all-reduce (SUM) plus a 2-word MAX for the
latency extrema, inside the timed region.

Prints ONE JSON line on rank 0 (contract in the task statement), with
`roofline` (dominant kernel = isim_walk, algorithmic bytes per launch =
16 B/trace records + program + stats, live HIP-event timing on the launch
stream) and `cpu_baseline` (the C oracle, OpenMP, bounded sample, rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "istio-isotope_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md)
N_CU = 256
CLOCK_HZ = 2.4e9
DEFAULT_BATCH = 1 << 24
# traces per rank per step of each config when --batch is left at its default
# (the parity suite checks these exact batches: tests/test_fullsize_gpu.py)
BENCH_BATCH = {
    "c1": 1_000_000,  # BASELINE config 1: 1M traces
    "c2": DEFAULT_BATCH,
    "c3": DEFAULT_BATCH,
    # the lane tree walk's per-launch cost (the tree copied to every
    # workgroup's LDS, the flush, the tail) amortises further: 2^24 / 2^25
    # / 2^26 traces per launch 5.82 / 6.06 / 6.23 G traces/s (1 GB of records)
    "c4": 1 << 26,
    # config 3's graph with a probability on every call: the lane tree walk
    # over a 10,000-position tree
    "c3p": 1 << 22,
    # the same graph in the generator's sequential shape (a ~30 s latency
    # bound: the lane tree walk with u64 time)
    "c3s": 1 << 22,
    # a 100k-service realistic graph at probability 30: a WIDE tree (100,000
    # positions and call sites, past the 8-byte nodes; round 5)
    "c4w": 1 << 22,
    # a DAG of shared callees past the unrolled tree (8^9 potential
    # invocations): the lane walk over the site graph (round 6)
    "cdag": 1 << 22,
    # the DES workspace is ~162 KB per trace on the 10k graph (rows sized
    # for u64: 170 GB at 2^20 of the 288 GB HBM); longer batches amortise
    # the pipelined queue pass's fill and drain (2^16 20.8,
    # 2^18 22.3, 2^20 23.9 M traces/s)
    "c5": 1 << 20,
    # DES of dynamic walks on the item engine: config 3's
    # graph at probability 50 (215 executed invocations per trace; 2^18 /
    # 2^19 / 2^20 traces per step 7.4 / 8.3 / 8.4 M traces/s, ~190 B per item)
    # and config 4's mesh with sleeps (a cyclic schedule: fixed-point passes;
    # 2^21 / 2^22 / 2^23: 4.3 / 6.2 / 7.4 M traces/s)
    # (2^19: 21 GB of item arrays; a step right after another process freed
    # ~170 GB — config 5's workspace — ran 4x slower at 2^20 while the driver
    # still held that memory)
    "c5p": 1 << 19,
    "c4d": 1 << 23,
}
DES_CONFIGS = ("c5", "c5p", "c4d")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    # 2^24 traces (256 MB of records) per launch: the per-launch flush and
    # tail amortise (config 3: 2^22 335, 2^23 339, 2^24 340 M traces/s)
    ap.add_argument("--batch", type=int, default=DEFAULT_BATCH, help="traces per rank per step")
    ap.add_argument("--config", default="c3",
                    choices=["c1", "c2", "c3", "c3p", "c3s", "c4", "c4w", "cdag", "c5", "c5p", "c4d"])
    ap.add_argument("--prob", type=int, default=0,
                    help="c3p / c3s / c4w / cdag: the probability on every call (1..99; 0: 50, c4w 30, cdag 10)")
    ap.add_argument("--no-wave-leg", action="store_true",
                    help="c3p / c3s: skip the wave-interpreter leg (kinds 2/3, ISIM_FLAG_WAVE_WALK) on the same graph")
    ap.add_argument("--fill", action="store_true", help="draw-free static walks (config 2): walk one trace and "
                    "fill the records (the library default) instead of walking every trace")
    ap.add_argument("--wide-rows", action="store_true", help="c5: 64-bit DES rows (default: 32-bit, "
                    "64-bit only when a batch's latencies reach 2^31 ns)")
    ap.add_argument("--mean-interarrival-ns", type=int, default=0,
                    help="DES (c5, c5p, c4d): mean gap of the open-loop Poisson arrivals (0: 6 ms for c5/c5p, "
                         "150 us for c4d)")
    ap.add_argument("--mode", default="A", choices=["A", "B"])
    ap.add_argument("--no-mode-b", action="store_true", help="c3: skip the extra mode-B legs")
    ap.add_argument("--mode-b-steps", type=int, default=5, help="c3: timed steps of each extra mode-B leg")
    ap.add_argument("--no-records", action="store_true")
    ap.add_argument("--no-svc-dur", action="store_true",
                    help="dynamic walks: skip the per-service duration histograms")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--cpu-traces", type=int, default=0, help="cpu_baseline sample size (0 = auto)")
    args = ap.parse_args()
    args.des_auto_batch = False  # c5 with the default batch: shrink it to the device's free HBM
    if not args.prob:
        args.prob = {"c4w": 30, "cdag": 10}.get(args.config, 50)
    if not args.mean_interarrival_ns:
        args.mean_interarrival_ns = 150_000 if args.config == "c4d" else 6_000_000
    return args


def build_graph(config: str, prob: int = 50):
    from isim.generators import (config2_topology, config3_topology, config3p_topology, config3s_topology,
                                 mesh_des_topology, mesh_topology, realistic_topology)
    from isim.yamljson import obj_to_json, yaml_to_json
    if config == "c1":
        j = yaml_to_json(open(os.path.join(ROOT, "tests", "golden", "topologies", "canonical.yaml"), "rb").read())
        desc = {"workload": "isotope example-topologies/canonical.yaml as written (4 services, entry d, 6 "
                            "invocations per trace), 1,000,000 traces",
                "services": 4}
    elif config == "c2":
        j = obj_to_json(config2_topology())
        desc = {"workload": "create_tree_topology.py tree depth 4 x fan-out 8, sequential requests (585 services)",
                "services": 585}
    elif config == "c4":
        j = obj_to_json(mesh_topology())
        desc = {"workload": "100k-service 8-layer mesh, fan-out 3 at probability 30, numReplicas + responseSize",
                "services": 100000}
    elif config == "c3p":
        j = obj_to_json(config3p_topology(prob))
        desc = {"workload": f"config 3's 10k-service graph with probability {prob} on every call (the reference "
                            "runtime's only randomness, executable.go:84-90): dynamic walk, lane tree walk",
                "services": 10000, "probability": prob}
    elif config == "c3s":
        j = obj_to_json(config3s_topology(prob))
        desc = {"workload": f"config 3's 10k-service graph in create_realistic_topology.py's sequential shape "
                            f"(one call step per child) with probability {prob} on every call: dynamic walk with a "
                            "~30 s latency bound, lane tree walk with u64 time",
                "services": 10000, "probability": prob}
    elif config == "c4w":
        # (the 100k-node generator takes ~40 s: the JSON is cached per probability under the temp dir)
        cache = os.path.join(tempfile.gettempdir(), f"isim_c4w_p{prob}.json")
        if os.path.exists(cache):
            j = open(cache).read()
        else:
            j = obj_to_json(realistic_topology(100000, concurrent=True, sleep_ms=(1, 5), error_rate=(0.0, 0.01),
                                               probability=prob))
            with open(cache + f".{os.getpid()}", "w") as f:
                f.write(j)
            os.replace(cache + f".{os.getpid()}", cache)
        desc = {"workload": f"create_realistic_topology.py multitier Barabasi 100k services (restated generator, "
                            f"seed 42), concurrent fan-out, sleep U{{1..5}}ms, errorRate U[0,1%], probability {prob} "
                            "on every call: a wide tree (100,000 positions and call sites), lane tree walk",
                "services": 100000, "probability": prob}
    elif config == "cdag":
        from isim.generators import layered_dag_topology
        j = obj_to_json(layered_dag_topology(probability=prob))
        desc = {"workload": "a layered DAG of shared callees (9 layers x 8 services, every service calls every "
                            "service of the next layer in one concurrent step at probability 10, sleep 1 ms, "
                            "errorRate 5 %): 8^9 = 134M potential invocations per trace, past the unrolled tree — "
                            "the lane walk over the site graph (one node per call site)",
                "services": 72, "probability": prob}
    elif config == "c5":
        j = obj_to_json(config3_topology())
        desc = {"workload": "config 3's 10k-service graph + per-replica worker-pool contention: open-loop Poisson "
                            "arrivals, one FIFO worker per replica held for the service's sleep (DES v1, DESIGN.md "
                            "§10), level-synchronous exact DES",
                "services": 10000}
    elif config == "c5p":
        j = obj_to_json(config3p_topology(prob))
        desc = {"workload": f"config 5 on a dynamic walk: config 3's 10k-service graph with probability {prob} on "
                            "every call + per-replica worker-pool contention (DES v1), item engine over the "
                            "executed invocations (DESIGN.md §10.9)",
                "services": 10000, "probability": prob}
    elif config == "c4d":
        j = obj_to_json(mesh_des_topology())
        desc = {"workload": "config 4's 100k-service mesh (fan-out 3 at probability 30, numReplicas) with a sleep "
                            "U{50..250} us per script under per-replica worker-pool contention (DES v1): item "
                            "engine, cyclic call-step schedule run to its fixed point (DESIGN.md §10.9)",
                "services": 100000}
    else:
        j = obj_to_json(config3_topology())
        desc = {"workload": "create_realistic_topology.py multitier Barabasi 10k services, concurrent fan-out, "
                            "sleep U{1..5}ms, errorRate U[0,1%] (restated generator, seed 42)",
                "services": 10000}
    return j, desc


def cpu_baseline(json_text: str, params, n_traces: int, trace_begin: int):
    """The C oracle (kind "port": no Go toolchain exists to run the reference)."""
    from oracle import executor as oc
    from oracle import graph_ref as gr
    from oracle.executor_py import SimGraph
    from oracle.executor_py import SimParams as OParams
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    sg = SimGraph(gr.unmarshal_service_graph(json_text))
    op = OParams(params.seed, params.hop_base_ns, params.req_ps_per_byte, params.resp_ps_per_byte,
                 params.error_mode)
    og = oc.OracleGraph(sg, op)
    auto = n_traces <= 0
    if auto:
        n_traces = 32768 * threads
    t0 = time.perf_counter()
    _, st = oc.run(sg, op, sg.entry(), trace_begin, n_traces, records=False, n_threads=threads, og=og)
    dt = time.perf_counter() - t0
    if auto and dt < 2.0:
        # a sample of ~10 s of CPU work (a fast graph finished the first one in under 2 s)
        n_traces = int(n_traces * min(256.0, 10.0 / max(dt, 1e-3)))
        t0 = time.perf_counter()
        _, st = oc.run(sg, op, sg.entry(), trace_begin, n_traces, records=False, n_threads=threads, og=og)
        dt = time.perf_counter() - t0
    return {"value": n_traces / dt, "unit": "traces/s", "cores": threads, "kind": "port",
            "sample": f"{n_traces} traces of the same workload (trace ids from {trace_begin}), "
                      f"C oracle oracle/isim_oracle.c with OpenMP, {dt:.3g} s",
            "hop_visits_per_s": float(st[2]) / dt}


def cpu_baseline_des(json_text: str, params, mean_ns: int, n_traces: int):
    """The DES oracle (oracle/des_oracle.c: sequential event-driven) on every
    host core: one DES of one arrival stream is sequential, so each thread runs
    an independent replica of n traces with its own trace ids (the same split
    as bench's N > 1 DES ranks, main_des); value = all threads' traces / wall
    time.  ctypes drops the GIL for the C call."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import des as od
    from oracle import graph_ref as gr
    from oracle.executor import OracleGraph
    from oracle.executor_py import SimGraph
    from oracle.executor_py import SimParams as OParams
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    sg = SimGraph(gr.unmarshal_service_graph(json_text))
    op = OParams(params.seed, params.hop_base_ns, params.req_ps_per_byte, params.resp_ps_per_byte,
                 params.error_mode)
    og = OracleGraph(sg, op)
    od.ln_table()  # the oracle's lazily built log table, built once before the threads start
    n = n_traces or 2048

    def one(r):
        return od.run(sg, op, sg.entry(), r * n, n, mean_ns, records=False, og=og)[1]

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        sts = list(ex.map(one, range(threads)))
    dt = time.perf_counter() - t0
    hops = sum(float(st[2]) for st in sts)
    return {"value": threads * n / dt, "unit": "traces/s", "cores": threads, "kind": "port",
            "sample": f"{threads} independent replicas (one per thread) x {n} traces of the same DES workload "
                      f"(replica r: trace ids from r*{n}, arrivals from time 0), event-driven C oracle "
                      f"oracle/des_oracle.c (binary heap, sequential per replica), {dt:.1f} s",
            "hop_visits_per_s": hops / dt}


def main_des(args, h, json_text, desc, params, rank, world, dev, multi=None, merge_label=""):
    """BASELINE config 5: one step = one DES batch of --batch traces per rank
    (arrivals from time 0, replicas idle), all kernels on one stream.  The DES
    does not shard a batch: with N ranks each runs an independent replica
    (its own trace ids, i.e. its own arrival stream) and the stats are summed
    with one RCCL all-reduce ("replicas only")."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import isim
    from isim.dist import shard_begin

    d = isim.DesHandler(h, args.mean_interarrival_ns)
    B = args.batch
    wsb = d.workspace_bytes(B)
    if args.des_auto_batch:
        # the default batch on a device with less free HBM than the 288 GB of
        # an MI355X: the largest halving whose workspace takes <= 80 % of it
        free = torch.cuda.mem_get_info(dev)[0]
        while B > 4096 and wsb > 0.8 * free:
            B //= 2
            wsb = d.workspace_bytes(B)
        if world > 1:  # one batch length on every rank (shard_begin)
            t = torch.tensor([B], dtype=torch.int64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            B = int(t.item())
        wsb = d.workspace_bytes(B)
        args.batch = B
    ws = torch.empty(wsb // 8 + 1, dtype=torch.int64, device=dev)
    stats = torch.zeros(h.info.stats_words, dtype=torch.int64, device=dev)
    table = torch.zeros(max(1, d.table_words), dtype=torch.int64, device=dev)
    recs = None if args.no_records else torch.empty((B, 2), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    # 32-bit rows unless a batch's latencies reach 2^31 ns (isim.h ISIM_ST_DES_RETRY): then 64-bit rows
    wide = [bool(args.wide_rows)]

    def step(s):
        begin = shard_begin(rank, world, s, B)
        d.serve_device(begin, B, recs.data_ptr() if recs is not None else 0, stats.data_ptr(), table.data_ptr(),
                       ws.data_ptr(), wsb, sptr, wide=wide[0])

    def retried():
        t = stats[isim.native.ST_DES_RETRY:isim.native.ST_DES_RETRY + 1].clone()
        if world > 1:
            dist.all_reduce(t)
        return int(t.item()) > 0

    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize()
    if retried():
        wide[0] = True
    for attempt in range(2):
        stats.zero_()
        table.zero_()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            ev[i][0].record(stream)
            step(args.warmup + i)
            ev[i][1].record(stream)
        torch.cuda.synchronize()
        if wide[0] or not retried():
            break
        wide[0] = True  # a timed batch overflowed the 32-bit rows: time the run again with 64-bit rows
    if world > 1:
        merge(h, multi, stats, sptr)
        if multi is not None:
            multi.allreduce_des_table(h, [table.data_ptr()], [sptr])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    folded = h.fold(stats.cpu().numpy().view(np.uint64))
    total = args.steps * B * world
    assert folded["n_traces"] == total, (folded["n_traces"], total)
    value = total / elapsed
    npos = d.info.n_positions
    # algorithmic bytes of one step, R = row bytes (4 or 8):
    # the rows the queue and finish passes read and write per trace
    # (isim_des_info row_reads / row_writes: the plan's own count — fused
    # leaves, caller-recorded durations, finishes without the start row), the
    # status bits (written once, read once: n_pos / 4 B), arrivals / per-trace
    # 500 counts / finalize ~44 B, records 16 B
    R = 8 if wide[0] else 4
    rows = d.info.row_reads + d.info.row_writes
    items = d.info.items == 1
    hops = folded["sum_hops"] / total
    batch = d.last_batch() if items else None
    if items:
        # the item engine: per executed invocation the
        # pre-walk writes 13 B, the renumbering moves 2 x 16 B, and every pass
        # over the rounds (a cyclic schedule's quiet passes and the recording
        # one: isim_des_last_batch) moves the queue's ~96 B (keys, the sort,
        # the scan's maps in and out, the start) and the finish's ~48 B
        # (start, arrival, callee maximum, finish); per trace the gaps,
        # arrivals, offsets, hops ~44 B and the record
        alg_bytes = int(B * (hops * (13 + 32 + (96 + 48) * batch["passes"]) + 44 +
                             (0 if args.no_records else 16)))
    else:
        alg_bytes = B * (R * rows + npos // 4 + 44 + (0 if args.no_records else 16))
    workspace_gbs = alg_bytes / (kern_ms * 1e-3) / 1e9
    # SURVEY §8(d)'s algorithmic bytes: what any
    # implementation must move — the 16-B record per trace, the statistics and
    # the DES table written once.  This is the line's roofline; it does not
    # grow with the fixed-point passes a cyclic schedule runs.
    compulsory = B * (0 if args.no_records else 16) + h.info.stats_words * 8 + d.table_words * 8
    achieved_gbs = compulsory / (kern_ms * 1e-3) / 1e9
    traffic = occupancy = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_summary_{args.config}.json")
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            if pmc.get("batch") == B:
                traffic = pmc.get("hbm_bytes_per_step")
                occupancy = pmc.get("occupancy")
        except Exception:
            traffic = None
    rows = d.fold(table.cpu().numpy().view(np.uint64))
    W = isim.native
    mean_wait = float(rows[:, W.DES_SUM_WAIT].sum()) / max(1, int(rows[:, W.DES_COUNT].sum()))
    line = {
        "metric": f"simulated request traces/sec (node), config {args.config} (DES)",
        "value": value, "unit": "traces/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "config": dict(desc, global_batch=B * world, traces_per_rank_per_step=B, error_mode=args.mode,
                       hop_visits_per_trace=folded["sum_hops"] / total,
                       mean_interarrival_ns=args.mean_interarrival_ns,
                       parallelism=f"replicas x{world}", merge=merge_label, records=not args.no_records,
                       des_levels=d.info.n_levels, des_max_width=d.info.max_width,
                       des_fused_leaves=d.info.n_fused,
                       des_engine="items (dynamic walk)" if items else "level-synchronous rows",
                       des_rows="u64" if wide[0] or items else "u32", des_cyclic=bool(d.info.cyclic),
                       workspace_bytes=wsb, rccl_ranks=multi.n_ranks if multi is not None else None,
                       traces_per_rank=args.steps * B,
                       des_passes_per_step=batch["passes"] if batch else 1,
                       des_syncs_per_step=batch["syncs"] if batch else None),
        "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": ("des_items k_* + rocPRIM sorts/scans per step" if items else
                                "des_* (arrivals, down and up passes of all levels, finalize) per step"),
                     "kernel_ms": kern_ms, "bytes_per_launch": compulsory,
                     "basis": "SURVEY §8(d): 16-B record per trace + stats buffer + DES table, written once"},
        # the builder's workspace model beside it (what the algorithm streams:
        # for the item engine it grows with the passes over the rounds), next
        # to the PMC traffic it is compared with
        "roofline_workspace": {"bytes_per_launch": alg_bytes, "achieved": workspace_gbs, "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": workspace_gbs / HBM_PEAK_GBS, "traffic": traffic,
                               "basis": ("per executed invocation 45 B once and ~144 B of item arrays and sort "
                                         "traffic per pass over the rounds (DESIGN.md §10.9)" if items else
                                         "the level-synchronous rows the algorithm streams (DESIGN.md §10.4)")},
        "occupancy": {"peak_waves_per_cu": 32, "measured": occupancy},
        "mean_latency_ns": folded["sum_latency"] / total,
        "mean_queue_wait_ns": mean_wait,
        "hop_visits_per_s": value * folded["sum_hops"] / total,
        "n_500_frac": folded["n_500"] / total,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline_des(json_text, params, args.mean_interarrival_ns, args.cpu_traces)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        teardown(multi)


def compute_roofline(stream: bool, info, B: int, kern_ms: float):
    """The draw-stream kernel is bound by integer VALU, not HBM: one
    Philox4x32-10 block per lane per group of 4 invocations.  Peak = the
    measured Philox block rate of tools/philox_peak.hip on MI355X
    (profiles/philox_peak.json)."""
    path = os.path.join(ROOT, "profiles", "philox_peak.json")
    if not stream or not os.path.exists(path):
        return None
    peak = json.load(open(path))["philox_blocks_per_s"]
    # only the groups of 4 invocations that hold an error draw cost a block
    # (the kernel skips all-zero-threshold groups)
    blocks = B * info.draw_groups
    if blocks == 0:
        return None
    achieved = blocks / (kern_ms * 1e-3)
    return {"bound": "valu", "achieved": achieved, "peak": peak, "unit": "Philox4x32-10 blocks/s",
            "frac": achieved / peak, "per_launch": blocks,
            "peak_source": "profiles/philox_peak.json (tools/philox_peak.hip)"}


def make_multi(rank, world, local):
    """libisim's RCCL communicator for the stats merge (isim_multi_init_rank;
    the 128-byte id travels over torch.distributed, as a Go host would send it
    out of band).  Returns (Multi or None, merge label).

    The choice is collective: every rank first loads RCCL and draws an id
    locally (isim_multi_get_id), the ranks agree on success (all_reduce MIN)
    before anyone enters the collective ncclCommInitRank, and agree again
    after it; on any failure every rank frees what it holds and all merge
    with torch.distributed together (no rank is left waiting in a collective
    the others skipped)."""
    import torch
    import torch.distributed as dist

    from isim.dist import Multi
    if world == 1:
        return None, "none (1 rank)"
    # the agreement all-reduces run on the process group's own device kind
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")

    def agree(ok: bool) -> bool:
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    err = ""
    mid = None
    try:
        # every local step that can fail runs here, before the collective
        # creation: RCCL loads, the device can be selected, an id can be drawn
        Multi.precheck(local)
        mid = Multi.get_id()  # rank 0's id is the one used
    except Exception as e:
        err = f"isim_multi_precheck / isim_multi_get_id failed on rank {rank}: {e}"
    if not agree(mid is not None):
        print(err or "isim_multi_precheck / isim_multi_get_id failed on another rank", file=sys.stderr)
        return None, "torch.distributed all_reduce (isim_multi_get_id failed)"
    obj = [mid if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    multi = None
    try:
        # collective; if a peer never enters it (a failure the pre-check could
        # not see), libisim's non-blocking creation gives up after
        # ISIM_MULTI_TIMEOUT_S with ECOMM, and the agreement below still runs
        multi = Multi.init_rank(obj[0], world, rank, local)
    except Exception as e:
        err = f"isim_multi_init_rank failed on rank {rank}: {e}"
    if not agree(multi is not None):
        if multi is not None:
            multi.close()
        print(err or "isim_multi_init_rank failed on another rank", file=sys.stderr)
        return None, "torch.distributed all_reduce (isim_multi_init_rank failed)"
    return multi, "isim_stats_allreduce_device (libisim RCCL)"


def teardown(multi):
    """Every rank frees libisim's communicator at the same point (after a
    barrier, while the process group still lives), then the process group:
    the communicator is never finalised at interpreter exit, in whatever order
    the ranks reach it."""
    import torch
    import torch.distributed as dist
    torch.cuda.synchronize()
    dist.barrier()
    if multi is not None:
        multi.close()
    dist.barrier()
    dist.destroy_process_group()


def merge(h, multi, stats, sptr):
    """SUM + extrema MAX of the per-rank stats buffers, on the launch stream."""
    from isim.dist import merge_stats
    if multi is not None:
        multi.allreduce_stats(h, [stats.data_ptr()], [sptr])
    else:
        merge_stats(stats)


def pmc_summary(name: str, batch: int, kernel: str):
    """profiles/pmc_summary_<name>.json if it profiled this very workload:
    the same configuration name, batch and kernel (name and template)."""
    path = os.path.join(ROOT, "profiles", f"pmc_summary_{name}.json")
    try:
        pmc = json.load(open(path))
    except Exception:
        return None
    if pmc.get("config") == name and pmc.get("batch") == batch and kernel in str(pmc.get("kernel", "")):
        return pmc
    return None


def kernel_name(launch) -> str:
    """The dominant kernel of a walk launch: the lane tree walk (kind 7) or
    the walk kernels (kinds 0-6)."""
    if launch["kernel_kind"] == 7:
        return "isim_tree"
    return f"isim_walk<{launch['kernel_kind']}"


def time_walk(h, steps, warmup, B, recs, stats, rank, world, dev, multi=None):
    """W untimed + K timed launches of isim_serve_device over B traces per
    rank (trace ids sharded globally), then the stats all-reduce; returns
    (max-over-ranks wall seconds of the K steps + merge, mean HIP-event
    kernel ms on the launch stream)."""
    import torch
    import torch.distributed as dist

    from isim.dist import shard_begin
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    def step(s):
        begin = shard_begin(rank, world, s, B)
        h.serve_device(begin, B, recs.data_ptr() if recs is not None else 0, stats.data_ptr(), sptr)

    for s in range(warmup):
        step(s)
    torch.cuda.synchronize()
    stats.zero_()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        ev[i][0].record(stream)
        step(warmup + i)
        ev[i][1].record(stream)
    if world > 1:
        merge(h, multi, stats, sptr)  # one RCCL all-reduce (SUM) + the 2-word extrema MAX
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / steps
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    return elapsed, kern_ms


def mode_b_legs(args, json_text, rank, world, dev, multi=None):
    """Config 3 in error mode B (the propagating EXT variant of
    executable.go:131-143): the same graph (every trace ends 500 at errorRate
    U[0, 1 %]) and an informative variant (errorRate U[0, 1e-4], entry 500 in
    ~40 % of the traces), both on the close-list kernel."""
    import numpy as np
    import torch

    import isim
    from isim.generators import realistic_topology
    from isim.yamljson import obj_to_json
    out = {}
    graphs = {"mode_b": json_text,
              "mode_b_informative": obj_to_json(realistic_topology(10_000, "multitier", 42, concurrent=True,
                                                                   sleep_ms=(1, 5), error_rate=(0.0, 1e-4)))}
    B = args.batch
    recs = None if args.no_records else torch.empty((B, 2), dtype=torch.int64, device=dev)
    for key, j in graphs.items():
        h = isim.Handler(isim.ServiceGraph.from_json(j), None,
                         isim.SimParams(error_mode=isim.MODE_B, flags=isim.native.FLAG_WALK_ALL))
        stats = torch.zeros(h.info.stats_words, dtype=torch.int64, device=dev)
        steps = max(1, args.mode_b_steps)
        elapsed, kern_ms = time_walk(h, steps, 1, B, recs, stats, rank, world, dev, multi)
        f = h.fold(stats.cpu().numpy().view(np.uint64))
        total = steps * B * world
        assert f["n_traces"] == total
        launch = h.launch_info(torch.cuda.current_device())
        out[key] = {"value": total / elapsed, "unit": "traces/s", "ms_per_step": elapsed * 1e3 / steps,
                    "kernel_ms": kern_ms, "steps": steps, "n_500_frac": f["n_500"] / total,
                    "kernel_kind": launch["kernel_kind"],
                    "errorRate": "U[0,1%]" if key == "mode_b" else "U[0,1e-4]"}
        if key == "mode_b":  # the mode-B profile (tools/profile_cfg.sh c3B "--config c3 --mode B --no-mode-b")
            pmc = pmc_summary("c3B", B, kernel_name(launch))
            out[key]["traffic"] = pmc.get("hbm_bytes_per_launch") if pmc else None
            out[key]["occupancy_measured"] = pmc.get("occupancy") if pmc else None
    return out


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import isim

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # ISIM_BENCH_BACKEND=gloo: a rehearsal of the N-rank flow on fewer GPUs
    # than ranks (ranks share devices; no RCCL, stats merged by gloo)
    backend = os.environ.get("ISIM_BENCH_BACKEND", "nccl")
    if world > 1:
        local = local % torch.cuda.device_count() if backend != "nccl" else local
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    if backend == "nccl":
        multi, merge_label = make_multi(rank, world, local)
    else:
        multi, merge_label = None, f"torch.distributed all_reduce ({backend} rehearsal)"
    json_text, desc = build_graph(args.config, args.prob)
    # every trace is walked unless --fill: a draw-free static walk (config 2)
    # is otherwise walked once and filled, which is not a walk rate
    params = isim.SimParams(error_mode=isim.MODE_B if args.mode == "B" else isim.MODE_A,
                            flags=(isim.native.FLAG_NO_SVC_DUR if args.no_svc_dur else 0) |
                            (0 if args.fill else isim.native.FLAG_WALK_ALL))
    h = isim.Handler(isim.ServiceGraph.from_json(json_text), None, params)
    if args.batch == DEFAULT_BATCH:
        args.batch = BENCH_BATCH[args.config]
        args.des_auto_batch = args.config == "c5"
    if args.config in DES_CONFIGS:
        return main_des(args, h, json_text, desc, params, rank, world, dev, multi, merge_label)
    info = h.info
    launch = h.launch_info(torch.cuda.current_device())
    B = args.batch
    stats = torch.zeros(info.stats_words, dtype=torch.int64, device=dev)
    recs = None if args.no_records else torch.empty((B, 2), dtype=torch.int64, device=dev)
    elapsed, kern_ms = time_walk(h, args.steps, args.warmup, B, recs, stats, rank, world, dev, multi)

    host_stats = stats.cpu().numpy().view(np.uint64)
    folded = h.fold(host_stats)
    total = args.steps * B * world
    assert folded["n_traces"] == total, (folded["n_traces"], total)
    value = total / elapsed
    hops_per_trace = folded["sum_hops"] / total

    # algorithmic bytes of one launch: 16 B records per trace + program read + stats written
    # (the draw stream is 8 B per invocation, padded to groups of 4; the interpreter 32 B per instruction)
    stream = launch["kernel_kind"] >= 4
    prog_bytes = (-(-info.hops_upper // 4) * 4 * 8 + info.n_slots * 4) if stream else info.program_len * 32
    alg_bytes = B * (0 if args.no_records else 16) + prog_bytes + info.stats_words * 8
    achieved_gbs = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = None
    occupancy = {"launched_waves_per_cu": launch["blocks_per_cu"] * launch["wg_threads"] // 64,
                 "peak_waves_per_cu": 32, "measured": None}
    # the PMC summary of this line's own configuration (profiles/pmc_summary_<name>.json,
    # tools/profile_cfg.sh + tools/pmc_summary.py; c3 in mode B: "c3B")
    pmc = pmc_summary(f"{args.config}B" if args.mode == "B" else args.config, B, kernel_name(launch))
    if pmc:
        traffic = pmc.get("hbm_bytes_per_launch")
        occupancy["measured"] = pmc.get("occupancy")

    line = {
        # BASELINE.json's metric verbatim (the roofline fraction is the "roofline" object)
        "metric": "simulated request traces/sec (node) + % HBM roofline, 10k-svc topology, 1/2/4/8 GPU"
        if args.config == "c3"
        else f"simulated request traces/sec (node), config {args.config}",
        "value": value,
        "unit": "traces/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic",
        "config": dict(desc, global_batch=B * world, traces_per_rank_per_step=B,
                       error_mode=args.mode, hop_visits_per_trace=hops_per_trace,
                       parallelism=f"trace-shard x{world}", merge=merge_label, records=not args.no_records,
                       static_walk=bool(info.static_walk), program_len=info.program_len,
                       launch=launch, rccl_ranks=multi.n_ranks if multi is not None else None,
                       traces_per_rank=args.steps * B),
        "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "isim_fill_const (draw-free walk: one trace walked, records filled)"
                     if launch["fill"] else kernel_name(launch), "kernel_ms": kern_ms, "bytes_per_launch": alg_bytes},
        "compute_roofline": None if launch["fill"] else compute_roofline(stream, info, B, kern_ms),
        "occupancy": occupancy,
        "hop_visits_per_s": value * hops_per_trace,
        "n_500_frac": folded["n_500"] / total,
    }
    if args.config == "c3" and args.mode == "A" and not args.no_mode_b:
        line.update(mode_b_legs(args, json_text, rank, world, dev, multi))
    if args.config in ("c3p", "c3s", "c4w", "cdag") and not args.no_wave_leg:
        line["wave_walk"] = wave_walk_leg(args, json_text, params, rank, world, dev, multi)
        line["speedup_vs_wave_walk"] = value / line["wave_walk"]["value"]
    if rank == 0 and world == 1 and not args.no_cpu:
        # config 1 is defined on the CPU interpreter: time it on the whole
        # 1M-trace workload; other configs on a bounded sample
        n_cpu = args.cpu_traces or (B if args.config == "c1" else 0)
        line["cpu_baseline"] = cpu_baseline(json_text, params, n_cpu, 0)
    if args.config == "c1":
        line["error_path"] = c1_error_path(args, json_text, params, rank, world, dev, multi)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        teardown(multi)


def wave_walk_leg(args, json_text, params, rank, world, dev, multi=None):
    """The same dynamic walk on the round-1 wave interpreter (kinds 2/3,
    ISIM_FLAG_WAVE_WALK: a wave walks its 64 traces in lock step over the
    union of their call paths), at a smaller batch: the rate the lane tree
    walk replaces."""
    import numpy as np
    import torch

    import isim
    p = isim.SimParams(error_mode=params.error_mode, flags=params.flags | isim.native.FLAG_WAVE_WALK)
    h = isim.Handler(isim.ServiceGraph.from_json(json_text), None, p)
    B = max(1 << 16, args.batch >> 4)
    stats = torch.zeros(h.info.stats_words, dtype=torch.int64, device=dev)
    recs = None if args.no_records else torch.empty((B, 2), dtype=torch.int64, device=dev)
    steps = 3
    elapsed, kern_ms = time_walk(h, steps, 1, B, recs, stats, rank, world, dev, multi)
    f = h.fold(stats.cpu().numpy().view(np.uint64))
    total = steps * B * world
    assert f["n_traces"] == total
    return {"value": total / elapsed, "unit": "traces/s", "batch": B, "steps": steps, "kernel_ms": kern_ms,
            "kernel_kind": h.launch_info(torch.cuda.current_device())["kernel_kind"],
            "hop_visits_per_trace": f["sum_hops"] / total}


def c1_error_path(args, json_text, params, rank, world, dev, multi=None):
    """SURVEY §8(d) config 1's error-path variant: canonical.yaml with
    errorRate 1 % on every service (the defaults block), same SimParams and
    trace range, on the GPU and — rank 0, one GPU — the whole workload on the
    CPU oracle."""
    import numpy as np
    import torch

    import isim
    doc = json.loads(json_text)
    doc.setdefault("defaults", {})
    doc["defaults"] = dict(doc["defaults"] or {}, errorRate="1%")
    j = json.dumps(doc)
    h = isim.Handler(isim.ServiceGraph.from_json(j), None, params)
    B = args.batch
    stats = torch.zeros(h.info.stats_words, dtype=torch.int64, device=dev)
    recs = None if args.no_records else torch.empty((B, 2), dtype=torch.int64, device=dev)
    elapsed, kern_ms = time_walk(h, args.steps, args.warmup, B, recs, stats, rank, world, dev, multi)
    f = h.fold(stats.cpu().numpy().view(np.uint64))
    total = args.steps * B * world
    assert f["n_traces"] == total
    out = {"errorRate": "1% (defaults)", "value": total / elapsed, "unit": "traces/s",
           "ms_per_step": elapsed * 1e3 / args.steps, "kernel_ms": kern_ms, "n_500_frac": f["n_500"] / total,
           "err_hops_per_trace": f["sum_err_hops"] / total,
           "kernel_kind": h.launch_info(torch.cuda.current_device())["kernel_kind"]}
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(j, params, args.cpu_traces or B, 0)
    return out


if __name__ == "__main__":
    main()
