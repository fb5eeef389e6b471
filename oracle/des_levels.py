"""Level-synchronous restatement of the DES timing (oracle — test
infrastructure only), in numpy.

A third, independent statement of isim DES semantics v1 used
to check that the level decomposition the GPU uses is exact: it unrolls the
invocation tree from the oracle's SimGraph (not from the product's plan),
computes the FIFO start times of each position over all traces with the
closed form of the single-server recurrence

    fin_t = max(fin_{t-1}, a_t) + P   =>   S_t = t*P + max_{s<=t}(a_s - s*P)

(per replica subsequence), then finish times bottom-up.  Latencies and queue
waits only (statuses come from the static walk, checked elsewhere).
"""
from __future__ import annotations

import numpy as np

from .des import exp_q24_py
from .executor_py import SimGraph, SimParams

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
M32 = np.uint64(0xFFFFFFFF)


def philox_np(c0, c1, c2, c3, seed: int):
    """Vectorized Philox4x32-10 over uint64 arrays holding 32-bit words."""
    c0, c1, c2, c3 = (np.asarray(x, np.uint64) & M32 for x in (c0, c1, c2, c3))
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> np.uint64(32)) ^ c1 ^ np.uint64(k0)) & M32, p1 & M32, \
                         ((p0 >> np.uint64(32)) ^ c3 ^ np.uint64(k1)) & M32, p0 & M32
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return c0, c1, c2, c3


def _sl(d):
    return d if d > 0 else 0


def unroll(sg: SimGraph, p: SimParams, entry: int):
    """Positions in hop order: dicts with svc, parent, off, hold, floor, post, leaf."""
    pos = []

    def shape(s):
        pre = cmax = post = hold = total = 0
        seen_call = False
        for st in sg.steps[s]:
            if st[0] == "sleep":
                d, calls, smax = _sl(st[1]), False, 0
                hold += d
            elif st[0] == "call":
                d, calls, smax = 0, True, 0
            else:
                smax = max([_sl(x[1]) for x in st[1] if x[0] == "sleep"] or [0])
                hold += sum(_sl(x[1]) for x in st[1] if x[0] == "sleep")
                calls = any(x[0] == "call" for x in st[1])
                d = smax
            if calls:
                seen_call = True
                cmax = smax
            elif not seen_call:
                pre += d
            else:
                post += d
            total += d
        return pre, cmax, post, hold, total, not seen_call

    def visit(s, parent, off):
        pre, cmax, post, hold, total, leaf = shape(s)
        i = len(pos)
        pos.append({"svc": s, "parent": parent, "off": off, "hold": hold, "post": post, "leaf": leaf,
                    "floor": total if leaf else pre + cmax, "children": [],
                    "reps": max(1, sg.g.services[s].num_replicas)})
        if parent >= 0:
            pos[parent]["children"].append(i)
        for st in sg.steps[s]:
            calls = [st] if st[0] == "call" else ([x for x in st[1] if x[0] == "call"] if st[0] == "conc" else [])
            for c in calls:
                visit(sg.sites[c[1]][1], i, pre + sg.hop_cost(c[1], p))
        return i

    visit(entry, -1, 0)
    depth = [0] * len(pos)
    for i, q in enumerate(pos):
        if q["parent"] >= 0:
            depth[i] = depth[q["parent"]] + 1
    return pos, depth


def fifo_starts(a: np.ndarray, hold: int) -> np.ndarray:
    """S_t = t*P + cummax(a_s - s*P) over an arrival sequence in service order."""
    a = a.astype(object) if a.dtype == object else a.astype(np.int64)
    idx = np.arange(len(a), dtype=np.int64) * hold
    return idx + np.maximum.accumulate(a - idx)


def run(sg: SimGraph, p: SimParams, entry: int, trace_begin: int, n: int, mean_ns: int):
    """Returns (latency[n], wait_sum[n_positions], wait_max[n_positions], positions)."""
    pos, depth = unroll(sg, p, entry)
    t = np.arange(trace_begin, trace_begin + n, dtype=np.uint64)
    lo, hi = t & M32, t >> np.uint64(32)
    u = philox_np(lo, hi, np.zeros(n, np.uint64), np.full(n, 0x80000001, np.uint64), p.seed)[0]
    x = np.array([(mean_ns * exp_q24_py(int(v))) >> 24 for v in u], np.int64)
    A = np.cumsum(x)
    S = np.zeros((len(pos), n), np.int64)
    wsum = np.zeros(len(pos), np.int64)
    wmax = np.zeros(len(pos), np.int64)
    for lvl in range(max(depth) + 1):
        for i in [k for k in range(len(pos)) if depth[k] == lvl]:
            q = pos[i]
            a = A if q["parent"] < 0 else S[q["parent"]] + q["off"]
            if q["reps"] > 1:
                r = philox_np(lo, hi, np.full(n, i, np.uint64), np.full(n, 0x80000002, np.uint64),
                              p.seed)[0] % np.uint64(q["reps"])
            else:
                r = np.zeros(n, np.uint64)
            for rep in range(q["reps"]):
                m = r == np.uint64(rep)
                if m.any():
                    sub = a[m]
                    assert np.all(np.diff(sub) >= 0), "arrivals out of trace order (outside DES v1)"
                    S[i, m] = fifo_starts(sub, q["hold"])
            w = S[i] - a
            wsum[i], wmax[i] = int(w.sum()), int(w.max()) if n else 0
    F = np.zeros_like(S)
    for i in reversed(range(len(pos))):  # children (later in hop order) before parents
        q = pos[i]
        if q["leaf"]:
            F[i] = S[i] + q["floor"]
        else:
            m = S[i] + q["floor"]
            for c in q["children"]:
                m = np.maximum(m, F[c])
            F[i] = m + q["post"]
    return F[0] - A, wsum, wmax, pos
