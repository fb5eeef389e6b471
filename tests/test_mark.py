"""CPU check of mode B by sparse ancestor marking (kernel kind 8,
kernel_abi.h kMarkPadKey, walk.hip walk_stream_mark), the algorithm alone:
on random preorder trees and random error sets, the per-invocation 500
counts and per-trace 500 hops the kernel's scheme derives — a running minimum
of key = depth << 24 | parent since the trace's last error, +1 at every
erring record, -1 at the LCA that minimum names, depth(e) - depth(LCA) new
500s, subtree sums of the marks — equal the direct definition (mode B: an
invocation responds 500 iff an invocation of its subtree drew an error,
handler.go:66-75 with the 500 propagated, executable.go:131-143).  The GPU
kernel itself is checked against the oracle in tests/test_walk_gpu.py and
tests/test_fullsize_gpu.py."""
import numpy as np
import pytest


def random_tree(rng, n, max_children):
    """Preorder tree of n records: parent, depth and subtree end per record."""
    parent = [-1]
    depth = [0]
    stack = [0]
    kids = [0]
    while len(parent) < n:
        # close frames at random (never the root while records remain)
        while len(stack) > 1 and (kids[stack[-1]] >= max_children or rng.random() < 0.3):
            stack.pop()
        p = stack[-1]
        kids[p] += 1
        r = len(parent)
        parent.append(p)
        depth.append(depth[p] + 1)
        kids.append(0)
        stack.append(r)
    end = list(range(n))
    for r in range(n - 1, 0, -1):
        end[parent[r]] = max(end[parent[r]], end[r])
    return np.array(parent), np.array(depth), np.array(end)


def direct(parent, errs):
    marked = set()
    for e in errs:
        v = e
        while v >= 0 and v not in marked:
            marked.add(v)
            v = parent[v]
    return marked


def marking(parent, depth, errs, n, marks):
    """The kernel's per-trace work: returns the trace's 500 count."""
    sentinel = n
    key = [(int(depth[r]) << 24) | (sentinel if r == 0 else int(parent[r])) for r in range(n)]
    err = set(errs)
    mk = 0xFFFFFFFF
    errh = 0
    for r in range(n):
        mk = min(mk, key[r])
        if r in err:
            marks[r] += 1
            marks[mk & 0xFFFFFF] -= 1
            errh += (key[r] >> 24) + 1 - (mk >> 24)
            mk = 0xFFFFFFFF
    return errh


@pytest.mark.parametrize("seed", range(12))
def test_marking_equals_root_path_union(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 400))
    parent, depth, end = random_tree(rng, n, int(rng.integers(1, 6)))
    marks = np.zeros(n + 1, np.int64)
    expect = np.zeros(n, np.int64)
    for _ in range(200):  # traces
        k = int(rng.integers(0, min(n, 12) + 1))
        errs = sorted(rng.choice(n, size=k, replace=False).tolist()) if k else []
        m = direct(parent, errs)
        for v in m:
            expect[v] += 1
        assert marking(parent, depth, errs, n, marks) == len(m)
    # subtree sums of the marks over prefix sums (isim_mark_fold), mod 2^32
    P = np.cumsum(marks[:n]) & 0xFFFFFFFF
    for v in range(n):
        s = (int(P[end[v]]) - (int(P[v - 1]) if v else 0)) & 0xFFFFFFFF
        assert s == expect[v], (v, s, expect[v])
