"""Topology generators for the benchmark configurations (the build's own
restatements of isotope's Python generators; they emit the same YAML schema).

* ``tree_topology``       ≡ isotope/create_tree_topology.py:37-80 (complete
  tree, BFS naming ``svc-0-1-2``, defaults requestSize/responseSize 128,
  numReplicas 1), plus a ``sequential`` switch: the reference's ``_call_all``
  (:79-80) puts all children in ONE concurrent step; ``sequential=True`` emits
  one call step per child (BASELINE config 2).
* ``realistic_topology``  ≡ isotope/create_realistic_topology.py:28-205:
  Barabási–Albert m=1 with ``power`` and ``zero_appeal`` (models star /
  multitier / auxiliary-services / star-auxiliary, :55-76), edges reversed so
  vertex 0 is the root (:34-47), names ``mock-<i>`` (:175), children from the
  adjacency list (:189-192).  igraph is not available, so the preferential
  attachment is restated with numpy's PCG64 (seeded): vertex i attaches to an
  existing vertex j with probability ∝ indeg(j)^power + zero_appeal.  Not
  igraph-identical; deterministic for a seed.  BASELINE config 3 adds a
  per-service sleep U{1..5} ms, errorRate U[0, 1%] and puts each service's
  children in one concurrent step.
* ``mesh_topology``       BASELINE config 4: layered DAG, each service calls
  ``fanout`` distinct services of the next layer with ``probability``,
  numReplicas U{1..8}, responseSize log-uniform in [128 B, 1 MiB].
"""
from __future__ import annotations

import collections
from typing import Any, Dict, List, Optional

import numpy as np

MODELS = {  # create_realistic_topology.py:55-76
    "star": (0.9, 0.01),
    "multitier": (0.9, 3.25),
    "auxiliary-services": (0.05, 3.25),
    "star-auxiliary": (0.05, 0.01),
}


def tree_topology(num_levels: int = 3, num_branches: int = 3, sequential: bool = False,
                  request_size: int = 128, response_size: int = 128,
                  num_replicas: int = 1) -> Dict[str, Any]:
    num_services = sum(num_branches ** i for i in range(num_levels))
    entry = {"name": "svc-0", "isEntrypoint": True}
    paths = collections.deque([(entry, ["0"])])
    services: List[Dict[str, Any]] = []
    for _ in range(num_services):
        cur, path = paths.popleft()
        services.append(cur)
        remaining = num_services - len(services) - len(paths)
        if remaining > 0:
            children = []
            for ci in range(min(num_branches, remaining)):
                cp = path + [str(ci)]
                child = {"name": "svc-{}".format("-".join(cp))}
                children.append(child)
                paths.append((child, cp))
            if sequential:
                cur["script"] = [{"call": c["name"]} for c in children]
            else:
                cur["script"] = [[{"call": c["name"]} for c in children]]
    return {"defaults": {"requestSize": request_size, "responseSize": response_size,
                         "numReplicas": num_replicas},
            "services": services}


def barabasi_tree(n: int, power: float, zero_appeal: float, seed: int) -> np.ndarray:
    """parent[i] for i >= 1 (parent[0] = -1): sequential preferential
    attachment, P(i -> j) ∝ indeg(j)^power + zero_appeal, j < i."""
    rng = np.random.Generator(np.random.PCG64(seed))
    parent = np.full(n, -1, np.int64)
    indeg = np.zeros(n, np.float64)
    w = np.zeros(n, np.float64)
    if n == 0:
        return parent
    w[0] = zero_appeal
    for i in range(1, n):
        c = np.cumsum(w[:i])
        r = rng.random() * c[-1]
        j = int(np.searchsorted(c, r, side="right"))
        j = min(j, i - 1)
        parent[i] = j
        indeg[j] += 1.0
        w[j] = indeg[j] ** power + zero_appeal
        w[i] = zero_appeal
    return parent


def realistic_topology(n: int = 10, model: str = "multitier", seed: int = 42,
                       concurrent: bool = False, sleep_ms=None, error_rate=None,
                       request_size: int = 128, response_size: int = 128,
                       num_replicas: int = 1, probability: Optional[int] = None) -> Dict[str, Any]:
    """sleep_ms=(lo, hi) adds a leading sleep U{lo..hi} ms per service;
    error_rate=(lo, hi) sets errorRate U[lo, hi] per service; probability
    (1..100) is set on every call command (request_command.go:30-32, the
    reference runtime's only randomness: executable.go:84-90)."""
    power, zero_appeal = MODELS[model]
    parent = barabasi_tree(n, power, zero_appeal, seed)
    children: List[List[int]] = [[] for _ in range(n)]
    for i in range(1, n):
        children[parent[i]].append(i)
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    services = []
    for i in range(n):
        svc: Dict[str, Any] = {"name": f"mock-{i}"}
        script: List[Any] = []
        if sleep_ms is not None:
            script.append({"sleep": f"{int(rng.integers(sleep_ms[0], sleep_ms[1] + 1))}ms"})
        calls = [{"call": f"mock-{c}"} if probability is None else
                 {"call": {"service": f"mock-{c}", "probability": probability}} for c in children[i]]
        if calls:
            script.extend([calls] if concurrent else calls)
        svc["script"] = script
        if error_rate is not None:
            svc["errorRate"] = float(error_rate[0] + (error_rate[1] - error_rate[0]) * rng.random())
        if i == 0:
            svc["isEntrypoint"] = True
        services.append(svc)
    return {"defaults": {"requestSize": request_size, "responseSize": response_size,
                         "numReplicas": num_replicas},
            "services": services}


def mesh_topology(n_services: int = 100_000, layers: int = 8, fanout: int = 3,
                  probability: int = 30, seed: int = 7) -> Dict[str, Any]:
    rng = np.random.Generator(np.random.PCG64(seed))
    per = n_services // layers
    services = []
    for layer in range(layers):
        for j in range(per):
            svc: Dict[str, Any] = {"name": f"l{layer}-{j}",
                                   "numReplicas": int(rng.integers(1, 9)),
                                   "responseSize": int(round(2.0 ** rng.uniform(7.0, 20.0)))}
            if layer + 1 < layers:
                targets = rng.choice(per, size=min(fanout, per), replace=False)
                svc["script"] = [{"call": {"service": f"l{layer + 1}-{int(t)}",
                                           "probability": probability}} for t in targets]
            if layer == 0 and j == 0:
                svc["isEntrypoint"] = True
            services.append(svc)
    return {"defaults": {"requestSize": 128, "responseSize": 128, "numReplicas": 1},
            "services": services}


def mesh_des_topology(n_services: int = 100_000, layers: int = 8, fanout: int = 3, probability: int = 30,
                      sleep_us=(50, 250), seed: int = 7) -> Dict[str, Any]:
    """Config 4's mesh with a sleep U{sleep_us} us at the start of every
    script: the worker of each replica is held (DES v1), so services shared
    by many callers queue under load; the three sequential probabilistic
    calls are three call steps (the DES item engine's step begins,
    DESIGN.md §10.9).  Sleeps in microseconds keep the static latency bound
    of the 3,280-position tree below 2^32 ns (the lane tree walk's u32 time)."""
    doc = mesh_topology(n_services, layers, fanout, probability, seed)
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    for s in doc["services"]:
        s["script"] = [{"sleep": f"{int(rng.integers(sleep_us[0], sleep_us[1] + 1))}us"}] + s.get("script", [])
    return doc


def layered_dag_topology(layers: int = 9, width: int = 8, probability: int = 10, error_rate: float = 0.05,
                         sleep: str = "1ms") -> Dict[str, Any]:
    """A DAG of shared callees: every service of a layer calls every service
    of the next in one concurrent step, each call at `probability`, after a
    sleep.  width^layers potential invocations per trace (8^9 = 134M: past the
    2^24 positions the unrolled tree of the lane tree walk holds, so kind 7
    runs over the site graph, Program::tree_dag), ~width * probability / 100
    expected callees per invocation.  Not a reference generator: a shape
    isotope's validation accepts (validation.go:28-57) that neither
    create_tree_topology.py nor create_realistic_topology.py emits."""
    services = []
    for layer in range(layers):
        for w in range(width):
            svc: Dict[str, Any] = {"name": f"l{layer}_{w}", "errorRate": error_rate, "script": [{"sleep": sleep}]}
            if layer + 1 < layers:
                svc["script"].append([{"call": {"service": f"l{layer + 1}_{v}", "probability": probability}}
                                      for v in range(width)])
            services.append(svc)
    services[0]["isEntrypoint"] = True
    return {"services": services}


def config3_topology(n: int = 10_000, seed: int = 42) -> Dict[str, Any]:
    """BASELINE config 3: realistic multitier 10k, concurrent fan-out,
    sleep U{1..5} ms, errorRate U[0, 1%]."""
    return realistic_topology(n, "multitier", seed, concurrent=True, sleep_ms=(1, 5),
                              error_rate=(0.0, 0.01))


def config3p_topology(probability: int = 50, n: int = 10_000, seed: int = 42) -> Dict[str, Any]:
    """Config 3's graph (same tree, sleeps and error rates) with `probability`
    on every call: a dynamic walk over a 10k-position tree (VERDICT r3 item 3,
    bench.py --config c3p)."""
    return realistic_topology(n, "multitier", seed, concurrent=True, sleep_ms=(1, 5),
                              error_rate=(0.0, 0.01), probability=probability)


def config3s_topology(probability: int = 50, n: int = 10_000, seed: int = 42) -> Dict[str, Any]:
    """Config 3's graph in the reference generator's SEQUENTIAL shape (each
    child called in its own step, create_realistic_topology.py:176-182) with
    config 3's sleeps and error rates and `probability` on every call: the
    latency bound is ~30 s, past the u32 nanosecond clock, so the lane tree
    walk keeps u64 time (bench.py --config c3s)."""
    return realistic_topology(n, "multitier", seed, concurrent=False, sleep_ms=(1, 5),
                              error_rate=(0.0, 0.01), probability=probability)


def config2_topology() -> Dict[str, Any]:
    """BASELINE config 2: tree depth 4 x fan-out 8, sequential requests."""
    return tree_topology(4, 8, sequential=True)
