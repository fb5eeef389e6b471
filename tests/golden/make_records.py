"""Per-trace record fixtures: the first traces of small
reference graphs under fixed SimParams, produced ONCE by the C oracle
(oracle/isim_oracle.c, oracle/des_oracle.c) after it passed the pins it has —
the reference's Go vectors (tests/golden/go_vectors.json), the Random123
Philox KATs and the hand-derived Appendix-B executor KATs.  They freeze isim
semantics v1: tests/test_golden_records.py checks that the oracle still
produces them, tests/test_golden_records_gpu.py that every HIP kernel kind
does.

Output: records/manifest.json (graph JSON, entry, params, trace range per
case) + records/<case>.npz (records [n, 2] u64: latency, hops | status/err <<
32; the oracle's raw stats buffer; DES cases also the per-service DES rows).

    python tests/golden/make_records.py      # needs the built oracle (oracle/Makefile)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "istio-isotope_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

OUT = os.path.join(HERE, "records")


def _topology(name):
    from isim.yamljson import yaml_to_json
    return yaml_to_json(open(os.path.join(HERE, "topologies", name), "rb").read())


def _with_defaults(j, **kw):
    doc = json.loads(j)
    d = doc.get("defaults") or {}
    d.update(kw)
    doc["defaults"] = d
    return json.dumps(doc)


def _small_mesh(layers=4, width=6, seed=7, prob=True):
    """A layered DAG in the shape of config 4 (probability-30..70 calls,
    numReplicas, responseSize, errorRate, sleeps) small enough for fixtures;
    prob=False: every call made (the DES takes static walks only)."""
    rng = np.random.default_rng(seed)
    svcs = []
    for l in range(layers):
        for i in range(width):
            s = {"name": f"m{l}-{i}", "numReplicas": int(rng.integers(1, 4)),
                 "responseSize": f"{int(rng.integers(64, 4096))}B", "errorRate": f"{int(rng.integers(0, 5))}%"}
            script = [{"sleep": f"{int(rng.integers(100, 3000))}us"}]
            if l + 1 < layers:
                tgt = rng.choice(width, size=3, replace=False)
                calls = [{"call": {"service": f"m{l + 1}-{int(t)}", "size": f"{int(rng.integers(0, 2048))}B",
                                   "probability": int(rng.integers(30, 71)) if prob else 0}} for t in tgt]
                script += [calls[:2], calls[2]]  # a concurrent step, then a sequential call
            s["script"] = script
            svcs.append(s)
    svcs[0]["isEntrypoint"] = True
    return json.dumps({"services": svcs})


def cases():
    import kat
    canon = _topology("canonical.yaml")
    gv = kat.graph_json("graphviz_test")
    tree = _topology("gen-tree-3x3-concurrent.yaml")
    mesh = _small_mesh()
    c1 = dict(seed=0x15070BE, hop_base_ns=250_000, req_ps_per_byte=80, resp_ps_per_byte=80)
    out = []

    def add(name, graph, entry, mode, begin=0, n=1024, des_mean=0, **p):
        prm = dict(c1, **p)
        prm["error_mode"] = mode
        out.append({"name": name, "graph": graph, "entry": entry, "params": prm, "begin": begin, "n": n,
                    "des_mean_ns": des_mean})

    # SURVEY §8(d) config 1 params; canonical as written, and with errorRate 1 %
    add("c1_canonical_A", canon, None, 0)
    add("c1_canonical_err1_A", _with_defaults(canon, errorRate="1%"), None, 0)
    add("c1_canonical_err1_B", _with_defaults(canon, errorRate="1%"), None, 1)
    # the graphviz_test graph (sleeps, concurrency, sizes), errorRate 10 %, ids straddling 2^32
    gv10 = _with_defaults(gv, errorRate="10%")
    add("graphviz_err10_A", gv10, "d", 0, begin=(1 << 32) - 512)
    add("graphviz_err10_B", gv10, "d", 1, begin=(1 << 32) - 512)
    # the reference generator's 3x3 tree, errorRate 5 %
    t5 = _with_defaults(tree, errorRate="5%")
    add("tree3x3_err5_A", t5, None, 0)
    add("tree3x3_err5_B", t5, None, 1)
    # probabilistic calls (dynamic walk), replicas, payload sizes
    add("mesh_A", mesh, None, 0, n=2048)
    add("mesh_B", mesh, None, 1, n=2048)
    # the per-replica DES (config 5 semantics) on the graphviz_test graph and the mesh
    # (light load; and an overloaded mesh whose late traces wait seconds: u64 rows)
    # (static walks only: no probabilistic calls, no mode-B aborts; light load,
    # and an overloaded mesh whose late traces wait seconds: the u64-row retry)
    mesh_s = _small_mesh(prob=False)
    add("des_graphviz_err10_A", gv10, "d", 0, n=512, des_mean=300_000_000)
    add("des_mesh_A", mesh_s, None, 0, n=1024, des_mean=60_000_000)
    add("des_mesh_A_overload", mesh_s, None, 0, n=1024, des_mean=2_000_000)
    tree_s = json.loads(t5)
    for sv in tree_s["services"]:
        sv["script"] = [{"sleep": "1ms"}] + (sv.get("script") or [])
    add("des_tree3x3_err5_B", json.dumps(tree_s), None, 1, n=1024, des_mean=3_000_000)
    return out


def main():
    from oracle import des as od
    from oracle import executor as oc
    from oracle import graph_ref as gr
    from oracle.executor_py import SimGraph, SimParams
    os.makedirs(OUT, exist_ok=True)
    manifest = []
    for c in cases():
        sg = SimGraph(gr.unmarshal_service_graph(c["graph"]))
        p = c["params"]
        op = SimParams(p["seed"], p["hop_base_ns"], p["req_ps_per_byte"], p["resp_ps_per_byte"], p["error_mode"])
        entry = sg.entry(c["entry"])
        if c["des_mean_ns"]:
            recs, stats, des = od.run(sg, op, entry, c["begin"], c["n"], c["des_mean_ns"])
            np.savez_compressed(os.path.join(OUT, c["name"] + ".npz"), records=recs, stats=stats, des=des)
        else:
            recs, stats = oc.run(sg, op, entry, c["begin"], c["n"])
            np.savez_compressed(os.path.join(OUT, c["name"] + ".npz"), records=recs, stats=stats)
        n500 = int(np.count_nonzero(recs[:, 1] >> np.uint64(63)))
        print(f"{c['name']}: {c['n']} traces, {n500} entry 500s, mean latency {recs[:, 0].mean():.0f} ns")
        manifest.append(c)
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump({"_source": __doc__.strip().split("\n\n")[0], "cases": manifest}, f, indent=1)


if __name__ == "__main__":
    main()
