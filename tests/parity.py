"""Shared helpers: run the HIP walk (through the C ABI) and the CPU oracle on
the same graph, params and trace range, and compare bit-exactly."""
from __future__ import annotations

import json

import numpy as np

import isim
from oracle import executor as oc
from oracle import graph_ref as gr
from oracle.executor_py import SimGraph
from oracle.executor_py import SimParams as OParams


def oracle_params(p: isim.SimParams) -> OParams:
    return OParams(p.seed, p.hop_base_ns, p.req_ps_per_byte, p.resp_ps_per_byte, p.error_mode)


class Case:
    """One graph (JSON text) + entry + params, for both implementations."""

    def __init__(self, json_text: str, entry=None, params: isim.SimParams = None):
        self.json = json_text
        self.entry = entry
        self.params = params or isim.SimParams()
        self.graph = isim.ServiceGraph.from_json(json_text)
        self.handler = isim.Handler(self.graph, entry, self.params)
        self.sg = SimGraph(gr.unmarshal_service_graph(json_text))
        self.og = oc.OracleGraph(self.sg, oracle_params(self.params))

    def gpu(self, begin: int, n: int, records=True, device=0):
        return self.handler.serve(begin, n, device=device, records=records)

    def cpu(self, begin: int, n: int, records=True, threads=0):
        return oc.run(self.sg, oracle_params(self.params), self.sg.entry(self.entry), begin, n,
                      records=records, n_threads=threads, og=self.og)

    def compare(self, begin: int, n: int, records=True):
        recs, stats = self.gpu(begin, n, records)
        orec, ost = self.cpu(begin, n, records)
        if records:
            assert_records_equal(recs, orec)
        assert_stats_equal(self.handler.fold(stats), oc.split_stats(ost, len(self.sg.g.services),
                                                                    len(self.sg.sites)))
        return recs, stats


def assert_records_equal(recs, orec):
    lat = recs["latency_ns"]
    packed = recs["hops"].astype(np.uint64) | (recs["status_err"].astype(np.uint64) << np.uint64(32))
    bad = np.nonzero((lat != orec[:, 0]) | (packed != orec[:, 1]))[0]
    if bad.size:
        i = int(bad[0])
        raise AssertionError(
            f"{bad.size} records differ; first at {i}: gpu=(lat {int(lat[i])}, hops {int(recs['hops'][i])}, "
            f"st {int(recs['status_err'][i]):#x}) oracle=(lat {int(orec[i, 0])}, hops {int(orec[i, 1]) & 0xffffffff}, "
            f"st {int(orec[i, 1]) >> 32:#x})")


def assert_stats_equal(f: dict, o: dict):
    for k in ("n_traces", "sum_latency", "sum_hops", "sum_err_hops", "n_500", "max_latency"):
        assert f[k] == o[k], f"{k}: gpu {f[k]} oracle {o[k]}"
    if o["n_traces"]:
        assert f["min_latency"] == o["min_latency"], (f["min_latency"], o["min_latency"])
    for k in ("lat_prom", "lat_log2", "svc_calls", "svc_errs", "site_calls"):
        assert np.array_equal(np.asarray(f[k], np.uint64), np.asarray(o[k], np.uint64)), k
    if f.get("svc_dur") is not None:
        fd, od = np.asarray(f["svc_dur"], np.uint64), np.asarray(o["svc_dur"], np.uint64)
        bad = np.argwhere(fd != od)
        assert bad.size == 0, f"svc_dur differs at (service, word) {bad[:4].tolist()}: gpu {fd[tuple(bad[0])]} " \
                              f"oracle {od[tuple(bad[0])]}"



def with_defaults(json_text: str, **defaults) -> str:
    doc = json.loads(json_text)
    d = doc.get("defaults") or {}
    d.update(defaults)
    doc["defaults"] = d
    return json.dumps(doc)
