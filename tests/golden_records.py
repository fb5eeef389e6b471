"""Loader of the per-trace record fixtures (tests/golden/records/, made once
by tests/golden/make_records.py with the C oracle)."""
from __future__ import annotations

import json
import os

import numpy as np

from conftest import GOLDEN

RECORDS = os.path.join(GOLDEN, "records")
MANIFEST = json.load(open(os.path.join(RECORDS, "manifest.json")))
CASES = MANIFEST["cases"]
WALK_CASES = [c for c in CASES if not c["des_mean_ns"]]
DES_CASES = [c for c in CASES if c["des_mean_ns"]]


def case_id(c) -> str:
    return c["name"]


def load(c) -> dict:
    with np.load(os.path.join(RECORDS, c["name"] + ".npz")) as z:  # allow_pickle stays False
        return {k: z[k] for k in z.files}


def oracle_graph(c):
    from oracle import executor as oc
    from oracle import graph_ref as gr
    from oracle.executor_py import SimGraph, SimParams
    sg = SimGraph(gr.unmarshal_service_graph(c["graph"]))
    p = c["params"]
    op = SimParams(p["seed"], p["hop_base_ns"], p["req_ps_per_byte"], p["resp_ps_per_byte"], p["error_mode"])
    return sg, op, oc.OracleGraph(sg, op)
