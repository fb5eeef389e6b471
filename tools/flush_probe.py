"""Timing probe (no result checks): mean HIP-event time of isim_serve_device
per batch size for configs 3 and 4, with the library named by ISIM_LIB (e.g.
a timing-only build without the workgroup flush).  Prints one line per case."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "istio-isotope_amd")]

import torch  # noqa: E402

import isim  # noqa: E402
from isim.generators import config3_topology, mesh_topology  # noqa: E402
from isim.yamljson import obj_to_json  # noqa: E402


def probe(name, doc, batches, reps=5):
    h = isim.Handler(isim.ServiceGraph.from_json(obj_to_json(doc)), None,
                     isim.SimParams(flags=isim.native.FLAG_WALK_ALL))
    dev = torch.device("cuda", 0)
    stats = torch.zeros(h.info.stats_words, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream()
    for B in batches:
        recs = torch.empty((B, 2), dtype=torch.int64, device=dev)
        h.serve_device(0, B, recs.data_ptr(), stats.data_ptr(), s.cuda_stream)
        ts = []
        for r in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            h.serve_device(r * B, B, recs.data_ptr(), stats.data_ptr(), s.cuda_stream)
            b.record(s)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        print(name, B, round(sum(ts) / len(ts), 4), "ms", flush=True)


probe("c3", config3_topology(), [1 << 16, 1 << 20, 1 << 22])
probe("c4", mesh_topology(), [1 << 16, 1 << 20, 1 << 22])
