"""The per-service Prometheus exposition rendered from a stats buffer the HIP
kernels produced (isim_serve on the GPU), compared with a registry fed one
Record* call at a time from the pure-Python oracle's event log — the
reference's own recording pattern (isotope/service/pkg/srv/prometheus/
handler.go:87-106).  Covers the static walks (draw stream, mode-B close
list: durations derived by isim_stats_fold_durations) and the dynamic lane
tree walk (durations recorded per invocation in the device table)."""
import pytest

import isim
from isim import prometheus as P
from oracle import executor_py as ex
from oracle import graph_ref as gr

from test_prometheus import GRAPHS, _registry_from_events

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(GRAPHS))
@pytest.mark.parametrize("begin,n", [(1000, 300), ((1 << 32) - 100, 257)])
def test_gpu_exposition_matches_event_registry(gpu, name, begin, n):
    text, mode = GRAPHS[name]
    graph = isim.ServiceGraph.from_json(text)
    h = isim.Handler(graph, None, isim.SimParams(error_mode=mode))
    _, stats = h.serve(begin, n, device=gpu)
    got = P.service_metrics(h, stats=stats)
    sg = ex.SimGraph(gr.unmarshal_service_graph(text))
    _, st = ex.run(sg, ex.SimParams(error_mode=mode), sg.entry(None), begin, n, events=True)
    want = _registry_from_events(sg, st.events, graph)
    for s in graph.services:
        assert got[s.name].exposition() == want[s.name].exposition(), s.name
