"""The C oracle still produces the committed per-trace record fixtures
(tests/golden/records/) bit for bit: records, the raw
stats buffer and, for the DES cases, the per-service DES rows.  The fixtures
freeze isim semantics v1 as the oracle stood once it passed the reference's
Go vectors, the Philox KATs and the Appendix-B executor KATs; the GPU side is
tests/test_golden_records_gpu.py."""
import numpy as np
import pytest

import golden_records as gr
from oracle import des as od
from oracle import executor as oc


def test_manifest_covers_every_fixture():
    import os
    files = {f[:-4] for f in os.listdir(gr.RECORDS) if f.endswith(".npz")}
    assert files == {c["name"] for c in gr.CASES}
    assert len(gr.WALK_CASES) >= 9 and len(gr.DES_CASES) >= 3


@pytest.mark.parametrize("case", gr.CASES, ids=gr.case_id)
def test_oracle_reproduces_fixture(case):
    fx = gr.load(case)
    sg, op, og = gr.oracle_graph(case)
    entry = sg.entry(case["entry"])
    if case["des_mean_ns"]:
        recs, stats, des = od.run(sg, op, entry, case["begin"], case["n"], case["des_mean_ns"], og=og)
        assert np.array_equal(des, fx["des"])
    else:
        recs, stats = oc.run(sg, op, entry, case["begin"], case["n"], og=og)
    assert recs.shape == (case["n"], 2)
    assert np.array_equal(recs, fx["records"])
    assert np.array_equal(stats, fx["stats"])


@pytest.mark.parametrize("case", gr.CASES, ids=gr.case_id)
def test_fixture_is_informative(case):
    """Every error-injecting fixture holds both 200 and 500 entries; the
    latencies vary wherever a queue or a probabilistic call is involved."""
    r = gr.load(case)["records"]
    st = r[:, 1] >> np.uint64(63)
    if case["name"] != "c1_canonical_A":
        assert 0 < int(st.sum()) < case["n"], case["name"]
    if case["des_mean_ns"] or case["name"].startswith("mesh"):
        assert len(np.unique(r[:, 0])) > case["n"] // 4
