"""A/B of the kind-7 occupancy variants on config 4's mesh WITH error draws
(errorRate 1 %: the DRAW kernels): the two-workgroups-per-CU kernel (80
VGPRs; its DRAW variants spill registers to scratch) against the one-
workgroup kernel (ISIM_TREE_OCC1).  Run on the GPU box:
  python tools/occ_ab.py            (prints one line per setting)"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "istio-isotope_amd"), ROOT]


def run_one():
    import torch

    import isim
    from isim.generators import mesh_topology
    from isim.yamljson import obj_to_json
    doc = mesh_topology()
    doc.setdefault("defaults", {})["errorRate"] = 0.01
    for s in doc["services"]:
        s["errorRate"] = 0.01
    h = isim.Handler(isim.ServiceGraph.from_json(obj_to_json(doc)), None, isim.SimParams())
    li = h.launch_info(0)
    n = 1 << 26
    dev = torch.device("cuda", 0)
    st = torch.zeros(h.stats_words, dtype=torch.int64, device=dev)
    rec = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(2):
        h.serve_device(0, n, rec.data_ptr(), st.data_ptr(), s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    k = 5
    for i in range(k):
        h.serve_device((i + 1) * n, n, rec.data_ptr(), st.data_ptr(), s)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / k
    print(json.dumps({"occ1": bool(os.environ.get("ISIM_TREE_OCC1")), "ms": dt * 1e3, "gtr_s": n / dt / 1e9,
                      "wg_threads": li["wg_threads"], "blocks_per_cu": li["blocks_per_cu"]}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run_one()
    else:
        for occ1 in ("", "1", "", "1"):
            env = dict(os.environ)
            env.pop("ISIM_TREE_OCC1", None)
            if occ1:
                env["ISIM_TREE_OCC1"] = occ1
            subprocess.run([sys.executable, __file__, "one"], env=env, check=True, timeout=300)
