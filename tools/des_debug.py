"""Debug helper: DES of one random test graph (tests/test_des_gpu.py) vs the oracle."""
import os
import sys
import numpy as np
sys.path[:0] = ["tests", "istio-isotope_amd", "."]
os.environ["ISIM_DES_DEBUG"] = "1"
import isim
from test_des_gpu import DesCase, _random_graph

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 5
doc = _random_graph(seed)
import json
print(json.dumps(doc))
mode = isim.MODE_B if seed % 3 == 0 else isim.MODE_A
mean = [60_000, 300_000, 2_000_000][seed % 3]
c = DesCase(doc, mean, error_mode=mode)
for n in (1, 2, 10, 100, 3000):
    try:
        r, s, t = c.d.serve(seed, n, wide=True)
        print(n, "ok", s[:8])
    except Exception as e:
        print(n, "fail", e)
