"""Debug helper: one DES device batch, narrow rows, print the stats header."""
import sys
import numpy as np
import torch
sys.path[:0] = ["tests", "istio-isotope_amd", "."]
import isim
from test_des_gpu import DesCase, _sleepy_tree

c = DesCase(_sleepy_tree(3, 3), 900_000)
n = 5000
dev = torch.device("cuda", 0)
st = torch.zeros(c.h.stats_words, dtype=torch.int64, device=dev)
tab = torch.zeros(max(1, c.d.table_words), dtype=torch.int64, device=dev)
wsb = c.d.workspace_bytes(n)
ws = torch.zeros(wsb // 8 + 1, dtype=torch.int64, device=dev)
s = torch.cuda.current_stream().cuda_stream
c.d.serve_device(0, n, 0, st.data_ptr(), tab.data_ptr(), ws.data_ptr(), wsb, s)
torch.cuda.synchronize()
print("header", st[:8].tolist())
_, s0, t0 = c.d.serve(0, n, records=False)
print("sync header", s0[:8].tolist())
