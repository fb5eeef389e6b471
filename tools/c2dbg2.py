import sys, os
os.environ["ISIM_LIB"] = "/root/repo/istio-isotope_amd/isim/libisim_dbg.so"
sys.path[:0] = ["/root/repo/tests", "/root/repo", "/root/repo/istio-isotope_amd"]
import isim
from isim.generators import tree_topology
from isim.yamljson import obj_to_json
from parity import with_defaults
j = with_defaults(obj_to_json(tree_topology(4, 8, sequential=True)), errorRate=0.01)
h = isim.Handler(isim.ServiceGraph.from_json(j), None, isim.SimParams(flags=isim.native.FLAG_DYNAMIC))
print(h.launch_info(0), flush=True)
try:
    recs, st = h.serve(0, 64)
    d = int(st[7])
    print("dbg word", hex(d), "code", d & 0xFF, "p", (d >> 8) & 0xFFFFFF, "f", d >> 32, flush=True)
    print(recs[:4])
except Exception as e:
    print("FAIL", e, flush=True)
