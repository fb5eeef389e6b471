import sys, os
sys.path[:0] = ["/root/repo/tests", "/root/repo", "/root/repo/istio-isotope_amd"]
import isim
from isim.generators import config2_topology, tree_topology
from isim.yamljson import obj_to_json
from parity import with_defaults, Case
for lv, br in [(3, 3), (3, 8), (4, 4), (4, 8)]:
    for er in (0.0, 0.01):
        j = with_defaults(obj_to_json(tree_topology(lv, br, sequential=True)), errorRate=er)
        c = Case(j, None, isim.SimParams(flags=isim.native.FLAG_DYNAMIC))
        li = c.handler.launch_info(0)
        print(lv, br, er, li, flush=True)
        try:
            c.compare(0, 64)
            print("ok", flush=True)
        except Exception as e:
            print("FAIL", e, flush=True)
            sys.exit(1)
