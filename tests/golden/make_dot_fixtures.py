"""Regenerates tests/golden/dot/*.dot: the Graphviz DOT text isotope's
`convert graphviz` would print for the committed topologies.

Run in the build container, where /root/reference is mounted (the GPU box
only reads the committed outputs).  The DOT text is produced by executing
the reference's OWN template — the `graphvizTemplate` raw-string constant,
read at generation time from
/root/reference/isotope/convert/pkg/graphviz/graphviz.go (it is not copied
into this repository) — with an independent text/template interpreter
(oracle/marshal_ref.py: execute_template) over the Graph value of the
oracle's ServiceGraphToGraph restatement, which tests/test_marshal.py pins
to the reference's TestServiceGraphToGraph vector.  The product's C++
emitter (libisim isim_graph_to_dot) hand-expands the template, so the
fixtures check its whitespace handling against the template itself.
"""
import glob
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "istio-isotope_amd"))

REF = "/root/reference/isotope/convert/pkg/graphviz/graphviz.go"


def reference_template() -> str:
    src = open(REF).read()
    m = re.search(r"const graphvizTemplate = `(.*?)`", src, re.S)
    assert m, "graphvizTemplate not found"
    return m.group(1)


def main():
    from oracle import graph_ref as gr
    from oracle import marshal_ref as mr
    from isim.yamljson import yaml_to_json

    tmpl = reference_template()
    out_dir = os.path.join(HERE, "dot")
    os.makedirs(out_dir, exist_ok=True)
    docs = {}
    for p in sorted(glob.glob(os.path.join(HERE, "topologies", "*.yaml"))):
        docs[os.path.basename(p)[:-5]] = yaml_to_json(open(p, "rb").read())
    vec = json.load(open(os.path.join(HERE, "go_vectors.json")))
    docs["graphviz_test"] = vec["graphviz_graph"]["input"]
    docs["empty"] = '{"services": []}'
    for name, j in docs.items():
        g = gr.unmarshal_service_graph(j)
        dot = mr.execute_template(tmpl, mr.service_graph_to_graph(g))
        with open(os.path.join(out_dir, name + ".dot"), "w") as f:
            f.write(dot)
        print(name, len(dot))


if __name__ == "__main__":
    main()
