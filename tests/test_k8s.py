"""Kubernetes manifests (isotope convert/pkg/kubernetes): the
C ABI isim_graph_to_k8s_manifests / isim_graph_marshal_yaml.  CPU only.

Parity unpinned: the reference has no tests for this package and
Go is absent, so the expected text comes from
  * hand-derived manifests for 1-service.yaml (every line written out below
    from kubernetes.go:56-270, fortio_client.go:28-78, consts.go and the
    k8s.io/api v0.18.0 json tags), and RBAC/RbacConfig text of rbac.go:25-71;
  * an independent restatement (oracle/k8s_ref.py) that renders the same
    objects with PyYAML's emitter (a port of the libyaml emitter yaml.v2
    carries) under yaml.v2's key order and quoting rules, on every committed
    topology, several parameter sets and hypothesis graphs with awkward names;
  * round trips: the ConfigMap payload decodes back to the same graph.
"""
import glob
import os

import pytest
import yaml
from hypothesis import HealthCheck, example, given, settings
from hypothesis import strategies as st

import isim
from isim.yamljson import obj_to_json, yaml_to_json
from oracle import graph_ref as gr
from oracle import k8s_ref

HERE = os.path.dirname(os.path.abspath(__file__))
TOPOS = sorted(glob.glob(os.path.join(HERE, "golden", "topologies", "*.yaml")))
TS = 1600000000  # 2020-09-13T12:26:40Z

ONE_SERVICE = """apiVersion: v1
kind: Namespace
metadata:
  creationTimestamp: "2020-09-13T12:26:40Z"
  labels:
    istio-injection: enabled
  name: service-graph
spec: {}
status: {}
---
apiVersion: v1
data:
  service-graph: |
    services:
    - isEntrypoint: true
      name: a
      numRbacPolicies: 0
      numReplicas: 1
      responseSize: 1KiB
      type: http
kind: ConfigMap
metadata:
  creationTimestamp: "2020-09-13T12:26:40Z"
  labels:
    app: service-graph
  name: service-graph-config
  namespace: service-graph
---
apiVersion: apps/v1
kind: Deployment
metadata:
  creationTimestamp: "2020-09-13T12:26:40Z"
  labels:
    app: service-graph
  name: a
  namespace: service-graph
spec:
  replicas: 1
  selector:
    matchLabels:
      name: a
  strategy: {}
  template:
    metadata:
      annotations:
        prometheus.io/scrape: "true"
      creationTimestamp: "2020-09-13T12:26:40Z"
      labels:
        name: a
        role: service
    spec:
      containers:
      - args:
        - --max-idle-connections-per-host=32
        env:
        - name: SERVICE_NAME
          value: a
        - name: PODNAME
          valueFrom:
            fieldRef:
              fieldPath: metadata.name
        - name: PODIP
          valueFrom:
            fieldRef:
              fieldPath: status.podIP
        - name: NAMESPACE
          valueFrom:
            fieldRef:
              fieldPath: metadata.namespace
        - name: NODENAME
          valueFrom:
            fieldRef:
              fieldPath: spec.nodeName
        image: tahler/isotope-service:1
        imagePullPolicy: IfNotPresent
        name: mock-service
        ports:
        - containerPort: 8080
        resources: {}
        volumeMounts:
        - mountPath: /etc/config
          name: config-volume
      nodeSelector:
        role: service
      volumes:
      - configMap:
          items:
          - key: service-graph
            path: service-graph.yaml
          name: service-graph-config
        name: config-volume
status: {}
---
apiVersion: v1
kind: Service
metadata:
  creationTimestamp: "2020-09-13T12:26:40Z"
  labels:
    app: service-graph
  name: a
  namespace: service-graph
spec:
  ports:
  - name: http-web
    port: 8080
    targetPort: 0
  selector:
    name: a
status:
  loadBalancer: {}
---
apiVersion: apps/v1
kind: Deployment
metadata:
  creationTimestamp: "2020-09-13T12:26:40Z"
  labels:
    app: client
  name: client
spec:
  selector:
    matchLabels:
      app: client
  strategy: {}
  template:
    metadata:
      creationTimestamp: "2020-09-13T12:26:40Z"
      labels:
        app: client
    spec:
      containers:
      - args:
        - server
        image: fortio/fortio:latest
        name: fortio-client
        ports:
        - containerPort: 8080
        - containerPort: 42422
        resources: {}
      nodeSelector:
        role: client
status: {}
---
apiVersion: v1
kind: Service
metadata:
  annotations:
    prometheus.io/scrape: "true"
  creationTimestamp: "2020-09-13T12:26:40Z"
  labels:
    app: client
  name: client
spec:
  ports:
  - port: 8080
    targetPort: 0
  selector:
    app: client
status:
  loadBalancer: {}
"""


def _graphs(path):
    j = yaml_to_json(open(path, "rb").read())
    return isim.ServiceGraph.from_json(j), gr.unmarshal_service_graph(j)


def _both(g, og, **kw):
    a = g.to_k8s_manifests(**kw)
    okw = dict(kw)
    okw["idle"] = okw.pop("service_max_idle_connections_per_host", 0)
    b = k8s_ref.manifests(og, **okw)
    return a, b


def test_one_service_hand_derived():
    g, og = _graphs(os.path.join(HERE, "golden", "topologies", "1-service.yaml"))
    kw = dict(service_node_selector={"role": "service"}, service_image="tahler/isotope-service:1",
              service_max_idle_connections_per_host=32, client_node_selector={"role": "client"},
              client_image="fortio/fortio:latest", creation_timestamp_s=TS)
    a, b = _both(g, og, **kw)
    assert a == ONE_SERVICE
    assert b == ONE_SERVICE


def test_rbac_under_istio():
    """rbac.go: numRbacPolicies rules + one allow-all per service, then the
    RbacConfig after the Fortio objects; only for environment ISTIO
    (strings.EqualFold) and numRbacPolicies > 0."""
    doc = {"defaults": {"numRbacPolicies": 2}, "services": [{"name": "a", "isEntrypoint": True},
                                                            {"name": "b", "numRbacPolicies": 0}]}
    g = isim.ServiceGraph.from_json(obj_to_json(doc))
    plain = g.to_k8s_manifests(creation_timestamp_s=TS)
    assert "rbac.istio.io" not in plain
    m = g.to_k8s_manifests(creation_timestamp_s=TS, environment_name="IsTiO", rbac_seed=7)
    docs = m.split("---\n")
    # Namespace, ConfigMap, a: Deployment Service + 3 x (ServiceRole, ServiceRoleBinding), b: 2, Fortio 2, RbacConfig
    assert len(docs) == 2 + 2 + 6 + 2 + 2 + 1
    roles = [d for d in docs if d.startswith('\napiVersion: "rbac.istio.io/v1alpha1"\nkind: ServiceRole\n')]
    binds = [d for d in docs if d.startswith('apiVersion: "rbac.istio.io/v1alpha1"\nkind: ServiceRoleBinding\n')]
    assert len(roles) == 3 and len(binds) == 3
    assert all('services: ["a.service-graph.*"]' in r for r in roles)
    names = [r.split("name: ")[1].split("\n")[0] for r in roles]
    assert len(set(names)) == 3
    for n in names:  # version-4 UUID text
        assert len(n) == 36 and n[14] == "4" and n[19] in "89ab"
    assert [b.count('user: "*"') for b in binds] == [0, 0, 1]
    assert docs[-1].startswith('\napiVersion: "rbac.istio.io/v1alpha1"\nkind: RbacConfig')
    assert "mode: 'ON_WITH_INCLUSION'" in docs[-1]
    # EXT: deterministic per seed
    assert g.to_k8s_manifests(creation_timestamp_s=TS, environment_name="ISTIO", rbac_seed=7) == m
    assert g.to_k8s_manifests(creation_timestamp_s=TS, environment_name="ISTIO", rbac_seed=8) != m


PARAMS = [
    dict(creation_timestamp_s=TS),
    dict(service_image="img:1", client_image="fortio", creation_timestamp_s=0,
         service_node_selector={"k": "v", "zone 1": "true", "0n": "yes"}, client_node_selector={"role": "client"},
         service_max_idle_connections_per_host=-5),
    dict(environment_name="ISTIO", rbac_seed=12345, creation_timestamp_s=253402300799),
]


@pytest.mark.parametrize("path", TOPOS, ids=os.path.basename)
@pytest.mark.parametrize("pi", range(len(PARAMS)))
def test_topologies_match_oracle(path, pi):
    g, og = _graphs(path)
    a, b = _both(g, og, **PARAMS[pi])
    assert a == b
    # every document parses, and the ConfigMap payload decodes to the same graph
    docs = list(yaml.safe_load_all(a.replace("\n---\n\napiVersion", "\n---\napiVersion")))
    cm = [d for d in docs if d and d.get("kind") == "ConfigMap"][0]
    back = isim.ServiceGraph.from_json(yaml_to_json(cm["data"]["service-graph"].encode()))
    assert back.canonical() == g.canonical()


def test_marshal_yaml_is_configmap_payload():
    g, og = _graphs(os.path.join(HERE, "golden", "topologies", "canonical.yaml"))
    y = g.marshal_yaml()
    assert y == k8s_ref.graph_yaml(og)
    assert "  service-graph: |\n    " + y[:-1].replace("\n", "\n    ") + "\n" in g.to_k8s_manifests()


@pytest.mark.parametrize("f,want", [(0.01, "0.01"), (1e-05, "1e-05"), (1e-07, "1e-07"), (0.5, "0.5"),
                                    (0.123456789, "0.123456789"), (1e6, "1e+06"), (123456.0, "123456"),
                                    (2.5e-4, "0.00025")])
def test_go_format_g(f, want):
    assert k8s_ref.go_format_g(f) == want


def test_error_rates_render_as_yaml_floats():
    doc = {"services": [{"name": "a", "isEntrypoint": True, "errorRate": 1e-7},
                        {"name": "b", "errorRate": "0.01%"}, {"name": "c", "errorRate": 0.5}]}
    g = isim.ServiceGraph.from_json(obj_to_json(doc))
    y = g.marshal_yaml()
    assert "errorRate: 1e-07\n" in y and "errorRate: 0.0001\n" in y and "errorRate: 0.5\n" in y
    assert y == k8s_ref.graph_yaml(gr.unmarshal_service_graph(obj_to_json(doc)))


def test_bad_params():
    g, _ = _graphs(os.path.join(HERE, "golden", "topologies", "1-service.yaml"))
    with pytest.raises(isim.IsimError):
        g.to_k8s_manifests(creation_timestamp_s=10 ** 12)  # year > 9999 (metav1.Time.MarshalJSON fails)


# names that exercise the scalar analysis: YAML 1.1 words, numbers, timestamps,
# indicators, ": " and " #", leading/trailing spaces, long texts with spaces
# (folded past column 80), quotes and backslashes, tabs, BMP letters
_tricky = st.sampled_from(["true", "no", "~", "null", "123", "0x1F", "1e3", "1:20", "2001-12-14", "2001-12-14t21:59:43.10Z",
                           "-dash", "- dash", "a: b", "a #b", "a#b", "?q", ":c", "[x]", "{y}", "*star", "&amp", "!bang",
                           "|pipe", ">gt", "'sq'", '"dq"', "%pct", "@at", "`bt", " lead", "trail ", "tab\tin",
                           "back\\slash", "café", " nbsp", "x" * 90, ("word " * 30).strip(), "---", "...",
                           "a,b", "y", "Off", ".5", "+1", "1_000", "0o17", "0b101"])
_names = st.one_of(_tricky, st.text(alphabet=st.characters(min_codepoint=0x20, max_codepoint=0x2000,
                                                          blacklist_categories=("Cs", "Zl", "Zp", "Cc")),
                                    min_size=1, max_size=40))


@st.composite
def _graph(draw):
    n = draw(st.integers(1, 4))
    names = draw(st.lists(_names, min_size=n, max_size=n, unique=True))
    svcs = []
    for nm in names:
        svc = {"name": nm, "numReplicas": draw(st.integers(0, 9)), "numRbacPolicies": draw(st.integers(0, 2)),
               "errorRate": draw(st.sampled_from([0, 0.01, 1e-7, 0.123456789, 1]))}
        if draw(st.booleans()):
            svc["script"] = [{"call": draw(st.sampled_from(names))}, {"sleep": "%dms" % draw(st.integers(0, 5000))}]
        svcs.append(svc)
    svcs[0]["isEntrypoint"] = True
    return {"services": svcs}


_ONE_TRUE = {"services": [{"name": "true", "numReplicas": 0, "numRbacPolicies": 0, "errorRate": 0,
                           "isEntrypoint": True}]}


@settings(max_examples=50, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(_graph(), st.sampled_from(["", "img", "my image:1 with spaces", "true"]),
       st.dictionaries(_names, _names, max_size=2))
# failures hypothesis found in round 3, pinned: a key outside ASCII, a key of
# 149 characters (complex key), and a double-quoted value after a 90-character
# key, which libyaml folds only at spaces (never right after an escape)
@example(doc=_ONE_TRUE, image="", sel={"true": "true", "\u0eb4": "true"})
@example(doc=_ONE_TRUE, image="", sel={("word " * 30).strip(): "true"})
@example(doc=_ONE_TRUE, image="", sel={"x" * 90: "tab\tin"})
@example(doc=_ONE_TRUE, image="", sel={"x" * 90: "tab\tin with spaces past the fold and \"quotes\" \\ and more"})
def test_hypothesis_graphs_match_oracle(doc, image, sel):
    j = obj_to_json(doc)
    g = isim.ServiceGraph.from_json(j)
    og = gr.unmarshal_service_graph(j)
    kw = dict(service_image=image, client_image=image, service_node_selector=sel, environment_name="ISTIO",
              rbac_seed=3, creation_timestamp_s=TS)
    a, b = _both(g, og, **kw)
    assert a == b


def test_key_order_unicode_classes():
    """yaml.v2 sorter.go keyList.Less classifies runes with Go's
    unicode.IsLetter (L*) and unicode.IsDigit (Nd), and a digit counts as
    rune - '0': a nonspacing mark (U+0EB4) is no letter, an Arabic-Indic
    three (U+0663) is a digit worth 1587, a superscript two no digit.
    Expected order derived by hand from those rules."""
    g, og = _graphs(os.path.join(HERE, "golden", "topologies", "1-service.yaml"))
    sel = {"true": "1", "ິ": "2", "a٣": "3", "a2": "4", "x²": "5"}
    a, b = _both(g, og, service_node_selector=sel, creation_timestamp_s=TS)
    assert a == b
    block = a.split("nodeSelector:\n", 1)[1].splitlines()[:5]
    assert [ln.strip().split(":")[0] for ln in block] == ["ິ", "a2", "a٣", '"true"', "x²"]


def test_complex_keys():
    """yaml.v2 (libyaml emitterc.go yaml_emitter_check_simple_key) writes a
    key of more than 128 BYTES as a complex key: "? key" (folded at 80
    columns), then ": value" at the mapping's indent.  Hand-derived layout."""
    g, og = _graphs(os.path.join(HERE, "golden", "topologies", "1-service.yaml"))
    sel = {"x" * 128: "a", "y" * 129: "b", "é" * 64: "c", "é" * 65: "d", ("word " * 30).strip(): "e"}
    a, b = _both(g, og, service_node_selector=sel, creation_timestamp_s=TS)
    assert a == b
    block = a.split("nodeSelector:\n", 1)[1].split("      volumes:", 1)[0]
    w = "word " * 15
    assert block == ("        ? " + w.strip() + "\n"  # keyList order: w < x < y < é (letters by code point)
                     "          " + w.strip() + "\n"
                     "        : e\n"
                     "        " + "x" * 128 + ": a\n"
                     "        ? " + "y" * 129 + "\n"
                     "        : b\n"
                     "        " + "é" * 64 + ": c\n"
                     "        ? " + "é" * 65 + "\n"
                     "        : d\n")


def test_double_quoted_folds_only_at_spaces():
    """libyaml (yaml.v2 emitterc.go yaml_emitter_write_double_quoted) folds a
    double-quoted scalar only at a single space past column 80, the space
    becoming the break; an escape sequence is never a break point.
    Hand-derived layout for a value after a 90-character key."""
    g, og = _graphs(os.path.join(HERE, "golden", "topologies", "1-service.yaml"))
    k = "x" * 90
    sel = {k: "tab\tin no-break"}
    a, b = _both(g, og, service_node_selector=sel, creation_timestamp_s=TS)
    assert a == b
    block = a.split("nodeSelector:\n", 1)[1].split("      volumes:", 1)[0]
    # column after `        <k>: "tab\tin` is 8 + 90 + 2 + 8 = 108 > 80: the space folds
    assert block == '        ' + k + ': "tab\\tin\n          no-break"\n'
