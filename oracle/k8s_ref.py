"""Restatement of isotope's Kubernetes manifest generator (oracle — test
infrastructure only; never imported by the product).

  ServiceGraphToKubernetesManifests  convert/pkg/kubernetes/kubernetes.go:56-137
  makeServiceGraphNamespace / makeConfigMap / makeService / makeDeployment
                                     kubernetes.go:150-270
  makeFortioDeployment / makeFortioService   fortio_client.go:28-78
  generateRbacPolicy / generateRbacConfig    rbac.go:25-71
  constants                                  convert/pkg/consts/consts.go

Each object is built as the JSON value encoding/json gives the k8s.io/api
v0.18.0 struct (omitempty drops empty strings, nil pointers and empty maps and
slices, never struct values), then rendered the way sigs.k8s.io/yaml v1.2.0
renders it: gopkg.in/yaml.v2 decodes the JSON (ints stay ints, floats become
float64) and encodes it again.  The encoding here is PyYAML's emitter — a
port of the same libyaml emitter yaml.v2 carries, so line layout, indentless
block sequences, scalar analysis, folding at 80 columns and escapes come from
an implementation independent of the product's (csrc/k8s.cpp) — driven with
yaml.v2's own choices restated on top: keys in keyList.Less order
(yaml.v2 sorter.go), strings that yaml.v2's resolve() would read back as
another type in double quotes, multi-line strings in literal style, numbers
with strconv.FormatFloat(f, 'g', -1, 64).  PyYAML departs from libyaml in
three places; two are replaced here: simple-key length (bytes vs characters,
`check_simple_key`) and double-quoted folding (libyaml breaks ONLY at a space
past column 80 and drops that space into the break; PyYAML also breaks right
after an escape sequence and keeps the space as `\\ `, so
`write_double_quoted` is libyaml's).  The third is not exercised by the tests:
in the scalar analysis that picks the style, NEL and characters beyond the BMP
count as printable for PyYAML but not for yaml.v2.

EXT rules shared with the product (the reference is not deterministic):
creationTimestamp = the caller's unix seconds (reference: time.Now()); RBAC
rule names = v4 UUIDs from Philox4x32-10((i_lo, i_hi, 0, 0x4B385300), seed)
(reference: uuid.New()).
"""
from __future__ import annotations

import datetime
import functools
import json
import re
import unicodedata
from typing import Any, Dict, List, Optional

import yaml

from . import philox
from .graph_ref import ServiceGraph
from .marshal_ref import marshal_service_graph

NAMESPACE = "service-graph"


# ------------------------------------------------------ yaml.v2 choices -----
def _is_letter(ch: str) -> bool:
    """Go unicode.IsLetter: categories Lu, Ll, Lt, Lm, Lo."""
    return unicodedata.category(ch) in ("Lu", "Ll", "Lt", "Lm", "Lo")


def _is_digit(ch: str) -> bool:
    """Go unicode.IsDigit: category Nd (str.isdigit would also take superscripts)."""
    return unicodedata.category(ch) == "Nd"


def _wrap64(x: int) -> int:
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >> 63 else x


def keylist_less(a: str, b: str) -> bool:
    """gopkg.in/yaml.v2 sorter.go keyList.Less for two string keys (Go int64
    arithmetic on rune - '0', so a non-ASCII digit counts by its code point)."""
    ar, br = list(a), list(b)
    for i in range(min(len(ar), len(br))):
        if ar[i] == br[i]:
            continue
        al, bl = _is_letter(ar[i]), _is_letter(br[i])
        if al and bl:
            return ar[i] < br[i]
        if al or bl:
            return bl
        an = bn = 0
        if ar[i] == "0" or br[i] == "0":
            j = i - 1
            while j >= 0 and _is_digit(ar[j]):
                if ar[j] != "0":
                    an = bn = 1
                    break
                j -= 1
        ai = i
        while ai < len(ar) and _is_digit(ar[ai]):
            an = _wrap64(an * 10 + ord(ar[ai]) - 48)
            ai += 1
        bi = i
        while bi < len(br) and _is_digit(br[bi]):
            bn = _wrap64(bn * 10 + ord(br[bi]) - 48)
            bi += 1
        if an != bn:
            return an < bn
        if ai != bi:
            return ai < bi
        return ar[i] < br[i]
    return len(ar) < len(br)


_FLOAT = re.compile(r"^[-+]?(\.[0-9]+|[0-9]+(\.[0-9]*)?)([eE][-+]?[0-9]+)?$")
_BASE60 = re.compile(r"^[-+]?[0-9][0-9_]*(?::[0-5]?[0-9])+(?:\.[0-9_]*)?$")
_WORDS = {"", "~", "null", "Null", "NULL", "y", "Y", "yes", "Yes", "YES", "n", "N", "no", "No", "NO",
          "true", "True", "TRUE", "false", "False", "FALSE", "on", "On", "ON", "off", "Off", "OFF",
          ".inf", ".Inf", ".INF", "+.inf", "+.Inf", "+.INF", "-.inf", "-.Inf", "-.INF", ".nan", ".NaN", ".NAN",
          "<<"}
_TS = [re.compile(r"^(\d{4})-(\d{1,2})-(\d{1,2})[Tt](\d{1,2}):(\d{1,2}):(\d{1,2})(?:[.,]\d+)?(?:Z|[+-]\d\d:\d\d)$"),
       re.compile(r"^(\d{4})-(\d{1,2})-(\d{1,2}) (\d{1,2}):(\d{1,2}):(\d{1,2})(?:[.,]\d+)?$"),
       re.compile(r"^(\d{4})-(\d{1,2})-(\d{1,2})$")]


def _go_int(s: str) -> bool:
    """strconv.ParseInt / ParseUint(s, 0, 64) succeed (range ignored: an
    out-of-range literal resolves to a float, also not a string)."""
    m = re.match(r"^[-+]?(0[xX][0-9a-fA-F]+|0[oO][0-7]+|0[bB][01]+|0[0-7]*|[1-9][0-9]*)$", s)
    return m is not None


def _timestamp(s: str) -> bool:
    for rx in _TS:
        m = rx.match(s)
        if not m:
            continue
        g = [int(x) for x in m.groups()]
        try:
            datetime.date(g[0], g[1], g[2])
        except ValueError:
            return False
        if len(g) > 3 and (g[3] > 23 or g[4] > 59 or g[5] > 59):
            return False
        return True
    return False


def resolves_non_string(s: str) -> bool:
    """yaml.v2 resolve("", s) returns a tag other than !!str, or isBase60Float."""
    if s in _WORDS:
        return True
    if s[0] in "+-.0123456789":
        plain = s.replace("_", "")
        if _go_int(plain) or _FLOAT.match(plain):
            return True
        if _timestamp(s):
            return True
    return bool(_BASE60.match(s))


def go_format_g(f: float) -> str:
    """strconv.FormatFloat(f, 'g', -1, 64)."""
    r = repr(float(f))  # shortest round-trip digits
    if "e" in r or "E" in r:
        mant, e = r.lower().split("e")
        exp = int(e)
    else:
        mant, exp = r, 0
    neg = mant.startswith("-")
    mant = mant.lstrip("-")
    ip, _, fp = mant.partition(".")
    digits = (ip + fp).lstrip("0")
    # decimal point position relative to the digit string
    lead = len(ip + fp) - len((ip + fp).lstrip("0"))
    dp = len(ip) - lead + exp
    digits = digits.rstrip("0") or "0"
    e10 = dp - 1
    sign = "-" if neg else ""
    if e10 < -4 or e10 >= 6:
        m = digits[0] + ("." + digits[1:] if len(digits) > 1 else "")
        return f"{sign}{m}e{'-' if e10 < 0 else '+'}{abs(e10):02d}"
    if dp <= 0:
        return sign + "0." + "0" * (-dp) + digits
    if dp >= len(digits):
        return sign + digits + "0" * (dp - len(digits))
    return sign + digits[:dp] + "." + digits[dp:]


class _Str(str):
    pass


class _Dumper(yaml.Dumper):
    """PyYAML's emitter with no implicit resolvers (every plain scalar reads
    back as a string to PyYAML), so the scalar style is exactly the one
    chosen below with yaml.v2's rules."""
    yaml_implicit_resolvers: Dict[str, Any] = {}

    def check_simple_key(self):
        """libyaml's (yaml.v2 emitterc.go yaml_emitter_check_simple_key) rule
        for a scalar key: at most 128 BYTES and not multiline, empty allowed
        (PyYAML: fewer than 128 characters, not empty)."""
        if isinstance(self.event, yaml.ScalarEvent):
            if self.analysis is None:
                self.analysis = self.analyze_scalar(self.event.value)
            return len(self.event.value.encode("utf-8")) <= 128 and not self.analysis.multiline
        return super().check_simple_key()

    def write_double_quoted(self, text, split=True):
        """libyaml's yaml_emitter_write_double_quoted (yaml.v2 emitterc.go):
        a line is folded ONLY at a single space past best_width that is not the
        scalar's first or last character; the space becomes the line break and a
        following space is escaped with a backslash.  PyYAML also breaks right
        after an escape sequence and keeps the folded space as an escaped
        break, so its own routine is replaced here."""
        self.write_indicator('"', True)
        spaces = False
        n = len(text)
        for i, ch in enumerate(text):
            printable = ('\x20' <= ch <= '\x7E' or (self.allow_unicode and (
                '\xA0' <= ch <= '\uD7FF' or '\uE000' <= ch <= '\uFFFD')))
            if not printable or ch in '"\\\x85\u2028\u2029\uFEFF':
                if ch in self.ESCAPE_REPLACEMENTS:
                    data = '\\' + self.ESCAPE_REPLACEMENTS[ch]
                elif ch <= '\xFF':
                    data = '\\x%02X' % ord(ch)
                elif ch <= '\uFFFF':
                    data = '\\u%04X' % ord(ch)
                else:
                    data = '\\U%08X' % ord(ch)
                spaces = False
            elif ch == ' ':
                if split and not spaces and self.column > self.best_width and 0 < i < n - 1:
                    self.write_indent()
                    data = '\\' if text[i + 1] == ' ' else ''
                else:
                    data = ' '
                spaces = True
            else:
                data = ch
                spaces = False
            if data:
                self.column += len(data)
                self.stream.write(data.encode(self.encoding) if self.encoding else data)
        self.write_indicator('"', False)


def _repr_str(d: yaml.Dumper, s: str):
    if "\n" in s:
        style = "|"
    elif resolves_non_string(s):
        style = '"'
    else:
        style = None
    return d.represent_scalar("tag:yaml.org,2002:str", s, style=style)


def _repr_plain(d: yaml.Dumper, s: "_Str"):
    return d.represent_scalar("tag:yaml.org,2002:str", str(s), style=None)


def _repr_dict(d: yaml.Dumper, m: dict):
    items = sorted(m.items(), key=functools.cmp_to_key(
        lambda x, y: -1 if keylist_less(x[0], y[0]) else (1 if keylist_less(y[0], x[0]) else 0)))
    return d.represent_mapping("tag:yaml.org,2002:map", items)


_Dumper.add_representer(str, _repr_str)
_Dumper.add_representer(_Str, _repr_plain)
_Dumper.add_representer(dict, _repr_dict)


def _v2_value(v):
    """yaml.v2's decode of a JSON value, with scalars pre-rendered as plain text."""
    if v is None:
        return _Str("null")
    if v is True or v is False:
        return _Str("true" if v else "false")
    if isinstance(v, int):
        return _Str(str(v))
    if isinstance(v, float):
        return _Str(go_format_g(v))
    if isinstance(v, list):
        return [_v2_value(x) for x in v]
    if isinstance(v, dict):
        return {k: _v2_value(x) for k, x in v.items()}
    return v


def _yaml_ints_floats(text: str):
    """json.Unmarshal-like parse keeping ints as int (yaml.v2 picks int/uint64 when the literal parses)."""
    return json.loads(text, parse_int=int, parse_float=float)


def sigs_yaml_marshal(obj) -> str:
    """sigs.k8s.io/yaml.Marshal of a JSON-shaped value."""
    return yaml.dump(_v2_value(obj), Dumper=_Dumper, default_flow_style=False, allow_unicode=True,
                     width=80, indent=2, sort_keys=False)


def graph_yaml(g: ServiceGraph) -> str:
    """yaml.Marshal(graph): JSONToYAML(json.Marshal(graph)) (kubernetes.go:161)."""
    return sigs_yaml_marshal(_yaml_ints_floats(marshal_service_graph(g).decode("utf-8")))


# ---------------------------------------------------------- the objects -----
def _ts(unix_s: int) -> str:
    return datetime.datetime.fromtimestamp(unix_s, datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def _meta(ts: str, name: str, ns: Optional[str], labels: Dict[str, str], annotations=None) -> dict:
    m: Dict[str, Any] = {"name": name, "creationTimestamp": ts}
    if ns:
        m["namespace"] = ns
    if labels:
        m["labels"] = dict(labels)
    if annotations:
        m["annotations"] = dict(annotations)
    return m


def make_namespace(ts):
    return {"kind": "Namespace", "apiVersion": "v1",
            "metadata": _meta(ts, NAMESPACE, None, {"istio-injection": "enabled"}), "spec": {}, "status": {}}


def make_config_map(ts, g: ServiceGraph):
    return {"kind": "ConfigMap", "apiVersion": "v1",
            "metadata": _meta(ts, "service-graph-config", NAMESPACE, {"app": "service-graph"}),
            "data": {"service-graph": graph_yaml(g)}}


def make_service(ts, s):
    return {"kind": "Service", "apiVersion": "v1",
            "metadata": _meta(ts, s.name, NAMESPACE, {"app": "service-graph"}),
            "spec": {"ports": [{"name": "http-web", "port": 8080, "targetPort": 0}], "selector": {"name": s.name}},
            "status": {"loadBalancer": {}}}


def make_deployment(ts, s, node_selector, image, idle):
    env = [{"name": "SERVICE_NAME", "value": s.name} if s.name else {"name": "SERVICE_NAME"}]
    for name, path in (("PODNAME", "metadata.name"), ("PODIP", "status.podIP"), ("NAMESPACE", "metadata.namespace"),
                       ("NODENAME", "spec.nodeName")):
        env.append({"name": name, "valueFrom": {"fieldRef": {"fieldPath": path}}})
    ctr: Dict[str, Any] = {"name": "mock-service", "args": ["--max-idle-connections-per-host=%d" % idle],
                           "ports": [{"containerPort": 8080}], "env": env, "resources": {},
                           "volumeMounts": [{"name": "config-volume", "mountPath": "/etc/config"}],
                           "imagePullPolicy": "IfNotPresent"}
    if image:
        ctr["image"] = image
    pod: Dict[str, Any] = {"volumes": [{"name": "config-volume", "configMap": {
        "name": "service-graph-config", "items": [{"key": "service-graph", "path": "service-graph.yaml"}]}}],
        "containers": [ctr]}
    if node_selector:
        pod["nodeSelector"] = dict(node_selector)
    return {"kind": "Deployment", "apiVersion": "apps/v1",
            "metadata": _meta(ts, s.name, NAMESPACE, {"app": "service-graph"}),
            "spec": {"replicas": s.num_replicas, "selector": {"matchLabels": {"name": s.name}},
                     "template": {"metadata": {"creationTimestamp": ts, "labels": {"role": "service", "name": s.name},
                                               "annotations": {"prometheus.io/scrape": "true"}},
                                  "spec": pod},
                     "strategy": {}},
            "status": {}}


def make_fortio_deployment(ts, node_selector, image):
    ctr: Dict[str, Any] = {"name": "fortio-client", "args": ["server"],
                           "ports": [{"containerPort": 8080}, {"containerPort": 42422}], "resources": {}}
    if image:
        ctr["image"] = image
    pod: Dict[str, Any] = {"containers": [ctr]}
    if node_selector:
        pod["nodeSelector"] = dict(node_selector)
    return {"kind": "Deployment", "apiVersion": "apps/v1", "metadata": _meta(ts, "client", None, {"app": "client"}),
            "spec": {"selector": {"matchLabels": {"app": "client"}},
                     "template": {"metadata": {"creationTimestamp": ts, "labels": {"app": "client"}}, "spec": pod},
                     "strategy": {}},
            "status": {}}


def make_fortio_service(ts):
    return {"kind": "Service", "apiVersion": "v1",
            "metadata": _meta(ts, "client", None, {"app": "client"}, {"prometheus.io/scrape": "true"}),
            "spec": {"ports": [{"port": 8080, "targetPort": 0}], "selector": {"app": "client"}},
            "status": {"loadBalancer": {}}}


def rule_uuid(seed: int, i: int) -> str:
    w = philox.philox4x32_10((i & 0xFFFFFFFF, i >> 32, 0, 0x4B385300), (seed & 0xFFFFFFFF, seed >> 32))
    b = bytearray(b"".join(int(x).to_bytes(4, "little") for x in w))
    b[6] = (b[6] & 0x0F) | 0x40
    b[8] = (b[8] & 0x3F) | 0x80
    h = b.hex()
    return f"{h[:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:]}"


def rbac_policy(name: str, allow_all: bool, rule: str) -> str:
    """rbac.go:25-57 (fmt.Sprintf of the template)."""
    user = "*" if allow_all else rule
    return (f'\napiVersion: "rbac.istio.io/v1alpha1"\nkind: ServiceRole\nmetadata:\n  name: {rule}\n'
            f'  namespace: {NAMESPACE}\nspec:\n  rules:\n  - services: ["{name}.{NAMESPACE}.*"]\n'
            f'    methods: ["*"]\n---\napiVersion: "rbac.istio.io/v1alpha1"\nkind: ServiceRoleBinding\n'
            f'metadata:\n  name: {rule}\n  namespace: {NAMESPACE}\nspec:\n  subjects:\n  - user: "{user}"\n'
            f'  roleRef:\n    kind: ServiceRole\n    name: "{rule}"\n')


def rbac_config() -> str:
    return (f'\napiVersion: "rbac.istio.io/v1alpha1"\nkind: RbacConfig\nmetadata:\n  name: default\n'
            f"spec:\n  mode: 'ON_WITH_INCLUSION'\n  inclusion:\n    namespaces: [\"{NAMESPACE}\"]\n")


def manifests(g: ServiceGraph, service_node_selector=None, service_image="", idle=0, client_node_selector=None,
              client_image="", environment_name="NONE", creation_timestamp_s=0, rbac_seed=0) -> str:
    """kubernetes.go:56-137."""
    ts = _ts(creation_timestamp_s)
    docs: List[str] = [sigs_yaml_marshal(make_namespace(ts)), sigs_yaml_marshal(make_config_map(ts, g))]
    istio = environment_name.lower() == "istio"
    has_rbac, rule = False, 0
    for s in g.services:
        docs.append(sigs_yaml_marshal(make_deployment(ts, s, service_node_selector, service_image, idle)))
        docs.append(sigs_yaml_marshal(make_service(ts, s)))
        if istio and s.num_rbac_policies > 0:
            has_rbac = True
            for _ in range(s.num_rbac_policies):
                docs.append(rbac_policy(s.name, False, rule_uuid(rbac_seed, rule)))
                rule += 1
            docs.append(rbac_policy(s.name, True, rule_uuid(rbac_seed, rule)))
            rule += 1
    docs.append(sigs_yaml_marshal(make_fortio_deployment(ts, client_node_selector, client_image)))
    docs.append(sigs_yaml_marshal(make_fortio_service(ts)))
    if has_rbac:
        docs.append(rbac_config())
    return "---\n".join(docs)
