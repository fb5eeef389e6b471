"""Restatement of isotope's graph encoders (oracle — test infrastructure only;
never imported by the product).

  json.Marshal(graph.ServiceGraph)
      svc/service.go:25-51            field order, json tags, omitempty
      script/script.go:24-31          Script.MarshalJSON
      script/command.go:30-53         commandsToMarshallable / commandToMarshallable
      script/request_command.go:26-33 RequestCommand fields
      size/byte_size.go:27-34         ByteSize.String / MarshalJSON (go-units BytesSize)
      pct/percentage.go:28-35         Percentage.String / MarshalJSON
      svctype/service_type.go:34-48   ServiceType.String / MarshalJSON
    plus Go 1.16 encoding/json's float and (HTML-escaping) string encoders.
  graphviz.ServiceGraphToGraph       convert/pkg/graphviz/graphviz.go:59-213
  text/template execution of the subset graphvizTemplate uses (range with and
  without variables, if, field and variable printing, {{- -}} trimming), so a
  DOT fixture can be rendered from the reference's own template text
  (tests/golden/make_dot_fixtures.py).
"""
from __future__ import annotations

import math
import re
from decimal import Decimal
from typing import Any, Dict, List

from . import gounits as gu
from .graph_ref import (SERVICE_GRPC, SERVICE_HTTP, ConcurrentCommand, RequestCommand, ServiceGraph,
                        SleepCommand)

# ------------------------------------------------------- encoding/json ------
_HEX = "0123456789abcdef"


def go_json_string(s) -> bytes:
    """encodeState.string(s, escapeHTML=true) (Go 1.16 encoding/json/encode.go)."""
    b = s.encode("utf-8", "surrogatepass") if isinstance(s, str) else bytes(s)
    out = bytearray(b'"')
    i = 0
    while i < len(b):
        c = b[i]
        if c < 0x80:
            if c >= 0x20 and c not in b'"\\<>&':
                out.append(c)
            elif c in b'"\\':
                out += b"\\" + bytes([c])
            elif c == 0x0A:
                out += b"\\n"
            elif c == 0x0D:
                out += b"\\r"
            elif c == 0x09:
                out += b"\\t"
            else:
                out += b"\\u00" + _HEX[c >> 4].encode() + _HEX[c & 15].encode()
            i += 1
            continue
        # utf8.DecodeRuneInString: longest valid sequence of 2..4 bytes
        size = 0
        for n in (2, 3, 4):
            try:
                ch = b[i:i + n].decode("utf-8")
            except UnicodeDecodeError:
                continue
            if len(ch) == 1:
                size = n
                break
        if size == 0:
            out += b"\\ufffd"
            i += 1
            continue
        r = ord(b[i:i + size].decode("utf-8"))
        if r in (0x2028, 0x2029):
            out += b"\\u202" + _HEX[r & 15].encode()
        else:
            out += b[i:i + size]
        i += size
    out += b'"'
    return bytes(out)


def go_json_float(f: float) -> bytes:
    """floatEncoder (bits 64): strconv.AppendFloat(f, 'f' | 'e', -1, 64), 'e'
    when |f| < 1e-6 or >= 1e21, then the e-0X cleanup."""
    if math.isnan(f) or math.isinf(f):
        raise ValueError("json: unsupported value")
    a = abs(f)
    d = Decimal(repr(f))  # repr: shortest digits that round-trip
    if a != 0 and (a < 1e-6 or a >= 1e21):
        sign, digits, exp = d.as_tuple()
        ds = "".join(map(str, digits)).rstrip("0") or "0"
        e10 = exp + len(digits) - 1
        mant = ds[0] + ("." + ds[1:] if len(ds) > 1 else "")
        s = ("-" if sign else "") + mant + "e" + ("-" if e10 < 0 else "+") + "%02d" % abs(e10)
        if len(s) >= 4 and s[-4] == "e" and s[-3] == "-" and s[-2] == "0":
            s = s[:-2] + s[-1]
        return s.encode()
    s = format(d, "f")
    if "." in s:
        s = s.rstrip("0").rstrip(".")
    if s in ("-0", ""):
        s = "-0" if math.copysign(1, f) < 0 else "0"
    return s.encode()


def _type_string(t: int) -> str:
    """svctype/service_type.go:34-42"""
    return {SERVICE_HTTP: "HTTP", SERVICE_GRPC: "gRPC"}.get(t, "")


def _marshal_cmd(c) -> bytes:
    """script/command.go:42-53"""
    if isinstance(c, SleepCommand):
        return b'{"sleep":' + go_json_string(gu.duration_string(c.ns)) + b"}"
    if isinstance(c, RequestCommand):
        o = b'{"call":{"service":' + go_json_string(c.service) + b',"size":' + \
            go_json_string(gu.bytes_size(float(c.size)))
        if c.probability:
            o += b',"probability":' + str(c.probability).encode()
        return o + b"}}"
    return b"[" + b",".join(_marshal_cmd(x) for x in c.commands) + b"]"


def marshal_service(s) -> bytes:
    """json.Marshal(svc.Service): svc/service.go:25-51 tags, omitempty."""
    o = b'{"name":' + go_json_string(s.name)
    if s.type != 0:
        o += b',"type":' + go_json_string(_type_string(s.type).lower())
    if s.num_replicas != 0:
        o += b',"numReplicas":' + str(s.num_replicas).encode()
    if s.is_entrypoint:
        o += b',"isEntrypoint":true'
    if s.error_rate != 0:
        o += b',"errorRate":' + go_json_float(s.error_rate)
    if s.response_size != 0:
        o += b',"responseSize":' + go_json_string(gu.bytes_size(float(s.response_size)))
    if s.script:
        o += b',"script":[' + b",".join(_marshal_cmd(c) for c in s.script) + b"]"
    return o + b',"numRbacPolicies":' + str(s.num_rbac_policies).encode() + b"}"


def marshal_service_graph(g: ServiceGraph) -> bytes:
    """json.Marshal(graph.ServiceGraph) (graph.go:21-23)."""
    if not g.services:
        return b'{"services":' + (b"null" if g.services_nil else b"[]") + b"}"
    return b'{"services":[' + b",".join(marshal_service(s) for s in g.services) + b"]}"


# ------------------------------------------------------------- graphviz -----
def _step_string(c) -> str:
    """graphviz.go:170-181 nonConcurrentCommandToString"""
    if isinstance(c, SleepCommand):
        return "SLEEP " + gu.duration_string(c.ns)
    return 'CALL "%s" %s' % (c.service, gu.bytes_size(float(c.size)))


def service_graph_to_graph(g: ServiceGraph) -> Dict[str, Any]:
    """graphviz.go:59-75 ServiceGraphToGraph / 147-168 toGraphvizNode /
    128-145 getEdgesFromExe / 183-213 executableToStringSlice."""
    nodes, edges = [], []
    for s in g.services:
        steps = []
        for idx, exe in enumerate(s.script):
            if isinstance(exe, ConcurrentCommand):
                steps.append([_step_string(c) for c in exe.commands])
                for c in exe.commands:
                    if isinstance(c, RequestCommand):
                        edges.append({"From": s.name, "To": c.service, "StepIndex": idx})
            else:
                steps.append([_step_string(exe)])
                if isinstance(exe, RequestCommand):
                    edges.append({"From": s.name, "To": exe.service, "StepIndex": idx})
        nodes.append({"Name": s.name, "Type": _type_string(s.type), "ErrorRate": gu.pct_string(s.error_rate),
                      "ResponseSize": gu.bytes_size(float(s.response_size)), "Steps": steps})
    return {"Nodes": nodes, "Edges": edges}


# ------------------------------------------------- text/template subset -----
_ACTION = re.compile(r"\{\{(- )?(.*?)( -)?\}\}", re.S)


def _parse(tmpl: str):
    """Split into text / action tokens applying the trim markers
    (text/template: "{{- " trims preceding, " -}}" following white space)."""
    toks: List[list] = []
    pos = 0
    for m in _ACTION.finditer(tmpl):
        toks.append(["text", tmpl[pos:m.start()]])
        toks.append(["act", m.group(2).strip(), bool(m.group(1)), bool(m.group(3))])
        pos = m.end()
    toks.append(["text", tmpl[pos:]])
    for i, t in enumerate(toks):
        if t[0] != "act":
            continue
        if t[2] and i > 0:
            toks[i - 1][1] = toks[i - 1][1].rstrip(" \t\r\n")
        if t[3] and i + 1 < len(toks):
            toks[i + 1][1] = toks[i + 1][1].lstrip(" \t\r\n")
    # build a tree
    root: List[Any] = []
    stack = [root]
    for t in toks:
        if t[0] == "text":
            if t[1]:
                stack[-1].append(("text", t[1]))
            continue
        a = t[1]
        if a.startswith("range ") or a.startswith("if "):
            node = (a.split(" ", 1)[0], a.split(" ", 1)[1], [])
            stack[-1].append(node)
            stack.append(node[2])
        elif a == "end":
            stack.pop()
        else:
            stack[-1].append(("print", a))
    assert len(stack) == 1, "unbalanced template"
    return root


def _eval(expr: str, dot, env):
    expr = expr.strip()
    if expr == ".":
        return dot
    if expr.startswith("$"):
        return env[expr]
    if expr.startswith("."):
        v = dot
        for f in expr[1:].split("."):
            v = v[f]
        return v
    raise ValueError("unsupported pipeline " + expr)


def _exec(nodes, dot, env, out: List[str]):
    for n in nodes:
        if n[0] == "text":
            out.append(n[1])
        elif n[0] == "print":
            v = _eval(n[1], dot, env)
            out.append(str(v) if not isinstance(v, bool) else ("true" if v else "false"))
        elif n[0] == "if":
            v = _eval(n[1], dot, env)
            if v:  # Go truth: non-zero number, non-empty string/slice
                _exec(n[2], dot, env, out)
        else:  # range [$i, $v :=] pipeline
            m = re.match(r"^\s*(\$\w+)\s*,\s*(\$\w+)\s*:=\s*(.*)$", n[1])
            seq = _eval(m.group(3) if m else n[1], dot, env)
            for i, item in enumerate(seq):
                e2 = dict(env)
                if m:
                    e2[m.group(1)] = i
                    e2[m.group(2)] = item
                _exec(n[2], item, e2, out)


def execute_template(tmpl: str, data) -> str:
    out: List[str] = []
    _exec(_parse(tmpl), data, {"$": data}, out)
    return "".join(out)
