"""YAML -> JSON conversion with the behaviour of sigs.k8s.io/yaml v1.2.0
(``yaml.Unmarshal`` = YAMLToJSON over gopkg.in/yaml.v2, then
``json.Unmarshal``), which is how the reference loads every service graph
(isotope/service/pkg/srv/graph.go:82-94, convert/cmd/graphviz.go:37-38).

The product's C++ loader (``isim_graph_from_json``) then applies
``(*ServiceGraph).UnmarshalJSON`` semantics to the JSON text produced here.

Conversion rules mirrored from sigs.k8s.io/yaml + encoding/json:
* YAML 1.1 scalars (PyYAML SafeLoader and yaml.v2 both implement YAML 1.1):
  ints stay ints, floats are re-encoded the way Go's ``json.Marshal`` formats
  a float64 (shortest round-trip digits, no exponent for 1e-6 <= |f| < 1e21,
  so ``1000.0`` becomes ``1000``), bools, nulls, strings.
* Non-string mapping keys are converted to strings as sigs.k8s.io/yaml does
  (ints via decimal, bools "true"/"false", floats via shortest form).
* Mapping order is emitted sorted by key, as Go's ``json.Marshal`` of a
  ``map[string]interface{}`` does.
"""
from __future__ import annotations

import json
import math
from decimal import Decimal

import yaml


def _go_float(f: float) -> str:
    if math.isnan(f) or math.isinf(f):
        raise ValueError(f"json: unsupported value: {f}")
    if f == 0:
        return "-0" if math.copysign(1.0, f) < 0 else "0"
    a = abs(f)
    r = repr(f)
    if 1e-6 <= a < 1e21:
        return format(Decimal(r).normalize(), "f")
    # 'e' format with Go's exponent cleanup (e-07 -> e-7)
    d = Decimal(r).normalize()
    sign, digits, exp = d.as_tuple()
    ds = "".join(map(str, digits))
    e = exp + len(ds) - 1
    mant = ds[0] + ("." + ds[1:] if len(ds) > 1 else "")
    return ("-" if sign else "") + mant + "e" + ("-" if e < 0 else "+") + ("%02d" % abs(e) if abs(e) >= 10 else "%d" % abs(e))


def _key(k) -> str:
    if isinstance(k, str):
        return k
    if isinstance(k, bool):
        return "true" if k else "false"
    if isinstance(k, int):
        return str(k)
    if isinstance(k, float):
        return _go_float(k)
    if k is None:
        return "null"
    raise ValueError(f"unsupported map key type {type(k).__name__}")


def _enc(v, out: list) -> None:
    if v is None:
        out.append("null")
    elif v is True:
        out.append("true")
    elif v is False:
        out.append("false")
    elif isinstance(v, int):
        out.append(str(v))
    elif isinstance(v, float):
        out.append(_go_float(v))
    elif isinstance(v, str):
        out.append(json.dumps(v, ensure_ascii=False))
    elif isinstance(v, dict):
        items = sorted((_key(k), val) for k, val in v.items())
        out.append("{")
        for i, (k, val) in enumerate(items):
            if i:
                out.append(",")
            out.append(json.dumps(k, ensure_ascii=False))
            out.append(":")
            _enc(val, out)
        out.append("}")
    elif isinstance(v, (list, tuple)):
        out.append("[")
        for i, x in enumerate(v):
            if i:
                out.append(",")
            _enc(x, out)
        out.append("]")
    else:
        # timestamps, binary, sets: yaml.v2 would produce strings for most of
        # these; keep them as strings of their YAML text form.
        out.append(json.dumps(str(v), ensure_ascii=False))


def yaml_to_json(text) -> str:
    """sigs.k8s.io/yaml YAMLToJSON for one document."""
    if isinstance(text, (bytes, bytearray)):
        text = text.decode("utf-8")
    doc = yaml.safe_load(text)
    out: list = []
    _enc(doc, out)
    return "".join(out)


def obj_to_json(obj) -> str:
    """Encode an in-memory YAML-like object (dicts/lists/scalars) exactly as
    ``yaml_to_json`` would encode its YAML dump."""
    out: list = []
    _enc(obj, out)
    return "".join(out)
