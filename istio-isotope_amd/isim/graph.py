"""Python mirror of isotope's graph API (isotope/convert/pkg/graph), backed by
the C++ loader in libisim.

    ServiceGraph.from_yaml(text)   ~ yaml.Unmarshal(bytes, &sg)  (sigs.k8s.io/yaml)
    ServiceGraph.from_json(text)   ~ json.Unmarshal(bytes, &sg)
                                     -> (*ServiceGraph).UnmarshalJSON, unmarshal.go:30-48
    size_from_string / duration_parse / percentage_from_string
                                   ~ size.FromString, time.ParseDuration, pct.FromString
    ServiceGraph.marshal_json()    ~ json.Marshal(sg)
    ServiceGraph.to_dot()          ~ graphviz.ServiceGraphToDotLanguage(sg)

Load errors raise ``GraphError`` carrying the Go error text.  The decoded
services are exposed as plain dataclasses with the Go field meanings
(svc/service.go:25-51, script/*.go).
"""
from __future__ import annotations

import ctypes as C
import json
from dataclasses import dataclass, field
from typing import Any, List, Optional

from . import native
from .yamljson import yaml_to_json

SERVICE_UNKNOWN, SERVICE_HTTP, SERVICE_GRPC = 0, 1, 2


class GraphError(ValueError):
    """A graph-load error; str() is the Go error text."""


@dataclass
class SleepCommand:
    ns: int


@dataclass
class RequestCommand:
    service: str
    size: int
    probability: int = 0


@dataclass
class ConcurrentCommand:
    commands: List[Any] = field(default_factory=list)


@dataclass
class Service:
    name: str
    type: int
    num_replicas: int
    is_entrypoint: bool
    error_rate: float
    response_size: int
    script: List[Any]
    num_rbac_policies: int


def _cmd(c):
    if c[0] == "sleep":
        return SleepCommand(c[1])
    if c[0] == "call":
        return RequestCommand(c[1], c[2], c[3])
    return ConcurrentCommand([_cmd(x) for x in c[1]])


class ServiceGraph:
    """A loaded, validated service graph (owns a native isim_graph)."""

    def __init__(self, handle: int, json_text: str):
        self._h = C.c_void_p(handle)
        self.json_text = json_text
        self._canon: Optional[dict] = None

    @classmethod
    def from_json(cls, text) -> "ServiceGraph":
        lib = native.load()
        if isinstance(text, str):
            text = text.encode("utf-8")
        out = C.c_void_p()
        rc = lib.isim_graph_unmarshal_json(text, len(text), C.byref(out))
        if rc == native.EPARSE:
            raise GraphError(native.last_error())
        native.check(rc)
        return cls(out.value, text.decode("utf-8"))

    @classmethod
    def from_yaml(cls, text) -> "ServiceGraph":
        return cls.from_json(yaml_to_json(text))

    @classmethod
    def from_yaml_file(cls, path: str) -> "ServiceGraph":
        with open(path, "rb") as f:
            return cls.from_yaml(f.read())

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and native._lib is not None:
            native._lib.isim_graph_free(h)
            self._h = None

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def _text(self, fn) -> bytes:
        n = C.c_size_t()
        native.check(fn(self._h, None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value)
        native.check(fn(self._h, buf, n.value, C.byref(n)))
        return buf.raw[:n.value - 1]

    def canonical(self) -> dict:
        if self._canon is None:
            self._canon = json.loads(self._text(native.load().isim_graph_canonical_json).decode("utf-8"))
        return self._canon

    def marshal_json(self) -> bytes:
        """json.Marshal(graph.ServiceGraph): the bytes Go would produce
        (svc/service.go json tags, script/command.go:30-53)."""
        return self._text(native.load().isim_graph_marshal_json)

    def to_dot(self) -> str:
        """graphviz.ServiceGraphToDotLanguage (convert/pkg/graphviz/graphviz.go:28-41)."""
        return self._text(native.load().isim_graph_to_dot).decode("utf-8")

    def marshal_yaml(self) -> str:
        """yaml.Marshal(graph) through sigs.k8s.io/yaml (the ConfigMap payload
        of convert/pkg/kubernetes/kubernetes.go:159-175)."""
        return self._text(native.load().isim_graph_marshal_yaml).decode("utf-8")

    def to_k8s_manifests(self, service_node_selector: Optional[dict] = None, service_image: str = "",
                         service_max_idle_connections_per_host: int = 0,
                         client_node_selector: Optional[dict] = None, client_image: str = "",
                         environment_name: str = "NONE", creation_timestamp_s: int = 0,
                         rbac_seed: int = 0) -> str:
        """kubernetes.ServiceGraphToKubernetesManifests (kubernetes.go:56-137),
        same argument order.  EXT: creationTimestamp and RBAC rule names are
        deterministic (creation_timestamp_s, rbac_seed) where the reference
        uses time.Now() and uuid.New()."""
        def kv(d):
            items = [x for k, v in (d or {}).items() for x in (str(k).encode(), str(v).encode())]
            arr = (C.c_char_p * max(1, len(items)))(*items)
            return arr, len(items) // 2
        sarr, sn = kv(service_node_selector)
        carr, cn = kv(client_node_selector)
        p = native.K8sParams(service_image.encode(), client_image.encode(), environment_name.encode(),
                             C.cast(sarr, C.c_void_p), C.cast(carr, C.c_void_p), sn, cn,
                             service_max_idle_connections_per_host, 0, creation_timestamp_s,
                             rbac_seed & ((1 << 64) - 1))
        lib = native.load()
        n = C.c_size_t()
        native.check(lib.isim_graph_to_k8s_manifests(self._h, C.byref(p), None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value)
        native.check(lib.isim_graph_to_k8s_manifests(self._h, C.byref(p), buf, n.value, C.byref(n)))
        return buf.raw[:n.value - 1].decode("utf-8")

    @property
    def services(self) -> List[Service]:
        import struct
        out = []
        for s in self.canonical()["services"]:
            out.append(Service(s["name"], s["type"], s["numReplicas"], s["isEntrypoint"],
                               struct.unpack("<d", struct.pack("<Q", s["errorRateBits"]))[0],
                               s["responseSize"], [_cmd(c) for c in s["script"]],
                               s["numRbacPolicies"]))
        return out

    def service_index(self, name: str) -> int:
        return native.load().isim_graph_service_index(self._h, name.encode("utf-8"))

    def __len__(self):
        return native.load().isim_graph_num_services(self._h)


def size_from_string(s: str) -> int:
    out = C.c_uint64()
    rc = native.load().isim_size_from_string(s.encode("utf-8"), C.byref(out))
    if rc == native.EPARSE:
        raise GraphError(native.last_error())
    native.check(rc)
    return out.value


def duration_parse(s: str) -> int:
    out = C.c_int64()
    rc = native.load().isim_duration_parse(s.encode("utf-8"), C.byref(out))
    if rc == native.EPARSE:
        raise GraphError(native.last_error())
    native.check(rc)
    return out.value


def percentage_from_string(s: str) -> float:
    out = C.c_double()
    rc = native.load().isim_percentage_from_string(s.encode("utf-8"), C.byref(out))
    if rc == native.EPARSE:
        raise GraphError(native.last_error())
    native.check(rc)
    return out.value
