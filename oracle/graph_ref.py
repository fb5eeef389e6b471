"""Restatement of the isotope service-graph loader (oracle — test
infrastructure only).

Follows, rule by rule:
  isotope/convert/pkg/graph/unmarshal.go:30-48   (*ServiceGraph).UnmarshalJSON
  isotope/convert/pkg/graph/unmarshal.go:50-62   parseJSONServiceGraphWithDefaults
  isotope/convert/pkg/graph/unmarshal.go:64-112  defaultDefaults / defaults / withGlobalDefaults
  isotope/convert/pkg/graph/validation.go:28-82  validate / validateCommands / errors
  isotope/convert/pkg/graph/svc/unmarshal.go:25-47 DefaultService / (*Service).UnmarshalJSON / ErrEmptyName
  isotope/convert/pkg/graph/svc/service.go:25-51 Service fields
  isotope/convert/pkg/graph/script/command.go:55-175 command decoding + errors
  isotope/convert/pkg/graph/script/request_command.go:26-68
  isotope/convert/pkg/graph/script/sleep_command.go:26-38
  isotope/convert/pkg/graph/size/byte_size.go:39-83
  isotope/convert/pkg/graph/pct/percentage.go:41-93
  isotope/convert/pkg/graph/svctype/service_type.go:51-85
and the parts of Go's encoding/json those methods rely on: case-insensitive
field matching (ASCII fold, exact match preferred), unknown keys ignored,
``null`` is a no-op for plain fields but is passed to custom UnmarshalJSON
methods, type mismatches on plain fields are *saved* (decoding continues,
the first is returned at the end of that json.Unmarshal call) while errors
from custom UnmarshalJSON methods abort.

Input is the JSON text sigs.k8s.io/yaml would hand to UnmarshalJSON; numbers
are kept as their literal text so integer-vs-float decoding follows Go.
"""
from __future__ import annotations

import json
import struct
from dataclasses import dataclass, field
from typing import Any, List, Optional

from . import gounits as gu


# ------------------------------------------------------------- JSON DOM ---
class Num(str):
    """A JSON number kept as its literal text."""


class Obj(list):
    """A JSON object as an ordered list of (key, value) pairs."""


def _reject_constant(c):
    raise ValueError(f"invalid character in JSON: {c}")


def loads(text) -> Any:
    if isinstance(text, (bytes, bytearray)):
        text = text.decode("utf-8")
    return json.loads(text, parse_int=Num, parse_float=Num,
                      parse_constant=_reject_constant, object_pairs_hook=Obj)


# ---------------------------------------------------------------- errors --
class UnmarshalTypeError(gu.GoError):
    def __init__(self, value: str, gotype: str):
        super().__init__(f"json: cannot unmarshal {value} into Go value of type {gotype}")


class ErrRequestToUndefinedService(gu.GoError):
    """validation.go:71-77"""

    def __init__(self, name: str):
        self.name = name
        super().__init__(f'cannot call undefined service "{name}"')


class ErrNestedConcurrentCommand(gu.GoError):
    """validation.go:79-82"""

    def __init__(self):
        super().__init__("concurrent commands may not be nested")


class ErrEmptyName(gu.GoError):
    """svc/unmarshal.go:45-47"""

    def __init__(self):
        super().__init__("services must have a name")


class UnknownCommandKeyError(gu.GoError):
    """script/command.go:167-175"""

    def __init__(self, key: str):
        self.key = key
        super().__init__(f"unknown command: {key}")


class MultipleKeysInCommandMapError(gu.GoError):
    """script/command.go:157-165"""

    def __init__(self, keys):
        self.keys = list(keys)
        super().__init__(f"multiple keys for command: {self.keys}")


class InvalidProbabilityError(gu.GoError):
    """script/request_command.go:61-63"""

    def __init__(self):
        super().__init__("math: invalid probability, outside range: [0,100]")


class InvalidServiceTypeStringError(gu.GoError):
    """svctype/service_type.go:77-85"""

    def __init__(self, s: str):
        self.s = s
        super().__init__(f"unknown service type: {s}")


# ----------------------------------------------------------------- model --
SERVICE_UNKNOWN, SERVICE_HTTP, SERVICE_GRPC = 0, 1, 2


@dataclass
class SleepCommand:
    ns: int                     # time.Duration (script/sleep_command.go:23)


@dataclass
class RequestCommand:
    service: str = ""
    size: int = 0
    probability: int = 0


@dataclass
class ConcurrentCommand:
    commands: List[Any] = field(default_factory=list)


@dataclass
class Service:
    name: str = ""
    type: int = SERVICE_HTTP
    num_replicas: int = 1
    is_entrypoint: bool = False
    error_rate: float = 0.0
    response_size: int = 0
    script: List[Any] = field(default_factory=list)
    num_rbac_policies: int = 0


@dataclass
class ServiceGraph:
    services: List[Service] = field(default_factory=list)
    services_nil: bool = True   # Go nil slice (key absent / null): json.Marshal writes null


# ------------------------------------------------------- decode helpers ---
def _kind(v) -> str:
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, Num):
        return "number"
    if isinstance(v, str):
        return "string"
    if isinstance(v, Obj):
        return "object"
    return "array"


class _Saver:
    """Go decodeState.saveError: keep the first plain-field type error."""

    def __init__(self):
        self.err: Optional[Exception] = None

    def save(self, e: Exception):
        if self.err is None:
            self.err = e

    def done(self):
        if self.err is not None:
            raise self.err


def _match_field(key: str, names: List[str]) -> Optional[str]:
    if key in names:
        return key
    low = key.lower()
    for n in names:
        if n.lower() == low:
            return n
    return None


def _dec_string(v, sv: _Saver, cur: str) -> str:
    if v is None:
        return cur
    if _kind(v) != "string":
        sv.save(UnmarshalTypeError(_kind(v), "string"))
        return cur
    return str(v)


def _dec_bool(v, sv: _Saver, cur: bool) -> bool:
    if v is None:
        return cur
    if not isinstance(v, bool):
        sv.save(UnmarshalTypeError(_kind(v), "bool"))
        return cur
    return v


def _dec_int(v, sv: _Saver, cur: int, bits: int) -> int:
    if v is None:
        return cur
    if _kind(v) != "number":
        sv.save(UnmarshalTypeError(_kind(v), f"int{bits}"))
        return cur
    try:
        return gu.parse_int(str(v), bits)
    except ValueError:
        sv.save(UnmarshalTypeError("number " + str(v), f"int{bits}"))
        return cur


def _unmarshal_float64(v) -> float:
    """json.Unmarshal(b, &f) for a float64 (its own Unmarshal call)."""
    if v is None:
        return 0.0
    if _kind(v) != "number":
        raise UnmarshalTypeError(_kind(v), "float64")
    try:
        return gu.parse_float(str(v))
    except gu.ParseFloatError:
        raise UnmarshalTypeError("number " + str(v), "float64") from None


def _unmarshal_string(v, gotype="string") -> str:
    if v is None:
        return ""
    if _kind(v) != "string":
        raise UnmarshalTypeError(_kind(v), gotype)
    return str(v)


def _unmarshal_int64(v) -> int:
    if v is None:
        return 0
    if _kind(v) != "number":
        raise UnmarshalTypeError(_kind(v), "int64")
    try:
        return gu.parse_int(str(v), 64)
    except ValueError:
        raise UnmarshalTypeError("number " + str(v), "int64") from None


# -------------------------------------------------- custom UnmarshalJSON --
def unmarshal_byte_size(v) -> int:
    """size/byte_size.go:39-63"""
    if _kind(v) == "string":
        return gu.size_from_string(str(v))
    return gu.size_from_int64(_unmarshal_int64(v))


def unmarshal_percentage(v) -> float:
    """pct/percentage.go:41-67"""
    if _kind(v) == "string":
        return gu.pct_from_string(str(v))
    return gu.pct_from_float(_unmarshal_float64(v))


def unmarshal_service_type(v) -> int:
    """svctype/service_type.go:51-76"""
    s = _unmarshal_string(v)
    if s == "http":
        return SERVICE_HTTP
    if s == "grpc":
        return SERVICE_GRPC
    raise InvalidServiceTypeStringError(s)


def unmarshal_sleep(v) -> SleepCommand:
    """script/sleep_command.go:26-38"""
    return SleepCommand(gu.parse_duration(_unmarshal_string(v)))


def unmarshal_request(v, default: RequestCommand) -> RequestCommand:
    """script/request_command.go:41-66"""
    c = RequestCommand(default.service, default.size, default.probability)
    if _kind(v) == "string":
        c.service = str(v)
        return c
    # json.Unmarshal(b, &unmarshallableRequestCommand)
    sv = _Saver()
    if v is None:
        pass
    elif _kind(v) != "object":
        raise UnmarshalTypeError(_kind(v), "script.unmarshallableRequestCommand")
    else:
        for key, val in v:
            f = _match_field(key, ["service", "size", "probability"])
            if f == "service":
                c.service = _dec_string(val, sv, c.service)
            elif f == "size":
                c.size = unmarshal_byte_size(val)
            elif f == "probability":
                c.probability = _dec_int(val, sv, c.probability, 64)
    sv.done()
    if c.probability < 0 or c.probability > 100:
        raise InvalidProbabilityError()
    return c


def _parse_command_key(v) -> str:
    """script/command.go:107-121 parseJSONCommandKey."""
    if v is None:
        return ""
    if _kind(v) != "object":
        raise UnmarshalTypeError(_kind(v), "map[string]interface {}")
    keys = []
    for k, _ in v:
        if k not in keys:
            keys.append(k)
    if len(keys) > 1:
        raise MultipleKeysInCommandMapError(keys)
    return keys[0] if keys else ""


def unmarshal_command(v, default_req: RequestCommand):
    """script/command.go:73-105 (*unmarshallableCommand).UnmarshalJSON."""
    if _kind(v) == "array":
        return ConcurrentCommand(parse_commands(v, default_req))
    key = _parse_command_key(v)
    if key == "sleep":
        cmd = None
        for k, val in v:
            if k == "sleep":
                cmd = unmarshal_sleep(val)
        return cmd
    if key == "call":
        cmd = None
        for k, val in v:
            if k == "call":
                cmd = unmarshal_request(val, default_req)
        return cmd
    raise UnknownCommandKeyError(key)


def parse_commands(v, default_req: RequestCommand) -> List[Any]:
    """script/command.go:55-68 parseJSONCommands (Script / ConcurrentCommand)."""
    if v is None:
        return []
    if _kind(v) != "array":
        raise UnmarshalTypeError(_kind(v), "[]script.unmarshallableCommand")
    return [unmarshal_command(e, default_req) for e in v]


_SERVICE_FIELDS = ["name", "type", "numReplicas", "isEntrypoint", "errorRate",
                   "responseSize", "script", "numRbacPolicies"]


def unmarshal_service(v, default: Service, default_req: RequestCommand) -> Service:
    """svc/unmarshal.go:29-41 (*Service).UnmarshalJSON."""
    s = Service(default.name, default.type, default.num_replicas, default.is_entrypoint,
                default.error_rate, default.response_size, list(default.script),
                default.num_rbac_policies)
    sv = _Saver()
    if v is None:
        pass
    elif _kind(v) != "object":
        raise UnmarshalTypeError(_kind(v), "svc.unmarshallableService")
    else:
        for key, val in v:
            f = _match_field(key, _SERVICE_FIELDS)
            if f == "name":
                s.name = _dec_string(val, sv, s.name)
            elif f == "type":
                s.type = unmarshal_service_type(val)
            elif f == "numReplicas":
                s.num_replicas = _dec_int(val, sv, s.num_replicas, 32)
            elif f == "isEntrypoint":
                s.is_entrypoint = _dec_bool(val, sv, s.is_entrypoint)
            elif f == "errorRate":
                s.error_rate = unmarshal_percentage(val)
            elif f == "responseSize":
                s.response_size = unmarshal_byte_size(val)
            elif f == "script":
                s.script = parse_commands(val, default_req)
            elif f == "numRbacPolicies":
                s.num_rbac_policies = _dec_int(val, sv, s.num_rbac_policies, 32)
    sv.done()
    if s.name == "":
        raise ErrEmptyName()
    return s


@dataclass
class Defaults:
    """unmarshal.go:78-86"""
    type: int = SERVICE_HTTP
    error_rate: float = 0.0
    response_size: int = 0
    script: List[Any] = field(default_factory=list)
    request_size: int = 0
    num_replicas: int = 1
    num_rbac_policies: int = 0


_DEFAULTS_FIELDS = ["type", "errorRate", "responseSize", "script", "requestSize",
                    "numReplicas", "numRbacPolicies"]


def _decode_defaults(doc) -> Defaults:
    """json.Unmarshal(b, &serviceGraphJSONMetadata{Defaults: defaultDefaults})
    (unmarshal.go:31-32). The default script is decoded with the *current*
    DefaultRequestCommand, i.e. the zero value (quirk F11)."""
    d = Defaults()
    sv = _Saver()
    zero_req = RequestCommand()
    if doc is None:
        return d
    if _kind(doc) != "object":
        raise UnmarshalTypeError(_kind(doc), "graph.serviceGraphJSONMetadata")
    for key, val in doc:
        if _match_field(key, ["defaults"]) is None or val is None:
            continue
        if _kind(val) != "object":
            sv.save(UnmarshalTypeError(_kind(val), "graph.defaults"))
            continue
        for k2, v2 in val:
            f = _match_field(k2, _DEFAULTS_FIELDS)
            if f == "type":
                d.type = unmarshal_service_type(v2)
            elif f == "errorRate":
                d.error_rate = unmarshal_percentage(v2)
            elif f == "responseSize":
                d.response_size = unmarshal_byte_size(v2)
            elif f == "script":
                d.script = parse_commands(v2, zero_req)
            elif f == "requestSize":
                d.request_size = unmarshal_byte_size(v2)
            elif f == "numReplicas":
                d.num_replicas = _dec_int(v2, sv, d.num_replicas, 32)
            elif f == "numRbacPolicies":
                d.num_rbac_policies = _dec_int(v2, sv, d.num_rbac_policies, 32)
    sv.done()
    return d


def validate(g: ServiceGraph) -> None:
    """validation.go:28-57"""
    names = {s.name for s in g.services}

    def contains_conc(cmds):
        return any(isinstance(c, ConcurrentCommand) for c in cmds)

    def validate_commands(cmds):
        for c in cmds:
            if isinstance(c, RequestCommand):
                if c.service not in names:
                    raise ErrRequestToUndefinedService(c.service)
            elif isinstance(c, ConcurrentCommand):
                validate_commands(c.commands)
                if contains_conc(c.commands):
                    raise ErrNestedConcurrentCommand()

    for s in g.services:
        validate_commands(s.script)


def unmarshal_service_graph(text) -> ServiceGraph:
    """(*ServiceGraph).UnmarshalJSON, unmarshal.go:30-48."""
    doc = loads(text)
    d = _decode_defaults(doc)
    # withGlobalDefaults (unmarshal.go:88-112)
    default_service = Service(name="", type=d.type, num_replicas=d.num_replicas,
                              is_entrypoint=False, error_rate=d.error_rate,
                              response_size=d.response_size, script=d.script,
                              num_rbac_policies=d.num_rbac_policies)
    default_req = RequestCommand(service="", size=d.request_size, probability=0)
    g = ServiceGraph()
    sv = _Saver()
    if doc is not None:
        for key, val in doc:
            if _match_field(key, ["services"]) is None:
                continue
            if val is None:
                g.services = []
                g.services_nil = True
                continue
            if _kind(val) != "array":
                sv.save(UnmarshalTypeError(_kind(val), "[]svc.Service"))
                continue
            g.services = [unmarshal_service(e, default_service, default_req) for e in val]
            g.services_nil = False
    sv.done()
    validate(g)
    return g


# ----------------------------------------------------- canonical dump -----
def _cmd_canon(c):
    if isinstance(c, SleepCommand):
        return ["sleep", c.ns]
    if isinstance(c, RequestCommand):
        return ["call", c.service, c.size, c.probability]
    return ["conc", [_cmd_canon(x) for x in c.commands]]


def canonical(g: ServiceGraph) -> dict:
    """Exact, implementation-neutral dump used to compare loaders."""
    return {"services": [{
        "name": s.name, "type": s.type, "numReplicas": s.num_replicas,
        "isEntrypoint": s.is_entrypoint,
        "errorRateBits": struct.unpack("<Q", struct.pack("<d", s.error_rate))[0],
        "responseSize": s.response_size, "numRbacPolicies": s.num_rbac_policies,
        "script": [_cmd_canon(c) for c in s.script]} for s in g.services]}
