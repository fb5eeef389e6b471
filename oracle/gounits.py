"""Restatement of the Go / third-party arithmetic used by the isotope graph
loader (oracle — test infrastructure only).

* ``ram_in_bytes`` / ``bytes_size``: github.com/docker/go-units v0.4.0
  (pinned by isotope/go.mod:6), called from
  isotope/convert/pkg/graph/size/byte_size.go:28 (``String``) and :68
  (``FromString``).  Published algorithm: regex
  ``^(\\d+(\\.\\d+)*) ?([kKmMgGtTpP])?[iI]?[bB]?$``, ``strconv.ParseFloat`` of
  group 1, multiplied by the binary unit 1024**k, converted to int64 by Go's
  truncating float->int conversion.  ``BytesSize`` = ``"%.4g%s"`` over
  ``B, KiB, MiB, ...`` dividing by 1024.
* ``parse_duration`` / ``duration_string``: Go stdlib ``time.ParseDuration``
  / ``Duration.String`` (go 1.14/1.16 per isotope/go.mod:3 and
  service/Dockerfile:4), used by script/sleep_command.go:32 and :41.
* ``parse_float``: Go ``strconv.ParseFloat(s, 64)`` syntax (decimal,
  hexadecimal with mandatory ``p`` exponent, inf/infinity/nan), used by
  pct/percentage.go:76 and encoding/json number decoding.
* ``pct_from_string`` / ``pct_from_float`` / ``pct_string``:
  isotope/convert/pkg/graph/pct/percentage.go:71-93 and :28-30.
"""
from __future__ import annotations

import math
import re

INT64_MAX = (1 << 63) - 1
INT64_MIN = -(1 << 63)


class GoError(Exception):
    """Base class: an error value the reference would return."""

    def go_type(self) -> str:
        return type(self).__name__


# ---------------------------------------------------------------- size ----
class NegativeSizeError(GoError):
    """size/error.go:19-26"""

    def __init__(self, size: int):
        self.size = size
        super().__init__(f"{size} must be non-negative")


class InvalidSizeError(GoError):
    """go-units parseSize: fmt.Errorf("invalid size: '%s'", sizeStr)."""

    def __init__(self, s: str):
        self.s = s
        super().__init__(f"invalid size: '{s}'")


_SIZE_RE = re.compile(r"(\d+(\.\d+)*) ?([kKmMgGtTpP])?[iI]?[bB]?\Z", re.ASCII)
_BINARY_MAP = {"k": 1 << 10, "m": 1 << 20, "g": 1 << 30, "t": 1 << 40, "p": 1 << 50}


def go_float_to_int64(f: float) -> int:
    """Go's float64 -> int64 conversion on amd64 (CVTTSD2SQ): truncation toward
    zero; out-of-range and NaN produce INT64_MIN ("integer indefinite")."""
    if math.isnan(f) or f >= 9223372036854775808.0 or f < -9223372036854775808.0:
        return INT64_MIN
    return int(f)


def ram_in_bytes(s: str) -> int:
    """go-units v0.4.0 RAMInBytes -> parseSize(s, binaryMap)."""
    m = _SIZE_RE.match(s)
    if m is None:
        raise InvalidSizeError(s)
    size = parse_float(m.group(1))  # ParseFloat error is returned as-is
    unit = (m.group(3) or "").lower()
    if unit in _BINARY_MAP:
        size *= float(_BINARY_MAP[unit])
    return go_float_to_int64(size)


def size_from_int64(x: int) -> int:
    """size/byte_size.go:76-83 FromInt64."""
    if x < 0:
        raise NegativeSizeError(x)
    return x


def size_from_string(s: str) -> int:
    """size/byte_size.go:67-73 FromString."""
    return size_from_int64(ram_in_bytes(s))


_BINARY_ABBRS = ["B", "KiB", "MiB", "GiB", "TiB", "PiB", "EiB", "ZiB", "YiB"]


def bytes_size(size: float) -> str:
    """go-units BytesSize: CustomSize("%.4g%s", size, 1024.0, binaryAbbrs)."""
    i = 0
    while size >= 1024.0 and i < len(_BINARY_ABBRS) - 1:
        size = size / 1024.0
        i += 1
    return "%.4g%s" % (size, _BINARY_ABBRS[i])


# ------------------------------------------------------------ ParseFloat --
class ParseFloatError(GoError):
    def __init__(self, s: str, why: str = "invalid syntax"):
        self.s = s
        super().__init__(f'strconv.ParseFloat: parsing "{s}": {why}')


_DEC_RE = re.compile(r"[+-]?(\d+(\.\d*)?|\.\d+)([eE][+-]?\d+)?\Z", re.ASCII)
_HEX_RE = re.compile(r"[+-]?0[xX]([0-9a-fA-F]+(\.[0-9a-fA-F]*)?|\.[0-9a-fA-F]+)[pP][+-]?\d+\Z", re.ASCII)


def parse_float(s: str) -> float:
    """Go strconv.ParseFloat(s, 64). Underscore digit separators (accepted by
    Go only after a base prefix) are rejected here: documented deviation."""
    low = s.lower()
    body = low[1:] if low[:1] in ("+", "-") else low
    if body in ("inf", "infinity"):
        return -math.inf if low[:1] == "-" else math.inf
    if low == "nan":
        return math.nan
    if _DEC_RE.match(s):
        f = float(s)
    elif _HEX_RE.match(s):
        sign = -1.0 if s[0] == "-" else 1.0
        f = sign * float.fromhex(s.lstrip("+-"))
    else:
        raise ParseFloatError(s)
    if math.isinf(f):
        raise ParseFloatError(s, "value out of range")
    return f


def parse_int(s: str, bits: int) -> int:
    """Go strconv.ParseInt(s, 10, bits) as used by encoding/json for integer
    fields: optional sign, decimal digits only."""
    if not re.fullmatch(r"[+-]?\d+", s, re.ASCII):
        raise ValueError(f'strconv.ParseInt: parsing "{s}": invalid syntax')
    v = int(s)
    lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
    if v < lo or v > hi:
        raise ValueError(f'strconv.ParseInt: parsing "{s}": value out of range')
    return v


# -------------------------------------------------------------- duration --
class DurationError(GoError):
    pass


_UNIT_NS = {
    b"ns": 1,
    b"us": 1000,
    "µs".encode(): 1000,  # U+00B5 micro sign
    "μs".encode(): 1000,  # U+03BC greek mu
    b"ms": 1000 * 1000,
    b"s": 1000 * 1000 * 1000,
    b"m": 60 * 1000 * 1000 * 1000,
    b"h": 3600 * 1000 * 1000 * 1000,
}


def _quote(b: bytes) -> str:
    return '"' + b.decode("utf-8", "replace") + '"'


def parse_duration(s: str) -> int:
    """Go time.ParseDuration -> int64 nanoseconds.
    Grammar [-+]?([0-9]*(\\.[0-9]*)?[a-z]+)+ ; exact integer arithmetic with
    the float64 fraction step Go uses."""
    orig = s.encode("utf-8")
    b = orig
    d = 0
    neg = False
    if b:
        c = b[:1]
        if c in (b"-", b"+"):
            neg = c == b"-"
            b = b[1:]
    if b == b"0":
        return 0
    if not b:
        raise DurationError("time: invalid duration " + _quote(orig))
    while b:
        if not (b[:1] == b"." or b"0" <= b[:1] <= b"9"):
            raise DurationError("time: invalid duration " + _quote(orig))
        # leadingInt
        pl = len(b)
        v = 0
        i = 0
        while i < len(b) and 48 <= b[i] <= 57:
            if v > INT64_MAX // 10:
                raise DurationError("time: invalid duration " + _quote(orig))
            v = v * 10 + (b[i] - 48)
            if v > INT64_MAX:
                raise DurationError("time: invalid duration " + _quote(orig))
            i += 1
        b = b[i:]
        pre = pl != len(b)
        post = False
        f = 0
        scale = 1.0
        if b[:1] == b".":
            b = b[1:]
            pl = len(b)
            # leadingFraction
            i = 0
            overflow = False
            while i < len(b) and 48 <= b[i] <= 57:
                if not overflow:
                    if f > INT64_MAX // 10:
                        overflow = True
                    else:
                        y = f * 10 + (b[i] - 48)
                        if y > INT64_MAX:
                            overflow = True
                        else:
                            f = y
                            scale *= 10.0
                i += 1
            b = b[i:]
            post = pl != len(b)
        if not pre and not post:
            raise DurationError("time: invalid duration " + _quote(orig))
        i = 0
        while i < len(b):
            c = b[i]
            if c == 46 or 48 <= c <= 57:
                break
            i += 1
        if i == 0:
            raise DurationError("time: missing unit in duration " + _quote(orig))
        u = b[:i]
        b = b[i:]
        if u not in _UNIT_NS:
            raise DurationError("time: unknown unit " + _quote(u) + " in duration " + _quote(orig))
        unit = _UNIT_NS[u]
        if v > INT64_MAX // unit:
            raise DurationError("time: invalid duration " + _quote(orig))
        v *= unit
        if f > 0:
            v += int(float(f) * (float(unit) / scale))
            if v > INT64_MAX:
                raise DurationError("time: invalid duration " + _quote(orig))
        d += v
        if d > INT64_MAX:
            raise DurationError("time: invalid duration " + _quote(orig))
    return -d if neg else d


def _fmt_frac(v: int, prec: int):
    out = ""
    printed = False
    for _ in range(prec):
        digit = v % 10
        printed = printed or digit != 0
        if printed:
            out = chr(48 + digit) + out
        v //= 10
    if printed:
        out = "." + out
    return out, v


def duration_string(d: int) -> str:
    """Go time.Duration.String()."""
    if d == 0:
        return "0s"
    neg = d < 0
    u = (-d) & ((1 << 64) - 1) if neg else d
    if u < 1000 * 1000 * 1000:
        if u < 1000:
            frac, u = _fmt_frac(u, 0)
            s = str(u) + frac + "ns"
        elif u < 1000 * 1000:
            frac, u = _fmt_frac(u, 3)
            s = str(u) + frac + "µs"
        else:
            frac, u = _fmt_frac(u, 6)
            s = str(u) + frac + "ms"
    else:
        frac, u = _fmt_frac(u, 9)
        s = str(u % 60) + frac + "s"
        u //= 60
        if u > 0:
            s = str(u % 60) + "m" + s
            u //= 60
            if u > 0:
                s = str(u) + "h" + s
    return ("-" if neg else "") + s


# ------------------------------------------------------------ percentage --
class InvalidPercentageStringError(GoError):
    """pct/error.go:19-28"""

    def __init__(self, s: str):
        self.s = s
        super().__init__(f'invalid percentage as string: {s} (must be between "0%" and "100%")')


class OutOfRangeError(GoError):
    """pct/error.go:30-38"""

    def __init__(self, f: float):
        self.f = f
        super().__init__(f"percentage {go_float_v(f)} is out of range (must be between 0.0 and 1.0)")


def go_float_v(f: float) -> str:
    """fmt %v of a float64 (strconv 'g' shortest, exponent when exp<-4||exp>=21)."""
    if math.isnan(f):
        return "NaN"
    if math.isinf(f):
        return "+Inf" if f > 0 else "-Inf"
    r = repr(f)
    if "e" in r or "E" in r:
        mant, exp = r.split("e")
        e = int(exp)
        if -4 <= e < 21:
            from decimal import Decimal
            return format(Decimal(r).normalize(), "f")
        return mant + "e" + ("-" if e < 0 else "+") + "%02d" % abs(e)
    if r.endswith(".0"):
        r = r[:-2]
    return r


def pct_from_float(f: float) -> float:
    """pct/percentage.go:85-93 FromFloat64."""
    if 0.0 <= f <= 1.0:
        return f
    raise OutOfRangeError(f)


def pct_from_string(s: str) -> float:
    """pct/percentage.go:71-82 FromString."""
    idx = s.find("%")
    if idx < 0:
        raise InvalidPercentageStringError(s)
    try:
        f = parse_float(s[:idx])
    except ParseFloatError:
        raise InvalidPercentageStringError(s) from None
    return pct_from_float(f / 100.0)


def pct_string(p: float) -> str:
    """pct/percentage.go:28-30: fmt.Sprintf("%0.2f%%", p*100)."""
    return "%0.2f%%" % (p * 100.0)


def error_threshold(p: float) -> int:
    """errorRate p -> u64 threshold over a u32 draw;
    2**32 means 'always'. Multiplying by 2**32 is exact; int() truncates."""
    if p >= 1.0:
        return 1 << 32
    if p <= 0.0:
        return 0
    return int(p * 4294967296.0)
