// Graph emitters (see marshal.h): Go's json.Marshal of a ServiceGraph and the
// graphviz DOT rendering of isotope's convert tool, byte for byte.
#include "marshal.h"

#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>

namespace isim {

// ---------------------------------------------------------------- formats --

// time.Duration.String() (Go src/time/time.go, fmtFrac / fmtInt): integer
// ns, the largest unit that keeps the integer part non-zero below 1 s,
// "h"/"m"/"s" composites above it, trailing fractional zeros dropped.
static void fmt_frac(std::string &frac, uint64_t &v, int prec) {
  bool printed = false;
  std::string out;
  for (int i = 0; i < prec; ++i) {
    const int digit = (int)(v % 10);
    printed = printed || digit != 0;
    if (printed) out.insert(out.begin(), (char)('0' + digit));
    v /= 10;
  }
  frac = printed ? "." + out : "";
}

std::string go_duration_string(int64_t d) {
  if (d == 0) return "0s";
  const bool neg = d < 0;
  uint64_t u = neg ? (uint64_t)0 - (uint64_t)d : (uint64_t)d;
  std::string s, frac;
  if (u < 1000000000ull) {
    const char *unit;
    int prec;
    if (u < 1000ull) {
      prec = 0;
      unit = "ns";
    } else if (u < 1000000ull) {
      prec = 3;
      unit = "\xC2\xB5s";  // U+00B5 MICRO SIGN, as Go writes it
    } else {
      prec = 6;
      unit = "ms";
    }
    fmt_frac(frac, u, prec);
    s = std::to_string(u) + frac + unit;
  } else {
    fmt_frac(frac, u, 9);
    s = std::to_string(u % 60) + frac + "s";
    u /= 60;
    if (u > 0) {
      s = std::to_string(u % 60) + "m" + s;
      u /= 60;
      if (u > 0) s = std::to_string(u) + "h" + s;
    }
  }
  return neg ? "-" + s : s;
}

// go-units v0.4.0: BytesSize(size) = CustomSize("%.4g%s", size, 1024.0,
// binaryAbbrs).  For the values reached here (< 1024 after the divisions)
// Go's %.4g and C's agree: same significant-digit rounding (exact, ties to
// even), same %e switch at exponent >= 4, trailing zeros dropped.
std::string go_bytes_size(double size) {
  static const char *abbrs[] = {"B", "KiB", "MiB", "GiB", "TiB", "PiB", "EiB", "ZiB", "YiB"};
  int i = 0;
  while (size >= 1024.0 && i < 8) {
    size = size / 1024.0;
    ++i;
  }
  char b[64];
  snprintf(b, sizeof b, "%.4g%s", size, abbrs[i]);
  return b;
}

// pct/percentage.go:28-30: fmt.Sprintf("%0.2f%%", p*100)
std::string pct_string(double p) {
  char b[64];
  snprintf(b, sizeof b, "%0.2f%%", p * 100.0);
  return b;
}

// svctype/service_type.go:34-42
std::string service_type_string(int32_t t) {
  if (t == kServiceHTTP) return "HTTP";
  if (t == kServiceGRPC) return "gRPC";
  return "";
}

// encoding/json floatEncoder (Go 1.16, bits = 64): shortest round-trip
// digits, 'f' format unless |f| < 1e-6 or >= 1e21 ('e'), then "e-07" -> "e-7".
void go_json_float(std::string &o, double f) {
  char b[64];
  const double a = std::fabs(f);
  const bool e = a != 0 && (a < 1e-6 || a >= 1e21);
  auto r = std::to_chars(b, b + sizeof b, f, e ? std::chars_format::scientific : std::chars_format::fixed);
  std::string s(b, r.ptr);
  if (e) {
    const size_t n = s.size();
    if (n >= 4 && s[n - 4] == 'e' && s[n - 3] == '-' && s[n - 2] == '0') s.erase(n - 2, 1);
  }
  o += s;
}

// utf8.DecodeRuneInString: returns the rune and its length; invalid -> (-1, 1)
static int decode_rune(const unsigned char *p, size_t n, int &len) {
  const unsigned char c = p[0];
  len = 1;
  if (c < 0x80) return c;
  int need;
  uint32_t r, lo = 0x80, hi = 0xBF;
  if (c >= 0xC2 && c <= 0xDF) {
    need = 1;
    r = c & 0x1F;
  } else if (c >= 0xE0 && c <= 0xEF) {
    need = 2;
    r = c & 0x0F;
    if (c == 0xE0) lo = 0xA0;
    if (c == 0xED) hi = 0x9F;  // no surrogates
  } else if (c >= 0xF0 && c <= 0xF4) {
    need = 3;
    r = c & 0x07;
    if (c == 0xF0) lo = 0x90;
    if (c == 0xF4) hi = 0x8F;
  } else {
    return -1;
  }
  if ((size_t)need >= n) return -1;
  for (int i = 1; i <= need; ++i) {
    const unsigned char x = p[i];
    if (x < (i == 1 ? lo : 0x80) || x > (i == 1 ? hi : 0xBF)) return -1;
    r = (r << 6) | (x & 0x3F);
  }
  len = need + 1;
  return (int)r;
}

// encoding/json encodeState.string with escapeHTML (json.Marshal, Go 1.16)
void go_json_string(std::string &o, const std::string &s) {
  static const char hex[] = "0123456789abcdef";
  o += '"';
  const unsigned char *p = (const unsigned char *)s.data();
  const size_t n = s.size();
  size_t i = 0;
  while (i < n) {
    const unsigned char b = p[i];
    if (b < 0x80) {
      if (b >= 0x20 && b != '"' && b != '\\' && b != '<' && b != '>' && b != '&') {
        o += (char)b;
      } else if (b == '"' || b == '\\') {
        o += '\\';
        o += (char)b;
      } else if (b == '\n') {
        o += "\\n";
      } else if (b == '\r') {
        o += "\\r";
      } else if (b == '\t') {
        o += "\\t";
      } else {
        o += "\\u00";
        o += hex[b >> 4];
        o += hex[b & 0xF];
      }
      ++i;
      continue;
    }
    int len;
    const int r = decode_rune(p + i, n - i, len);
    if (r < 0) {
      o += "\\ufffd";
    } else if (r == 0x2028 || r == 0x2029) {
      o += "\\u202";
      o += hex[r & 0xF];
    } else {
      o.append((const char *)p + i, (size_t)len);
    }
    i += (size_t)len;
  }
  o += '"';
}

// ------------------------------------------------------------ json.Marshal --

// script/command.go:42-53 commandToMarshallable: sleep -> {"sleep": "<d>"},
// request -> {"call": RequestCommand}, concurrent -> nested array.
// RequestCommand fields (request_command.go:26-33): service, size
// (ByteSize.MarshalJSON = its String()), probability omitempty.
static void marshal_cmd(std::string &o, const Command &c) {
  if (c.kind == Command::Sleep) {
    o += "{\"sleep\":";
    go_json_string(o, go_duration_string(c.sleep_ns));
    o += '}';
  } else if (c.kind == Command::Request) {
    o += "{\"call\":{\"service\":";
    go_json_string(o, c.service);
    o += ",\"size\":";
    go_json_string(o, go_bytes_size((double)c.size));
    if (c.probability != 0) o += ",\"probability\":" + std::to_string(c.probability);
    o += "}}";
  } else {
    o += '[';
    for (size_t i = 0; i < c.commands.size(); ++i) {
      if (i) o += ',';
      marshal_cmd(o, c.commands[i]);
    }
    o += ']';
  }
}

// svc/service.go:25-51 field order and omitempty; graph.go:21-23.
std::string marshal_json(const ServiceGraph &g) {
  std::string o = "{\"services\":";
  if (g.services.empty()) {
    o += g.services_nil ? "null}" : "[]}";
    return o;
  }
  o += '[';
  for (size_t i = 0; i < g.services.size(); ++i) {
    const Service &s = g.services[i];
    if (i) o += ',';
    o += "{\"name\":";
    go_json_string(o, s.name);
    if (s.type != kServiceUnknown) {
      std::string t = service_type_string(s.type);
      for (char &ch : t) ch = (char)tolower((unsigned char)ch);  // MarshalJSON lower-cases String()
      o += ",\"type\":";
      go_json_string(o, t);
    }
    if (s.num_replicas != 0) o += ",\"numReplicas\":" + std::to_string(s.num_replicas);
    if (s.is_entrypoint) o += ",\"isEntrypoint\":true";
    if (s.error_rate != 0) {
      o += ",\"errorRate\":";
      go_json_float(o, s.error_rate);
    }
    if (s.response_size != 0) {
      o += ",\"responseSize\":";
      go_json_string(o, go_bytes_size((double)s.response_size));
    }
    if (!s.script.empty()) {
      o += ",\"script\":[";
      for (size_t j = 0; j < s.script.size(); ++j) {
        if (j) o += ',';
        marshal_cmd(o, s.script[j]);
      }
      o += ']';
    }
    o += ",\"numRbacPolicies\":" + std::to_string(s.num_rbac_policies) + "}";
  }
  o += "]}";
  return o;
}

// ---------------------------------------------------------------- graphviz --

// graphviz.go:170-181 nonConcurrentCommandToString
static std::string step_string(const Command &c) {
  if (c.kind == Command::Sleep) return "SLEEP " + go_duration_string(c.sleep_ns);
  return "CALL \"" + c.service + "\" " + go_bytes_size((double)c.size);
}

// graphviz.go:99-126 graphvizTemplate, with text/template's whitespace
// trimming ({{- / -}}) applied: per node a header row and one row per step
// (a concurrent step's commands joined by <BR />), then one line per edge
// "From":StepIndex -> "To" (getEdgesFromExe, graphviz.go:128-145).  Values
// are inserted unescaped (text/template).
std::string to_dot(const ServiceGraph &g) {
  std::string o =
      "digraph {\n  node [\n    fontsize = \"16\"\n    fontname = \"courier\"\n    shape = plaintext\n  ];\n\n  ";
  std::string edges;
  for (const Service &s : g.services) {
    o += "\"" + s.name + "\" [label=<\n<TABLE BORDER=\"0\" CELLBORDER=\"1\" CELLSPACING=\"0\">\n  <TR><TD><B>" +
         s.name + "</B><BR />Type: " + service_type_string(s.type) + "<BR />Err: " + pct_string(s.error_rate) +
         "</TD></TR>";
    for (size_t i = 0; i < s.script.size(); ++i) {
      const Command &c = s.script[i];
      o += "\n  <TR><TD PORT=\"" + std::to_string(i) + "\">";
      if (c.kind == Command::Concurrent) {
        for (size_t j = 0; j < c.commands.size(); ++j) {
          if (j) o += "<BR />";
          o += step_string(c.commands[j]);
        }
      } else {
        o += step_string(c);
      }
      o += "</TD></TR>";
      auto edge = [&](const Command &r) {
        if (r.kind == Command::Request) edges += "\n  \"" + s.name + "\":" + std::to_string(i) + " -> \"" + r.service + "\"";
      };
      if (c.kind == Command::Concurrent)
        for (const Command &sub : c.commands) edge(sub);
      else
        edge(c);
    }
    o += "\n</TABLE>>];\n\n  ";
  }
  o += edges;
  o += "\n}\n";
  return o;
}

}  // namespace isim
