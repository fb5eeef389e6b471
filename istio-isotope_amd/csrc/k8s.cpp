// Kubernetes manifests of a service graph: the C++ host restatement of
// isotope's `convert kubernetes` (second half).
//
//   ServiceGraphToKubernetesManifests  convert/pkg/kubernetes/kubernetes.go:56-137
//   makeServiceGraphNamespace          kubernetes.go:150-157
//   makeConfigMap                      kubernetes.go:159-175
//   makeService / makeDeployment       kubernetes.go:177-270
//   makeFortioDeployment / Service     fortio_client.go:28-78
//   generateRbacPolicy / RbacConfig    rbac.go:25-71
//   constants                          convert/pkg/consts/consts.go
//
// Every object goes through sigs.k8s.io/yaml v1.2.0 Marshal in the reference:
// encoding/json of the k8s.io/api v0.18.0 struct (field tags, omitempty —
// which never drops a struct-valued field, hence `spec: {}`, `status: {}`,
// `resources: {}`, `strategy: {}`, `loadBalancer: {}` and the IntOrString
// `targetPort: 0`), then JSONToYAML: gopkg.in/yaml.v2 v2.2.8 decodes the JSON
// (numbers resolved as int / uint64 / float64) and encodes it again (keys in
// yaml.v2's keyList order, scalar styles chosen by resolve() and libyaml's
// scalar analysis, block sequences not indented inside mappings, plain and
// double-quoted scalars folded at spaces past column 80).  Both halves are
// restated here on a small value tree; the ConfigMap payload is
// yaml.Marshal(graph) = JSONToYAML(isim_graph_marshal_json).
//
// EXT (the reference is not deterministic): every creationTimestamp is the
// caller's `creation_timestamp_s` (the reference stamps time.Now()), and the
// RBAC rule names are version-4 UUIDs drawn from Philox4x32-10 keyed by
// `rbac_seed` (the reference calls uuid.New() after rand.Seed(time.Now())).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <charconv>
#include <string>
#include <utility>
#include <vector>

#include "../../include/isim.h"
#include "graph.h"
#include "json.h"
#include "k8s.h"
#include "marshal.h"
#include "tree_walk.h"

namespace isim {
namespace k8s {

// ---- value tree (what yaml.v2 unmarshals JSON into) -------------------------
struct Y {
  enum Kind { Null, Bool, Int, Float, Str, Map, Seq } kind = Null;
  std::string s;                              // Int/Float: formatted text; Str: the string
  bool b = false;
  std::vector<std::pair<std::string, Y>> map; // Map: string keys (sorted at emit)
  std::vector<Y> seq;
};

static Y str(const std::string &s) {
  Y y;
  y.kind = Y::Str;
  y.s = s;
  return y;
}
static Y num(long long v) {
  Y y;
  y.kind = Y::Int;
  y.s = std::to_string(v);
  return y;
}
static Y map() {
  Y y;
  y.kind = Y::Map;
  return y;
}
static Y seq() {
  Y y;
  y.kind = Y::Seq;
  return y;
}
static Y &put(Y &m, const std::string &k, Y v) {
  for (auto &kv : m.map)
    if (kv.first == k) {
      kv.second = std::move(v);
      return kv.second;
    }
  m.map.emplace_back(k, std::move(v));
  return m.map.back().second;
}
static Y labels(std::initializer_list<std::pair<const char *, std::string>> kv) {
  Y m = map();
  for (auto &p : kv) put(m, p.first, str(p.second));
  return m;
}

// strconv.FormatFloat(f, 'g', -1, 64) (yaml.v2 encoder.floatv)
static std::string go_format_g(double f) {
  if (std::isnan(f)) return ".nan";
  if (std::isinf(f)) return f > 0 ? ".inf" : "-.inf";
  if (f == 0) return std::signbit(f) ? "-0" : "0";
  char b[64];
  auto r = std::to_chars(b, b + sizeof b, f, std::chars_format::scientific);  // shortest digits
  std::string t(b, r.ptr);
  const bool neg = t[0] == '-';
  if (neg) t.erase(0, 1);
  const size_t e = t.find('e');
  std::string digs;
  for (size_t i = 0; i < e; ++i)
    if (t[i] != '.') digs += t[i];
  const int exp10 = std::atoi(t.c_str() + e + 1);  // value = 0.d1d2.. x 10^(exp10+1)
  const int nd = (int)digs.size(), dp = exp10 + 1;
  std::string o = neg ? "-" : "";
  if (exp10 < -4 || exp10 >= 6) {  // %e, shortest: precision 6 decides
    o += digs[0];
    if (nd > 1) o += "." + digs.substr(1);
    o += exp10 < 0 ? "e-" : "e+";
    const int a = exp10 < 0 ? -exp10 : exp10;
    if (a < 10) o += '0';
    o += std::to_string(a);
    return o;
  }
  if (dp <= 0) {
    o += "0." + std::string(-dp, '0') + digs;
  } else if (dp >= nd) {
    o += digs + std::string(dp - nd, '0');
  } else {
    o += digs.substr(0, dp) + "." + digs.substr(dp);
  }
  return o;
}

// yaml.v2 resolve() of a JSON number literal: int, uint64, else float64
static Y from_json_number(const std::string &lit) {
  Y y;
  long long iv = 0;
  auto r = std::from_chars(lit.data(), lit.data() + lit.size(), iv);
  if (r.ec == std::errc() && r.ptr == lit.data() + lit.size()) {
    y.kind = Y::Int;
    y.s = std::to_string(iv);
    return y;
  }
  unsigned long long uv = 0;
  r = std::from_chars(lit.data(), lit.data() + lit.size(), uv);
  if (r.ec == std::errc() && r.ptr == lit.data() + lit.size()) {
    y.kind = Y::Int;
    y.s = std::to_string(uv);
    return y;
  }
  y.kind = Y::Float;
  y.s = go_format_g(std::strtod(lit.c_str(), nullptr));
  return y;
}

static Y from_json(const JVal &v) {
  switch (v.kind) {
    case JVal::Null: return Y{};
    case JVal::Bool: {
      Y y;
      y.kind = Y::Bool;
      y.b = v.b;
      return y;
    }
    case JVal::Num: return from_json_number(v.s);
    case JVal::Str: return str(v.s);
    case JVal::Arr: {
      Y y = seq();
      for (const JVal &e : v.arr) y.seq.push_back(from_json(e));
      return y;
    }
    default: {
      Y y = map();
      for (const auto &kv : v.obj) put(y, kv.first, from_json(kv.second));  // duplicate keys: last wins
      return y;
    }
  }
}

// ---- yaml.v2 key order (sorter.go keyList.Less) ------------------------------
static std::vector<uint32_t> runes(const std::string &s) {
  std::vector<uint32_t> r;
  for (size_t i = 0; i < s.size();) {
    const unsigned char c = (unsigned char)s[i];
    int n = c < 0x80 ? 1 : c < 0xE0 ? 2 : c < 0xF0 ? 3 : 4;
    uint32_t v = n == 1 ? c : n == 2 ? (c & 0x1F) : n == 3 ? (c & 0x0F) : (c & 0x07);
    for (int k = 1; k < n && i + k < s.size(); ++k) v = (v << 6) | ((unsigned char)s[i + k] & 0x3F);
    r.push_back(v);
    i += n;
  }
  return r;
}
#include "unicode_tables.inc"
static bool in_ranges(const uint32_t (*t)[2], size_t n, uint32_t r) {
  size_t lo = 0, hi = n;  // first range whose end >= r
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (t[mid][1] < r) lo = mid + 1;
    else hi = mid;
  }
  return lo < n && t[lo][0] <= r;
}
// unicode.IsLetter / unicode.IsDigit (Go), as sorter.go uses them
static bool is_letter(uint32_t r) {
  if (r < 0x80) return (r >= 'a' && r <= 'z') || (r >= 'A' && r <= 'Z');
  return in_ranges(kUniLetter, sizeof(kUniLetter) / sizeof(kUniLetter[0]), r);
}
static bool is_udigit(uint32_t r) {
  if (r < 0x80) return r >= '0' && r <= '9';
  return in_ranges(kUniDigit, sizeof(kUniDigit) / sizeof(kUniDigit[0]), r);
}
static bool is_digit(uint32_t r) { return r >= '0' && r <= '9'; }
static bool key_less(const std::string &as, const std::string &bs) {
  const std::vector<uint32_t> a = runes(as), b = runes(bs);
  for (size_t i = 0; i < a.size() && i < b.size(); ++i) {
    if (a[i] == b[i]) continue;
    const bool al = is_letter(a[i]), bl = is_letter(b[i]);
    if (al && bl) return a[i] < b[i];
    if (al || bl) return bl;
    // Go int64 arithmetic on rune - '0' (wrapping; any Nd digit counts)
    uint64_t an = 0, bn = 0;
    size_t ai, bi;
    if (a[i] == '0' || b[i] == '0') {
      for (long j = (long)i - 1; j >= 0 && is_udigit(a[j]); --j)
        if (a[j] != '0') {
          an = 1;
          bn = 1;
          break;
        }
    }
    for (ai = i; ai < a.size() && is_udigit(a[ai]); ++ai) an = an * 10 + (uint64_t)((int64_t)a[ai] - '0');
    for (bi = i; bi < b.size() && is_udigit(b[bi]); ++bi) bn = bn * 10 + (uint64_t)((int64_t)b[bi] - '0');
    if (an != bn) return (int64_t)an < (int64_t)bn;
    if (ai != bi) return ai < bi;
    return a[i] < b[i];
  }
  return a.size() < b.size();
}

// yaml.v2 parseTimestamp: YYYY- then time.Parse against its allowed layouts
static bool is_timestamp(const std::string &s) {
  size_t i = 0;
  auto num = [&](int &v) -> bool {  // Go getnum(value, false): one or two digits
    if (i >= s.size() || !is_digit((unsigned char)s[i])) return false;
    v = s[i++] - '0';
    if (i < s.size() && is_digit((unsigned char)s[i])) v = v * 10 + (s[i++] - '0');
    return true;
  };
  while (i < s.size() && is_digit((unsigned char)s[i])) ++i;
  if (i != 4 || i == s.size() || s[i] != '-') return false;
  const int year = std::atoi(s.substr(0, 4).c_str());
  ++i;
  int mon, day;
  if (!num(mon) || i >= s.size() || s[i] != '-') return false;
  ++i;
  if (!num(day)) return false;
  if (mon < 1 || mon > 12) return false;
  static const int dim[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  const bool leap = (year % 4 == 0 && year % 100 != 0) || year % 400 == 0;
  if (day < 1 || day > dim[mon - 1] + (mon == 2 && leap ? 1 : 0)) return false;
  if (i == s.size()) return true;  // "2006-1-2"
  const char sep = s[i];
  if (sep != 'T' && sep != 't' && sep != ' ') return false;
  ++i;
  int hh, mm, ss;
  if (!num(hh) || i >= s.size() || s[i] != ':') return false;
  ++i;
  if (!num(mm) || i >= s.size() || s[i] != ':') return false;
  ++i;
  if (!num(ss)) return false;
  if (hh > 23 || mm > 59 || ss > 59) return false;
  if (i + 1 < s.size() && (s[i] == '.' || s[i] == ',') && is_digit((unsigned char)s[i + 1])) {
    ++i;
    while (i < s.size() && is_digit((unsigned char)s[i])) ++i;
  }
  if (sep == ' ') return i == s.size();
  if (i < s.size() && s[i] == 'Z') return i + 1 == s.size();
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) {  // Z07:00
    ++i;
    if (s.size() - i != 5 || !is_digit((unsigned char)s[i]) || !is_digit((unsigned char)s[i + 1]) || s[i + 2] != ':' ||
        !is_digit((unsigned char)s[i + 3]) || !is_digit((unsigned char)s[i + 4]))
      return false;
    return (s[i] - '0') * 10 + (s[i + 1] - '0') <= 24 && (s[i + 3] - '0') * 10 + (s[i + 4] - '0') <= 59;
  }
  return false;
}

// ---- yaml.v2 resolve(): does a plain scalar read back as something else? ----
static bool resolves_non_string(const std::string &s) {
  if (s.empty()) return true;  // null
  static const char *words[] = {"~",    "null", "Null", "NULL", "y",    "Y",    "yes",  "Yes",   "YES",
                                "n",    "N",    "no",   "No",   "NO",   "true", "True", "TRUE",  "false",
                                "False", "FALSE", "on",  "On",   "ON",   "off",  "Off",  "OFF",   ".inf",
                                ".Inf", ".INF", "+.inf", "+.Inf", "+.INF", "-.inf", "-.Inf", "-.INF", ".nan",
                                ".NaN", ".NAN", "<<"};
  for (const char *w : words)
    if (s == w) return true;
  const char c = s[0];
  if (!(c == '+' || c == '-' || c == '.' || (c >= '0' && c <= '9'))) return false;
  std::string plain;
  for (char ch : s)
    if (ch != '_') plain += ch;
  // strconv.ParseInt / ParseUint with base 0 (sign, 0x / 0o / 0b / leading-0 octal)
  {
    std::string t = plain;
    size_t i = 0;
    if (i < t.size() && (t[i] == '+' || t[i] == '-')) ++i;
    int base = 10;
    std::string body = t.substr(i);
    if (body.size() > 1 && body[0] == '0') {
      const char p = body[1];
      if (p == 'x' || p == 'X') base = 16, body = body.substr(2);
      else if (p == 'o' || p == 'O') base = 8, body = body.substr(2);
      else if (p == 'b' || p == 'B') base = 2, body = body.substr(2);
      else base = 8, body = body.substr(1);
    }
    bool ok = !body.empty();
    for (char ch : body) {
      int d = (ch >= '0' && ch <= '9') ? ch - '0' : (ch >= 'a' && ch <= 'f') ? ch - 'a' + 10
                                                 : (ch >= 'A' && ch <= 'F') ? ch - 'A' + 10 : 99;
      if (d >= base) ok = false;
    }
    if (ok) return true;  // an int (range errors fall through to float in Go too; both non-string)
  }
  // yamlStyleFloat ^[-+]?(\.[0-9]+|[0-9]+(\.[0-9]*)?)([eE][-+]?[0-9]+)?$
  {
    size_t i = 0;
    const std::string &t = plain;
    if (i < t.size() && (t[i] == '+' || t[i] == '-')) ++i;
    bool ok = false;
    if (i < t.size() && t[i] == '.') {
      ++i;
      size_t j = i;
      while (i < t.size() && is_digit((unsigned char)t[i])) ++i;
      ok = i > j;
    } else {
      size_t j = i;
      while (i < t.size() && is_digit((unsigned char)t[i])) ++i;
      ok = i > j;
      if (ok && i < t.size() && t[i] == '.') {
        ++i;
        while (i < t.size() && is_digit((unsigned char)t[i])) ++i;
      }
    }
    if (ok && i < t.size() && (t[i] == 'e' || t[i] == 'E')) {
      ++i;
      if (i < t.size() && (t[i] == '+' || t[i] == '-')) ++i;
      size_t j = i;
      while (i < t.size() && is_digit((unsigned char)t[i])) ++i;
      ok = i > j;
    }
    if (ok && i == t.size()) return true;
  }
  // timestamps: yaml.v2 parseTimestamp (resolve.go), time.Parse of
  // "2006-1-2T15:4:5.999999999Z07:00" (T or t), "2006-1-2 15:4:5.999999999", "2006-1-2"
  return is_timestamp(s);
  return false;
}

// isBase60Float ^[-+]?[0-9][0-9_]*(?::[0-5]?[0-9])+(?:\.[0-9_]*)?$
static bool is_base60_float(const std::string &s) {
  size_t i = 0;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
  if (i >= s.size() || !is_digit((unsigned char)s[i])) return false;
  while (i < s.size() && (is_digit((unsigned char)s[i]) || s[i] == '_')) ++i;
  int groups = 0;
  while (i < s.size() && s[i] == ':') {
    ++i;
    size_t j = i;
    while (i < s.size() && is_digit((unsigned char)s[i]) && i - j < 2) ++i;
    if (i == j) return false;
    if (i - j == 2 && s[j] > '5') return false;
    ++groups;
  }
  if (!groups) return false;
  if (i < s.size() && s[i] == '.') {
    ++i;
    while (i < s.size() && (is_digit((unsigned char)s[i]) || s[i] == '_')) ++i;
  }
  return i == s.size();
}

// ---- libyaml emitter (as yaml.v2 drives it: best_indent 2, best_width 80, unicode) ----
struct Emitter {
  std::string out;
  int column = 0;
  bool whitespace = true, indention = true;
  static constexpr int kWidth = 80;

  void put_char(char c) {
    out += c;
    ++column;
  }
  void put_break() {
    out += '\n';
    column = 0;
  }
  void write_raw(const std::string &s) {  // no line breaks inside
    out += s;
    column += (int)runes(s).size();
  }
  void write_indent(int indent) {
    if (indent < 0) indent = 0;
    if (!indention || column > indent || (column == indent && !whitespace)) put_break();
    while (column < indent) put_char(' ');
    whitespace = true;
    indention = true;
  }
  void indicator(const char *ind, bool need_ws, bool is_ws, bool is_indention) {
    if (need_ws && !whitespace) put_char(' ');
    write_raw(ind);
    whitespace = is_ws;
    indention = indention && is_indention;
  }
};

struct Analysis {
  bool multiline = false, flow_plain = true, block_plain = true, single_quoted = true, block = true;
};

static size_t utf8_width(unsigned char c) { return c < 0x80 ? 1 : (c & 0xE0) == 0xC0 ? 2 : (c & 0xF0) == 0xE0 ? 3 : 4; }
static bool is_break_at(const std::string &v, size_t i) {
  const unsigned char c = (unsigned char)v[i];
  if (c == '\r' || c == '\n') return true;
  if (c == 0xC2 && i + 1 < v.size() && (unsigned char)v[i + 1] == 0x85) return true;
  if (c == 0xE2 && i + 2 < v.size() && (unsigned char)v[i + 1] == 0x80 &&
      ((unsigned char)v[i + 2] == 0xA8 || (unsigned char)v[i + 2] == 0xA9))
    return true;
  return false;
}
static bool is_blankz_at(const std::string &v, size_t i) {
  if (i >= v.size()) return true;
  return v[i] == ' ' || v[i] == '\t' || is_break_at(v, i) || v[i] == 0;
}
static bool is_printable_at(const std::string &v, size_t i) {  // yaml.v2 yamlprivateh.go is_printable
  const unsigned char b0 = (unsigned char)v[i];
  const unsigned char b1 = i + 1 < v.size() ? (unsigned char)v[i + 1] : 0;
  const unsigned char b2 = i + 2 < v.size() ? (unsigned char)v[i + 2] : 0;
  return b0 == 0x0A || (b0 >= 0x20 && b0 <= 0x7E) || (b0 == 0xC2 && b1 >= 0xA0) || (b0 > 0xC2 && b0 < 0xED) ||
         (b0 == 0xED && b1 < 0xA0) || b0 == 0xEE ||
         (b0 == 0xEF && !(b1 == 0xBB && b2 == 0xBF) && !(b1 == 0xBF && (b2 == 0xBE || b2 == 0xBF)));
}

static Analysis analyze(const std::string &v) {
  Analysis a;
  if (v.empty()) {
    a.flow_plain = false;
    a.block_plain = true;
    a.single_quoted = true;
    a.block = false;
    return a;
  }
  bool block_ind = false, flow_ind = false, line_breaks = false, special = false;
  bool leading_space = false, leading_break = false, trailing_space = false, trailing_break = false;
  bool break_space = false, space_break = false, prev_space = false, prev_break = false;
  if (v.size() >= 3 && ((v[0] == '-' && v[1] == '-' && v[2] == '-') || (v[0] == '.' && v[1] == '.' && v[2] == '.'))) {
    block_ind = true;
    flow_ind = true;
  }
  bool preceded_ws = true;
  bool followed_ws = is_blankz_at(v, utf8_width((unsigned char)v[0]));
  for (size_t i = 0; i < v.size();) {
    const char c = v[i];
    if (i == 0) {
      switch (c) {
        case '#': case ',': case '[': case ']': case '{': case '}': case '&': case '*': case '!': case '|':
        case '>': case '\'': case '"': case '%': case '@': case '`':
          flow_ind = block_ind = true;
          break;
        case '?': case ':':
          flow_ind = true;
          if (followed_ws) block_ind = true;
          break;
        case '-':
          if (followed_ws) flow_ind = block_ind = true;
          break;
        default: break;
      }
    } else {
      switch (c) {
        case ',': case '?': case '[': case ']': case '{': case '}':
          flow_ind = true;
          break;
        case ':':
          flow_ind = true;
          if (followed_ws) block_ind = true;
          break;
        case '#':
          if (preceded_ws) flow_ind = block_ind = true;
          break;
        default: break;
      }
    }
    if (!is_printable_at(v, i)) special = true;
    const size_t w = utf8_width((unsigned char)c);
    if (c == ' ') {
      if (i == 0) leading_space = true;
      if (i + w == v.size()) trailing_space = true;
      if (prev_break) break_space = true;
      prev_space = true;
      prev_break = false;
    } else if (is_break_at(v, i)) {
      line_breaks = true;
      if (i == 0) leading_break = true;
      if (i + w == v.size()) trailing_break = true;
      if (prev_space) space_break = true;
      prev_space = false;
      prev_break = true;
    } else {
      prev_space = prev_break = false;
    }
    preceded_ws = is_blankz_at(v, i);
    i += w;
    if (i < v.size()) followed_ws = is_blankz_at(v, i + utf8_width((unsigned char)v[i]));
  }
  a.multiline = line_breaks;
  if (leading_space || leading_break || trailing_space || trailing_break) a.flow_plain = a.block_plain = false;
  if (trailing_space) a.block = false;
  if (break_space) a.flow_plain = a.block_plain = a.single_quoted = false;
  if (space_break || special) a.flow_plain = a.block_plain = a.single_quoted = a.block = false;
  if (line_breaks) a.flow_plain = a.block_plain = false;
  if (flow_ind) a.flow_plain = false;
  if (block_ind) a.block_plain = false;
  return a;
}

enum Style { Plain, Single, Double, Literal };

// encoder.stringv style, then yaml_emitter_select_scalar_style (block context)
static Style string_style(const std::string &s, bool simple_key) {
  Style st;
  const bool can_plain = !resolves_non_string(s) && !is_base60_float(s);
  if (s.find('\n') != std::string::npos) st = Literal;
  else if (can_plain) st = Plain;
  else st = Double;
  const Analysis a = analyze(s);
  if (st == Plain) {
    if (!a.block_plain || (simple_key && a.multiline) || (s.empty() && simple_key)) st = Single;
  }
  if (st == Single && !a.single_quoted) st = Double;
  if (st == Literal && (!a.block || simple_key)) st = Double;
  return st;
}

static void write_plain(Emitter &e, const std::string &v, bool allow_breaks, int indent) {
  if (!e.whitespace) e.put_char(' ');
  bool spaces = false;
  for (size_t i = 0; i < v.size();) {
    if (v[i] == ' ') {
      if (allow_breaks && !spaces && e.column > Emitter::kWidth && !(i + 1 < v.size() && v[i + 1] == ' ')) {
        e.write_indent(indent);
        ++i;
      } else {
        e.put_char(' ');
        ++i;
      }
      spaces = true;
    } else {
      const size_t w = utf8_width((unsigned char)v[i]);
      e.out.append(v, i, w);
      ++e.column;
      i += w;
      e.indention = false;
      spaces = false;
    }
  }
  e.whitespace = false;
  e.indention = false;
}

static void write_single(Emitter &e, const std::string &v, bool allow_breaks, int indent) {
  e.indicator("'", true, false, false);
  bool spaces = false;
  for (size_t i = 0; i < v.size();) {
    if (v[i] == ' ') {
      if (allow_breaks && !spaces && e.column > Emitter::kWidth && i != 0 && i != v.size() - 1 &&
          !(i + 1 < v.size() && v[i + 1] == ' ')) {
        e.write_indent(indent);
        ++i;
      } else {
        e.put_char(' ');
        ++i;
      }
      spaces = true;
    } else {
      if (v[i] == '\'') e.put_char('\'');
      const size_t w = utf8_width((unsigned char)v[i]);
      e.out.append(v, i, w);
      ++e.column;
      i += w;
      e.indention = false;
      spaces = false;
    }
  }
  e.indicator("'", false, false, false);
}

static void write_double(Emitter &e, const std::string &v, bool allow_breaks, int indent) {
  e.indicator("\"", true, false, false);
  bool spaces = false;
  for (size_t i = 0; i < v.size();) {
    const unsigned char c = (unsigned char)v[i];
    const bool bom = c == 0xEF && i + 2 < v.size() && (unsigned char)v[i + 1] == 0xBB && (unsigned char)v[i + 2] == 0xBF;
    if (!is_printable_at(v, i) || bom || is_break_at(v, i) || c == '"' || c == '\\') {
      const size_t w = utf8_width(c);
      uint32_t r = w == 1 ? c : w == 2 ? (c & 0x1F) : w == 3 ? (c & 0x0F) : (c & 0x07);
      for (size_t k = 1; k < w && i + k < v.size(); ++k) r = (r << 6) | ((unsigned char)v[i + k] & 0x3F);
      i += w;
      e.put_char('\\');
      switch (r) {
        case 0x00: e.put_char('0'); break;
        case 0x07: e.put_char('a'); break;
        case 0x08: e.put_char('b'); break;
        case 0x09: e.put_char('t'); break;
        case 0x0A: e.put_char('n'); break;
        case 0x0B: e.put_char('v'); break;
        case 0x0C: e.put_char('f'); break;
        case 0x0D: e.put_char('r'); break;
        case 0x1B: e.put_char('e'); break;
        case 0x22: e.put_char('"'); break;
        case 0x5C: e.put_char('\\'); break;
        case 0x85: e.put_char('N'); break;
        case 0xA0: e.put_char('_'); break;
        case 0x2028: e.put_char('L'); break;
        case 0x2029: e.put_char('P'); break;
        default: {
          int n;
          if (r <= 0xFF) {
            e.put_char('x');
            n = 2;
          } else if (r <= 0xFFFF) {
            e.put_char('u');
            n = 4;
          } else {
            e.put_char('U');
            n = 8;
          }
          for (int k = (n - 1) * 4; k >= 0; k -= 4) {
            const uint32_t d = (r >> k) & 0xF;
            e.put_char((char)(d < 10 ? '0' + d : 'A' + d - 10));
          }
        }
      }
      spaces = false;
    } else if (c == ' ') {
      if (allow_breaks && !spaces && e.column > Emitter::kWidth && i != 0 && i != v.size() - 1) {
        e.write_indent(indent);
        if (i + 1 < v.size() && v[i + 1] == ' ') e.put_char('\\');
        ++i;
      } else {
        e.put_char(' ');
        ++i;
      }
      spaces = true;
    } else {
      const size_t w = utf8_width(c);
      e.out.append(v, i, w);
      ++e.column;
      i += w;
      spaces = false;
    }
  }
  e.indicator("\"", false, false, false);
}

static void write_literal(Emitter &e, const std::string &v, int indent) {
  e.indicator("|", true, false, false);
  if (!v.empty() && (v[0] == ' ' || is_break_at(v, 0))) e.indicator("2", false, false, false);
  // chomping: '-' without a final break, '+' with two or more (or only one break)
  char chomp = 0;
  if (v.empty()) {
    chomp = '-';
  } else {
    long i = (long)v.size() - 1;
    while (i > 0 && ((unsigned char)v[i] & 0xC0) == 0x80) --i;
    if (!is_break_at(v, (size_t)i)) {
      chomp = '-';
    } else if (i == 0) {
      chomp = '+';
    } else {
      --i;
      while (i > 0 && ((unsigned char)v[i] & 0xC0) == 0x80) --i;
      if (is_break_at(v, (size_t)i)) chomp = '+';
    }
  }
  if (chomp) {
    const char s[2] = {chomp, 0};
    e.indicator(s, false, false, false);
  }
  e.put_break();
  e.indention = true;
  e.whitespace = true;
  bool breaks = true;
  for (size_t i = 0; i < v.size();) {
    if (is_break_at(v, i)) {
      i += (v[i] == '\r' && i + 1 < v.size() && v[i + 1] == '\n') ? 2 : utf8_width((unsigned char)v[i]);
      e.put_break();
      e.indention = true;
      breaks = true;
    } else {
      if (breaks) {
        e.write_indent(indent);
        breaks = false;
      }
      const size_t w = utf8_width((unsigned char)v[i]);
      e.out.append(v, i, w);
      ++e.column;
      i += w;
      e.indention = false;
    }
  }
}

// A scalar at the current position; `indent` = the scalar's indentation
// (its parent collection's indent + 2: yaml_emitter_emit_scalar's increase).
static void emit_scalar(Emitter &e, const Y &y, int indent, bool simple_key) {
  switch (y.kind) {
    case Y::Null: write_plain(e, "null", !simple_key, indent); return;
    case Y::Bool: write_plain(e, y.b ? "true" : "false", !simple_key, indent); return;
    case Y::Int:
    case Y::Float: write_plain(e, y.s, !simple_key, indent); return;
    default: break;
  }
  switch (string_style(y.s, simple_key)) {
    case Plain: write_plain(e, y.s, !simple_key, indent); break;
    case Single: write_single(e, y.s, !simple_key, indent); break;
    case Double: write_double(e, y.s, !simple_key, indent); break;
    case Literal: write_literal(e, y.s, indent); break;
  }
}

static bool empty_coll(const Y &y) {
  return (y.kind == Y::Map && y.map.empty()) || (y.kind == Y::Seq && y.seq.empty());
}

static void emit_node(Emitter &e, const Y &y, int parent_indent, bool in_mapping_value);

// yaml_emitter_check_simple_key (emitterc.go) for a string key: at most 128
// bytes and no line break; else a complex key ("? key" then ": value")
static bool simple_key(const std::string &k) {
  if (k.size() > 128) return false;
  for (size_t i = 0; i < k.size(); i += utf8_width((unsigned char)k[i]))
    if (is_break_at(k, i)) return false;
  return true;
}

// block mapping whose keys sit at column `indent`
static void emit_map(Emitter &e, const Y &m, int indent) {
  std::vector<const std::pair<std::string, Y> *> kv;
  for (const auto &p : m.map) kv.push_back(&p);
  std::stable_sort(kv.begin(), kv.end(), [](auto *a, auto *b) { return key_less(a->first, b->first); });
  for (const auto *p : kv) {
    e.write_indent(indent);
    if (simple_key(p->first)) {  // yaml_emitter_emit_block_mapping_key / _value, simple
      emit_scalar(e, str(p->first), indent + 2, true);
      e.indicator(":", false, false, false);
      emit_node(e, p->second, indent, true);
    } else {
      // "? " key (breaks allowed), then ": " at the mapping's indent; the
      // value follows at an indention point, so a sequence there is indented
      e.indicator("?", true, false, true);
      emit_scalar(e, str(p->first), indent + 2, false);
      e.write_indent(indent);
      e.indicator(":", true, false, true);
      emit_node(e, p->second, indent, false);
    }
  }
}

// block sequence whose "- " sit at column `indent`
static void emit_seq(Emitter &e, const Y &s, int indent) {
  for (const Y &item : s.seq) {
    e.write_indent(indent);
    e.indicator("-", true, false, true);
    emit_node(e, item, indent, false);
  }
}

// a value after "key:" (in_mapping_value) or after "- "; parent_indent = the
// enclosing collection's indent
static void emit_node(Emitter &e, const Y &y, int parent_indent, bool in_mapping_value) {
  if (empty_coll(y)) {
    e.indicator(y.kind == Y::Map ? "{" : "[", true, true, false);
    e.indicator(y.kind == Y::Map ? "}" : "]", false, false, false);
    return;
  }
  if (y.kind == Y::Map) {
    emit_map(e, y, parent_indent + 2);
  } else if (y.kind == Y::Seq) {
    // a sequence directly inside a mapping is not indented (indentless), unless
    // the mapping value starts at an indention point (never, after "key:")
    emit_seq(e, y, in_mapping_value ? parent_indent : parent_indent + 2);
  } else {
    emit_scalar(e, y, parent_indent + 2, false);
  }
}

// yaml.Marshal of a top-level value (a mapping for every object here)
static std::string marshal(const Y &doc) {
  Emitter e;
  if (doc.kind == Y::Map && !doc.map.empty()) {
    emit_map(e, doc, 0);
  } else if (doc.kind == Y::Seq && !doc.seq.empty()) {
    emit_seq(e, doc, 0);
  } else {
    emit_node(e, doc, -2, false);
  }
  e.write_indent(0);  // yaml_emitter_emit_document_end: a final break unless one was just written
  return e.out;
}

// ---- the manifests -----------------------------------------------------------
constexpr const char *kNamespace = "service-graph";          // consts.ServiceGraphNamespace
constexpr const char *kConfigName = "service-graph-config";  // kubernetes.go:43
constexpr const char *kConfigVolume = "config-volume";       // kubernetes.go:42
constexpr const char *kConfigKey = "service-graph";          // consts.ServiceGraphConfigMapKey
constexpr const char *kConfigPath = "/etc/config";           // consts.ConfigPath
constexpr const char *kGraphFile = "service-graph.yaml";     // consts.ServiceGraphYAMLFileName
constexpr const char *kContainer = "mock-service";           // consts.ServiceContainerName
constexpr int kServicePort = 8080;                           // consts.ServicePort
constexpr const char *kServicePortName = "http-web";         // consts.ServicePortName
constexpr int kFortioMetricsPort = 42422;                    // consts.FortioMetricsPort

struct Ctx {
  Y ts;  // creationTimestamp (metav1.Time.MarshalJSON: RFC 3339, UTC, seconds)
  Y service_selector, client_selector;
  std::string service_image, client_image;
  int idle_conns = 0;
};

static Y object(const char *api, const char *kind) {
  Y o = map();
  put(o, "apiVersion", str(api));
  put(o, "kind", str(kind));
  return o;
}
static Y meta(const Ctx &c, const std::string &name, const char *ns, Y lab) {
  Y m = map();
  put(m, "creationTimestamp", c.ts);
  if (!name.empty()) put(m, "name", str(name));
  if (ns) put(m, "namespace", str(ns));
  if (!lab.map.empty()) put(m, "labels", std::move(lab));
  return m;
}
static Y env_field(const char *name, const char *path) {
  Y ev = map();
  put(ev, "name", str(name));
  Y fr = map();
  put(fr, "fieldPath", str(path));
  Y src = map();
  put(src, "fieldRef", std::move(fr));
  put(ev, "valueFrom", std::move(src));
  return ev;
}
static Y port_entry(int port) {
  Y p = map();
  put(p, "containerPort", num(port));
  return p;
}
static Y service_port(const char *name, int port) {
  Y p = map();
  if (name) put(p, "name", str(name));
  put(p, "port", num(port));
  put(p, "targetPort", num(0));  // intstr.IntOrString{} marshals as 0
  return p;
}

// makeServiceGraphNamespace (kubernetes.go:150-157)
static Y make_namespace(const Ctx &c) {
  Y o = object("v1", "Namespace");
  put(o, "metadata", meta(c, kNamespace, nullptr, labels({{"istio-injection", "enabled"}})));
  put(o, "spec", map());
  put(o, "status", map());
  return o;
}

// makeConfigMap (kubernetes.go:159-175)
static Y make_config_map(const Ctx &c, const std::string &graph_yaml) {
  Y o = object("v1", "ConfigMap");
  Y d = map();
  put(d, kConfigKey, str(graph_yaml));
  put(o, "data", std::move(d));
  put(o, "metadata", meta(c, kConfigName, kNamespace, labels({{"app", "service-graph"}})));
  return o;
}

// makeService (kubernetes.go:177-187)
static Y make_service(const Ctx &c, const Service &s) {
  Y o = object("v1", "Service");
  put(o, "metadata", meta(c, s.name, kNamespace, labels({{"app", "service-graph"}})));
  Y spec = map();
  Y ports = seq();
  ports.seq.push_back(service_port(kServicePortName, kServicePort));
  put(spec, "ports", std::move(ports));
  put(spec, "selector", labels({{"name", s.name}}));
  put(o, "spec", std::move(spec));
  Y st = map();
  put(st, "loadBalancer", map());
  put(o, "status", std::move(st));
  return o;
}

// makeDeployment (kubernetes.go:189-270)
static Y make_deployment(const Ctx &c, const Service &s) {
  Y o = object("apps/v1", "Deployment");
  put(o, "metadata", meta(c, s.name, kNamespace, labels({{"app", "service-graph"}})));
  Y spec = map();
  put(spec, "replicas", num(s.num_replicas));
  Y sel = map();
  put(sel, "matchLabels", labels({{"name", s.name}}));
  put(spec, "selector", std::move(sel));
  put(spec, "strategy", map());
  Y tmeta = map();
  put(tmeta, "annotations", labels({{"prometheus.io/scrape", "true"}}));
  put(tmeta, "creationTimestamp", c.ts);
  put(tmeta, "labels", labels({{"role", "service"}, {"name", s.name}}));
  Y ctr = map();
  Y args = seq();
  args.seq.push_back(str("--max-idle-connections-per-host=" + std::to_string(c.idle_conns)));
  put(ctr, "args", std::move(args));
  Y env = seq();
  {
    Y ev = map();
    put(ev, "name", str("SERVICE_NAME"));  // consts.ServiceNameEnvKey
    if (!s.name.empty()) put(ev, "value", str(s.name));
    env.seq.push_back(std::move(ev));
  }
  env.seq.push_back(env_field("PODNAME", "metadata.name"));
  env.seq.push_back(env_field("PODIP", "status.podIP"));
  env.seq.push_back(env_field("NAMESPACE", "metadata.namespace"));
  env.seq.push_back(env_field("NODENAME", "spec.nodeName"));
  put(ctr, "env", std::move(env));
  if (!c.service_image.empty()) put(ctr, "image", str(c.service_image));
  put(ctr, "imagePullPolicy", str("IfNotPresent"));
  put(ctr, "name", str(kContainer));
  Y ports = seq();
  ports.seq.push_back(port_entry(kServicePort));
  put(ctr, "ports", std::move(ports));
  put(ctr, "resources", map());
  Y vm = map();
  put(vm, "mountPath", str(kConfigPath));
  put(vm, "name", str(kConfigVolume));
  Y vms = seq();
  vms.seq.push_back(std::move(vm));
  put(ctr, "volumeMounts", std::move(vms));
  Y pod = map();
  Y ctrs = seq();
  ctrs.seq.push_back(std::move(ctr));
  put(pod, "containers", std::move(ctrs));
  if (!c.service_selector.map.empty()) put(pod, "nodeSelector", c.service_selector);
  Y item = map();
  put(item, "key", str(kConfigKey));
  put(item, "path", str(kGraphFile));
  Y items = seq();
  items.seq.push_back(std::move(item));
  Y cm = map();
  put(cm, "items", std::move(items));
  put(cm, "name", str(kConfigName));
  Y vol = map();
  put(vol, "configMap", std::move(cm));
  put(vol, "name", str(kConfigVolume));
  Y vols = seq();
  vols.seq.push_back(std::move(vol));
  put(pod, "volumes", std::move(vols));
  Y tmpl = map();
  put(tmpl, "metadata", std::move(tmeta));
  put(tmpl, "spec", std::move(pod));
  put(spec, "template", std::move(tmpl));
  put(o, "spec", std::move(spec));
  put(o, "status", map());
  return o;
}

// makeFortioDeployment (fortio_client.go:28-66)
static Y make_fortio_deployment(const Ctx &c) {
  Y o = object("apps/v1", "Deployment");
  put(o, "metadata", meta(c, "client", nullptr, labels({{"app", "client"}})));
  Y spec = map();
  Y sel = map();
  put(sel, "matchLabels", labels({{"app", "client"}}));
  put(spec, "selector", std::move(sel));
  put(spec, "strategy", map());
  Y tmeta = map();
  put(tmeta, "creationTimestamp", c.ts);
  put(tmeta, "labels", labels({{"app", "client"}}));
  Y ctr = map();
  Y args = seq();
  args.seq.push_back(str("server"));
  put(ctr, "args", std::move(args));
  if (!c.client_image.empty()) put(ctr, "image", str(c.client_image));
  put(ctr, "name", str("fortio-client"));
  Y ports = seq();
  ports.seq.push_back(port_entry(kServicePort));
  ports.seq.push_back(port_entry(kFortioMetricsPort));
  put(ctr, "ports", std::move(ports));
  put(ctr, "resources", map());
  Y pod = map();
  Y ctrs = seq();
  ctrs.seq.push_back(std::move(ctr));
  put(pod, "containers", std::move(ctrs));
  if (!c.client_selector.map.empty()) put(pod, "nodeSelector", c.client_selector);
  Y tmpl = map();
  put(tmpl, "metadata", std::move(tmeta));
  put(tmpl, "spec", std::move(pod));
  put(spec, "template", std::move(tmpl));
  put(o, "spec", std::move(spec));
  put(o, "status", map());
  return o;
}

// makeFortioService (fortio_client.go:68-78)
static Y make_fortio_service(const Ctx &c) {
  Y o = object("v1", "Service");
  Y m = meta(c, "client", nullptr, labels({{"app", "client"}}));
  put(m, "annotations", labels({{"prometheus.io/scrape", "true"}}));
  put(o, "metadata", std::move(m));
  Y spec = map();
  Y ports = seq();
  ports.seq.push_back(service_port(nullptr, kServicePort));
  put(spec, "ports", std::move(ports));
  put(spec, "selector", labels({{"app", "client"}}));
  put(o, "spec", std::move(spec));
  Y st = map();
  put(st, "loadBalancer", map());
  put(o, "status", std::move(st));
  return o;
}

// EXT: uuid.New() (a random version-4 UUID, google/uuid v1.1.1) replaced by
// the bytes of Philox4x32-10((i_lo, i_hi, 0, 0x4B385300), seed), i = the
// rule's index in generation order; version and variant bits as RFC 4122.
static std::string rule_uuid(uint64_t seed, uint64_t i) {
  uint32_t c0 = (uint32_t)i, c1 = (uint32_t)(i >> 32), c2 = 0, c3 = 0x4B385300u;
  tw::philox10(c0, c1, c2, c3, (uint32_t)seed, (uint32_t)(seed >> 32));
  const uint32_t w[4] = {c0, c1, c2, c3};
  unsigned char b[16];
  for (int k = 0; k < 16; ++k) b[k] = (unsigned char)(w[k / 4] >> (8 * (k % 4)));
  b[6] = (unsigned char)((b[6] & 0x0F) | 0x40);
  b[8] = (unsigned char)((b[8] & 0x3F) | 0x80);
  static const char *hex = "0123456789abcdef";
  std::string s;
  for (int k = 0; k < 16; ++k) {
    if (k == 4 || k == 6 || k == 8 || k == 10) s += '-';
    s += hex[b[k] >> 4];
    s += hex[b[k] & 0xF];
  }
  return s;
}

// generateRbacPolicy (rbac.go:25-57): fmt.Sprintf of a fixed template
static std::string rbac_policy(const Service &s, bool allow_all, const std::string &rule) {
  const std::string ns = kNamespace, user = allow_all ? "*" : rule;
  return "\napiVersion: \"rbac.istio.io/v1alpha1\"\nkind: ServiceRole\nmetadata:\n  name: " + rule +
         "\n  namespace: " + ns + "\nspec:\n  rules:\n  - services: [\"" + s.name + "." + ns +
         ".*\"]\n    methods: [\"*\"]\n---\napiVersion: \"rbac.istio.io/v1alpha1\"\nkind: ServiceRoleBinding\n"
         "metadata:\n  name: " + rule + "\n  namespace: " + ns + "\nspec:\n  subjects:\n  - user: \"" + user +
         "\"\n  roleRef:\n    kind: ServiceRole\n    name: \"" + rule + "\"\n";
}

// generateRbacConfig (rbac.go:59-71)
static std::string rbac_config() {
  return std::string("\napiVersion: \"rbac.istio.io/v1alpha1\"\nkind: RbacConfig\nmetadata:\n  name: default\n"
                     "spec:\n  mode: 'ON_WITH_INCLUSION'\n  inclusion:\n    namespaces: [\"") +
         kNamespace + "\"]\n";
}

static bool equal_fold(const char *a, const char *b) {  // strings.EqualFold for ASCII
  for (; *a && *b; ++a, ++b) {
    char x = *a, y = *b;
    if (x >= 'A' && x <= 'Z') x = (char)(x - 'A' + 'a');
    if (y >= 'A' && y <= 'Z') y = (char)(y - 'A' + 'a');
    if (x != y) return false;
  }
  return *a == *b;
}

}  // namespace k8s

// yaml.Marshal(graph): JSONToYAML(json.Marshal(graph)) (kubernetes.go:161)
std::string graph_yaml(const ServiceGraph &g) {
  const std::string j = marshal_json(g);
  JVal v;
  std::string err;
  if (!json_parse(j.data(), j.size(), v, err)) return std::string();
  return k8s::marshal(k8s::from_json(v));
}

int k8s_manifests(const ServiceGraph &g, const isim_k8s_params &p, std::string &out, std::string &err) {
  using namespace k8s;
  Ctx c;
  {
    const time_t t = (time_t)p.creation_timestamp_s;
    struct tm u {};
    if (!gmtime_r(&t, &u) || u.tm_year + 1900 < 0 || u.tm_year + 1900 > 9999) {
      err = "creation timestamp outside years 0-9999 (metav1.Time.MarshalJSON)";
      return ISIM_EINVAL;
    }
    char b[32];
    std::snprintf(b, sizeof b, "%04d-%02d-%02dT%02d:%02d:%02dZ", u.tm_year + 1900, u.tm_mon + 1, u.tm_mday,
                  u.tm_hour, u.tm_min, u.tm_sec);
    c.ts = str(b);
  }
  auto selector = [&](const char *const *kv, int32_t n, Y &out_sel) -> bool {
    out_sel = map();
    if (n < 0 || (n > 0 && !kv)) return false;
    for (int32_t i = 0; i < n; ++i) {
      if (!kv[2 * i] || !kv[2 * i + 1]) return false;
      put(out_sel, kv[2 * i], str(kv[2 * i + 1]));
    }
    return true;
  };
  if (!selector(p.service_node_selector, p.n_service_node_selector, c.service_selector) ||
      !selector(p.client_node_selector, p.n_client_node_selector, c.client_selector)) {
    err = "bad node selector (n key/value pairs expected)";
    return ISIM_EINVAL;
  }
  c.service_image = p.service_image ? p.service_image : "";
  c.client_image = p.client_image ? p.client_image : "";
  c.idle_conns = p.service_max_idle_connections_per_host;
  const bool istio = p.environment_name && equal_fold(p.environment_name, "ISTIO");

  std::vector<std::string> docs;
  docs.push_back(marshal(make_namespace(c)));
  const std::string gy = graph_yaml(g);
  if (gy.empty()) {
    err = "graph marshal failed";
    return ISIM_EINVAL;
  }
  docs.push_back(marshal(make_config_map(c, gy)));
  bool has_rbac = false;
  uint64_t rule = 0;
  for (const Service &s : g.services) {
    docs.push_back(marshal(make_deployment(c, s)));
    docs.push_back(marshal(make_service(c, s)));
    if (istio && s.num_rbac_policies > 0) {
      has_rbac = true;
      for (int32_t i = 0; i < s.num_rbac_policies; ++i) docs.push_back(rbac_policy(s, false, rule_uuid(p.rbac_seed, rule++)));
      docs.push_back(rbac_policy(s, true, rule_uuid(p.rbac_seed, rule++)));
    }
  }
  docs.push_back(marshal(make_fortio_deployment(c)));
  docs.push_back(marshal(make_fortio_service(c)));
  if (has_rbac) docs.push_back(rbac_config());
  out.clear();
  for (size_t i = 0; i < docs.size(); ++i) {
    if (i) out += "---\n";
    out += docs[i];
  }
  return ISIM_OK;
}

}  // namespace isim
