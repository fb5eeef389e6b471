#include "gounits.h"

#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace isim {
namespace {

const int64_t kInt64Max = INT64_MAX;

bool lower_eq(const std::string &a, const char *b) {
  size_t n = strlen(b);
  if (a.size() != n) return false;
  for (size_t i = 0; i < n; ++i)
    if (tolower((unsigned char)a[i]) != b[i]) return false;
  return true;
}

bool is_dec(char c) { return c >= '0' && c <= '9'; }
bool is_hex(char c) { return is_dec(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }

// [+-]?(\d+(\.\d*)?|\.\d+)([eE][+-]?\d+)?
bool dec_syntax(const std::string &s) {
  size_t i = 0, n = s.size();
  if (i < n && (s[i] == '+' || s[i] == '-')) ++i;
  size_t d0 = i;
  while (i < n && is_dec(s[i])) ++i;
  bool intd = i > d0;
  bool fracd = false;
  if (i < n && s[i] == '.') {
    ++i;
    size_t f0 = i;
    while (i < n && is_dec(s[i])) ++i;
    fracd = i > f0;
  }
  if (!intd && !fracd) return false;
  if (i < n && (s[i] == 'e' || s[i] == 'E')) {
    ++i;
    if (i < n && (s[i] == '+' || s[i] == '-')) ++i;
    size_t e0 = i;
    while (i < n && is_dec(s[i])) ++i;
    if (i == e0) return false;
  }
  return i == n;
}

// [+-]?0[xX](h+(\.h*)?|\.h+)[pP][+-]?\d+
bool hex_syntax(const std::string &s) {
  size_t i = 0, n = s.size();
  if (i < n && (s[i] == '+' || s[i] == '-')) ++i;
  if (!(i + 1 < n && s[i] == '0' && (s[i + 1] == 'x' || s[i + 1] == 'X'))) return false;
  i += 2;
  size_t d0 = i;
  while (i < n && is_hex(s[i])) ++i;
  bool intd = i > d0, fracd = false;
  if (i < n && s[i] == '.') {
    ++i;
    size_t f0 = i;
    while (i < n && is_hex(s[i])) ++i;
    fracd = i > f0;
  }
  if (!intd && !fracd) return false;
  if (!(i < n && (s[i] == 'p' || s[i] == 'P'))) return false;
  ++i;
  if (i < n && (s[i] == '+' || s[i] == '-')) ++i;
  size_t e0 = i;
  while (i < n && is_dec(s[i])) ++i;
  return i > e0 && i == n;
}

std::string quote(const std::string &s) { return "\"" + s + "\""; }

}  // namespace

bool go_parse_float(const std::string &s, double &out, std::string &err) {
  std::string body = s;
  bool neg = false;
  if (!body.empty() && (body[0] == '+' || body[0] == '-')) {
    neg = body[0] == '-';
    body = body.substr(1);
  }
  if (lower_eq(body, "inf") || lower_eq(body, "infinity")) {
    out = neg ? -INFINITY : INFINITY;
    return true;
  }
  if (lower_eq(s, "nan")) {
    out = NAN;
    return true;
  }
  if (!dec_syntax(s) && !hex_syntax(s)) {
    err = "strconv.ParseFloat: parsing " + quote(s) + ": invalid syntax";
    return false;
  }
  errno = 0;
  char *endp = nullptr;
  double v = strtod(s.c_str(), &endp);
  if (std::isinf(v)) {
    err = "strconv.ParseFloat: parsing " + quote(s) + ": value out of range";
    return false;
  }
  out = v;
  return true;
}

bool go_parse_int(const std::string &s, int bits, int64_t &out) {
  size_t i = 0, n = s.size();
  bool neg = false;
  if (i < n && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; ++i; }
  if (i == n) return false;
  unsigned __int128 v = 0;
  for (; i < n; ++i) {
    if (!is_dec(s[i])) return false;
    v = v * 10 + (unsigned)(s[i] - '0');
    if (v > ((unsigned __int128)1 << 64)) v = ((unsigned __int128)1 << 64);  // saturate
  }
  unsigned __int128 lim_pos = ((unsigned __int128)1 << (bits - 1)) - 1;
  unsigned __int128 lim_neg = ((unsigned __int128)1 << (bits - 1));
  if (neg ? v > lim_neg : v > lim_pos) return false;
  out = neg ? (int64_t)(-(__int128)v) : (int64_t)v;
  return true;
}

// go-units v0.4.0 parseSize(sizeStr, binaryMap):
//   regex ^(\d+(\.\d+)*) ?([kKmMgGtTpP])?[iI]?[bB]?$ ; ParseFloat(group1);
//   size *= unit; return int64(size)
bool go_ram_in_bytes(const std::string &s, int64_t &out, std::string &err) {
  size_t i = 0, n = s.size();
  size_t g0 = i;
  auto digits = [&]() {
    size_t st = i;
    while (i < n && is_dec(s[i])) ++i;
    return i > st;
  };
  bool ok = digits();
  while (ok && i + 1 < n && s[i] == '.' && is_dec(s[i + 1])) {
    ++i;
    digits();
  }
  size_t g1 = i;
  if (ok && i < n && s[i] == ' ') ++i;
  char unit = 0;
  if (ok && i < n && strchr("kKmMgGtTpP", s[i])) unit = (char)tolower((unsigned char)s[i++]);
  if (ok && i < n && (s[i] == 'i' || s[i] == 'I')) ++i;
  if (ok && i < n && (s[i] == 'b' || s[i] == 'B')) ++i;
  if (!ok || i != n) {
    err = "invalid size: '" + s + "'";
    return false;
  }
  double size;
  if (!go_parse_float(s.substr(g0, g1 - g0), size, err)) return false;
  double mul = 1.0;
  switch (unit) {
    case 'k': mul = 1024.0; break;
    case 'm': mul = 1048576.0; break;
    case 'g': mul = 1073741824.0; break;
    case 't': mul = 1099511627776.0; break;
    case 'p': mul = 1125899906842624.0; break;
    default: break;
  }
  if (unit) size *= mul;
  // Go float64 -> int64 on amd64: truncation; out of range / NaN -> INT64_MIN
  if (std::isnan(size) || size >= 9223372036854775808.0 || size < -9223372036854775808.0)
    out = INT64_MIN;
  else
    out = (int64_t)size;
  return true;
}

bool size_from_int64(int64_t x, uint64_t &out, std::string &err) {
  if (x < 0) {
    err = std::to_string(x) + " must be non-negative";
    return false;
  }
  out = (uint64_t)x;
  return true;
}

bool size_from_string(const std::string &s, uint64_t &out, std::string &err) {
  int64_t x;
  if (!go_ram_in_bytes(s, x, err)) return false;
  return size_from_int64(x, out, err);
}

// Go time.ParseDuration (go 1.14-1.16).
bool go_parse_duration(const std::string &orig, int64_t &out, std::string &err) {
  std::string s = orig;
  int64_t d = 0;
  bool neg = false;
  auto invalid = [&]() {
    err = "time: invalid duration " + quote(orig);
    return false;
  };
  if (!s.empty() && (s[0] == '-' || s[0] == '+')) {
    neg = s[0] == '-';
    s = s.substr(1);
  }
  if (s == "0") { out = 0; return true; }
  if (s.empty()) return invalid();
  size_t i = 0, n = s.size();
  while (i < n) {
    int64_t v = 0, f = 0;
    double scale = 1.0;
    if (!(s[i] == '.' || is_dec(s[i]))) return invalid();
    size_t pl = i;
    while (i < n && is_dec(s[i])) {
      if (v > kInt64Max / 10) return invalid();
      v = v * 10 + (s[i] - '0');
      if (v < 0) return invalid();
      ++i;
    }
    bool pre = i != pl;
    bool post = false;
    if (i < n && s[i] == '.') {
      ++i;
      size_t fl = i;
      bool overflow = false;
      while (i < n && is_dec(s[i])) {
        if (!overflow) {
          if (f > kInt64Max / 10) {
            overflow = true;
          } else {
            int64_t y = f * 10 + (s[i] - '0');
            if (y < 0) overflow = true;
            else { f = y; scale *= 10.0; }
          }
        }
        ++i;
      }
      post = i != fl;
    }
    if (!pre && !post) return invalid();
    size_t u0 = i;
    while (i < n && !(s[i] == '.' || is_dec(s[i]))) ++i;
    if (i == u0) {
      err = "time: missing unit in duration " + quote(orig);
      return false;
    }
    std::string u = s.substr(u0, i - u0);
    int64_t unit;
    if (u == "ns") unit = 1;
    else if (u == "us" || u == "\xC2\xB5s" || u == "\xCE\xBCs") unit = 1000;
    else if (u == "ms") unit = 1000000;
    else if (u == "s") unit = 1000000000LL;
    else if (u == "m") unit = 60LL * 1000000000LL;
    else if (u == "h") unit = 3600LL * 1000000000LL;
    else {
      err = "time: unknown unit " + quote(u) + " in duration " + quote(orig);
      return false;
    }
    if (v > kInt64Max / unit) return invalid();
    v *= unit;
    if (f > 0) {
      v += (int64_t)((double)f * ((double)unit / scale));
      if (v < 0) return invalid();
    }
    d += v;
    if (d < 0) return invalid();
  }
  out = neg ? -d : d;
  return true;
}

std::string go_float_v(double f) {
  if (std::isnan(f)) return "NaN";
  if (std::isinf(f)) return f > 0 ? "+Inf" : "-Inf";
  // shortest round-trip digits
  char buf[64];
  for (int prec = 1; prec <= 17; ++prec) {
    snprintf(buf, sizeof buf, "%.*e", prec - 1, f);
    if (strtod(buf, nullptr) == f) break;
  }
  // buf = d.ddde[+-]XX ; Go %v uses %e when exp < -4 || exp >= 21
  std::string m(buf);
  size_t e = m.find('e');
  int exp = atoi(m.c_str() + e + 1);
  std::string mant = m.substr(0, e);
  bool negv = mant[0] == '-';
  if (negv) mant = mant.substr(1);
  std::string digs;
  for (char c : mant)
    if (c != '.') digs += c;
  while (digs.size() > 1 && digs.back() == '0') digs.pop_back();
  std::string r;
  if (exp < -4 || exp >= 21) {
    r = digs.substr(0, 1);
    if (digs.size() > 1) r += "." + digs.substr(1);
    char eb[16];
    snprintf(eb, sizeof eb, "e%c%02d", exp < 0 ? '-' : '+', exp < 0 ? -exp : exp);
    r += eb;
  } else if (exp < 0) {
    r = "0." + std::string((size_t)(-exp - 1), '0') + digs;
  } else if ((size_t)exp + 1 >= digs.size()) {
    r = digs + std::string((size_t)exp + 1 - digs.size(), '0');
  } else {
    r = digs.substr(0, (size_t)exp + 1) + "." + digs.substr((size_t)exp + 1);
  }
  return (negv ? "-" : "") + r;
}

bool pct_from_float(double f, double &out, std::string &err) {
  if (0.0 <= f && f <= 1.0) {
    out = f;
    return true;
  }
  err = "percentage " + go_float_v(f) + " is out of range (must be between 0.0 and 1.0)";
  return false;
}

bool pct_from_string(const std::string &s, double &out, std::string &err) {
  size_t idx = s.find('%');
  std::string inv = "invalid percentage as string: " + s + " (must be between \"0%\" and \"100%\")";
  if (idx == std::string::npos) {
    err = inv;
    return false;
  }
  double f;
  std::string e2;
  if (!go_parse_float(s.substr(0, idx), f, e2)) {
    err = inv;
    return false;
  }
  return pct_from_float(f / 100.0, out, err);
}

uint64_t error_threshold(double p) {
  if (!(p > 0.0)) return 0;
  if (p >= 1.0) return 1ull << 32;
  return (uint64_t)(p * 4294967296.0);
}

}  // namespace isim
