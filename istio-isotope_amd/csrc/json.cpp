#include "json.h"

#include <cstdio>

namespace isim {
namespace {

struct Parser {
  const char *p;
  const char *end;
  const char *begin;
  std::string err;
  int depth = 0;

  bool fail(const char *what) {
    if (err.empty()) {
      char buf[160];
      if (p >= end)
        snprintf(buf, sizeof buf, "unexpected end of JSON input");
      else
        snprintf(buf, sizeof buf, "invalid character '%c' %s (offset %ld)", *p, what,
                 (long)(p - begin));
      err = buf;
    }
    return false;
  }
  void ws() {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  static void put_utf8(std::string &o, unsigned cp) {
    if (cp < 0x80) {
      o += (char)cp;
    } else if (cp < 0x800) {
      o += (char)(0xC0 | (cp >> 6));
      o += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      o += (char)(0xE0 | (cp >> 12));
      o += (char)(0x80 | ((cp >> 6) & 0x3F));
      o += (char)(0x80 | (cp & 0x3F));
    } else {
      o += (char)(0xF0 | (cp >> 18));
      o += (char)(0x80 | ((cp >> 12) & 0x3F));
      o += (char)(0x80 | ((cp >> 6) & 0x3F));
      o += (char)(0x80 | (cp & 0x3F));
    }
  }
  bool hex4(unsigned &v) {
    v = 0;
    for (int i = 0; i < 4; ++i) {
      if (p >= end) return fail("in string escape code");
      char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (unsigned)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (unsigned)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (unsigned)(c - 'A' + 10);
      else { --p; return fail("in \\u hexadecimal character escape"); }
    }
    return true;
  }
  bool str(std::string &o) {
    ++p;  // opening quote
    while (true) {
      if (p >= end) return fail("in string literal");
      unsigned char c = (unsigned char)*p;
      if (c == '"') { ++p; return true; }
      if (c < 0x20) return fail("in string literal");
      if (c != '\\') { o += (char)c; ++p; continue; }
      ++p;
      if (p >= end) return fail("in string escape code");
      char e = *p++;
      switch (e) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          unsigned v;
          if (!hex4(v)) return false;
          if (v >= 0xD800 && v < 0xDC00) {
            // surrogate pair; a lone surrogate decodes to U+FFFD as in Go
            if (p + 6 <= end && p[0] == '\\' && p[1] == 'u') {
              const char *save = p;
              p += 2;
              unsigned lo;
              if (!hex4(lo)) return false;
              if (lo >= 0xDC00 && lo < 0xE000) {
                put_utf8(o, 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00));
              } else {
                put_utf8(o, 0xFFFD);
                p = save;
              }
            } else {
              put_utf8(o, 0xFFFD);
            }
          } else if (v >= 0xDC00 && v < 0xE000) {
            put_utf8(o, 0xFFFD);
          } else {
            put_utf8(o, v);
          }
          break;
        }
        default: --p; return fail("in string escape code");
      }
    }
  }
  bool num(std::string &o) {
    const char *s = p;
    if (*p == '-') ++p;
    if (p >= end) return fail("in numeric literal");
    if (*p == '0') {
      ++p;
    } else if (*p >= '1' && *p <= '9') {
      while (p < end && *p >= '0' && *p <= '9') ++p;
    } else {
      return fail("in numeric literal");
    }
    if (p < end && *p == '.') {
      ++p;
      if (p >= end || !(*p >= '0' && *p <= '9')) return fail("after decimal point in numeric literal");
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    if (p < end && (*p == 'e' || *p == 'E')) {
      ++p;
      if (p < end && (*p == '+' || *p == '-')) ++p;
      if (p >= end || !(*p >= '0' && *p <= '9')) return fail("in exponent of numeric literal");
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    o.assign(s, p - s);
    return true;
  }
  bool lit(const char *w, size_t n) {
    if ((size_t)(end - p) < n) { p = end; return fail("in literal"); }
    for (size_t i = 0; i < n; ++i)
      if (p[i] != w[i]) { p += i; return fail("in literal"); }
    p += n;
    return true;
  }
  bool value(JVal &v) {
    if (++depth > 10000) return fail("exceeded max depth");
    ws();
    if (p >= end) return fail("looking for beginning of value");
    bool ok = true;
    switch (*p) {
      case '{': {
        v.kind = JVal::Obj;
        ++p;
        ws();
        if (p < end && *p == '}') { ++p; break; }
        while (true) {
          ws();
          if (p >= end || *p != '"') { ok = fail("looking for beginning of object key string"); break; }
          std::string k;
          if (!str(k)) { ok = false; break; }
          ws();
          if (p >= end || *p != ':') { ok = fail("after object key"); break; }
          ++p;
          v.obj.emplace_back(std::move(k), JVal());
          if (!value(v.obj.back().second)) { ok = false; break; }
          ws();
          if (p < end && *p == ',') { ++p; continue; }
          if (p < end && *p == '}') { ++p; break; }
          ok = fail("after object key:value pair");
          break;
        }
        break;
      }
      case '[': {
        v.kind = JVal::Arr;
        ++p;
        ws();
        if (p < end && *p == ']') { ++p; break; }
        while (true) {
          v.arr.emplace_back();
          if (!value(v.arr.back())) { ok = false; break; }
          ws();
          if (p < end && *p == ',') { ++p; continue; }
          if (p < end && *p == ']') { ++p; break; }
          ok = fail("after array element");
          break;
        }
        break;
      }
      case '"': v.kind = JVal::Str; ok = str(v.s); break;
      case 't': v.kind = JVal::Bool; v.b = true; ok = lit("true", 4); break;
      case 'f': v.kind = JVal::Bool; v.b = false; ok = lit("false", 5); break;
      case 'n': v.kind = JVal::Null; ok = lit("null", 4); break;
      default:
        if (*p == '-' || (*p >= '0' && *p <= '9')) { v.kind = JVal::Num; ok = num(v.s); }
        else ok = fail("looking for beginning of value");
    }
    --depth;
    return ok;
  }
};

}  // namespace

bool json_parse(const char *text, size_t len, JVal &out, std::string &err) {
  Parser ps{text, text + len, text, std::string()};
  out = JVal();
  if (!ps.value(out)) { err = ps.err; return false; }
  ps.ws();
  if (ps.p != ps.end) { ps.fail("after top-level value"); err = ps.err; return false; }
  return true;
}

}  // namespace isim
