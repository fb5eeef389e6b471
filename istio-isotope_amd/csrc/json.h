// Minimal JSON DOM for the graph loader: RFC 8259 syntax as Go's
// encoding/json checkValid accepts it; numbers are kept as literal text so the
// decoder can apply Go's per-type conversions (ParseInt vs ParseFloat).
#pragma once
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace isim {

struct JVal {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  bool b = false;
  std::string s;                                   // Num: literal text; Str: decoded UTF-8
  std::vector<JVal> arr;                           // Arr
  std::vector<std::pair<std::string, JVal>> obj;   // Obj: in document order (duplicates kept)

  const char *kind_name() const {
    switch (kind) {
      case Null: return "null";
      case Bool: return "bool";
      case Num: return "number";
      case Str: return "string";
      case Arr: return "array";
      default: return "object";
    }
  }
};

// Parses `text`; on failure returns false and sets `err` to a Go-style
// syntax error message.
bool json_parse(const char *text, size_t len, JVal &out, std::string &err);

}  // namespace isim
