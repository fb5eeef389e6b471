// Service-graph loader: (*graph.ServiceGraph).UnmarshalJSON semantics over a
// JSON DOM.  Each function cites the Go code it mirrors
// (paths relative to isotope/convert/pkg/graph/).
//
// Go encoding/json behaviours reproduced (they shape what UnmarshalJSON
// accepts): object keys match struct fields exactly first, else ASCII
// case-insensitively; unknown keys are ignored; JSON null is a no-op for
// plain fields but IS passed to custom UnmarshalJSON methods (ByteSize,
// Percentage, ServiceType, Script, SleepCommand, RequestCommand, Service);
// type mismatches on plain fields are saved and reported at the end of the
// enclosing json.Unmarshal call, errors from custom methods abort at once.
#include <cstdio>
#include <cstring>
#include <unordered_set>

#include "gounits.h"
#include "graph.h"

namespace isim {
namespace {

struct Saver {
  std::string err;
  bool has = false;
  void save(const std::string &e) {
    if (!has) { has = true; err = e; }
  }
};

std::string type_err(const std::string &what, const char *gotype) {
  return "json: cannot unmarshal " + what + " into Go value of type " + gotype;
}

bool ascii_ieq(const std::string &a, const char *b) {
  size_t n = strlen(b);
  if (a.size() != n) return false;
  for (size_t i = 0; i < n; ++i) {
    char x = a[i], y = b[i];
    if (x >= 'A' && x <= 'Z') x = (char)(x - 'A' + 'a');
    if (y >= 'A' && y <= 'Z') y = (char)(y - 'A' + 'a');
    if (x != y) return false;
  }
  return true;
}

// Field lookup: exact match preferred, then case-insensitive; -1 = unknown key.
int match_field(const std::string &key, const char *const *names, int n) {
  for (int i = 0; i < n; ++i)
    if (key == names[i]) return i;
  for (int i = 0; i < n; ++i)
    if (ascii_ieq(key, names[i])) return i;
  return -1;
}

void dec_string(const JVal &v, Saver &sv, std::string &cur) {
  if (v.kind == JVal::Null) return;
  if (v.kind != JVal::Str) { sv.save(type_err(v.kind_name(), "string")); return; }
  cur = v.s;
}

void dec_bool(const JVal &v, Saver &sv, bool &cur) {
  if (v.kind == JVal::Null) return;
  if (v.kind != JVal::Bool) { sv.save(type_err(v.kind_name(), "bool")); return; }
  cur = v.b;
}

template <typename T>
void dec_int(const JVal &v, Saver &sv, T &cur, int bits) {
  char ty[16];
  snprintf(ty, sizeof ty, "int%d", bits);
  if (v.kind == JVal::Null) return;
  if (v.kind != JVal::Num) { sv.save(type_err(v.kind_name(), ty)); return; }
  int64_t x;
  if (!go_parse_int(v.s, bits, x)) { sv.save(type_err("number " + v.s, ty)); return; }
  cur = (T)x;
}

// json.Unmarshal(b, &string) as its own call (custom methods use it).
bool unmarshal_string(const JVal &v, std::string &out, std::string &err) {
  if (v.kind == JVal::Null) { out.clear(); return true; }
  if (v.kind != JVal::Str) { err = type_err(v.kind_name(), "string"); return false; }
  out = v.s;
  return true;
}

// size/byte_size.go:39-63 (*ByteSize).UnmarshalJSON
bool unmarshal_byte_size(const JVal &v, uint64_t &out, std::string &err) {
  if (v.kind == JVal::Str) return size_from_string(v.s, out, err);
  int64_t x = 0;
  if (v.kind == JVal::Num) {
    if (!go_parse_int(v.s, 64, x)) { err = type_err("number " + v.s, "int64"); return false; }
  } else if (v.kind != JVal::Null) {
    err = type_err(v.kind_name(), "int64");
    return false;
  }
  return size_from_int64(x, out, err);
}

// pct/percentage.go:41-67 (*Percentage).UnmarshalJSON
bool unmarshal_percentage(const JVal &v, double &out, std::string &err) {
  if (v.kind == JVal::Str) return pct_from_string(v.s, out, err);
  double f = 0.0;
  if (v.kind == JVal::Num) {
    std::string e2;
    if (!go_parse_float(v.s, f, e2)) { err = type_err("number " + v.s, "float64"); return false; }
  } else if (v.kind != JVal::Null) {
    err = type_err(v.kind_name(), "float64");
    return false;
  }
  return pct_from_float(f, out, err);
}

// svctype/service_type.go:51-76
bool unmarshal_service_type(const JVal &v, int32_t &out, std::string &err) {
  std::string s;
  if (!unmarshal_string(v, s, err)) return false;
  if (s == "http") { out = kServiceHTTP; return true; }
  if (s == "grpc") { out = kServiceGRPC; return true; }
  err = "unknown service type: " + s;
  return false;
}

// script/sleep_command.go:26-38
bool unmarshal_sleep(const JVal &v, Command &c, std::string &err) {
  std::string s;
  if (!unmarshal_string(v, s, err)) return false;
  int64_t d;
  if (!go_parse_duration(s, d, err)) return false;
  c = Command();
  c.kind = Command::Sleep;
  c.sleep_ns = d;
  return true;
}

// script/request_command.go:41-66 (*RequestCommand).UnmarshalJSON
bool unmarshal_request(const JVal &v, const Command &def, Command &c, std::string &err) {
  c = def;
  c.kind = Command::Request;
  if (v.kind == JVal::Str) { c.service = v.s; return true; }
  Saver sv;
  if (v.kind == JVal::Obj) {
    static const char *const kF[] = {"service", "size", "probability"};
    for (const auto &kv : v.obj) {
      switch (match_field(kv.first, kF, 3)) {
        case 0: dec_string(kv.second, sv, c.service); break;
        case 1: if (!unmarshal_byte_size(kv.second, c.size, err)) return false; break;
        case 2: dec_int(kv.second, sv, c.probability, 64); break;
        default: break;
      }
    }
  } else if (v.kind != JVal::Null) {
    err = type_err(v.kind_name(), "script.unmarshallableRequestCommand");
    return false;
  }
  if (sv.has) { err = sv.err; return false; }
  if (c.probability < 0 || c.probability > 100) {
    err = "math: invalid probability, outside range: [0,100]";
    return false;
  }
  return true;
}

bool parse_commands(const JVal &v, const Command &def_req, std::vector<Command> &out, std::string &err);

// script/command.go:73-105 (*unmarshallableCommand).UnmarshalJSON
bool unmarshal_command(const JVal &v, const Command &def_req, Command &c, std::string &err) {
  if (v.kind == JVal::Arr) {
    c = Command();
    c.kind = Command::Concurrent;
    return parse_commands(v, def_req, c.commands, err);
  }
  // parseJSONCommandKey (command.go:107-121)
  std::string key;
  if (v.kind == JVal::Obj) {
    std::vector<std::string> keys;
    for (const auto &kv : v.obj) {
      bool seen = false;
      for (const auto &k : keys) seen = seen || k == kv.first;
      if (!seen) keys.push_back(kv.first);
    }
    if (keys.size() > 1) {
      std::string m = "multiple keys for command: map[";
      for (size_t i = 0; i < keys.size(); ++i) m += (i ? " " : "") + keys[i] + ":...";
      err = m + "]";
      return false;
    }
    if (!keys.empty()) key = keys[0];
  } else if (v.kind != JVal::Null) {
    err = type_err(v.kind_name(), "map[string]interface {}");
    return false;
  }
  if (key == "sleep") {
    for (const auto &kv : v.obj)
      if (!unmarshal_sleep(kv.second, c, err)) return false;
    return true;
  }
  if (key == "call") {
    for (const auto &kv : v.obj)
      if (!unmarshal_request(kv.second, def_req, c, err)) return false;
    return true;
  }
  err = "unknown command: " + key;
  return false;
}

// script/command.go:55-68 parseJSONCommands (Script, ConcurrentCommand)
bool parse_commands(const JVal &v, const Command &def_req, std::vector<Command> &out, std::string &err) {
  out.clear();
  if (v.kind == JVal::Null) return true;
  if (v.kind != JVal::Arr) {
    err = type_err(v.kind_name(), "[]script.unmarshallableCommand");
    return false;
  }
  out.resize(v.arr.size());
  for (size_t i = 0; i < v.arr.size(); ++i)
    if (!unmarshal_command(v.arr[i], def_req, out[i], err)) return false;
  return true;
}

const char *const kServiceFields[] = {"name", "type", "numReplicas", "isEntrypoint",
                                      "errorRate", "responseSize", "script", "numRbacPolicies"};

// svc/unmarshal.go:29-41 (*Service).UnmarshalJSON starting from DefaultService
bool unmarshal_service(const JVal &v, const Service &def, const Command &def_req, Service &s,
                       std::string &err) {
  s = def;
  Saver sv;
  if (v.kind == JVal::Obj) {
    for (const auto &kv : v.obj) {
      const JVal &x = kv.second;
      switch (match_field(kv.first, kServiceFields, 8)) {
        case 0: dec_string(x, sv, s.name); break;
        case 1: if (!unmarshal_service_type(x, s.type, err)) return false; break;
        case 2: dec_int(x, sv, s.num_replicas, 32); break;
        case 3: dec_bool(x, sv, s.is_entrypoint); break;
        case 4: if (!unmarshal_percentage(x, s.error_rate, err)) return false; break;
        case 5: if (!unmarshal_byte_size(x, s.response_size, err)) return false; break;
        case 6: if (!parse_commands(x, def_req, s.script, err)) return false; break;
        case 7: dec_int(x, sv, s.num_rbac_policies, 32); break;
        default: break;
      }
    }
  } else if (v.kind != JVal::Null) {
    err = type_err(v.kind_name(), "svc.unmarshallableService");
    return false;
  }
  if (sv.has) { err = sv.err; return false; }
  if (s.name.empty()) {
    err = "services must have a name";
    return false;
  }
  return true;
}

struct Defaults {  // unmarshal.go:78-86, defaultDefaults :67-70
  int32_t type = kServiceHTTP;
  double error_rate = 0.0;
  uint64_t response_size = 0;
  std::vector<Command> script;
  uint64_t request_size = 0;
  int32_t num_replicas = 1;
  int32_t num_rbac_policies = 0;
};

const char *const kDefaultsFields[] = {"type", "errorRate", "responseSize", "script",
                                       "requestSize", "numReplicas", "numRbacPolicies"};

// json.Unmarshal(b, &serviceGraphJSONMetadata{Defaults: defaultDefaults}),
// unmarshal.go:31-32.  The default script is decoded while
// script.DefaultRequestCommand is still the zero value (quirk F11).
bool decode_defaults(const JVal &doc, Defaults &d, std::string &err) {
  Saver sv;
  Command zero_req;
  zero_req.kind = Command::Request;
  if (doc.kind == JVal::Null) return true;
  if (doc.kind != JVal::Obj) {
    err = type_err(doc.kind_name(), "graph.serviceGraphJSONMetadata");
    return false;
  }
  static const char *const kTop[] = {"defaults"};
  for (const auto &kv : doc.obj) {
    if (match_field(kv.first, kTop, 1) != 0) continue;
    const JVal &v = kv.second;
    if (v.kind == JVal::Null) continue;
    if (v.kind != JVal::Obj) { sv.save(type_err(v.kind_name(), "graph.defaults")); continue; }
    for (const auto &f : v.obj) {
      const JVal &x = f.second;
      switch (match_field(f.first, kDefaultsFields, 7)) {
        case 0: if (!unmarshal_service_type(x, d.type, err)) return false; break;
        case 1: if (!unmarshal_percentage(x, d.error_rate, err)) return false; break;
        case 2: if (!unmarshal_byte_size(x, d.response_size, err)) return false; break;
        case 3: if (!parse_commands(x, zero_req, d.script, err)) return false; break;
        case 4: if (!unmarshal_byte_size(x, d.request_size, err)) return false; break;
        case 5: dec_int(x, sv, d.num_replicas, 32); break;
        case 6: dec_int(x, sv, d.num_rbac_policies, 32); break;
        default: break;
      }
    }
  }
  if (sv.has) { err = sv.err; return false; }
  return true;
}

bool contains_concurrent(const std::vector<Command> &cmds) {
  for (const auto &c : cmds)
    if (c.kind == Command::Concurrent) return true;
  return false;
}

// validation.go:41-57 validateCommands
bool validate_commands(const std::vector<Command> &cmds, const std::unordered_set<std::string> &names,
                       std::string &err) {
  for (const auto &c : cmds) {
    if (c.kind == Command::Request) {
      if (!names.count(c.service)) {
        err = "cannot call undefined service \"" + c.service + "\"";
        return false;
      }
    } else if (c.kind == Command::Concurrent) {
      if (!validate_commands(c.commands, names, err)) return false;
      if (contains_concurrent(c.commands)) {
        err = "concurrent commands may not be nested";
        return false;
      }
    }
  }
  return true;
}

// validation.go:28-39 validate
bool validate(const ServiceGraph &g, std::string &err) {
  std::unordered_set<std::string> names;
  for (const auto &s : g.services) names.insert(s.name);
  for (const auto &s : g.services)
    if (!validate_commands(s.script, names, err)) return false;
  return true;
}

void json_str(std::string &o, const std::string &s) {
  o += '"';
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') { o += '\\'; o += (char)c; }
    else if (c < 0x20) {
      char b[8];
      snprintf(b, sizeof b, "\\u%04x", c);
      o += b;
    } else o += (char)c;
  }
  o += '"';
}

void canon_cmd(std::string &o, const Command &c) {
  char b[96];
  if (c.kind == Command::Sleep) {
    snprintf(b, sizeof b, "[\"sleep\",%lld]", (long long)c.sleep_ns);
    o += b;
  } else if (c.kind == Command::Request) {
    o += "[\"call\",";
    json_str(o, c.service);
    snprintf(b, sizeof b, ",%llu,%lld]", (unsigned long long)c.size, (long long)c.probability);
    o += b;
  } else {
    o += "[\"conc\",[";
    for (size_t i = 0; i < c.commands.size(); ++i) {
      if (i) o += ',';
      canon_cmd(o, c.commands[i]);
    }
    o += "]]";
  }
}

}  // namespace

bool unmarshal_service_graph(const char *json, size_t len, ServiceGraph &g, std::string &err) {
  JVal doc;
  if (!json_parse(json, len, doc, err)) return false;
  Defaults d;
  if (!decode_defaults(doc, d, err)) return false;
  // withGlobalDefaults (unmarshal.go:88-112)
  Service def;
  def.type = d.type;
  def.num_replicas = d.num_replicas;
  def.error_rate = d.error_rate;
  def.response_size = d.response_size;
  def.script = d.script;
  def.num_rbac_policies = d.num_rbac_policies;
  Command def_req;
  def_req.kind = Command::Request;
  def_req.size = d.request_size;
  g.services.clear();
  g.services_nil = true;
  Saver sv;
  static const char *const kTop[] = {"services"};
  if (doc.kind == JVal::Obj) {
    for (const auto &kv : doc.obj) {
      if (match_field(kv.first, kTop, 1) != 0) continue;
      const JVal &v = kv.second;
      if (v.kind == JVal::Null) { g.services.clear(); g.services_nil = true; continue; }
      if (v.kind != JVal::Arr) { sv.save(type_err(v.kind_name(), "[]svc.Service")); continue; }
      g.services.assign(v.arr.size(), Service());
      g.services_nil = false;
      for (size_t i = 0; i < v.arr.size(); ++i)
        if (!unmarshal_service(v.arr[i], def, def_req, g.services[i], err)) return false;
    }
  }
  if (sv.has) { err = sv.err; return false; }
  return validate(g, err);
}

std::string canonical_json(const ServiceGraph &g) {
  std::string o = "{\"services\":[";
  char b[256];
  for (size_t i = 0; i < g.services.size(); ++i) {
    const Service &s = g.services[i];
    if (i) o += ',';
    o += "{\"name\":";
    json_str(o, s.name);
    uint64_t bits;
    memcpy(&bits, &s.error_rate, 8);
    snprintf(b, sizeof b,
             ",\"type\":%d,\"numReplicas\":%d,\"isEntrypoint\":%s,\"errorRateBits\":%llu,"
             "\"responseSize\":%llu,\"numRbacPolicies\":%d,\"script\":[",
             s.type, s.num_replicas, s.is_entrypoint ? "true" : "false", (unsigned long long)bits,
             (unsigned long long)s.response_size, s.num_rbac_policies);
    o += b;
    for (size_t j = 0; j < s.script.size(); ++j) {
      if (j) o += ',';
      canon_cmd(o, s.script[j]);
    }
    o += "]}";
  }
  o += "]}";
  return o;
}

}  // namespace isim
