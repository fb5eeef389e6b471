// Go / third-party arithmetic the isotope graph loader depends on, restated
// in C++ for the product loader.
//   go-units v0.4.0 RAMInBytes      (isotope/go.mod:6; size/byte_size.go:68)
//   Go strconv.ParseFloat / ParseInt syntax (pct/percentage.go:76; encoding/json)
//   Go time.ParseDuration           (script/sleep_command.go:32)
//   pct.FromString / FromFloat64    (pct/percentage.go:71-93)
#pragma once
#include <cstdint>
#include <string>

namespace isim {

// Each returns true on success; on failure `err` holds the Go error text.
bool go_parse_float(const std::string &s, double &out, std::string &err);
bool go_parse_int(const std::string &s, int bits, int64_t &out);
bool go_ram_in_bytes(const std::string &s, int64_t &out, std::string &err);
bool size_from_int64(int64_t x, uint64_t &out, std::string &err);
bool size_from_string(const std::string &s, uint64_t &out, std::string &err);
bool go_parse_duration(const std::string &s, int64_t &out, std::string &err);
bool pct_from_float(double f, double &out, std::string &err);
bool pct_from_string(const std::string &s, double &out, std::string &err);
// fmt %v of a float64
std::string go_float_v(double f);
// errorRate -> threshold over a u32 draw (2^32 = always). SURVEY A.1 (EXT).
uint64_t error_threshold(double p);

}  // namespace isim
