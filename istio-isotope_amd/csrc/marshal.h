// Graph emitters: the encode side of the isotope graph API.
//   json.Marshal(graph.ServiceGraph)      svc/service.go:25-51 (json tags, omitempty),
//                                          script/script.go:24-31, script/command.go:30-53,
//                                          size/byte_size.go:27-34, pct/percentage.go:28-35,
//                                          svctype/service_type.go:34-48
//   graphviz.ServiceGraphToDotLanguage    convert/pkg/graphviz/graphviz.go:28-213
// plus the Go formatting they rest on (time.Duration.String, go-units
// BytesSize, encoding/json float and string encoding).
#pragma once
#include <cstdint>
#include <string>

#include "graph.h"

namespace isim {

std::string go_duration_string(int64_t d);      // time.Duration.String()
std::string go_bytes_size(double size);          // go-units v0.4.0 BytesSize
std::string pct_string(double p);                // pct.Percentage.String()
std::string service_type_string(int32_t t);      // svctype.ServiceType.String()
void go_json_float(std::string &o, double f);    // encoding/json float64 encoder
void go_json_string(std::string &o, const std::string &s);  // encoding/json string encoder (escapeHTML)

std::string marshal_json(const ServiceGraph &g);
std::string to_dot(const ServiceGraph &g);

}  // namespace isim
