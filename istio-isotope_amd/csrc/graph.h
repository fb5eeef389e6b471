// Service-graph model and loader: the C++ host side of the isotope graph API
// (isotope/convert/pkg/graph).  Types mirror the Go ones:
//   graph.ServiceGraph   convert/pkg/graph/graph.go:21-23
//   svc.Service          convert/pkg/graph/svc/service.go:25-51
//   script.Command       convert/pkg/graph/script/{sleep,request,concurrent}_command.go
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "json.h"

namespace isim {

enum ServiceType : int32_t { kServiceUnknown = 0, kServiceHTTP = 1, kServiceGRPC = 2 };

struct Command {
  enum Kind : int32_t { Sleep = 0, Request = 1, Concurrent = 2 } kind = Sleep;
  int64_t sleep_ns = 0;            // SleepCommand (time.Duration)
  std::string service;             // RequestCommand.ServiceName
  uint64_t size = 0;               // RequestCommand.Size (size.ByteSize)
  int64_t probability = 0;         // RequestCommand.Probability (0 = always)
  std::vector<Command> commands;   // ConcurrentCommand
};

struct Service {
  std::string name;
  int32_t type = kServiceHTTP;
  int32_t num_replicas = 1;
  bool is_entrypoint = false;
  double error_rate = 0.0;         // pct.Percentage
  uint64_t response_size = 0;      // size.ByteSize
  std::vector<Command> script;     // script.Script
  int32_t num_rbac_policies = 0;
};

struct ServiceGraph {
  std::vector<Service> services;
  bool services_nil = true;  // Go: a nil slice (key absent or null) marshals as null, [] as []
};

// (*ServiceGraph).UnmarshalJSON (convert/pkg/graph/unmarshal.go:30-48):
// defaults, per-service defaults, command decoding and validate().  On error
// returns false with the Go error text in `err`.
bool unmarshal_service_graph(const char *json, size_t len, ServiceGraph &g, std::string &err);

// Implementation-neutral exact dump, compared against the
// oracle's restatement in the parity tests.
std::string canonical_json(const ServiceGraph &g);

}  // namespace isim
