// Wave-level simulation of the lane tree walk loop (tree.hip, kernel kind 7)
// on the CPU: 64 lanes stepping tree_walk.h's Lane in lock step with the
// kernel's refill, counting wave iterations and Philox executions (the open
// site runs when any lane of the wave opens a calling invocation) per 64
// traces, and which Philox sites (a call block past the fourth call, an error
// block, the skip residues of an open) the wave runs per iteration.  Build
// (g++, from the repo root; -DTW_... selects tree_walk.h variants):
//   C=istio-isotope_amd/csrc; g++ -O2 -std=c++17 -Iinclude -I$C tools/tree_wave_sim.cpp \
//     $C/json.cpp $C/gounits.cpp $C/graph.cpp $C/program.cpp $C/marshal.cpp -o /tmp/tree_wave_sim
//   /tmp/tree_wave_sim graph.json [waves]
// ("Round 3 — macro steps": config 4 at 10.4 iterations per 64
// traces, 12.5 without the end-of-step close, 25.9 for round 2's one-position
// steps.)
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <vector>

#include "graph.h"
#include "kernel_abi.h"
#include "program.h"
#include "tree_walk.h"

using namespace isim;

namespace {
struct NullSink {
  void call(uint32_t) {}
  void resp(uint32_t, uint32_t, uint32_t, bool) {}
  void resp_leaf(uint32_t, bool) {}
};
}  // namespace

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  std::ifstream f(argv[1]);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string js = ss.str();
  ServiceGraph g;
  std::string err;
  if (!unmarshal_service_graph(js.data(), js.size(), g, err)) return 2;
  int32_t entry = 0;
  for (size_t i = 0; i < g.services.size(); ++i)
    if (g.services[i].is_entrypoint) {
      entry = (int32_t)i;
      break;
    }
  isim_params p{};
  p.seed = 0x15070be;
  p.hop_base_ns = 250000;
  p.req_ps_per_byte = 80;
  p.resp_ps_per_byte = 80;
  p.flags = ISIM_FLAG_DYNAMIC;
  Program prog;
  if (compile_program(g, entry, p, prog, err) != ISIM_OK || prog.tree_nodes.empty()) return 3;
  const tw::CpuNodes nodes{prog.tree_nodes.data()};
  const TreeExt *ext = prog.tree_ext.data();
  const TreeStep *stp = prog.tree_step.data();
  NullSink sk;
  const int waves = argc > 2 ? atoi(argv[2]) : 100, per_wave = 1024;
  uint64_t next = 0, it = 0, execs = 0, lanes = 0, hops = 0, siteA = 0, siteB = 0, merged = 0;
  for (int w = 0; w < waves; ++w) {
    std::vector<tw::Lane<16, true, true>> L(64);
    std::vector<bool> act(64, false);
    int issued = 0;
    while (true) {
      for (int l = 0; l < 64; ++l)
        if (act[l] && L[l].done) {
          act[l] = false;
          hops += L[l].hops();
        }
      for (int l = 0; l < 64; ++l)
        if (!act[l] && issued < per_wave) {
          L[l].start(next++);
          act[l] = true;
          ++issued;
        }
      bool any = false;
      for (int l = 0; l < 64; ++l) any = any || act[l];
      if (!any) break;
      uint32_t opening = 0, nA = 0, nB = 0, maxBC = 0;
      for (int l = 0; l < 64; ++l) {
        if (!act[l] || L[l].done) continue;
        const uint32_t d0 = L[l].d, eb = L[l].ek_blk, fp = L[l].f_pos, kb = L[l].f_kb();
        const bool entry_step = L[l].p == 0;
        L[l].step(nodes, ext, stp, sk, (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
        const bool C = L[l].d > d0 || (entry_step && !L[l].done);  // drew its skip residues at an open
        const bool B = L[l].ek_blk != eb;                          // drew an error block
        const bool A = !C && L[l].d == d0 && L[l].f_pos == fp && L[l].f_kb() != kb;
        opening += C;
        nA += A;
        nB += B;
        maxBC = std::max<uint32_t>(maxBC, (uint32_t)B + (uint32_t)C);
      }
      if (opening) {
        ++execs;
        lanes += opening;
      }
      siteA += nA > 0;
      siteB += nB > 0;
      merged += maxBC;
      ++it;
    }
  }
  const double n64 = (double)waves * per_wave / 64;
  std::printf("wave iterations per 64 traces %.2f; Philox open-site executions per 64 traces %.2f (%.1f lanes each); "
              "hops per trace %.3f\n", it / n64, execs / n64, execs ? (double)lanes / execs : 0.0,
              hops / (n64 * 64));
  std::printf("per 64 traces: block-residue site %.2f, error site %.2f, open site %.2f; error + open sites merged %.2f\n",
              siteA / n64, siteB / n64, execs / n64, merged / n64);
  return 0;
}
