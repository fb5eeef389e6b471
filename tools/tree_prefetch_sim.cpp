// CPU simulation of a skip-residue prefetch for the lane tree walk (kernel
// kind 7): 64 lanes step tree_walk.h's Lane in lock
// step with the kernel's refill; each lane keeps a FIFO of K prefetched
// Philox residue blocks for its next hop ids, refilled in a wave-wide phase
// when at least T lanes have room; an open whose block is not ready draws it
// inline.  Prints the Philox executions per 64 traces of the kernel as built
// (one open site per iteration) and of the prefetch policy.  Build (repo root):
//   C=istio-isotope_amd/csrc; g++ -O2 -std=c++17 -Iinclude -I$C tools/tree_prefetch_sim.cpp \
//     $C/json.cpp $C/gounits.cpp $C/graph.cpp $C/program.cpp -o /tmp/tree_prefetch_sim
//   /tmp/tree_prefetch_sim graph.json K T
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <vector>
#include "graph.h"
#include "kernel_abi.h"
#include "program.h"
#include "tree_walk.h"
using namespace isim;
struct NullSink { const Program *pg; int opened = 0; void call(uint32_t slot) { opened = !(pg->slot_tbkt[slot] & kTreeLeafSlot); } void resp(uint32_t, uint32_t, uint32_t, bool) {} void resp_leaf(uint32_t, bool) {} };
int main(int argc, char **argv) {
  std::ifstream f(argv[1]); std::stringstream ss; ss << f.rdbuf(); const std::string js = ss.str();
  ServiceGraph g; std::string err;
  if (!unmarshal_service_graph(js.data(), js.size(), g, err)) return 2;
  int32_t entry = 0;
  for (size_t i = 0; i < g.services.size(); ++i) if (g.services[i].is_entrypoint) { entry = (int32_t)i; break; }
  isim_params p{}; p.seed = 0x15070be; p.hop_base_ns = 250000; p.req_ps_per_byte = 80; p.resp_ps_per_byte = 80; p.flags = ISIM_FLAG_DYNAMIC;
  Program prog;
  if (compile_program(g, entry, p, prog, err) != ISIM_OK || prog.tree_nodes.empty()) return 3;
  const tw::CpuNodes nodes{prog.tree_nodes.data()};
  const int K = atoi(argv[2]), T = atoi(argv[3]);  // FIFO depth, phase threshold (lanes needing refill)
  const int waves = 200, per_wave = 1024;
  NullSink sk; sk.pg = &prog;
  uint64_t next = 0, it = 0, base_ex = 0, base_l = 0, inl_ex = 0, inl_l = 0, ph_ex = 0, ph_l = 0, waste = 0, used = 0;
  for (int w = 0; w < waves; ++w) {
    std::vector<tw::Lane<16, false, true>> L(64);
    std::vector<bool> act(64, false);
    std::vector<uint32_t> qh(64, 0), qn(64, 0);
    int issued = 0;
    while (true) {
      for (int l = 0; l < 64; ++l) if (act[l] && L[l].done) act[l] = false;
      for (int l = 0; l < 64; ++l) if (!act[l] && issued < per_wave) { L[l].start(next++); act[l] = true; ++issued; qh[l] = 0; qn[l] = 0; }
      bool any = false;
      for (int l = 0; l < 64; ++l) any = any || act[l];
      if (!any) break;
      uint32_t opening = 0, miss = 0;
      for (int l = 0; l < 64; ++l) {
        if (!act[l] || L[l].done) continue;
        const uint32_t h0 = L[l].hops(); const bool es = L[l].p == 0;
        sk.opened = 0;
        L[l].step(nodes, prog.tree_ext.data(), prog.tree_step.data(), sk, (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
        const bool open = es ? !(prog.tree_nodes[0].flags & TF_LEAF) : (sk.opened && L[l].hops() > h0);
        const uint32_t h1 = L[l].hops();
        for (uint32_t h = h0; h < h1; ++h) {
          const bool hit = qn[l] > 0 && qh[l] == h;
          if (open && h == h1 - 1) { opening++; if (!hit) miss++; else used++; }
          else if (hit) waste++;
          if (hit) { qh[l]++; qn[l]--; } else if (qn[l] == 0) qh[l] = h + 1; else { qh[l] = h + 1; qn[l] = 0; }
        }
      }
      if (opening) { base_ex++; base_l += opening; }
      if (miss) { inl_ex++; inl_l += miss; }
      // prefetch phase
      uint32_t need = 0;
      for (int l = 0; l < 64; ++l) if (act[l] && !L[l].done && qn[l] < (uint32_t)K) need++;
      if (need >= (uint32_t)T && need) {
        ph_ex++; ph_l += need;
        for (int l = 0; l < 64; ++l) if (act[l] && !L[l].done && qn[l] < (uint32_t)K) { if (qn[l] == 0) qh[l] = L[l].hops(); qn[l]++; }
      }
      ++it;
    }
  }
  const double n64 = (double)waves * per_wave / 64;
  printf("K=%d T=%d: iterations %.2f; baseline open execs %.2f (%.1f lanes); prefetch: inline %.2f (%.1f lanes) + phases %.2f (%.1f lanes) = %.2f execs; used %.2f wasted %.2f per 64 traces\n",
         K, T, it / n64, base_ex / n64, base_ex ? (double)base_l / base_ex : 0, inl_ex / n64, inl_ex ? (double)inl_l / inl_ex : 0,
         ph_ex / n64, ph_ex ? (double)ph_l / ph_ex : 0, (inl_ex + ph_ex) / n64, used / n64, waste / n64);
}
