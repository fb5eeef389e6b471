// CPU run of the lane tree walk (tree_walk.h, kernel kind 7) over the
// product's own loader and program compiler: the per-lane code the HIP
// kernel executes, with the kernel's accounting of the statistics (per-slot
// counters, per-row duration sums, static-bucket rows derived from the
// counters at the end, the entry's row from the trace results).  Prints the
// results in the oracle's terms so tests/test_tree_walk.py can compare them
// with oracle/executor.py bit for bit.  Test infrastructure only.
//   tree_walk_check <graph.json> <mode 0|1> <seed> <hop_base> <req_ps> <resp_ps> <begin> <n>
// Output (one line each): "why <reason>" and exit 3 if no tree; else
//   rec <lat> <hops> <status500> <err_hops>          per trace
//   site <calls...>                                   per call site
//   svc <calls...> / err <errs...>                    per service
//   dur <svc> <68 words>                              per reachable service
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <sstream>
#include <vector>

#include "graph.h"
#include "kernel_abi.h"
#include "program.h"
#include "tree_walk.h"

using namespace isim;

namespace {

struct Sink {
  const Program *prog = nullptr;
  std::vector<uint64_t> calls, errs;                // per slot
  std::vector<uint64_t> sum200, sum500;             // per row (HBM in the kernel, or its LDS sums)
  std::vector<std::vector<uint64_t>> gbucket;       // per row: [2][33] the global-atomic buckets
  std::map<uint32_t, std::vector<uint64_t>> dyn;    // the LDS code-200 bucket tables, by header offset
  std::map<uint32_t, uint32_t> hdr;                 // their header words (b_lo | width << 8)
  bool out_of_table = false;
  bool wide = false;  // a wide tree (tree.hip WideSink): every response's bucket and sum at once
  // a wide tree's node gives a hot site's LDS counter | kSiteLds (tree_walk.h NodeW4::site)
  uint32_t slot_of(uint32_t site) const {
    return (wide && (site & tw::kSiteLds)) ? prog->tree_lds_slot[site & 0xFFFFu] : site;
  }
  uint64_t ev_hot = 0, ev_cold = 0, row_hot = 0, row_cold = 0, leaf_cold = 0;  // wide: event kinds (stderr)
  void call(uint32_t site) {
    calls[slot_of(site)] += 1;
    ((wide && (site & tw::kSiteLds)) ? ev_hot : ev_cold) += 1;
  }
  void resp_leaf(uint32_t site, bool st) {
    const uint32_t slot = slot_of(site);
    if (st) errs[slot] += 1;
    if (!wide) return;
    if (!(site & tw::kSiteLds)) leaf_cold += 1;
    const uint32_t w = prog->slot_tbkt[slot], r = w & (kTreeLeafSlot - 1u);
    gbucket[r][(st ? ISIM_N_PROM : 0) + (w >> 24)] += 1;
    (st ? sum500 : sum200)[r] += prog->slot_tc[slot];
  }
  void resp(uint32_t site, uint32_t roww, uint64_t T, bool st) {
    const uint32_t slot = slot_of(site);
    if (wide) {  // (a hot row: bit 31 | its sum index << 16 | table offset — counted in LDS, same totals)
      const uint32_t r = (roww & 0x80000000u) ? prog->sum_row[(roww >> 16) & 0x7FFFu] : roww;
      ((roww & 0x80000000u) ? row_hot : row_cold) += 1;
      if (st) errs[slot] += 1;
      gbucket[r][(st ? ISIM_N_PROM : 0) + prom_bucket_ns(T)] += 1;
      (st ? sum500 : sum200)[r] += T;
      return;
    }
    const uint32_t idx = roww & 0xFFFFu, place = roww >> 16;
    if (st) errs[slot] += 1;
    if (place == kTreeGlobalDyn || place == kTreeGlobalStatic) {  // as tree.hip TreeSink::resp: a row in global memory
      if (place == kTreeGlobalDyn) gbucket[idx][(st ? ISIM_N_PROM : 0) + prom_bucket_ns(T)] += 1;
      (st ? sum500 : sum200)[idx] += T;
      return;
    }
    const uint32_t row = prog->sum_row[idx];
    if (place != kTreeStaticRow) {  // an LDS bucket table (code 200), with the range check made an error
      std::vector<uint64_t> &tb = dyn.at(place);
      const uint32_t lo = hdr.at(place) & 0xFFu, w = hdr.at(place) >> 8, b = prom_bucket_ns(T);
      if (st) gbucket[row][ISIM_N_PROM + b] += 1;  // 500s: global atomics in the kernel
      else if (b < lo || b >= lo + w) out_of_table = true;
      else tb[b - lo] += 1;
    }
    (st ? sum500 : sum200)[row] += T;
  }
};
}  // namespace

int main(int argc, char **argv) {
  if (argc < 9) return 2;
  std::ifstream f(argv[1]);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string js = ss.str();
  ServiceGraph g;
  std::string err;
  if (!unmarshal_service_graph(js.data(), js.size(), g, err)) {
    std::fprintf(stderr, "parse: %s\n", err.c_str());
    return 2;
  }
  int32_t entry = -1;
  for (size_t i = 0; i < g.services.size() && entry < 0; ++i)
    if (g.services[i].is_entrypoint) entry = (int32_t)i;
  isim_params p{};
  p.error_mode = (uint32_t)std::atoi(argv[2]);
  p.seed = std::strtoull(argv[3], nullptr, 0);
  p.hop_base_ns = std::strtoull(argv[4], nullptr, 0);
  p.req_ps_per_byte = std::strtoull(argv[5], nullptr, 0);
  p.resp_ps_per_byte = std::strtoull(argv[6], nullptr, 0);
  p.flags = ISIM_FLAG_DYNAMIC;  // static graphs too: the tree walk is the general path
  if (std::getenv("ISIM_TW_WIDE")) p.flags |= ISIM_FLAG_TREE_WIDE;  // every tree in the wide format
  if (std::getenv("ISIM_TW_DAG")) p.flags |= ISIM_FLAG_TREE_DAG;    // every walk over the site graph
  const uint64_t begin = std::strtoull(argv[7], nullptr, 0), n = std::strtoull(argv[8], nullptr, 0);
  Program prog;
  if (compile_program(g, entry, p, prog, err) != ISIM_OK) {
    std::fprintf(stderr, "compile: %s\n", err.c_str());
    return 2;
  }
  if (!prog.has_tree()) {
    std::printf("why %s\n", prog.tree_why.c_str());
    return 3;
  }
  std::fprintf(stderr, "positions %u frames %u lds %u nodes_lds %u wg_per_cu %u lds_rows %u wide %d dag %d\n",
               prog.tree_positions(), prog.tree_frames, prog.tree_layout.bytes, prog.tree_layout.nodes_lds,
               prog.tree_layout.wg_per_cu, prog.tree_layout.n_sum, prog.tree_wide ? 1 : 0, prog.tree_dag ? 1 : 0);
  const uint32_t S = (uint32_t)prog.n_slots, R = (uint32_t)prog.row_svc.size();
  Sink sk;
  sk.prog = &prog;
  sk.wide = prog.tree_wide;
  sk.calls.assign(S, 0);
  sk.errs.assign(S, 0);
  sk.sum200.assign(R, 0);
  sk.sum500.assign(R, 0);
  sk.gbucket.assign(R, std::vector<uint64_t>(2 * ISIM_N_PROM, 0));
  for (const TreeDynRow &d : prog.tree_dyn) {
    sk.hdr[d.off] = d.b_lo | (d.width << 8);
    sk.dyn[d.off].assign(d.width, 0);
  }
  std::vector<uint64_t> root_hist(2 * ISIM_N_PROM, 0), root_sum(2, 0);
  const bool modeb = p.error_mode == ISIM_MODE_B;
  // one Lane per depth variant, reused trace after trace as a GPU lane is
  // (tree.hip hands a lane its next trace as soon as one responds); the
  // spilling variant keeps its deep frames in a vector, one column (stride 1)
  std::vector<uint32_t> spill((size_t)kTreeMaxFrames * 12, 0);  // (rows of 16-B aligned frames)
  tw::Lane<4, true> b4;
  tw::Lane<8, true> b8;
  tw::Lane<16, true> b16;
  tw::Lane<8, true, true, true> bs;
  tw::Lane<4, false> a4;
  tw::Lane<8, false> a8;
  tw::Lane<16, false> a16;
  tw::Lane<8, false, true, true> as;
  // u64 time (Program::tree_t64): the kernel's 8- and 16-frame and spilling variants
  tw::Lane<8, true, true, false, true, uint64_t> c8;
  tw::Lane<16, true, true, false, true, uint64_t> c16;
  tw::Lane<8, true, true, true, true, uint64_t> cs;
  tw::Lane<8, false, true, false, true, uint64_t> d8;
  tw::Lane<16, false, true, false, true, uint64_t> d16;
  tw::Lane<8, false, true, true, true, uint64_t> ds;
  std::vector<uint32_t> spill64((size_t)kTreeMaxFrames * 12, 0);
  bs.sp = as.sp = spill.data();
  cs.sp = ds.sp = spill64.data();
  // wide trees (Program::tree_wide): the kernel's variants — 6 register frames (u32 time) or 4 (u64),
  // and the same + the spill (kernel_abi.h tree_wide_reg_frames)
  tw::Lane<6, true, true, false, true, uint32_t, true> wb16;
  tw::Lane<6, true, true, true, true, uint32_t, true> wbs;
  tw::Lane<6, false, true, false, true, uint32_t, true> wa16;
  tw::Lane<6, false, true, true, true, uint32_t, true> was;
  tw::Lane<4, true, true, false, true, uint64_t, true> wc16;
  tw::Lane<4, true, true, true, true, uint64_t, true> wcs;
  tw::Lane<4, false, true, false, true, uint64_t, true> wd16;
  tw::Lane<4, false, true, true, true, uint64_t, true> wds;
  std::vector<uint32_t> spillw((size_t)kTreeMaxFrames * 12, 0);
  wbs.sp = was.sp = wcs.sp = wds.sp = spillw.data();
  const tw::CpuNodes nodes{prog.tree_nodes.data()};
  const tw::CpuNodesW nodes_w{prog.tree_nodes_w.data()};
  const tw::CpuNodesD nodes_d{prog.tree_nodes_w.data()};  // the site graph (Program::tree_dag)
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t lat = 0;
    uint32_t hops = 0, errh = 0;
    bool r500 = false;
    auto run = [&](auto &L) {
      L.start(begin + i);
      while (!L.done) {
        if (prog.tree_dag)
          L.step(nodes_d, prog.tree_ext.data(), prog.tree_step.data(), sk, (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
        else if (prog.tree_wide)
          L.step(nodes_w, prog.tree_ext.data(), prog.tree_step.data(), sk, (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
        else
          L.step(nodes, prog.tree_ext.data(), prog.tree_step.data(), sk, (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
      }
      lat = L.lat;
      hops = L.hops();
      errh = L.errs();
      r500 = L.root500;
    };
    // the register-stack depth the device compiles for this graph (tree.hip tree_kernel)
    const uint32_t fr = prog.tree_frames;
    const bool spills = fr > kTreeRegFrames || std::getenv("ISIM_TW_SPILL") != nullptr;
    if (prog.tree_wide) {
      const bool sp = fr > tree_wide_reg_frames(prog.tree_t64) || std::getenv("ISIM_TW_SPILL") != nullptr;
      if (prog.tree_t64) {
        if (modeb) sp ? run(wcs) : run(wc16);
        else sp ? run(wds) : run(wd16);
      } else {
        if (modeb) sp ? run(wbs) : run(wb16);
        else sp ? run(was) : run(wa16);
      }
    } else if (prog.tree_t64) {
      if (modeb) {
        if (spills) run(cs);
        else if (fr <= 8) run(c8);
        else run(c16);
      } else {
        if (spills) run(ds);
        else if (fr <= 8) run(d8);
        else run(d16);
      }
    } else if (modeb) {
      if (spills) run(bs);
      else if (fr <= 4) run(b4);
      else if (fr <= 8) run(b8);
      else run(b16);
    } else {
      if (spills) run(as);
      else if (fr <= 4) run(a4);
      else if (fr <= 8) run(a8);
      else run(a16);
    }
    std::printf("rec %llu %u %d %u\n", (unsigned long long)lat, hops, r500 ? 1 : 0, errh);
    root_hist[(r500 ? ISIM_N_PROM : 0) + prom_bucket_ns(lat)] += 1;
    root_sum[r500 ? 1 : 0] += lat;
  }
  if (sk.wide)
    std::fprintf(stderr, "wide events per trace: calls hot %.2f cold %.2f, rows hot %.2f cold %.2f, cold leaves %.2f "
                 "(hot sites %zu, hot rows %zu)\n", (double)sk.ev_hot / n, (double)sk.ev_cold / n,
                 (double)sk.row_hot / n, (double)sk.row_cold / n, (double)sk.leaf_cold / n, prog.tree_lds_slot.size(),
                 prog.sum_row.size());
  // per call site and per service, as isim_stats_fold
  std::vector<uint64_t> site(prog.n_sites, 0), svc_calls(prog.n_services, 0), svc_errs(prog.n_services, 0);
  for (uint32_t s = 0; s < S; ++s) {
    site[prog.slot_site[s]] += sk.calls[s];
    svc_calls[prog.slot_callee[s]] += sk.calls[s];
    svc_errs[prog.slot_callee[s]] += sk.errs[s];
  }
  uint64_t n500 = 0;
  for (uint32_t b = 0; b < ISIM_N_PROM; ++b) n500 += root_hist[ISIM_N_PROM + b];
  svc_calls[prog.entry] += n;
  svc_errs[prog.entry] += n500;
  std::printf("site");
  for (uint64_t v : site) std::printf(" %llu", (unsigned long long)v);
  std::printf("\nsvc");
  for (uint64_t v : svc_calls) std::printf(" %llu", (unsigned long long)v);
  std::printf("\nerr");
  for (uint64_t v : svc_errs) std::printf(" %llu", (unsigned long long)v);
  std::printf("\n");
  // duration rows: the kernel's flush (static buckets from the slot counters)
  std::vector<std::vector<uint64_t>> row(R, std::vector<uint64_t>(ISIM_SVC_DUR_WORDS, 0));
  if (sk.out_of_table) {
    std::fprintf(stderr, "a duration fell outside its row's bucket table (tmin/tmax bounds wrong)\n");
    return 4;
  }
  for (uint32_t r = 0; r < R; ++r) {
    row[r][2 * ISIM_N_PROM] = sk.sum200[r];
    row[r][2 * ISIM_N_PROM + 1] = sk.sum500[r];
    for (uint32_t w = 0; w < 2 * ISIM_N_PROM; ++w) row[r][w] += sk.gbucket[r][w];
  }
  for (const TreeDynRow &d : prog.tree_dyn)
    for (uint32_t j = 0; j < d.width; ++j) row[d.row][d.b_lo + j] += sk.dyn[d.off][j];
  for (uint32_t s = 0; s < S && !prog.tree_wide; ++s) {  // the kernel's flush: static buckets and leaf sums from the counters
    const uint32_t w = prog.slot_tbkt[s], r = w & kTreeRowMask, b = w >> 24;
    if (b != kTreeDynBucket) {
      row[r][b] += sk.calls[s] - sk.errs[s];
      row[r][ISIM_N_PROM + b] += sk.errs[s];
    }
    if (w & kTreeLeafSlot) {
      row[r][2 * ISIM_N_PROM] += (uint64_t)prog.slot_tc[s] * (sk.calls[s] - sk.errs[s]);
      row[r][2 * ISIM_N_PROM + 1] += (uint64_t)prog.slot_tc[s] * sk.errs[s];
    }
  }
  for (uint32_t w = 0; w < 2 * ISIM_N_PROM; ++w) row[0][w] += root_hist[w];
  row[0][2 * ISIM_N_PROM] += root_sum[0];
  row[0][2 * ISIM_N_PROM + 1] += root_sum[1];
  for (uint32_t r = 0; r < R; ++r) {
    std::printf("dur %d", prog.row_svc[r]);
    for (uint64_t v : row[r]) std::printf(" %llu", (unsigned long long)v);
    std::printf("\n");
  }
  return 0;
}
