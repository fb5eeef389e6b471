// CPU restatement of the DES item engine (istio-isotope_amd/csrc/
// des_items.hip) over the product's own plan
// (build_des_plan with DesPlan::items) and pre-walk (tree_walk.h Lane): the
// same arrivals, items, rounds, queue order (row, replica, arrival, item),
// finishes and fixed-point passes, in plain loops.  Test infrastructure
// only: tests/test_des_items.py runs it and compares its records, stats and
// DES table with the event-driven oracle (oracle/des_oracle.c) — the
// algorithm checked on the CPU, the HIP kernels by tests/test_des_items_gpu.py.
//   des_items_check <graph.json> <seed> <hop_base> <req_ps> <resp_ps> <mean_ns> <begin> <n> <out prefix> [mode]
// (mode 1: error mode B — a failed call step ends its script)
// writes <prefix>.rec (n x 16 B), <prefix>.stats (u64), <prefix>.table (u64 rows)
#include <algorithm>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <tuple>
#include <vector>

#include "des.h"
#include "graph.h"
#include "kernel_abi.h"
#include "program.h"
#include "tree_walk.h"

using namespace isim;

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;

uint32_t draw0(uint64_t t, uint32_t w2, uint32_t w3, uint64_t seed) {
  uint32_t a = (uint32_t)t, b = (uint32_t)(t >> 32), c = w2, d = w3;
  tw::philox10(a, b, c, d, (uint32_t)seed, (uint32_t)(seed >> 32));
  return a;
}

uint32_t prom_bucket(uint64_t t) {
  static const uint64_t e[32] = {7000000ull,   8000000ull,   9000000ull,   10000000ull,  11000000ull,
                                 12000000ull,  14000000ull,  16000000ull,  18000000ull,  20000000ull,
                                 25000000ull,  30000000ull,  35000000ull,  40000000ull,  45000000ull,
                                 50000000ull,  60000000ull,  70000000ull,  80000000ull,  90000000ull,
                                 100000000ull, 120000000ull, 140000000ull, 160000000ull, 180000000ull,
                                 200000000ull, 250000000ull, 300000000ull, 350000000ull, 400000000ull,
                                 450000000ull, 500000000ull};
  for (uint32_t j = 0; j < 32; ++j)
    if (t <= e[j]) return j;
  return 32;
}

struct Item {
  uint32_t pos, par, t;
  uint8_t own;
};

struct Sink {
  std::vector<Item> *items;
  std::vector<uint64_t> *dur_of;  // per item: its duration without contention
  uint64_t base;
  uint32_t t;
  void call(uint32_t) {}
  void resp_leaf(uint32_t, bool) {}
  void resp(uint32_t, uint32_t, uint64_t, bool) {}
  // (after exec: the status replaces the own error — they differ only when a
  // mode-B step failed)
  void dur(uint32_t hop, uint64_t T, bool st) {
    if (dur_of->size() <= base + hop) dur_of->resize(base + hop + 1);
    (*dur_of)[base + hop] = T;
    (*items)[base + hop].own = st ? 1 : 0;
  }
  void exec(uint32_t p, uint32_t hop, uint32_t caller, bool own) {
    if (items->size() <= base + hop) items->resize(base + hop + 1);
    (*items)[base + hop] = Item{p, caller == tw::kNoCaller ? kNone : (uint32_t)(base + caller), t,
                                (uint8_t)(own ? 1 : 0)};
  }
};

template <bool MB, bool W, class Nodes>
void walk_all(const Program &prog, const Nodes &nodes, uint64_t seed, uint64_t begin, uint64_t n,
              std::vector<Item> &items, std::vector<uint64_t> &dur_of, std::vector<uint64_t> &toff,
              std::vector<uint32_t> &terr) {
  tw::Lane<kTreeMaxFrames + 1, MB, true, false, true, uint64_t, W> L;
  for (uint64_t t = 0; t < n; ++t) {
    Sink s{&items, &dur_of, toff[t], (uint32_t)t};
    L.start(begin + t);
    while (!L.done) L.step(nodes, prog.tree_ext.data(), prog.tree_step.data(), s, (uint32_t)seed,
                           (uint32_t)(seed >> 32));
    toff[t + 1] = toff[t] + L.hops();
    items.resize(toff[t + 1]);
    items[toff[t]].own = L.root500 ? 1 : 0;
    terr[t] = (L.root500 ? 0x80000000u : 0u) | L.errs();
  }
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 10) return 2;
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
  isim_params prm{};
  prm.seed = std::stoull(argv[2]);
  prm.hop_base_ns = std::stoull(argv[3]);
  prm.req_ps_per_byte = std::stoull(argv[4]);
  prm.resp_ps_per_byte = std::stoull(argv[5]);
  const bool modeb = argc > 10 && std::stoi(argv[10]) == 1;
  prm.error_mode = modeb ? ISIM_MODE_B : ISIM_MODE_A;
  prm.flags = ISIM_FLAG_DYNAMIC;
  const uint64_t mean = std::stoull(argv[6]), begin = std::stoull(argv[7]), n = std::stoull(argv[8]);
  const std::string out = argv[9];
  Program prog;
  if (compile_program(g, entry, prm, prog, err) != ISIM_OK) {
    std::fprintf(stderr, "compile: %s\n", err.c_str());
    return 2;
  }
  DesPlan pl;
  if (build_des_plan(g, prog, modeb, pl, err) != ISIM_OK || !pl.items) {
    std::fprintf(stderr, "plan: %s\n", err.c_str());
    return 3;
  }
  const uint64_t seed = prm.seed;
  // 1. arrivals
  std::vector<uint64_t> A(n);
  uint64_t now = 0;
  for (uint64_t t = 0; t < n; ++t) {
    now += (mean * des_exp_q24_host(draw0(begin + t, 0u, 0x80000001u, seed))) >> 24;
    A[t] = now;
  }
  // 2. pre-walk
  std::vector<Item> items;
  std::vector<uint64_t> dur_of;
  std::vector<uint64_t> toff(n + 1, 0);
  std::vector<uint32_t> terr(n);
  const tw::CpuNodes nodes{prog.tree_nodes.data()};
  const tw::CpuNodesW nodes_w{prog.tree_nodes_w.data()};
  if (prog.tree_wide) {  // a wide tree (ISIM_FLAG_TREE_WIDE or past the 8-byte nodes): 16-byte nodes, 32-bit frames
    if (modeb) walk_all<true, true>(prog, nodes_w, seed, begin, n, items, dur_of, toff, terr);
    else walk_all<false, true>(prog, nodes_w, seed, begin, n, items, dur_of, toff, terr);
  } else {
    if (modeb) walk_all<true, false>(prog, nodes, seed, begin, n, items, dur_of, toff, terr);
    else walk_all<false, false>(prog, nodes, seed, begin, n, items, dur_of, toff, terr);
  }
  const uint64_t M = items.size();
  // mode B: an invocation with a callee that responded 500 failed at that
  // callee's call step (the last one it ran: no later step has callees)
  std::vector<uint32_t> fst(M, kNone);
  if (modeb)
    for (uint64_t i = 0; i < M; ++i)
      if (items[i].par != kNone && items[i].own)
        fst[items[i].par] = std::min<uint32_t>(fst[items[i].par], pl.item_pos[items[i].pos].kstep);
  const uint32_t aw = pl.item_acc, bw = std::max<uint32_t>(1, pl.item_bk);
  std::vector<uint64_t> IA(M, 0), IS(M, 0), IF(M, 0), bk(M * bw, 0), acc(M * aw, 0), accp(M * aw, 0);
  const uint32_t n_slots = (uint32_t)prog.n_slots;
  const uint32_t R = pl.rounds();
  std::vector<uint64_t> stats(ISIM_ST_SITES + 2 * (uint64_t)n_slots, 0);
  std::vector<uint64_t> table(prog.row_svc.size() * (uint64_t)ISIM_DES_ROW_WORDS, 0);
  // items per queue round / finish group (item order within each)
  std::vector<std::vector<uint64_t>> qlist(R), flist(pl.fin_off.size() - 1);
  for (uint64_t i = 0; i < M; ++i) {
    const DesItemPos &p = pl.item_pos[items[i].pos];
    qlist[p.qround].push_back(i);
    flist[p.fgroup].push_back(i);
  }
  // the engine's own choices, restated: the first quiet pass of a cyclic
  // schedule starts its cut step begins from the contention-free callee
  // maxima (des_items.hip k_relmax), and a round the plan marks sort-free
  // (DesPlan::round_nosort) takes its items in (position, item) order, a
  // zero-hold item starting at its own arrival (k_pairs0)
  dur_of.resize(M, 0);
  std::vector<uint64_t> relmax(M * aw, 0);
  for (uint64_t i = 0; i < M; ++i) {
    const uint32_t par = items[i].par;
    if (par == kNone) continue;
    const DesItemPos &p = pl.item_pos[items[i].pos], &pp = pl.item_pos[items[par].pos];
    if (pp.nsteps < 2) continue;
    const uint64_t h = pl.pos[items[i].pos].off - (p.kstep == 0 ? pl.steps[pp.bk_first].add : 0ull);
    uint64_t &m = relmax[(uint64_t)par * aw + p.kstep];
    m = std::max(m, h + dur_of[i]);
  }
  bool first_pass = pl.cyclic;
  bool changed = false;
  auto store = [&](uint64_t &dst, uint64_t v) {
    if (dst != v) changed = true;
    dst = v;
  };
  auto pass = [&](bool quiet) {
    std::swap(acc, accp);
    std::fill(acc.begin(), acc.end(), 0);
    for (uint32_t r = 0; r < R; ++r) {
      // step begins
      for (uint64_t i = 0; i < M; ++i) {
        const DesItemPos &p = pl.item_pos[items[i].pos];
        if (p.nsteps < 2) continue;
        for (uint32_t s = 0; s < p.nsteps && s <= fst[i]; ++s) {  // (a failed script's later steps never begin)
          const uint32_t b = p.bk_first + s, sr = pl.step_round[b];
          if ((sr & ~kDesStepCut) != r) continue;
          const DesStep &st = pl.steps[b];
          uint64_t v;
          if (s == 0) {
            v = IS[i];
          } else {
            v = bk[i * bw + s - 1] + st.smax;
            uint64_t c = ((sr & kDesStepCut) ? accp : acc)[i * aw + s - 1];
            if ((sr & kDesStepCut) && first_pass) c = bk[i * bw + s - 1] + relmax[i * aw + s - 1];
            v = std::max(v, c);
          }
          store(bk[i * bw + s], v + st.add);
        }
      }
      // queues: (row, replica, arrival, item) order, one FIFO per (row, replica)
      std::vector<std::tuple<uint32_t, uint32_t, uint64_t, uint64_t>> q;
      for (uint64_t i : qlist[r]) {
        const Item &it = items[i];
        const DesPos &P = pl.pos[it.pos];
        uint64_t a;
        if (it.par == kNone) {
          a = A[it.t];
        } else {
          const uint32_t ks = pl.item_pos[it.pos].kstep;
          a = (ks == 0 ? IS[it.par] : bk[(uint64_t)it.par * bw + ks]) + P.off;
        }
        IA[i] = a;
        uint32_t rep = 0;
        if (P.reps > 1) rep = draw0(begin + it.t, (uint32_t)(i - toff[it.t]), 0x80000002u, seed) % P.reps;
        // sort-free round: the key is (position, item); a zero-hold item its own queue
        if (pl.round_nosort[r])
          q.emplace_back(it.pos, P.hold ? 0u : (uint32_t)i, P.hold ? i : 0u, i);
        else
          q.emplace_back(P.row, rep, a, i);
      }
      std::sort(q.begin(), q.end());
      for (size_t j = 0; j < q.size(); ++j) {
        const uint64_t i = std::get<3>(q[j]);
        const DesPos &P = pl.pos[items[i].pos];
        const bool first = j == 0 || std::get<0>(q[j - 1]) != std::get<0>(q[j]) ||
                           std::get<1>(q[j - 1]) != std::get<1>(q[j]);
        if (pl.round_nosort[r]) std::get<2>(q[j]) = IA[i];
        const uint64_t a = std::get<2>(q[j]);
        const uint64_t free_at = first ? 0 : IS[std::get<3>(q[j - 1])] + P.hold;
        store(IS[i], std::max(a, free_at));
        if (!quiet) {
          uint64_t *tr = table.data() + (uint64_t)P.row * ISIM_DES_ROW_WORDS;
          const uint64_t w = IS[i] - a;
          tr[ISIM_DES_COUNT] += 1;
          tr[ISIM_DES_SUM_WAIT] += w;
          tr[ISIM_DES_MAX_WAIT] = std::max(tr[ISIM_DES_MAX_WAIT], w);
          tr[ISIM_DES_SUM_HOLD] += P.hold;
        }
      }
      // finishes, deepest group first
      for (uint32_t gi = pl.fin_round_off[r]; gi < pl.fin_round_off[r + 1]; ++gi) {
        for (uint64_t i : flist[gi]) {
          const Item &it = items[i];
          const DesPos &P = pl.pos[it.pos];
          const DesItemPos &p = pl.item_pos[it.pos];
          uint64_t F;
          if (P.flags & kDesFlagLeaf) {
            F = IS[i] + P.floor;
          } else if (fst[i] != kNone) {
            // failed at call step j: the step's end — its begin plus its longest
            // sleep, or its callees' finishes — and no later command
            const uint32_t j = fst[i];
            const uint64_t b0 = p.nsteps >= 2 ? bk[i * bw + j] : IS[i];
            const uint64_t sm = p.nsteps >= 2 && j + 1u < p.nsteps ? pl.steps[p.bk_first + j + 1].smax : P.floor;
            F = std::max(b0 + sm, acc[i * aw + j]);
          } else {
            const uint32_t last = p.nsteps >= 2 ? p.nsteps - 1u : 0u;
            F = (p.nsteps >= 2 ? bk[i * bw + last] : IS[i]) + P.floor;
            F = std::max(F, acc[i * aw + last]) + P.post;
          }
          store(IF[i], F);
          if (it.par != kNone) {
            uint64_t &m = acc[(uint64_t)it.par * aw + p.kstep];
            m = std::max(m, F);
          }
          if (quiet) continue;
          const uint64_t dur = F - IA[i];
          uint64_t *tr = table.data() + (uint64_t)P.row * ISIM_DES_ROW_WORDS;
          tr[it.own * ISIM_N_PROM + prom_bucket(dur)] += 1;
          tr[2 * ISIM_N_PROM + it.own] += dur;
          if (it.par != kNone) {
            stats[ISIM_ST_SITES + P.slot] += 1;
            stats[ISIM_ST_SITES + n_slots + P.slot] += it.own;
          }
        }
      }
    }
  };
  if (pl.cyclic) {
    uint32_t p = 0;
    for (; p < 256; ++p) {
      changed = false;
      pass(true);
      first_pass = false;
      if (!changed) break;
    }
    if (p == 256) return 5;
  }
  pass(false);
  // 5. records and statistics
  std::vector<uint64_t> rec(2 * n);
  stats[ISIM_ST_NOT_MIN_LATENCY] = 0;
  uint64_t mn = ~0ull;
  for (uint64_t t = 0; t < n; ++t) {
    const uint64_t L = IF[toff[t]] - A[t];
    const uint64_t hops = toff[t + 1] - toff[t];
    const uint32_t st = terr[t] >> 31;
    rec[2 * t] = L;
    rec[2 * t + 1] = hops | ((uint64_t)terr[t] << 32);
    stats[ISIM_ST_N_TRACES] += 1;
    stats[ISIM_ST_SUM_LATENCY] += L;
    stats[ISIM_ST_SUM_HOPS] += hops;
    stats[ISIM_ST_SUM_ERR_HOPS] += terr[t] & 0x7FFFFFFFu;
    stats[ISIM_ST_N_500] += st;
    mn = std::min(mn, L);
    stats[ISIM_ST_MAX_LATENCY] = std::max(stats[ISIM_ST_MAX_LATENCY], L);
    stats[ISIM_ST_PROM + st * ISIM_N_PROM + prom_bucket(L)] += 1;
    stats[ISIM_ST_LOG2 + st * ISIM_N_LOG2 + (L ? 64u - (uint32_t)__builtin_clzll(L) : 0u)] += 1;
  }
  if (n) stats[ISIM_ST_NOT_MIN_LATENCY] = ~mn;
  auto dump = [&](const std::string &path, const std::vector<uint64_t> &v) {
    std::FILE *o = std::fopen(path.c_str(), "wb");
    if (!o) return false;
    const bool ok = std::fwrite(v.data(), 8, v.size(), o) == v.size();
    return std::fclose(o) == 0 && ok;
  };
  if (!dump(out + ".rec", rec) || !dump(out + ".stats", stats) || !dump(out + ".table", table)) return 4;
  std::printf("items %llu rounds %u cyclic %d\n", (unsigned long long)M, R, pl.cyclic ? 1 : 0);
  return 0;
}
