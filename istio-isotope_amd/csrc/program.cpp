// Graph -> device program.  See program.h and DESIGN.md §4.
#include "program.h"

#include <algorithm>
#include <cstdlib>
#include <unordered_map>

#include "gounits.h"

namespace isim {
namespace {

constexpr uint64_t kTimeCap = 1ull << 63;  // latencies must stay below 2^63 ns

struct Site {
  int32_t caller, callee;
  uint64_t size;
  int64_t prob;
  uint32_t k;     // index of the call command within the caller's script
  bool conc;
  uint64_t hop;   // H
};

uint64_t sat_add(uint64_t a, uint64_t b) {
  uint64_t r = a + b;
  return (r < a || r >= kTimeCap) ? kTimeCap : r;
}

uint64_t sleep_ns(int64_t d) { return d > 0 ? (uint64_t)d : 0; }

// Shape of a script for the lane tree walk: per call command (document
// order) its step's facts; the time outside call steps.
struct CallShape {
  bool step_first, conc;
  uint64_t pre;    // step_first: non-call step time since the previous call step
  uint64_t cmax0;  // conc: the step's longest sleep sub-command
};
struct ScriptTimes {
  std::vector<CallShape> calls;
  uint64_t tail = 0;  // non-call step time after the last call step (the whole script for a leaf)
};

ScriptTimes script_times(const Service &sv) {
  ScriptTimes r;
  uint64_t pending = 0;  // non-call step time not yet assigned
  for (const Command &c : sv.script) {
    if (c.kind == Command::Sleep) {
      pending = sat_add(pending, sleep_ns(c.sleep_ns));
    } else if (c.kind == Command::Request) {
      r.calls.push_back(CallShape{true, false, pending, 0});
      pending = 0;
    } else {
      uint64_t m = 0;
      size_t first = r.calls.size();
      for (const Command &x : c.commands) {
        if (x.kind == Command::Request) r.calls.push_back(CallShape{r.calls.size() == first, true, 0, 0});
        else m = std::max(m, sleep_ns(x.sleep_ns));
      }
      if (r.calls.size() == first) {  // a concurrent step of sleeps only: a timed step
        pending = sat_add(pending, m);
      } else {
        r.calls[first].pre = pending;
        r.calls[first].cmax0 = m;
        pending = 0;
      }
    }
  }
  r.tail = pending;
  return r;
}

}  // namespace

// LDS layout of the lane tree walk (kernel_abi.h TreeLayout): the per-slot
// counters always; the nodes when they fit; then the non-leaf callees'
// duration rows (a u64 sum, and a bucket table when the bucket varies),
// hottest first (expected invocations per trace), the rest in global memory.
// Tried in order: nodes in LDS within half the CU (two 1024-thread workgroups
// per CU), nodes in LDS within the whole CU, nodes in global memory within
// half, then within the whole CU; the first whose fixed part fits and which
// holds every row wins, else the first whose fixed part fits.
// LDS bytes of a calling row (kernel_abi.h TreeLayout): wide — a u64
// code-200 sum, and when the bucket varies a header word and [2][width] u32
// counts; compact — a u32 sum (carries to HBM), a header word and the code-200
// counts as guarded u16 pairs (500s are errorRate-rare: HBM)
static uint32_t row_lds_bytes(uint32_t bw, bool compact) {
  if (compact) return 4u + (bw ? 4u + 4u * ((bw + 1u) / 2u) : 0u);
  return 8u + (bw ? 4u + 8u * bw : 0u);
}

static bool place_tree(Program &out, const std::vector<double> &row_heat, const std::vector<uint32_t> &row_bw,
                       const std::vector<char> &row_nonleaf) {
  const uint32_t P = (uint32_t)out.tree_nodes_w.size(), S = (uint32_t)out.n_slots;
  const uint32_t R = (uint32_t)out.row_svc.size();
  const uint32_t head = kLdsAccBytes + kHistWords * 4u + kTreeLutBytes;  // + the duration-bucket LUT
  // per-slot counters: guarded 16-bit pairs (4 B per slot)
  const uint32_t cb = 4u;
  // rows by heat (the entry's row, 0, is the end-to-end histogram: no LDS row)
  std::vector<uint32_t> order;
  for (uint32_t r = 1; r < R; ++r)
    if (row_nonleaf[r]) order.push_back(r);
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return row_heat[a] > row_heat[b]; });
  struct Cand {
    bool nodes;
    uint32_t limit;
  };
  const Cand cands[4] = {{true, kTreeLdsHalf}, {true, kTreeLdsFull}, {false, kTreeLdsHalf}, {false, kTreeLdsFull}};
  int pick = -1;
  // wide rows unless they do not all fit in any candidate and compact ones
  // hold more
  bool compact = false;
  const int first = 0, last = 4;
  // walks deeper than 8 calling invocations run kernels built for 4 waves per
  // SIMD (tree.hip): one 1024-thread workgroup per CU whatever the layout, so
  // the half-CU layouts would only leave LDS unused
  const bool one_wg = out.tree_frames > 8;
  const bool force_c = false, force_w = false;
  // passes: every row fits (wide, then compact), else the fixed part fits (compact: more rows)
  for (int pass = 0; pass < 3 && pick < 0; ++pass) {
    compact = force_c || (!force_w && pass >= 1);
    if (force_c && pass == 1) continue;
    for (int i = first; i < last && pick < 0; ++i) {
      if (one_wg && cands[i].limit == kTreeLdsHalf) continue;
      uint32_t fixed = ((head + cb * S + 7u) & ~7u) + (cands[i].nodes ? 8u * P + 8u : 0u);
      if (fixed > cands[i].limit) continue;
      uint32_t all = fixed;
      for (uint32_t r : order) all += row_lds_bytes(row_bw[r], compact);
      if (pass == 2 || all <= cands[i].limit) pick = i;
    }
  }
  if (pick < 0) return false;
  const Cand c = cands[pick];
  TreeLayout &L = out.tree_layout;
  L = TreeLayout{};
  L.nodes_lds = c.nodes ? 1u : 0u;
  L.wg_per_cu = c.limit == kTreeLdsHalf ? 2u : 1u;
  L.off_cnt = head;
  L.cnt16 = cb == 4u ? 1u : 0u;
  L.compact = compact ? 1u : 0u;
  L.off_sums = (head + cb * S + 7u) & ~7u;
  uint32_t room = c.limit - L.off_sums - (c.nodes ? 8u * P + 8u : 0u);
  // rows into LDS while they fit: a sum word, and the bucket table when the bucket varies
  out.tree_row_place.assign(R, kTreeGlobalStatic);
  out.sum_row.clear();
  out.tree_dyn.clear();
  out.tree_dyn_words = 0;
  std::vector<uint32_t> lds_rows;
  for (uint32_t r : order) {
    const uint32_t need = row_lds_bytes(row_bw[r], compact);
    if (need <= room && out.sum_row.size() < 0xFFFFu && out.tree_dyn_words + 4096u < 0xFFF0u) {
      room -= need;
      lds_rows.push_back(r);
      out.sum_row.push_back(r);
    } else {
      out.tree_row_place[r] = row_bw[r] ? kTreeGlobalDyn : kTreeGlobalStatic;
    }
  }
  out.tree_row_index.assign(R, 0);
  for (uint32_t i = 0; i < (uint32_t)out.sum_row.size(); ++i) {
    const uint32_t r = out.sum_row[i];
    out.tree_row_index[r] = i;
    if (row_bw[r]) {
      out.tree_row_place[r] = out.tree_dyn_words;
      out.tree_dyn.push_back(TreeDynRow{r, out.tree_dyn_words, out.tree_row_blo[r], row_bw[r]});
      out.tree_dyn_words += 1u + (compact ? (row_bw[r] + 1u) / 2u : 2u * row_bw[r]);
    } else {
      out.tree_row_place[r] = kTreeStaticRow;
    }
  }
  for (uint32_t r = 0; r < R; ++r)
    if (out.tree_row_place[r] == kTreeGlobalDyn || out.tree_row_place[r] == kTreeGlobalStatic)
      out.tree_row_index[r] = r;
  L.n_sum = (uint32_t)out.sum_row.size();
  L.off_dyn = L.off_sums + (compact ? 4u : 8u) * L.n_sum;
  L.off_nodes = (L.off_dyn + 4u * out.tree_dyn_words + 7u) & ~7u;
  L.bytes = L.off_nodes + (c.nodes ? 8u * P : 0u);
  return L.bytes <= c.limit;
}

// The unrolled tree of potential invocations for the lane tree walk
// (kernel_abi.h TreeNode/TreeExt, tree_walk.h); leaves the trees empty with
// the reason in out.tree_why when the walk does not fit it.  A tree past the
// 8-byte nodes' 16-bit fields (positions, call sites, rows) or whose per-slot
// counters do not fit in LDS is built WIDE (kernel_abi.h TreeNodeW;
// ISIM_FLAG_TREE_WIDE: always, an independent check of the narrow format).
constexpr uint32_t kTreeMaxWidePositions = 1u << 24;
constexpr uint32_t kDagLdsPaths = 4096;  // site graph: LDS rows only for services reached <= this often per trace
static void build_tree(const ServiceGraph &g, Program &out, const std::vector<Site> &sites,
                       const std::vector<std::vector<int32_t>> &svc_sites, const std::vector<uint64_t> &thr,
                       const std::vector<uint64_t> &tmin, const std::vector<char> &leaf, bool modeb,
                       bool force_wide, bool force_dag) {
  out.tree_dag = false;
  out.tree_nodes.clear();
  out.tree_nodes_w.clear();
  out.tree_ext.clear();
  out.tree_step.clear();
  out.tree_wide = false;
  auto give_up = [&](const char *why) {
    out.tree_nodes.clear();
    out.tree_nodes_w.clear();
    out.tree_ext.clear();
    out.tree_step.clear();
    out.tree_wide = false;
    out.tree_dag = false;
    out.tree_why = why;
  };
  // u64 time when the latency bound reaches 2^32 ns; each position's own
  // figures (hop cost, callee time, step facts, leaf latency) stay 32-bit
  out.tree_t64 = out.max_latency >= (1ull << 32);
  constexpr uint64_t k32 = 1ull << 32;
  // ISIM_FLAG_TREE_WIDE: the wide format for any tree (an independent check of the narrow one)
  bool wide = force_wide || out.n_slots > (int32_t)kTreeMaxPositions;
  if ((uint32_t)out.n_slots >= kSlotRoot) return give_up("more than 2^24 call sites");
  const int32_t n = (int32_t)g.services.size();
  std::vector<ScriptTimes> shape(n);
  std::vector<char> shaped(n, 0);
  auto shape_of = [&](int32_t s) -> const ScriptTimes & {
    if (!shaped[s]) {
      shape[s] = script_times(g.services[s]);
      shaped[s] = 1;
    }
    return shape[s];
  };
  const uint32_t R = (uint32_t)out.row_svc.size();
  if (R > kTreeGlobalStatic) wide = true;
  if (R >= kTreeLeafSlot) return give_up("more than 2^23 reachable services");
  // per row: bucket range of the durations (a table when it spans several buckets), non-leaf
  std::vector<uint32_t> row_bw(R, 0);
  std::vector<char> row_nonleaf(R, 0);
  std::vector<double> row_heat(R, 0.0);
  out.tree_row_blo.assign(R, 0);
  for (uint32_t r = 1; r < R; ++r) {
    const int32_t s = out.row_svc[r];
    row_nonleaf[r] = leaf[s] ? 0 : 1;
    const uint32_t lo = prom_bucket_ns(tmin[s]), hi = prom_bucket_ns(out.svc_time[s]);
    out.tree_row_blo[r] = lo;
    if (lo != hi && !leaf[s]) row_bw[r] = hi - lo + 1;
  }
  // the time a script spends outside its call steps when every step runs (mode A: folded into tc)
  auto own_time = [&](int32_t s) -> uint64_t {
    const ScriptTimes &t = shape_of(s);
    uint64_t v = t.tail;
    if (!modeb)
      for (const CallShape &cs : t.calls) v += cs.step_first ? cs.pre : 0;
    return v;
  };
  auto err_flags = [&](int32_t s) -> uint8_t {
    if (thr[s] >= (1ull << 32)) return TF_ERR_ALWAYS;
    return thr[s] > 0 ? (uint8_t)TF_ERR_DRAW : (uint8_t)0;
  };
  // per service: a probabilistic call among its first 4 call commands (TF_PROBK0); script length bound
  std::vector<char> probk0(n, 0);
  for (int32_t s = 0; s < n; ++s)
    for (int32_t si : svc_sites[s]) {
      const Site &st = sites[si];
      if (st.k < 4 && st.prob >= 1 && st.prob <= 99) probk0[s] = 1;
      if (st.k >= kTreeMaxCalls) return give_up("a script with more than 8188 calls");
    }
  out.tree_flags = 0;
  std::vector<uint32_t> through(out.n_slots, 0);
  std::vector<double> slot_heat(out.n_slots, 0.0);  // expected calls per trace (a wide tree's LDS counters)
  std::vector<uint32_t> row_through(R, 0);
  std::vector<int32_t> pos_callee;  // per position: the callee service
  // preorder DFS over call sites; frame = (service, next call index, position, path probability)
  struct Frame {
    int32_t svc;
    size_t next;
    uint32_t pos;
    double heat;
  };
  std::vector<Frame> stack;
  const int32_t e = out.entry;
  // the node of call site j of service s (flags, ext, step facts): shared by
  // the unrolled tree (one per potential invocation) and the site graph (one
  // per reachable call site); false when a figure does not fit 32 bits
  auto site_node = [&](int32_t s, size_t j, TreeNodeW &nd, TreeExt &x, TreeStep &tsp) -> bool {
    const Site &st = sites[svc_sites[s][j]];
    const CallShape &cs = shape_of(s).calls[j];
    const int32_t c = st.callee;
    nd = TreeNodeW{};
    nd.k = st.k;
    nd.prob = (st.prob >= 1 && st.prob <= 99) ? (uint8_t)st.prob : (uint8_t)0;
    const bool xpre = modeb && cs.step_first && cs.pre != 0;
    const bool xcmax = cs.step_first && cs.conc && cs.cmax0 != 0;
    nd.flags = (uint8_t)((cs.step_first ? TF_STEP : 0) | (cs.conc ? TF_CONC : 0) | (leaf[c] ? TF_LEAF : 0) |
                         err_flags(c) | (probk0[c] ? TF_PROBK0 : 0) | (xpre ? TF_XPRE : 0) | (xcmax ? TF_XCMAX : 0));
    if (nd.prob) out.tree_flags |= kTreeAnyProb;
    if (nd.flags & TF_CONC) out.tree_flags |= kTreeAnyConc;
    if (nd.flags & TF_ERR_DRAW) out.tree_flags |= kTreeAnyDraw;
    nd.slot = (uint32_t)out.site_slot[svc_sites[s][j]];
    if (st.hop >= k32 || own_time(c) >= k32 || cs.pre >= k32 || cs.cmax0 >= k32) return false;
    x = TreeExt{};
    x.H = (uint32_t)st.hop;
    x.tc = (uint32_t)own_time(c);
    x.thr = thr[c] >= (1ull << 32) ? 0u : (uint32_t)thr[c];
    tsp = TreeStep{(uint32_t)cs.pre, (uint32_t)cs.cmax0};
    return true;
  };
  // per service (reachable, DAG order): expected invocations per trace, and
  // potential invocations per trace (the site graph's launch-split guard)
  std::vector<double> svc_heat, svc_paths;
  bool dag = force_dag;
  TreeNodeW root{};
  root.flags = (uint8_t)((leaf[e] ? TF_LEAF : 0) | err_flags(e) | (probk0[e] ? TF_PROBK0 : 0));
  if (root.flags & TF_ERR_DRAW) out.tree_flags |= kTreeAnyDraw;
  TreeExt rx{};
  if (own_time(e) >= k32) return give_up("a script whose time outside its call steps is >= 2^32 ns");
  rx.tc = (uint32_t)own_time(e);
  rx.thr = thr[e] >= (1ull << 32) ? 0u : (uint32_t)thr[e];
  out.tree_nodes_w.push_back(root);
  out.tree_ext.push_back(rx);
  out.tree_step.push_back(TreeStep{});
  pos_callee.push_back(e);
  uint32_t max_open = leaf[e] ? 0u : 1u;
  if (!dag && !leaf[e]) stack.push_back({e, 0, 0, 1.0});
  while (!dag && !stack.empty()) {
    Frame &top = stack.back();
    if (top.next < svc_sites[top.svc].size()) {
      const size_t j = top.next++;
      const int32_t c = sites[svc_sites[top.svc][j]].callee;
      if (out.tree_nodes_w.size() >= kTreeMaxPositions) wide = true;
      if (out.tree_nodes_w.size() >= kTreeMaxWidePositions) {
        // shared callees multiply the potential invocations past the tree: the site graph
        dag = true;
        break;
      }
      TreeNodeW nd;
      TreeExt x;
      TreeStep tsp;
      if (!site_node(top.svc, j, nd, x, tsp)) return give_up("a hop cost, script time or step sleep >= 2^32 ns");
      const uint32_t slot = nd.slot;
      through[slot] += 1;
      const uint32_t row = (uint32_t)out.svc_row[c];
      if (row_bw[row]) row_through[row] += 1;
      const double heat = top.heat * (nd.prob ? nd.prob / 100.0 : 1.0);
      row_heat[row] += heat;
      slot_heat[slot] += heat;
      const uint32_t pos = (uint32_t)out.tree_nodes_w.size();
      out.tree_nodes_w.push_back(nd);
      out.tree_ext.push_back(x);
      out.tree_step.push_back(tsp);
      pos_callee.push_back(c);
      if (!leaf[c]) {
        stack.push_back({c, 0, pos, heat});
        max_open = std::max<uint32_t>(max_open, (uint32_t)stack.size());
      }
    } else {
      out.tree_nodes_w[top.pos].size = (uint32_t)(out.tree_nodes_w.size() - top.pos);
      stack.pop_back();
    }
  }
  if (dag) {
    // the site graph (tree_walk.h NodeD4): node 0 the entry, then each
    // reachable calling service's sites, contiguous in script order; the
    // services in reverse post-order of the call DAG (callers before callees)
    if (out.hops_upper >= (1ull << 31)) return give_up("more than 2^31 invocations per trace in the site graph");
    out.tree_nodes_w.resize(1);
    out.tree_ext.resize(1);
    out.tree_step.resize(1);
    pos_callee.resize(1);
    std::fill(row_heat.begin(), row_heat.end(), 0.0);
    std::fill(slot_heat.begin(), slot_heat.end(), 0.0);
    out.tree_flags = (out.tree_nodes_w[0].flags & TF_ERR_DRAW) ? kTreeAnyDraw : 0u;
    wide = true;
    std::vector<int32_t> order;  // post-order of the reachable calling services
    {
      std::vector<char> seen(n, 0);
      std::vector<std::pair<int32_t, size_t>> st;
      if (!leaf[e]) {
        st.push_back({e, 0});
        seen[e] = 1;
      }
      while (!st.empty()) {
        auto &[s, j] = st.back();
        if (j < svc_sites[s].size()) {
          const int32_t c = sites[svc_sites[s][j++]].callee;
          if (!leaf[c] && !seen[c]) {
            seen[c] = 1;
            st.push_back({c, 0});
          }
        } else {
          order.push_back(s);
          st.pop_back();
        }
      }
    }
    std::reverse(order.begin(), order.end());  // callers first (a DAG: cycles were rejected)
    std::vector<uint32_t> first(n, 0), chain(n, 1);
    uint32_t next = 1;
    for (int32_t s : order) {
      first[s] = next;
      next += (uint32_t)svc_sites[s].size();
    }
    if (next >= kTreeMaxWidePositions) return give_up("more than 2^24 call sites in the site graph");
    svc_heat.assign(n, 0.0);
    svc_paths.assign(n, 0.0);
    svc_heat[e] = svc_paths[e] = 1.0;
    for (int32_t s : order) {
      for (size_t j = 0; j < svc_sites[s].size(); ++j) {
        TreeNodeW nd;
        TreeExt x;
        TreeStep tsp;
        if (!site_node(s, j, nd, x, tsp)) return give_up("a hop cost, script time or step sleep >= 2^32 ns");
        const int32_t c = sites[svc_sites[s][j]].callee;
        nd.size = leaf[c] ? 0u : first[c];
        nd.k = nd.k | ((leaf[c] ? 0u : (uint32_t)svc_sites[c].size()) << 16);
        const double heat = svc_heat[s] * (nd.prob ? nd.prob / 100.0 : 1.0);
        svc_heat[c] += heat;
        svc_paths[c] += svc_paths[s];
        row_heat[(uint32_t)out.svc_row[c]] += heat;
        slot_heat[nd.slot] += heat;
        out.tree_nodes_w.push_back(nd);
        out.tree_ext.push_back(x);
        out.tree_step.push_back(tsp);
        pos_callee.push_back(c);
      }
    }
    // nested calling invocations: the longest chain of calling services from the entry
    for (auto it = order.rbegin(); it != order.rend(); ++it) {  // callees first
      const int32_t s = *it;
      for (int32_t si : svc_sites[s]) {
        const int32_t c = sites[si].callee;
        if (!leaf[c]) chain[s] = std::max(chain[s], 1u + chain[c]);
      }
    }
    max_open = leaf[e] ? 0u : chain[e];
    out.tree_nodes_w[0].size = leaf[e] ? 0u : first[e];
    out.tree_nodes_w[0].k = (leaf[e] ? 0u : (uint32_t)svc_sites[e].size()) << 16;
    out.tree_dag = true;
  }
  if (!out.tree_dag) {
    if (out.tree_nodes_w.size() == 1) out.tree_nodes_w[0].size = 1;
    for (size_t i = 0; i < out.tree_nodes_w.size(); ++i)
      if (out.tree_nodes_w[i].size == 0) out.tree_nodes_w[i].size = 1;  // leaf positions
  }
  out.tree_frames = max_open ? max_open - 1 : 0;
  if (out.tree_frames > kTreeMaxFrames) return give_up("more than 65 nested calling invocations");
  if (!wide) {  // the 8-byte device nodes and the LDS layout
    out.tree_nodes.resize(out.tree_nodes_w.size());
    for (size_t i = 0; i < out.tree_nodes_w.size(); ++i) {
      const TreeNodeW &w = out.tree_nodes_w[i];
      out.tree_nodes[i] = TreeNode{(uint16_t)w.size, (uint16_t)w.k, w.prob, w.flags, (uint16_t)w.slot};
    }
    if (!place_tree(out, row_heat, row_bw, row_nonleaf)) {  // the per-slot counters do not fit in LDS
      wide = true;
      out.tree_nodes.clear();
    }
  }
  out.tree_wide = wide;
  if (wide) {  // LDS: the accumulators, histograms, bucket LUT, then the hottest rows and call sites
    TreeLayout &L = out.tree_layout;
    L = TreeLayout{};
    const uint32_t head = kLdsAccBytes + kHistWords * 4u + kTreeLutBytes;
    // the hottest calling rows (expected invocations per trace) in up to half
    // the CU's LDS, as the 8-byte kernel's wide rows (a u64 code-200 sum and
    // a [2][width] bucket table — width 1 for a static bucket, so every hot
    // row counts its buckets in LDS); the rest by global atomics
    std::vector<uint32_t> rorder;
    for (uint32_t r = 1; r < R; ++r)
      if (row_nonleaf[r]) rorder.push_back(r);
    std::stable_sort(rorder.begin(), rorder.end(), [&](uint32_t a, uint32_t b) { return row_heat[a] > row_heat[b]; });
    out.sum_row.clear();
    out.tree_dyn.clear();
    out.tree_dyn_words = 0;
    out.tree_row_place.assign(R, kTreeGlobalDyn);
    out.tree_row_index.assign(R, 0);
    uint32_t room = kTreeLdsHalf - head;
    for (uint32_t r : rorder) {
      // (the site graph: a row reached by more than kDagLdsPaths potential
      // invocations per trace keeps global atomics, so its u32 LDS buckets
      // do not force tiny launches — Program::tree_mult)
      if (out.tree_dag && svc_paths[out.row_svc[r]] > (double)kDagLdsPaths) continue;
      // (round 6: the code-200 buckets only — a 500, errorRate-rare, goes to
      // HBM with its sum — so a hot row takes 12 + 4 w bytes, not 12 + 8 w)
      const uint32_t w = std::max<uint32_t>(1u, row_bw[r]);
      const uint32_t need = 12u + 4u * w;
      if (need > room || out.sum_row.size() >= 0x7FFFu || out.tree_dyn_words + 1u + w >= 0xFFF0u) continue;
      room -= need;
      out.tree_row_index[r] = (uint32_t)out.sum_row.size();
      out.tree_row_place[r] = out.tree_dyn_words;
      out.sum_row.push_back(r);
      out.tree_dyn.push_back(TreeDynRow{r, out.tree_dyn_words, out.tree_row_blo[r], w});
      out.tree_dyn_words += 1u + w;
    }
    L.n_sum = (uint32_t)out.sum_row.size();
    // the hottest call sites (expected calls per trace) keep guarded 16-bit
    // counter pairs in LDS, as the 8-byte kernel's (one word each, the rest
    // of the CU); the index rides in TreeNodeW.lidx (0xFFFF: global atomics)
    const uint32_t rows_bytes = 8u * L.n_sum + 4u * out.tree_dyn_words;
    std::vector<uint32_t> order(out.n_slots);
    for (uint32_t i = 0; i < (uint32_t)out.n_slots; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return slot_heat[a] > slot_heat[b]; });
    const uint32_t K =
        std::min<uint32_t>({(uint32_t)out.n_slots, (kTreeLdsFull - head - rows_bytes - 8u) / 4u, 0xFFFEu});
    out.tree_slot_lds.assign(out.n_slots, 0xFFFFu);
    out.tree_lds_slot.assign(order.begin(), order.begin() + K);
    for (uint32_t i = 0; i < K; ++i) out.tree_slot_lds[order[i]] = (uint16_t)i;
    for (TreeNodeW &nd : out.tree_nodes_w) nd.lidx = out.tree_slot_lds.empty() ? 0xFFFFu : out.tree_slot_lds[nd.slot];
    out.tree_nodes_w[0].lidx = 0xFFFFu;  // the entry has no call site
    L.off_cnt = head;
    L.cnt16 = 1;
    L.off_sums = (head + 4u * K + 7u) & ~7u;
    L.off_dyn = L.off_sums + 8u * L.n_sum;
    L.off_nodes = L.bytes = L.off_dyn + 4u * out.tree_dyn_words;
    L.wg_per_cu = 1;
  }
  // the row words of the non-leaf callees (the entry's row is filled from the histograms)
  for (size_t i = 1; i < out.tree_nodes_w.size(); ++i) {
    const int32_t c = pos_callee[i];
    if (leaf[c]) continue;
    const uint32_t r = (uint32_t)out.svc_row[c];
    // (a wide tree: a hot row's sum index << 16 | its table's LDS offset, flagged by bit 31; else the row)
    out.tree_ext[i].row = !wide                                  ? out.tree_row_index[r] | (out.tree_row_place[r] << 16)
                          : out.tree_row_place[r] != kTreeGlobalDyn ? 0x80000000u | (out.tree_row_index[r] << 16) |
                                                                          out.tree_row_place[r]
                                                                    : r;
  }
  out.tree_ext[0].row = wide ? 0u : kTreeStaticRow << 16;
  // per slot: the callee's row, its static bucket (kTreeDynBucket when it varies), leaf flag and latency
  out.slot_tbkt.assign(out.n_slots, 0);
  out.slot_tc.assign(out.n_slots, 0);
  for (int32_t sl = 0; sl < out.n_slots; ++sl) {
    const int32_t s = out.slot_callee[sl];
    const uint32_t r = (uint32_t)out.svc_row[s];
    const uint32_t b = (leaf[s] || !row_bw[r]) ? prom_bucket_ns(tmin[s]) : kTreeDynBucket;
    out.slot_tbkt[sl] = r | (leaf[s] ? kTreeLeafSlot : 0u) | (b << 24);
    if (leaf[s] && out.svc_time[s] >= k32) return give_up("a leaf latency >= 2^32 ns");
    out.slot_tc[sl] = leaf[s] ? (uint32_t)out.svc_time[s] : 0u;
  }
  out.tree_mult = 1;
  if (wide) {  // a hot row's u32 LDS bucket counts: the positions into it (the launch split's guard)
    std::vector<uint32_t> into(R, 0);
    if (out.tree_dag) {  // the site graph: the potential invocations per trace
      for (uint32_t r = 1; r < R; ++r) into[r] = (uint32_t)std::min<double>(svc_paths[out.row_svc[r]], 4e9);
    } else {
      for (size_t i = 1; i < out.tree_nodes_w.size(); ++i) into[(uint32_t)out.svc_row[pos_callee[i]]] += 1;
    }
    for (uint32_t r : out.sum_row) out.tree_mult = std::max(out.tree_mult, into[r]);
  } else {
    for (uint32_t m : through) out.tree_mult = std::max(out.tree_mult, m);
    for (uint32_t r = 0; r < R; ++r)
      if (out.tree_row_place[r] < kTreeGlobalStatic) out.tree_mult = std::max(out.tree_mult, row_through[r]);
  }
  out.tree_why.clear();
}

uint32_t prom_bucket_ns(uint64_t t) {
  static const uint64_t edges_ms[32] = {7,  8,  9,  10, 11,  12,  14,  16,  18,  20,  25,  30,  35,  40,  45,  50,
                                        60, 70, 80, 90, 100, 120, 140, 160, 180, 200, 250, 300, 350, 400, 450, 500};
  for (uint32_t i = 0; i < 32; ++i)
    if (t <= edges_ms[i] * 1000000ull) return i;
  return 32;
}

int32_t service_index(const ServiceGraph &g, const std::string &name) {
  for (size_t i = 0; i < g.services.size(); ++i)
    if (g.services[i].name == name) return (int32_t)i;
  return -1;
}

int compile_program(const ServiceGraph &g, int32_t entry, const isim_params &p, Program &out,
                    std::string &err) {
  const int32_t n = (int32_t)g.services.size();
  if (entry < 0 || entry >= n) {
    err = "entry service out of range";
    return ISIM_EINVAL;
  }
  if (p.error_mode > ISIM_MODE_B) {
    err = "error_mode must be ISIM_MODE_A or ISIM_MODE_B";
    return ISIM_EINVAL;
  }
  const uint32_t max_depth = p.max_depth == 0 ? 64 : p.max_depth;
  if (max_depth > 64) {
    err = "max_depth must be <= 64";
    return ISIM_EINVAL;
  }
  const bool modeb = p.error_mode == ISIM_MODE_B;
  std::unordered_map<std::string, int32_t> index;
  for (int32_t i = 0; i < n; ++i) index.emplace(g.services[i].name, i);  // first wins

  // ---- call sites in document order: services, steps, concurrent sub-commands
  std::vector<Site> sites;
  std::vector<std::vector<int32_t>> svc_sites(n);
  std::vector<uint64_t> thr(n);
  for (int32_t s = 0; s < n; ++s) thr[s] = error_threshold(g.services[s].error_rate);
  auto add_site = [&](int32_t s, const Command &c, uint32_t k, bool conc) -> bool {
    Site st;
    st.caller = s;
    auto it = index.find(c.service);
    if (it == index.end()) {  // impossible after validate(); keep the guard
      err = "cannot call undefined service \"" + c.service + "\"";
      return false;
    }
    st.callee = it->second;
    st.size = c.size;
    st.prob = c.probability;
    st.k = k;
    st.conc = conc;
    unsigned __int128 h = (unsigned __int128)p.hop_base_ns +
                          ((unsigned __int128)c.size * p.req_ps_per_byte +
                           (unsigned __int128)g.services[st.callee].response_size * p.resp_ps_per_byte) /
                              1000;
    st.hop = h >= kTimeCap ? kTimeCap : (uint64_t)h;
    svc_sites[s].push_back((int32_t)sites.size());
    sites.push_back(st);
    return true;
  };
  for (int32_t s = 0; s < n; ++s) {
    uint32_t k = 0;
    for (const Command &c : g.services[s].script) {
      if (c.kind == Command::Request) {
        if (!add_site(s, c, k++, false)) return ISIM_EPARSE;
      } else if (c.kind == Command::Concurrent) {
        for (const Command &x : c.commands)
          if (x.kind == Command::Request && !add_site(s, x, k++, true)) return ISIM_EPARSE;
      }
    }
  }

  // ---- reachability, cycle check (EXT, F12) and post-order from the entry
  std::vector<int8_t> color(n, 0);  // 0 white, 1 grey, 2 black
  std::vector<int32_t> post, pre;
  {
    std::vector<std::pair<int32_t, size_t>> stack;
    stack.push_back({entry, 0});
    color[entry] = 1;
    pre.push_back(entry);
    while (!stack.empty()) {
      auto &top = stack.back();
      int32_t s = top.first;
      if (top.second < svc_sites[s].size()) {
        int32_t c = sites[svc_sites[s][top.second++]].callee;
        if (color[c] == 1) {
          err = "call cycle through service \"" + g.services[c].name + "\"";
          return ISIM_ECYCLE;
        }
        if (color[c] == 0) {
          color[c] = 1;
          pre.push_back(c);
          stack.push_back({c, 0});
        }
      } else {
        color[s] = 2;
        post.push_back(s);
        stack.pop_back();
      }
    }
  }

  // ---- per-service static facts, children before parents
  std::vector<uint64_t> tmax(n, 0), hops(n, 0);
  // tmin: a lower bound of any invocation's duration (sleeps, always-made
  // calls, and in mode B nothing after a step that can fail); tree-walk
  // rows whose bound and tmax share a duration bucket never vary in bucket
  std::vector<uint64_t> tmin(n, 0);
  std::vector<int32_t> depth(n, 0), frames(n, 0);
  std::vector<char> leaf(n, 1), can_fail(n, 0);
  bool any_prob = false, nonstatic_abort = false;
  for (int32_t s : post) {
    const Service &sv = g.services[s];
    uint64_t T = 0, H = 1, Tl = 0;
    bool lb_open = true;  // no step that can fail (mode B) seen yet: later steps always run
    int32_t d = 1, fr = 0;
    bool fail = thr[s] > 0;
    size_t si = 0;  // walks svc_sites[s] in document order
    const size_t nsteps = sv.script.size();
    for (size_t step = 0; step < nsteps; ++step) {
      const Command &c = sv.script[step];
      bool step_fallible = false;
      auto visit_call = [&](uint64_t &dt, uint64_t &dl) {
        const Site &st = sites[svc_sites[s][si++]];
        leaf[s] = 0;
        const bool maybe = st.prob >= 1 && st.prob <= 99;
        if (maybe) any_prob = true;
        dt = sat_add(st.hop, tmax[st.callee]);
        dl = maybe ? 0 : sat_add(st.hop, tmin[st.callee]);
        H = std::min<uint64_t>(H + hops[st.callee], kTimeCap);
        d = std::max(d, 1 + depth[st.callee]);
        fr = std::max(fr, frames[st.callee]);
        if (modeb && can_fail[st.callee]) step_fallible = true;
      };
      uint64_t dl = 0;
      if (c.kind == Command::Sleep) {
        T = sat_add(T, sleep_ns(c.sleep_ns));
        dl = sleep_ns(c.sleep_ns);
      } else if (c.kind == Command::Request) {
        uint64_t dt;
        visit_call(dt, dl);
        T = sat_add(T, dt);
      } else {
        uint64_t m = 0;
        for (const Command &x : c.commands) {
          uint64_t dt = 0, xl = 0;
          if (x.kind == Command::Request) visit_call(dt, xl);
          else dt = xl = sleep_ns(x.sleep_ns);
          m = std::max(m, dt);
          dl = std::max(dl, xl);
        }
        T = sat_add(T, m);
      }
      if (lb_open) Tl = sat_add(Tl, dl);
      if (step_fallible) {
        fail = true;
        lb_open = false;
        if (step + 1 < nsteps) nonstatic_abort = true;  // a failure would skip later steps
      }
    }
    tmin[s] = Tl;
    tmax[s] = T;
    hops[s] = H;
    depth[s] = d;
    frames[s] = leaf[s] ? 0 : 1 + fr;
    can_fail[s] = fail;
  }
  if (tmax[entry] >= kTimeCap) {
    err = "latency bound of the entry overflows int64 nanoseconds";
    return ISIM_ERANGE;
  }
  if ((uint32_t)depth[entry] > max_depth) {
    err = "call depth " + std::to_string(depth[entry]) + " exceeds max_depth " + std::to_string(max_depth);
    return ISIM_EDEPTH;
  }

  out = Program();
  out.entry = entry;
  out.n_services = n;
  out.n_sites = (int32_t)sites.size();
  out.max_depth = depth[entry];
  out.max_frames = std::max(1, frames[entry]);
  out.static_walk = !any_prob && !(modeb && nonstatic_abort) && !(p.flags & ISIM_FLAG_DYNAMIC);
  out.max_latency = tmax[entry];
  out.hops_upper = hops[entry];
  out.time_bits = tmax[entry] < (1ull << 32) ? 32 : 64;
  out.site_callee.resize(sites.size());
  out.site_slot.assign(sites.size(), -1);
  out.site_hop.resize(sites.size());
  for (size_t i = 0; i < sites.size(); ++i) {
    out.site_callee[i] = sites[i].callee;
    out.site_hop[i] = sites[i].hop;
  }
  // stats slots: reachable call sites in document order
  for (size_t i = 0; i < sites.size(); ++i) {
    if (color[sites[i].caller] == 2) {
      out.site_slot[i] = (int32_t)out.slot_site.size();
      out.slot_site.push_back((int32_t)i);
      out.slot_callee.push_back(sites[i].callee);
    }
  }
  out.n_slots = (int32_t)out.slot_site.size();
  // per-service duration table rows: reachable services in preorder (entry = row 0)
  if (pre.size() > (size_t)kDurRowMask) {
    err = "more than 2^24 services reachable from the entry";
    return ISIM_ERANGE;
  }
  out.svc_time = tmax;
  out.svc_row.assign(n, -1);
  for (int32_t s : pre) {
    out.svc_row[s] = (int32_t)out.row_svc.size();
    out.row_svc.push_back(s);
  }
  auto dur_word = [&](int32_t callee) -> uint32_t {
    return (uint32_t)out.svc_row[callee] | ((leaf[callee] ? prom_bucket_ns(tmax[callee]) : 0u) << 24);
  };
  for (int32_t sl = 0; sl < out.n_slots; ++sl) out.slot_dur.push_back(dur_word(out.slot_callee[sl]));
  out.root_dur = dur_word(entry);

  // ---- emit
  auto err_flags = [&](int32_t callee) -> uint32_t {
    if (thr[callee] >= (1ull << 32)) return F_ERR_ALWAYS;
    return thr[callee] > 0 ? (uint32_t)F_ERR_DRAW : 0u;
  };
  auto make_invoke = [&](int32_t callee, uint64_t hop, uint32_t flags, uint32_t prob, uint32_t k,
                         uint32_t slot) {
    Ins in{};
    const bool lf = leaf[callee];
    flags |= err_flags(callee);
    in.opf = (uint32_t)(lf ? OP_LEAF : OP_CALL) | (flags << 8) | (prob << 16);
    in.k = k;
    in.thr = (uint32_t)thr[callee];
    in.slot = slot;
    in.a_lo = (uint32_t)hop;
    in.a_hi = (uint32_t)(hop >> 32);
    if (lf) {
      in.b_lo = (uint32_t)tmax[callee];
      in.b_hi = (uint32_t)(tmax[callee] >> 32);
    } else {
      in.b_lo = (uint32_t)callee;  // patched to the body's pc below
    }
    return in;
  };
  std::vector<Ins> &code = out.code;
  code.push_back(make_invoke(entry, 0, F_ROOT, 0, 0, 0));
  Ins halt{};
  halt.opf = OP_HALT;
  code.push_back(halt);
  std::vector<int32_t> body_pc(n, -1);
  for (int32_t s : pre) {  // bodies in DFS preorder from the entry (streaming locality)
    if (leaf[s]) continue;
    body_pc[s] = (int32_t)code.size();
    size_t si = 0;
    for (const Command &c : g.services[s].script) {
      Ins in{};
      if (c.kind == Command::Sleep) {
        uint64_t d = sleep_ns(c.sleep_ns);
        in.opf = OP_SLEEP;
        in.a_lo = (uint32_t)d;
        in.a_hi = (uint32_t)(d >> 32);
        code.push_back(in);
      } else if (c.kind == Command::Request) {
        int32_t sid = svc_sites[s][si++];
        const Site &st = sites[sid];
        uint32_t prob = (st.prob >= 1 && st.prob <= 99) ? (uint32_t)st.prob : 0;
        code.push_back(make_invoke(st.callee, st.hop, prob ? (uint32_t)F_PROB : 0u, prob, st.k,
                                   (uint32_t)out.site_slot[sid]));
      } else {
        in.opf = OP_CBEGIN;
        code.push_back(in);
        for (const Command &x : c.commands) {
          Ins sub{};
          if (x.kind == Command::Sleep) {
            uint64_t d = sleep_ns(x.sleep_ns);
            sub.opf = OP_CSLEEP;
            sub.a_lo = (uint32_t)d;
            sub.a_hi = (uint32_t)(d >> 32);
            code.push_back(sub);
          } else {
            int32_t sid = svc_sites[s][si++];
            const Site &st = sites[sid];
            uint32_t prob = (st.prob >= 1 && st.prob <= 99) ? (uint32_t)st.prob : 0;
            code.push_back(make_invoke(st.callee, st.hop, F_CONC | (prob ? (uint32_t)F_PROB : 0u), prob, st.k,
                                       (uint32_t)out.site_slot[sid]));
          }
        }
        Ins e{};
        e.opf = OP_CEND;
        code.push_back(e);
      }
    }
    Ins r{};
    r.opf = OP_RET;
    code.push_back(r);
  }
  for (Ins &in : code)
    if ((in.opf & 0xFF) == OP_CALL) in.b_lo = (uint32_t)body_pc[in.b_lo];

  // ---- draw stream of a static walk: the unrolled invocation tree in hop order
  if (out.static_walk && hops[entry] <= kMaxStreamNodes) {
    auto rec = [&](int32_t callee, uint32_t slot) {
      Node nd;
      nd.thr = thr[callee] >= (1ull << 32) ? 0u : (uint32_t)thr[callee];
      nd.meta = (slot & 0xFFFFFFu) | (thr[callee] >= (1ull << 32) ? 0x80000000u : 0u);
      out.stream.push_back(nd);
    };
    struct Frame {
      int32_t svc;
      size_t next;  // next call site of the script
      uint32_t pre;  // stream position of the invocation
      uint32_t slot;
    };
    // kind 8 (sparse ancestor marking): per record its depth and parent
    std::vector<uint32_t> depth_of, parent_of;
    struct Pop {
      uint32_t pre, end, slot;  // a calling invocation: its subtree spans records [pre, end]
    };
    std::vector<Frame> stack;
    std::vector<Pop> pops;
    out.stream_end.clear();
    rec(entry, kSlotRoot);
    depth_of.push_back(0);
    parent_of.push_back(~0u);  // the sentinel, set below
    out.stream_end.push_back(0);
    stack.push_back({entry, 0, 0u, kSlotRoot});
    while (!stack.empty()) {
      Frame &top = stack.back();
      if (top.next < svc_sites[top.svc].size()) {
        const int32_t sid = svc_sites[top.svc][top.next++];
        const uint32_t slot = (uint32_t)out.site_slot[sid];
        const uint32_t pre = (uint32_t)out.stream.size();
        depth_of.push_back((uint32_t)stack.size());
        parent_of.push_back(top.pre);
        out.stream_end.push_back(0);
        rec(sites[sid].callee, slot);
        stack.push_back({sites[sid].callee, 0, pre, slot});
      } else {
        const uint32_t end = (uint32_t)out.stream.size() - 1;
        if (top.pre != end && top.slot != kSlotRoot) pops.push_back({top.pre, end, top.slot});
        out.stream_end[top.pre] = end;
        stack.pop_back();
        out.stream.back().meta += 1u << 24;  // the subtree ending here closes after this record
      }
    }
    out.stream_nodes = (uint32_t)out.stream.size();
    // the mark stream (kind 8): thr | always | depth | parent; the entry's
    // parent is the sentinel record n (depth <= max_depth - 1 <= 63: 7 bits)
    out.stream_mark.clear();
    for (uint32_t r = 0; r < out.stream_nodes; ++r) {
      const Node &nd = out.stream[r];
      const uint32_t par = r == 0 ? out.stream_nodes : parent_of[r];
      out.stream_mark.push_back(Node{nd.thr, (nd.meta & 0x80000000u) | (depth_of[r] << 24) | (par & kMarkPosMask)});
    }
    out.stream_mult.assign((size_t)out.n_slots, 0u);
    for (const Node &nd : out.stream)
      if ((nd.meta & 0xFFFFFFu) != kSlotRoot) out.stream_mult[nd.meta & 0xFFFFFFu] += 1;
    while (out.stream.size() % 4) out.stream.push_back(Node{0u, kSlotPad});
    while (out.stream_mark.size() % 4) out.stream_mark.push_back(Node{0u, kMarkPadKey});
    // close list of the mode-B stream kernel (kernel_abi.h, StreamClose)
    const uint32_t n_rec = (uint32_t)out.stream.size();
    const uint32_t n_chunks = (n_rec + kChunkRecords - 1) / kChunkRecords;
    out.stream_close_end.assign(n_chunks, 0u);
    out.stream_closes.clear();
    out.stream_close_slot.clear();
    for (const Pop &q : pops) {
      const uint32_t c = q.end / kChunkRecords, cb = c * kChunkRecords;
      const uint32_t n = std::min(kChunkRecords, n_rec - cb);  // records walked in the chunk
      const uint32_t lo = std::max(q.pre, cb);
      uint32_t m = 0;
      for (uint32_t r = lo; r <= q.end; ++r) m |= 1u << (n - 1 - (r - cb));
      out.stream_closes.push_back(StreamClose{q.pre < cb ? q.pre + 1 : 0xFFFFFFFFu, m});
      out.stream_close_slot.push_back(q.slot);
      out.stream_close_end[c] = (uint32_t)out.stream_closes.size();
    }
    for (uint32_t c = 1; c < n_chunks; ++c)
      out.stream_close_end[c] = std::max(out.stream_close_end[c], out.stream_close_end[c - 1]);
  }
  if (code.size() >= (1u << 30)) {
    err = "program too large";
    return ISIM_EINVAL;
  }
  if (!out.static_walk) build_tree(g, out, sites, svc_sites, thr, tmin, leaf, p.error_mode == ISIM_MODE_B,
                                        (p.flags & ISIM_FLAG_TREE_WIDE) != 0, (p.flags & ISIM_FLAG_TREE_DAG) != 0);
  return ISIM_OK;
}

}  // namespace isim
