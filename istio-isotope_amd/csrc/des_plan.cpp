// DES plan builder (des.h); the kernels are in des.hip.
//
// The plan unrolls the static walk's invocation tree (one POSITION per
// invocation, hop order = the draw stream's order) and schedules the exact
// DES of a batch as ROUNDS; a round runs, in this order,
//   1. step begins   BK rows of call steps k > 1 (and k = 1 of multi-step
//                    scripts) whose inputs are settled,
//   2. queues        the FIFO scan of every service whose arrivals are all
//                    known (fast path, or sort path),
//   3. finishes      F of positions whose start and callees are settled,
//                    deepest first.
// Every operation goes in the earliest round its inputs allow (longest path
// over the dependency graph).  A dependency cycle — a service with a hold
// invoked both inside a call step and after it within one caller's script —
// is cut at the back edges of a depth-first search and the schedule runs as
// repeated passes to its fixed point (des.hip).  Zero-hold services (no
// sleeps) never queue: each of their positions starts at its arrival, one op
// each.  Graphs whose scripts have at most one call step
// get the shortest schedule: queues by service level, all finishes last.
#include "des.h"

#include <algorithm>
#include <cstdlib>

namespace isim {
namespace {

uint64_t sleep_of(int64_t d) { return d > 0 ? (uint64_t)d : 0; }

// A script as [sleeps] (call step [sleeps])* (DESIGN.md §10.1).
struct ScriptShape {
  uint64_t pre = 0;                  // sleeps before the first call step (leaf: the script time)
  std::vector<uint64_t> smax, gap;   // per call step: longest concurrent sleep; sleeps after it
  std::vector<uint32_t> call_step;   // per call command (document order): its call step
  uint64_t hold = 0;                 // sum of all sleeps (the worker hold time)
  bool leaf() const { return smax.empty(); }
};

ScriptShape shape_of(const Service &s) {
  ScriptShape r;
  for (const Command &c : s.script) {
    uint64_t dur = 0, smax = 0;
    uint32_t calls = 0;
    if (c.kind == Command::Sleep) {
      dur = sleep_of(c.sleep_ns);
      r.hold += dur;
    } else if (c.kind == Command::Request) {
      calls = 1;
    } else {
      for (const Command &x : c.commands) {
        if (x.kind == Command::Request) {
          ++calls;
        } else {
          smax = std::max(smax, sleep_of(x.sleep_ns));
          r.hold += sleep_of(x.sleep_ns);
        }
      }
      dur = smax;
    }
    if (calls) {
      for (uint32_t i = 0; i < calls; ++i) r.call_step.push_back((uint32_t)r.smax.size());
      r.smax.push_back(smax);
      r.gap.push_back(0);
    } else if (r.smax.empty()) {
      r.pre += dur;
    } else {
      r.gap.back() += dur;
    }
  }
  return r;
}

}  // namespace

void des_row_traffic(const DesPlan &plan, uint32_t &reads, uint32_t &writes) {
  reads = writes = 0;
  const uint32_t np = (uint32_t)plan.pos.size();
  // flagged callees per caller (des_up records their durations)
  std::vector<uint32_t> nd(np, 0);
  for (uint32_t v = 1; v < np; ++v)
    if (plan.pos[v].flags & kDesFlagParentDur) ++nd[plan.pos[v].parent];
  for (uint32_t v = 0; v < np; ++v) {
    const DesPos &q = plan.pos[v];
    // queue pass (fast, zero-hold or sort path): the arrival row (the entry's
    // arrivals are per-trace extras), the start or fused finish row
    reads += v ? 1 : 0;
    writes += 1;
    if (q.flags & kDesFlagFused) continue;
    // finish pass: the children's finishes, the start row unless the finish
    // needs none and no callee's duration is recorded here, the arrival row
    // when the position records its own durations, the finish row
    reads += q.child_cnt;
    reads += (q.flags & kDesFlagNoStart) && nd[v] == 0 && q.child_cnt <= kDesUpChildLds ? 0 : 1;
    reads += v && !(q.flags & kDesFlagParentDur) ? 1 : 0;
    writes += 1;
  }
  reads += (uint32_t)plan.steps.size() * 2;  // step begins: a row read and written per BK row
  writes += (uint32_t)plan.steps.size();
}

int build_des_plan(const ServiceGraph &g, const Program &p, bool modeb, DesPlan &out, std::string &err) {
  out = DesPlan();
  out.modeb = modeb;
  // the positions: a static walk's draw stream (every invocation executes in
  // every trace), or — probabilistic calls, or mode-B aborts (a call step
  // after one that can fail) — the lane tree walk's unrolled tree of
  // POTENTIAL invocations (kernel_abi.h TreeNode): the item engine
  // (des_items.hip) simulates the executed ones only
  struct Src {
    uint32_t slot, parent, thr;
    bool always;
  };
  std::vector<Src> src;
  if (p.static_walk && p.stream_nodes) {
    std::vector<uint32_t> stack;
    for (uint32_t i = 0; i < p.stream_nodes; ++i) {
      const Node &nd = p.stream[i];
      src.push_back({nd.meta & 0xFFFFFFu, stack.empty() ? kDesNoParent : stack.back(), nd.thr,
                     (nd.meta & 0x80000000u) != 0});
      stack.push_back(i);
      for (uint32_t k = (nd.meta >> 24) & 0x7Fu; k > 0; --k) stack.pop_back();
    }
  } else if (!p.static_walk && p.has_tree() && !p.tree_dag) {
    out.items = true;
    std::vector<std::pair<uint32_t, uint32_t>> stack;  // (position, end of its subtree)
    for (uint32_t i = 0; i < p.tree_positions(); ++i) {
      while (!stack.empty() && i >= stack.back().second) stack.pop_back();
      const TreeNodeW &nd = p.tree_nodes_w[i];
      src.push_back({i ? (uint32_t)nd.slot : kSlotRoot, stack.empty() ? kDesNoParent : stack.back().first,
                     p.tree_ext[i].thr, (nd.flags & TF_ERR_ALWAYS) != 0});
      stack.push_back({i, i + std::max<uint32_t>(1, nd.size)});
    }
  } else {
    err = p.static_walk ? "DES needs a static walk of at most 2^24 invocations"
          : p.tree_dag  ? std::string("DES of a dynamic walk needs the lane tree walk's unrolled tree (this walk runs "
                                      "on the site graph: more than 2^24 potential invocations)")
                        : "DES of a dynamic walk needs the lane tree walk's unrolled tree (" + p.tree_why + ")";
    return ISIM_EINVAL;
  }
  const int32_t n = (int32_t)g.services.size();
  std::vector<ScriptShape> shape(n);
  std::vector<char> shaped(n, 0);
  const uint32_t np = (uint32_t)src.size();
  out.pos.resize(np);
  out.ext.assign(np, DesPosExt{kDesNone, kDesNone, 0, 0});
  std::vector<std::vector<uint32_t>> kids(np);
  std::vector<uint32_t> depth(np, 0), kstep(np, 0);  // kstep: the caller's call step of the position
  std::vector<int32_t> pos_svc(np, -1);
  std::vector<std::vector<uint32_t>> svc_pos(n);
  for (uint32_t i = 0; i < np; ++i) {
    const uint32_t slot = src[i].slot;
    const int32_t svc = slot == kSlotRoot ? p.entry : p.slot_callee[slot];
    if (!shaped[svc]) {
      shape[svc] = shape_of(g.services[svc]);
      shaped[svc] = 1;
      if (std::max<int32_t>(1, g.services[svc].num_replicas) > 65536) {
        err = "service \"" + g.services[svc].name + "\" has more than 65536 replicas (DES limit)";
        return ISIM_EINVAL;
      }
    }
    const ScriptShape &sh = shape[svc];
    DesPos &ps = out.pos[i];
    ps.parent = src[i].parent;
    ps.row = (uint32_t)p.svc_row[svc];
    ps.slot = slot;
    ps.reps = (uint32_t)std::max<int32_t>(1, g.services[svc].num_replicas);
    ps.hold = sh.hold;
    out.max_hold = std::max(out.max_hold, sh.hold);
    // one call step: F = max(S + floor, max_c F_c) + post; several: F =
    // max(BK_last + floor, max_c(last step) F_c) + post
    ps.floor = sh.leaf() ? sh.pre : (sh.smax.size() == 1 ? sh.pre + sh.smax[0] : sh.smax.back());
    ps.post = sh.leaf() ? 0 : sh.gap.back();
    ps.thr = src[i].thr;
    ps.flags = src[i].always ? kDesFlagAlways : 0u;
    if (sh.leaf()) ps.flags |= kDesFlagLeaf;
    pos_svc[i] = svc;
    svc_pos[svc].push_back(i);
    if (ps.parent != kDesNoParent) {
      const uint32_t par = ps.parent;
      const ScriptShape &ph = shape[pos_svc[par]];
      kstep[i] = ph.call_step[kids[par].size()];  // j-th callee = j-th call command (static walk)
      const uint64_t h = p.site_hop[p.slot_site[slot]];
      ps.off = kstep[i] == 0 ? ph.pre + h : h;     // step 1: start(parent) + pre + H; later: BK + H
      kids[par].push_back(i);
      depth[i] = depth[par] + 1;
    }
  }
  for (uint32_t i = 0; i < np; ++i) {
    out.pos[i].child_off = (uint32_t)out.child.size();
    out.pos[i].child_cnt = (uint32_t)kids[i].size();
    out.child.insert(out.child.end(), kids[i].begin(), kids[i].end());
  }
  out.n_levels = np ? 1 + *std::max_element(depth.begin(), depth.end()) : 0;
  {
    std::vector<uint32_t> w(out.n_levels, 0);
    for (uint32_t i = 0; i < np; ++i) out.max_width = std::max(out.max_width, ++w[depth[i]]);
  }

  // ---- BK rows: every call step of a multi-step script
  std::vector<std::vector<uint32_t>> pos_bk(np);  // per position: BK row of each of its call steps
  for (uint32_t i = 0; i < np; ++i) {
    const ScriptShape &sh = shape[pos_svc[i]];
    if (sh.smax.size() < 2) continue;
    out.general = true;
    uint32_t c0 = out.pos[i].child_off, cprev = 0, nprev = 0;
    for (uint32_t k = 0; k < sh.smax.size(); ++k) {
      DesStep st{};
      st.pos = i;
      st.prev = k ? pos_bk[i][k - 1] : kDesNone;
      st.add = k ? sh.gap[k - 1] : sh.pre;
      st.smax = k ? sh.smax[k - 1] : 0;
      st.child_off = cprev;
      st.child_cnt = nprev;
      pos_bk[i].push_back((uint32_t)out.steps.size());
      out.steps.push_back(st);
      // the callees of step k follow in the children list
      uint32_t cnt = 0;
      for (uint32_t j = 0; j < kids[i].size(); ++j) cnt += kstep[kids[i][j]] == k ? 1u : 0u;
      cprev = c0;
      nprev = cnt;
      c0 += cnt;
    }
    out.ext[i].bk_last = pos_bk[i].back();
    out.ext[i].last_child = out.pos[i].child_cnt - nprev;
  }
  for (uint32_t i = 0; i < np; ++i) {
    const uint32_t par = out.pos[i].parent;
    if (par != kDesNoParent && kstep[i] > 0) out.ext[i].bk_in = pos_bk[par][kstep[i]];
  }

  // ---- arrivals in trace order (no sort needed): a first-step callee of a
  // single-replica caller whose own arrivals are in order
  std::vector<char> arr_sorted(np, 1), s_sorted(np, 1);
  for (uint32_t i = 0; i < np; ++i) {
    const uint32_t par = out.pos[i].parent;
    arr_sorted[i] = par == kDesNoParent ? 1 : (s_sorted[par] && kstep[i] == 0);
    s_sorted[i] = arr_sorted[i] && (out.pos[i].reps == 1 || out.pos[i].hold == 0);
  }

  // ---- the schedule: op ids  Q(s) = service s, F(v) = n + v, A(b) = n + np + b,
  // Z(v) = n + np + nb + v: the start of a position of a zero-hold service
  // (start = arrival, no queue: one op per position, so such a service can be
  // called both inside a call step and after it)
  const uint32_t nq = (uint32_t)n, nb = (uint32_t)out.steps.size();
  const uint32_t n_ops = nq + np + nb + np;
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> pred(n_ops);  // (op, weight)
  auto zero = [&](uint32_t v) { return out.pos[v].hold == 0; };
  auto Q = [&](uint32_t v) { return zero(v) ? nq + np + nb + v : (uint32_t)pos_svc[v]; };
  auto F = [&](uint32_t v) { return nq + v; };
  auto Ab = [&](uint32_t b) { return nq + np + b; };
  for (uint32_t v = 0; v < np; ++v) {
    const uint32_t par = out.pos[v].parent;
    // queue(svc v) after the arrival of v is known
    if (par != kDesNoParent) {
      if (kstep[v] == 0) pred[Q(v)].push_back({Q(par), 1});          // start(parent), earlier round
      else pred[Q(v)].push_back({Ab(out.ext[v].bk_in), 0});          // BK row, same round or later
    }
    pred[F(v)].push_back({Q(v), 0});
    for (uint32_t c : kids[v]) pred[F(v)].push_back({F(c), 0});        // same round: deeper first
    if (out.ext[v].bk_last != kDesNone) pred[F(v)].push_back({Ab(out.ext[v].bk_last), 0});
  }
  for (uint32_t b = 0; b < nb; ++b) {
    const DesStep &st = out.steps[b];
    if (st.prev == kDesNone) {
      pred[Ab(b)].push_back({Q(st.pos), 1});
    } else {
      pred[Ab(b)].push_back({Ab(st.prev), 1});  // step begins of one round run in one launch
      for (uint32_t j = 0; j < st.child_cnt; ++j) pred[Ab(b)].push_back({F(out.child[st.child_off + j]), 1});
    }
  }
  std::vector<char> used(n_ops, 0), step_cut(nb, 0);
  for (uint32_t v = 0; v < np; ++v) used[Q(v)] = used[F(v)] = 1;
  for (uint32_t b = 0; b < nb; ++b) used[Ab(b)] = 1;
  // cycles (a service with a hold invoked both inside a caller's call step
  // and after it): every cycle of the operation graph runs through an edge
  // F(v) -> A(b) (a step begin waiting for the previous step's callees) —
  // positions form a tree and the service graph is acyclic, so without
  // those edges paths only go down (queues, step begins) or up among
  // finishes.  Those edges inside a strongly connected component are cut;
  // the schedule then runs as repeated passes to its fixed point
  // (des_launch), the cut step begins reading the previous pass's finish
  // rows (F rows hold their final value at the end of a pass).
  {
    // Tarjan's strongly connected components, iterative
    std::vector<std::vector<uint32_t>> succ(n_ops);
    for (uint32_t o = 0; o < n_ops; ++o)
      for (auto &e : pred[o]) succ[e.first].push_back(o);
    std::vector<int32_t> idx(n_ops, -1), low(n_ops, 0), comp(n_ops, -1);
    std::vector<char> on(n_ops, 0);
    std::vector<uint32_t> stk, comp_size;
    std::vector<std::pair<uint32_t, uint32_t>> call;  // (op, next successor)
    int32_t counter = 0;
    for (uint32_t r0 = 0; r0 < n_ops; ++r0) {
      if (!used[r0] || idx[r0] >= 0) continue;
      call.push_back({r0, 0});
      idx[r0] = low[r0] = counter++;
      stk.push_back(r0);
      on[r0] = 1;
      while (!call.empty()) {
        const uint32_t u = call.back().first;
        if (call.back().second < succ[u].size()) {
          const uint32_t w = succ[u][call.back().second++];
          if (idx[w] < 0) {
            idx[w] = low[w] = counter++;
            stk.push_back(w);
            on[w] = 1;
            call.push_back({w, 0});
          } else if (on[w]) {
            low[u] = std::min(low[u], idx[w]);
          }
        } else {
          call.pop_back();
          if (!call.empty()) low[call.back().first] = std::min(low[call.back().first], low[u]);
          if (low[u] == idx[u]) {
            const int32_t c = (int32_t)comp_size.size();
            uint32_t n_in = 0, w;
            do {
              w = stk.back();
              stk.pop_back();
              on[w] = 0;
              comp[w] = c;
              ++n_in;
            } while (w != u);
            comp_size.push_back(n_in);
          }
        }
      }
    }
    auto is_f = [&](uint32_t o) { return o >= nq && o < nq + np; };
    step_cut.assign(nb, 0);
    auto is_a = [&](uint32_t o) { return o >= nq + np && o < nq + np + nb; };
    for (uint32_t o = 0; o < n_ops; ++o) {
      if (!used[o] || !is_a(o) || comp_size[comp[o]] < 2) continue;
      auto &pl = pred[o];
      const size_t before = pl.size();
      pl.erase(std::remove_if(pl.begin(), pl.end(),
                              [&](const std::pair<uint32_t, uint32_t> &e) {
                                return is_f(e.first) && comp[e.first] == comp[o];
                              }),
               pl.end());
      if (pl.size() != before) {
        out.cyclic = true;
        step_cut[o - (nq + np)] = 1;
      }
    }
  }
  // longest path in topological order (acyclic now): O(ops + edges).  A
  // relaxation sweep in op-index order needed one sweep per link of the
  // longest chain, and sequential call steps chain every position of the
  // tree (quadratic in the positions of a deep DAG)
  std::vector<uint32_t> rnd(n_ops, 0);
  {
    std::vector<uint32_t> indeg(n_ops, 0), succ_off(n_ops + 1, 0);
    for (uint32_t o = 0; o < n_ops; ++o)
      for (auto &e : pred[o]) {
        ++indeg[o];
        ++succ_off[e.first + 1];
      }
    for (uint32_t o = 0; o < n_ops; ++o) succ_off[o + 1] += succ_off[o];
    std::vector<std::pair<uint32_t, uint32_t>> succ(succ_off[n_ops]);
    {
      std::vector<uint32_t> at(succ_off.begin(), succ_off.end() - 1);
      for (uint32_t o = 0; o < n_ops; ++o)
        for (auto &e : pred[o]) succ[at[e.first]++] = {o, e.second};
    }
    std::vector<uint32_t> ready;
    for (uint32_t o = 0; o < n_ops; ++o)
      if (used[o] && indeg[o] == 0) ready.push_back(o);
    size_t done = 0;
    while (!ready.empty()) {
      const uint32_t o = ready.back();
      ready.pop_back();
      ++done;
      for (uint32_t j = succ_off[o]; j < succ_off[o + 1]; ++j) {
        const uint32_t w = succ[j].first;
        rnd[w] = std::max(rnd[w], rnd[o] + succ[j].second);
        if (--indeg[w] == 0) ready.push_back(w);
      }
    }
    size_t n_used = 0;
    for (uint32_t o = 0; o < n_ops; ++o) n_used += used[o] ? 1 : 0;
    if (done != n_used) {
      err = "DES schedule: dependency cycle left after removing back edges (internal error)";
      return ISIM_EINVAL;
    }
  }
  uint32_t R = 0;
  for (uint32_t o = 0; o < n_ops; ++o)
    if (used[o]) R = std::max(R, rnd[o] + 1);
  if (!out.general) {
    // no step begins depend on finishes: all finishes in one last round
    for (uint32_t v = 0; v < np; ++v) rnd[F(v)] = R;
    R += 1;
  }
  if (R > kDesMaxRounds) {
    // every round is a few launches over the whole batch: a schedule this
    // long (sequential call steps chaining a deep tree) is no batch-parallel
    // simulation any more
    err = "DES schedule needs " + std::to_string(R) + " rounds (sequential call steps chain the invocation tree); "
          "the limit is " + std::to_string(kDesMaxRounds);
    return ISIM_EINVAL;
  }
  // ---- lay the rounds out
  std::vector<std::vector<uint32_t>> arr(R), fast(R), zpos(R);
  std::vector<std::vector<int32_t>> srt(R);
  for (uint32_t b = 0; b < nb; ++b) arr[rnd[Ab(b)]].push_back(b);
  for (uint32_t v = 0; v < np; ++v)
    if (zero(v)) zpos[rnd[Q(v)]].push_back(v);
  for (int32_t s = 0; s < n; ++s) {
    if (svc_pos[s].empty() || shape[s].hold == 0) continue;
    // the one-workgroup-per-position pass keeps per-replica carries in LDS
    // (<= kDesMaxReplicas); more replicas: the sort path's segmented scan
    bool need = svc_pos[s].size() > 1 || std::max<int32_t>(1, g.services[s].num_replicas) > (int32_t)kDesMaxReplicas;
    for (uint32_t v : svc_pos[s]) need = need || !arr_sorted[v];
    if (need) {
      srt[rnd[s]].push_back(s);
    } else {
      const uint32_t v = svc_pos[s][0];
      fast[rnd[s]].push_back(v);
      // a leaf's finish needs only its start: the queue pass writes F (every
      // reader of F(v) runs in a later stage of Q(v)'s round or later)
      if (!out.items && (out.pos[v].flags & kDesFlagLeaf)) out.pos[v].flags |= kDesFlagFused;
    }
  }
  // finish groups: by round, deepest first, most children first within a
  // depth (the costliest blocks start first)
  std::vector<uint32_t> fin;
  for (uint32_t v = 0; v < np; ++v)
    if (!(out.pos[v].flags & kDesFlagFused)) fin.push_back(v);
  std::stable_sort(fin.begin(), fin.end(), [&](uint32_t a, uint32_t b) {
    if (rnd[F(a)] != rnd[F(b)]) return rnd[F(a)] < rnd[F(b)];
    if (depth[a] != depth[b]) return depth[a] > depth[b];
    return out.pos[a].child_cnt > out.pos[b].child_cnt;
  });
  size_t fi = 0;
  out.arr_off.assign(R + 1, 0);
  out.fast_off.assign(R + 1, 0);
  out.zero_off.assign(R + 1, 0);
  out.fast_split.assign(5 * R, 0);
  out.sorted_off.assign(R + 1, 0);
  out.fin_round_off.assign(R + 1, 0);
  out.fin_off.assign(1, 0);
  for (uint32_t r = 0; r < R; ++r) {
    out.arr_ops.insert(out.arr_ops.end(), arr[r].begin(), arr[r].end());
    out.arr_off[r + 1] = (uint32_t)out.arr_ops.size();
    // grouped by kernel variant: single replica (no routing draw) or not, fused leaf or not
    // fused leaves first: in a launch mixing both, the costlier workgroups
    // start first and the last wave of workgroups is the cheaper kind
    auto variant = [&](uint32_t v) {
      return (out.pos[v].reps > 1 ? 2u : 0u) + ((out.pos[v].flags & kDesFlagFused) ? 0u : 1u);
    };
    std::stable_sort(fast[r].begin(), fast[r].end(),
                     [&](uint32_t a, uint32_t b) { return variant(a) < variant(b); });
    uint32_t at = out.fast_off[r];
    for (uint32_t j = 0; j < 4; ++j) {
      out.fast_split[5 * r + j] = at;
      for (uint32_t v : fast[r]) at += variant(v) == j ? 1u : 0u;
    }
    out.fast_split[5 * r + 4] = at;
    out.fast_pos.insert(out.fast_pos.end(), fast[r].begin(), fast[r].end());
    out.fast_off[r + 1] = (uint32_t)out.fast_pos.size();
    out.zero_pos.insert(out.zero_pos.end(), zpos[r].begin(), zpos[r].end());
    out.zero_off[r + 1] = (uint32_t)out.zero_pos.size();
    for (int32_t s : srt[r]) {
      DesSortSvc ss;
      ss.row = (uint32_t)p.svc_row[s];
      ss.reps = (uint32_t)std::max<int32_t>(1, g.services[s].num_replicas);
      ss.pos_off = (uint32_t)out.sort_pos.size();
      ss.pos_cnt = (uint32_t)svc_pos[s].size();
      ss.hold = shape[s].hold;
      out.sort_pos.insert(out.sort_pos.end(), svc_pos[s].begin(), svc_pos[s].end());
      out.max_sort_pos = std::max(out.max_sort_pos, ss.pos_cnt);
      uint32_t rb = 0;
      while (ss.reps > 1 && ((ss.reps - 1) >> rb) != 0) ++rb;
      out.max_rep_bits = std::max(out.max_rep_bits, rb);
      out.sorted.push_back(ss);
    }
    out.sorted_off[r + 1] = (uint32_t)out.sorted.size();
    while (fi < fin.size() && rnd[F(fin[fi])] == r) {
      const uint32_t d = depth[fin[fi]];
      while (fi < fin.size() && rnd[F(fin[fi])] == r && depth[fin[fi]] == d) out.fin_pos.push_back(fin[fi++]);
      out.fin_off.push_back((uint32_t)out.fin_pos.size());
    }
    out.fin_round_off[r + 1] = (uint32_t)out.fin_off.size() - 1;
  }
  // ---- pipelined queue segments
  auto pipeable = [&](uint32_t r) {
    return !out.items && out.arr_off[r + 1] == out.arr_off[r] && out.zero_off[r + 1] == out.zero_off[r] &&
           out.sorted_off[r + 1] == out.sorted_off[r] && out.fast_split[5 * r + 2] == out.fast_off[r + 1] &&
           out.fast_off[r + 1] > out.fast_off[r];
  };
  std::vector<uint32_t> seg_of(np, kDesNone);
  for (uint32_t r = 0; r < R;) {
    if (!pipeable(r)) {
      ++r;
      continue;
    }
    uint32_t e = r + 1;  // the run [r, e): round e - 1 has no finishes, round e is pipeable
    while (e < R && pipeable(e) && out.fin_round_off[e] == out.fin_round_off[e - 1]) ++e;
    if (e - r >= 2) {
      const uint32_t id = (uint32_t)out.pipe.size();
      DesPlan::PipeSeg sg{r, e - 1, (uint32_t)out.pipe_pos.size(), 0};
      for (uint32_t x = r; x < e; ++x)
        for (uint32_t fused = 0; fused < 2; ++fused)
          for (uint32_t i = out.fast_off[x]; i < out.fast_off[x + 1]; ++i) {
            const uint32_t v = out.fast_pos[i];
            if (((out.pos[v].flags & kDesFlagFused) != 0) != (fused != 0)) continue;
            seg_of[v] = id;
            out.pipe_pos.push_back(v);
          }
      sg.cnt = (uint32_t)out.pipe_pos.size() - sg.off;
      for (uint32_t i = sg.off; i < sg.off + sg.cnt; ++i) {
        const uint32_t v = out.pipe_pos[i], u = out.pos[v].parent;
        // the arrival row is the caller's start row, written in this launch
        const bool wait = u != kDesNoParent && out.ext[v].bk_in == kDesNone && seg_of[u] == id;
        out.pipe_dep.push_back(wait ? u : kDesNone);
      }
      out.pipe.push_back(sg);
    }
    r = e;
  }
  out.up_n32 = !out.general && !out.cyclic;
  for (const DesPos &ps : out.pos)
    out.up_n32 = out.up_n32 && ps.off < (1ull << 30) && ps.floor < (1ull << 30) && ps.post < (1ull << 30);
  out.pipe_n32 = !out.pipe.empty();
  for (uint32_t v : out.pipe_pos) {
    const DesPos &ps = out.pos[v];
    out.pipe_n32 = out.pipe_n32 && ps.hold < kDesN32HoldMax && ps.off < (1ull << 30) &&
                   (!(ps.flags & kDesFlagFused) || ps.floor < (1ull << 30));
  }
  // finishes without the start row (kDesFlagNoStart)
  if (!out.items && !out.general && !out.cyclic) {
    for (uint32_t v = 0; v < np; ++v) {
      if ((out.pos[v].flags & kDesFlagFused) || kids[v].empty()) continue;
      const ScriptShape &sh = shape[pos_svc[v]];
      const uint64_t smax = sh.smax.empty() ? 0 : sh.smax[0];
      bool ok = true;
      for (uint32_t c : kids[v]) ok = ok && out.pos[c].off >= sh.pre + smax;  // off = pre + H
      if (ok) out.pos[v].flags |= kDesFlagNoStart;
    }
  }
  // durations recorded by the caller (des.hip des_up): one call step per
  // script (every arrival is start(caller) + off), no fixed-point passes, the
  // caller's first kDesDurKids non-fused callees
  if (!out.items && !out.general && !out.cyclic) {
    for (uint32_t v = 0; v < np; ++v) {
      if (kids[v].size() > kDesUpChildLds) continue;
      uint32_t j = 0;
      for (uint32_t c : kids[v]) {
        if ((out.pos[c].flags & kDesFlagFused) || j >= kDesDurKids) continue;
        out.pos[c].flags |= kDesFlagParentDur | (j++ << kDesDurShift);
      }
    }
  }
  out.slot_mult = p.stream_mult;
  if (out.items) {
    // per position: its queue round, finish group, call step in its caller,
    // and its own call steps' BK ids (des_items.hip)
    out.item_pos.assign(np, DesItemPos{0, 0, 0, 0, kDesNone});
    for (uint32_t v = 0; v < np; ++v) {
      DesItemPos &ip = out.item_pos[v];
      ip.qround = rnd[Q(v)];
      ip.kstep = kstep[v];
      const ScriptShape &sh = shape[pos_svc[v]];
      ip.nsteps = (uint32_t)sh.smax.size();
      out.item_acc = std::max<uint32_t>(out.item_acc, std::max<uint32_t>(1, ip.nsteps));
      if (ip.nsteps >= 2) {
        ip.bk_first = out.ext[v].bk_last - (ip.nsteps - 1);
        out.item_bk = std::max<uint32_t>(out.item_bk, ip.nsteps);
      }
    }
    // the finish sort keys hold group | position bits (des_items.hip)
    if (out.fin_off.size() - 1 > 65535) {
      err = "DES of a dynamic walk: more than 65535 finish groups";
      return ISIM_EINVAL;
    }
    for (uint32_t gi = 0; gi + 1 < out.fin_off.size(); ++gi)
      for (uint32_t j = out.fin_off[gi]; j < out.fin_off[gi + 1]; ++j) out.item_pos[out.fin_pos[j]].fgroup = gi;
    out.round_nosort.assign(R, 1);
    for (uint32_t v = 0; v < np; ++v) {
      const DesPos &q = out.pos[v];
      const bool free = q.hold == 0 ||
                        (svc_pos[pos_svc[v]].size() == 1 && q.reps == 1 && arr_sorted[v]);
      if (!free) out.round_nosort[rnd[Q(v)]] = 0;
    }
    out.step_round.resize(nb);
    for (uint32_t b = 0; b < nb; ++b) out.step_round[b] = rnd[Ab(b)] | (step_cut[b] ? kDesStepCut : 0u);
  }
  return ISIM_OK;
}

}  // namespace isim
