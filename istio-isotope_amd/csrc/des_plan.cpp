// DES plan builder (des.h); the kernels are in des.hip.
#include "des.h"

#include <algorithm>

namespace isim {
namespace {

uint64_t sleep_of(int64_t d) { return d > 0 ? (uint64_t)d : 0; }

struct ScriptShape {
  bool ok = true;     // at most one step contains calls
  bool leaf = true;   // no call step
  uint64_t pre = 0, cmax = 0, post = 0, total = 0, hold = 0;
};

// Splits a script into [sleeps] [call step] [sleeps].
ScriptShape shape_of(const Service &s) {
  ScriptShape r;
  for (const Command &c : s.script) {
    uint64_t dur = 0, smax = 0;
    bool calls = false;
    if (c.kind == Command::Sleep) {
      dur = sleep_of(c.sleep_ns);
      r.hold += dur;
    } else if (c.kind == Command::Request) {
      calls = true;
    } else {
      for (const Command &x : c.commands) {
        if (x.kind == Command::Request) {
          calls = true;
        } else {
          smax = std::max(smax, sleep_of(x.sleep_ns));
          r.hold += sleep_of(x.sleep_ns);
        }
      }
      dur = smax;
    }
    if (calls) {
      if (!r.leaf) r.ok = false;
      r.leaf = false;
      r.cmax = smax;
    } else if (r.leaf) {
      r.pre += dur;
    } else {
      r.post += dur;
    }
    r.total += dur;
  }
  return r;
}

}  // namespace

int build_des_plan(const ServiceGraph &g, const Program &p, DesPlan &out, std::string &err) {
  out = DesPlan();
  if (!p.static_walk || p.stream_nodes == 0) {
    err = "DES needs a static walk (no probabilistic calls, no mode-B aborts) of at most 2^24 invocations";
    return ISIM_EINVAL;
  }
  const int32_t n = (int32_t)g.services.size();
  std::vector<ScriptShape> shape(n);
  std::vector<char> shaped(n, 0);
  const uint32_t np = p.stream_nodes;
  out.pos.resize(np);
  std::vector<std::vector<uint32_t>> kids(np);
  std::vector<uint32_t> depth(np, 0);
  std::vector<int32_t> pos_svc(np, -1);
  std::vector<std::vector<uint32_t>> svc_pos(n);
  std::vector<uint32_t> stack;
  for (uint32_t i = 0; i < np; ++i) {
    const Node &nd = p.stream[i];
    const uint32_t slot = nd.meta & 0xFFFFFFu;
    const int32_t svc = slot == kSlotRoot ? p.entry : p.slot_callee[slot];
    if (!shaped[svc]) {
      shape[svc] = shape_of(g.services[svc]);
      shaped[svc] = 1;
      if (!shape[svc].ok) {
        err = "service \"" + g.services[svc].name +
              "\" has more than one step with calls; the DES needs every call sent when the script's call step "
              "begins (a call after a call waits for the first callee's queueing)";
        return ISIM_EINVAL;
      }
      if (std::max<int32_t>(1, g.services[svc].num_replicas) > (int32_t)kDesMaxReplicas) {
        err = "service \"" + g.services[svc].name + "\" has more than 64 replicas (DES limit)";
        return ISIM_EINVAL;
      }
    }
    DesPos &ps = out.pos[i];
    ps.parent = stack.empty() ? kDesNoParent : stack.back();
    ps.row = (uint32_t)p.svc_row[svc];
    ps.slot = slot;
    ps.reps = (uint32_t)std::max<int32_t>(1, g.services[svc].num_replicas);
    ps.hold = shape[svc].hold;
    ps.floor = shape[svc].leaf ? shape[svc].total : shape[svc].pre + shape[svc].cmax;
    ps.post = shape[svc].post;
    ps.thr = nd.thr;
    ps.flags = (nd.meta & 0x80000000u) ? kDesFlagAlways : 0u;
    if (shape[svc].leaf) ps.flags |= kDesFlagLeaf;
    pos_svc[i] = svc;
    svc_pos[svc].push_back(i);
    if (ps.parent != kDesNoParent) {
      // calls are sent when the caller's call step begins: its pre-call sleeps after its start
      ps.off = shape[pos_svc[ps.parent]].pre + p.site_hop[p.slot_site[slot]];
      kids[ps.parent].push_back(i);
      depth[i] = depth[ps.parent] + 1;
    }
    stack.push_back(i);
    for (uint32_t k = (nd.meta >> 24) & 0x7Fu; k > 0; --k) stack.pop_back();
  }
  for (uint32_t i = 0; i < np; ++i) {
    out.pos[i].child_off = (uint32_t)out.child.size();
    out.pos[i].child_cnt = (uint32_t)kids[i].size();
    out.child.insert(out.child.end(), kids[i].begin(), kids[i].end());
  }
  // up pass: positions by depth
  const uint32_t levels = np ? 1 + *std::max_element(depth.begin(), depth.end()) : 0;
  out.level_off.assign(levels + 1, 0);
  for (uint32_t i = 0; i < np; ++i) out.level_off[depth[i] + 1]++;
  for (uint32_t l = 0; l < levels; ++l) {
    out.max_width = std::max(out.max_width, out.level_off[l + 1]);
    out.level_off[l + 1] += out.level_off[l];
  }
  out.level_pos.resize(np);
  std::vector<uint32_t> fill(out.level_off.begin(), out.level_off.end() - 1);
  for (uint32_t i = 0; i < np; ++i) out.level_pos[fill[depth[i]]++] = i;

  // down pass: a service's queue needs ALL its arrivals, so services go by
  // service level (longest call path from the entry; positions in hop order
  // visit callers before callees, so one sweep settles it)
  std::vector<uint32_t> slev(n, 0);
  {
    // longest path over the service DAG of the reachable services (Kahn)
    std::vector<std::vector<int32_t>> out_e(n);
    std::vector<uint32_t> indeg(n, 0);
    std::vector<std::pair<int32_t, int32_t>> edges;
    for (uint32_t i = 0; i < np; ++i)
      if (out.pos[i].parent != kDesNoParent) edges.push_back({pos_svc[out.pos[i].parent], pos_svc[i]});
    std::sort(edges.begin(), edges.end());
    edges.erase(std::unique(edges.begin(), edges.end()), edges.end());
    for (auto &e : edges) {
      out_e[e.first].push_back(e.second);
      indeg[e.second]++;
    }
    std::vector<int32_t> q{p.entry};
    for (size_t h = 0; h < q.size(); ++h)
      for (int32_t c : out_e[q[h]]) {
        slev[c] = std::max(slev[c], slev[q[h]] + 1);
        if (--indeg[c] == 0) q.push_back(c);
      }
  }
  // arrivals in trace order (the FIFO scan needs no sort) when the caller's
  // start times are: a single-replica caller whose own arrivals are in order
  std::vector<char> arr_sorted(np, 1), s_sorted(np, 1);
  for (uint32_t i = 0; i < np; ++i) {
    const uint32_t par = out.pos[i].parent;
    arr_sorted[i] = par == kDesNoParent ? 1 : s_sorted[par];
    s_sorted[i] = arr_sorted[i] && out.pos[i].reps == 1;
  }
  uint32_t n_slev = 0;
  for (int32_t s = 0; s < n; ++s)
    if (!svc_pos[s].empty()) n_slev = std::max(n_slev, slev[s] + 1);
  std::vector<std::vector<uint32_t>> fast(n_slev);
  std::vector<std::vector<int32_t>> srt(n_slev);
  for (int32_t s = 0; s < n; ++s) {
    if (svc_pos[s].empty()) continue;
    bool need = svc_pos[s].size() > 1;
    for (uint32_t v : svc_pos[s]) need = need || !arr_sorted[v];
    if (need) srt[slev[s]].push_back(s);
    else fast[slev[s]].push_back(svc_pos[s][0]);
  }
  out.fast_off.assign(n_slev + 1, 0);
  out.fast_multi.assign(n_slev, 0);
  out.sorted_off.assign(n_slev + 1, 0);
  for (uint32_t l = 0; l < n_slev; ++l) {
    // single-replica positions first: they run a kernel variant without the routing draw
    std::stable_partition(fast[l].begin(), fast[l].end(), [&](uint32_t v) { return out.pos[v].reps == 1; });
    out.fast_multi[l] = out.fast_off[l];
    for (uint32_t v : fast[l]) out.fast_multi[l] += out.pos[v].reps == 1 ? 1u : 0u;
    out.fast_pos.insert(out.fast_pos.end(), fast[l].begin(), fast[l].end());
    out.fast_off[l + 1] = (uint32_t)out.fast_pos.size();
    for (int32_t s : srt[l]) {
      DesSortSvc ss;
      ss.row = (uint32_t)p.svc_row[s];
      ss.reps = (uint32_t)std::max<int32_t>(1, g.services[s].num_replicas);
      ss.pos_off = (uint32_t)out.sort_pos.size();
      ss.pos_cnt = (uint32_t)svc_pos[s].size();
      ss.hold = shape[s].hold;
      out.sort_pos.insert(out.sort_pos.end(), svc_pos[s].begin(), svc_pos[s].end());
      out.max_sort_pos = std::max(out.max_sort_pos, ss.pos_cnt);
      out.sorted.push_back(ss);
    }
    out.sorted_off[l + 1] = (uint32_t)out.sorted.size();
  }
  out.slot_mult = p.stream_mult;
  return ISIM_OK;
}

}  // namespace isim
