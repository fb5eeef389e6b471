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
    err = "DES v1 needs a static walk (no probabilistic calls, no mode-B aborts) of at most 2^24 invocations";
    return ISIM_EINVAL;
  }
  const int32_t n = (int32_t)g.services.size();
  if ((uint64_t)p.stream_nodes > (uint64_t)n) {
    err = "a service is invoked more than once per trace; DES v1 needs a tree-shaped invocation graph";
    return ISIM_EINVAL;
  }
  std::vector<ScriptShape> shape(n);
  std::vector<int32_t> seen(n, -1);
  const uint32_t np = p.stream_nodes;
  out.pos.resize(np);
  std::vector<std::vector<uint32_t>> kids(np);
  std::vector<uint32_t> depth(np, 0);
  std::vector<int32_t> pos_svc(np, -1);
  std::vector<uint32_t> stack;
  for (uint32_t i = 0; i < np; ++i) {
    const Node &nd = p.stream[i];
    const uint32_t slot = nd.meta & 0xFFFFFFu;
    const int32_t svc = slot == kSlotRoot ? p.entry : p.slot_callee[slot];
    if (seen[svc] >= 0) {
      err = "service \"" + g.services[svc].name +
            "\" is invoked more than once per trace; DES v1 needs a tree-shaped invocation graph";
      return ISIM_EINVAL;
    }
    seen[svc] = (int32_t)i;
    shape[svc] = shape_of(g.services[svc]);
    if (!shape[svc].ok) {
      err = "service \"" + g.services[svc].name +
            "\" has more than one step with calls; DES v1 needs every call sent when the script's call step begins";
      return ISIM_EINVAL;
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
    if (ps.parent != kDesNoParent) {
      // calls are sent when the caller's call step begins: its pre-call sleeps after its start
      ps.off = shape[pos_svc[ps.parent]].pre + p.site_hop[p.slot_site[slot]];
      kids[ps.parent].push_back(i);
      depth[i] = depth[ps.parent] + 1;
    }
    if (ps.reps > 1 && !shape[svc].leaf) {
      err = "service \"" + g.services[svc].name +
            "\" has numReplicas > 1 and makes calls; DES v1 keeps callee arrivals in trace order only below "
            "single-replica callers";
      return ISIM_EINVAL;
    }
    if (ps.reps > kDesMaxReplicas) {
      err = "service \"" + g.services[svc].name + "\" has more than 64 replicas (DES v1 limit)";
      return ISIM_EINVAL;
    }
    stack.push_back(i);
    for (uint32_t k = (nd.meta >> 24) & 0x7Fu; k > 0; --k) stack.pop_back();
  }
  for (uint32_t i = 0; i < np; ++i) {
    out.pos[i].child_off = (uint32_t)out.child.size();
    out.pos[i].child_cnt = (uint32_t)kids[i].size();
    out.child.insert(out.child.end(), kids[i].begin(), kids[i].end());
  }
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
  out.slot_mult = p.stream_mult;
  return ISIM_OK;
}

}  // namespace isim
