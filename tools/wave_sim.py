"""Lock-step wave simulation of the lane tree walk (kernel kind 7) on the CPU.

Runs tree_walk.h's Lane::step for 64 lanes in lock step, refilling a lane with
the next trace as soon as its trace responds (tree.hip), and counts what a
wave executes: wave steps per 64 traces, and for each code site (the Philox
draws, the close, leaf / open / skip) the share of wave steps in which ANY lane runs it — a divergent wave
issues a site's instructions whenever one of its lanes needs it — against
the share of lane-steps that use it.  This is how round 6's step changes were
sized (the close at the start of a step dropped, a one-Philox-
block step measured and dropped).  Analysis tool only: it compiles an
instrumented COPY of tree_walk.h in a temporary directory.

    python tools/wave_sim.py --config c3p [--traces 20000] [-D TW_SCAN=2]
"""
import argparse
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "istio-isotope_amd", "csrc")

# (anchor in tree_walk.h, replacement) — each marks a site in tw_mask
PATCHES = [
    ("namespace tw {\n", "namespace tw {\nextern unsigned tw_mask;\n"),
    ("        f_res = residues(cur_hop(), kb, k0, k1);", "        tw_mask |= 1u;\n        f_res = residues(cur_hop(), kb, k0, k1);"),
    ("    if (b != ek_blk) {\n", "    if (b != ek_blk) {\n      tw_mask |= 2u;\n"),
    ("    f_res = pk ? residues(hop, 0, k0, k1) : 0u;", "    if (pk) tw_mask |= 4u;\n    f_res = pk ? residues(hop, 0, k0, k1) : 0u;"),
    ("    if (!done && p >= end) close(nodes, ext, sink);",
     "    if (!done && p >= end) { tw_mask |= 8u; close(nodes, ext, sink); }"),
    ("    if (fl & TF_LEAF) {\n      const TreeExt x", "    if (fl & TF_LEAF) {\n      tw_mask |= 16u;\n      const TreeExt x"),
    ("    if (!entry) push();", "    tw_mask |= 32u;\n    if (!entry) push();"),
    ("      if (skipped(n)) {\n", "      if (skipped(n)) {\n        tw_mask |= 64u;\n"),
]
SITES = ["res_kb", "err_blk", "res_open", "close", "leaf", "open", "skip"]

MAIN = r'''
namespace isim { namespace tw { unsigned tw_mask = 0; } }
template <class L, class Nodes>
void sim(std::vector<L> &lanes, const Nodes &nodes, const Program &prog, Sink &sk, uint64_t n, uint32_t k0,
         uint32_t k1) {
  uint64_t next = 0, wave_steps = 0, lane_steps = 0, site_w[7] = {0}, site_l[7] = {0};
  std::vector<bool> act(64, false);
  while (true) {
    for (int l = 0; l < 64; ++l)
      if (!act[l] && next < n) { lanes[l].start(next++); act[l] = true; }
    bool any = false;
    unsigned um = 0;
    for (int l = 0; l < 64; ++l) {
      if (!act[l]) continue;
      any = true;
      tw::tw_mask = 0;
      lanes[l].step(nodes, prog.tree_ext.data(), prog.tree_step.data(), sk, k0, k1);
      ++lane_steps;
      for (int b = 0; b < 7; ++b) if (tw::tw_mask >> b & 1) site_l[b]++;
      um |= tw::tw_mask;
      if (lanes[l].done) act[l] = false;
    }
    if (!any) break;
    ++wave_steps;
    for (int b = 0; b < 7; ++b) if (um >> b & 1) site_w[b]++;
  }
  std::printf("traces %llu wave_steps_per_64 %.3f lane_util %.4f\n", (unsigned long long)n, wave_steps * 64.0 / n,
              lane_steps / (64.0 * wave_steps));
  for (int b = 0; b < 7; ++b)
    std::printf("site %d wave %.4f lane %.4f\n", b, site_w[b] / (double)wave_steps, site_l[b] / (double)lane_steps);
}

int main(int argc, char **argv) {
  std::ifstream f(argv[1]);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string js = ss.str();
  ServiceGraph g;
  std::string err;
  if (!unmarshal_service_graph(js.data(), js.size(), g, err)) return 2;
  int32_t entry = -1;
  for (size_t i = 0; i < g.services.size() && entry < 0; ++i)
    if (g.services[i].is_entrypoint) entry = (int32_t)i;
  isim_params p{};
  p.error_mode = (uint32_t)std::atoi(argv[2]);
  p.seed = 0x15070BE;
  p.hop_base_ns = 250000;
  p.req_ps_per_byte = 80;
  p.resp_ps_per_byte = 80;
  p.flags = ISIM_FLAG_DYNAMIC;
  const uint64_t n = std::strtoull(argv[3], nullptr, 0);
  Program prog;
  if (compile_program(g, entry, p, prog, err) != ISIM_OK || !prog.has_tree()) return 3;
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
  std::vector<uint32_t> spill((size_t)kTreeMaxFrames * 12 * 64, 0);
  const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
  const bool draw = (prog.tree_flags & kTreeAnyDraw) != 0;
  std::printf("positions %u frames %u wide %d t64 %d draw %d\n", prog.tree_positions(), prog.tree_frames,
              prog.tree_wide ? 1 : 0, prog.tree_t64 ? 1 : 0, draw ? 1 : 0);
  auto go = [&](auto &L, const auto &nodes) {
    for (int l = 0; l < 64; ++l) {
      L[l].sp = spill.data() + l;
      L[l].sp_stride = 64;
    }
    sim(L, nodes, prog, sk, n, k0, k1);
  };
  // the kernel's variants (tree.hip tree_pick), spilling frames everywhere (same walk, same steps)
  if (prog.tree_wide) {
    if (draw) { std::vector<tw::Lane<6, false, true, true, true, uint32_t, true>> L(64); go(L, tw::CpuNodesW{prog.tree_nodes_w.data()}); }
    else { std::vector<tw::Lane<6, false, true, true, false, uint32_t, true>> L(64); go(L, tw::CpuNodesW{prog.tree_nodes_w.data()}); }
  } else if (draw) {
    std::vector<tw::Lane<8, false, true, true, true>> L(64);
    go(L, tw::CpuNodes{prog.tree_nodes.data()});
  } else {
    std::vector<tw::Lane<8, false, true, true, false>> L(64);
    go(L, tw::CpuNodes{prog.tree_nodes.data()});
  }
  return 0;
}
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3p", help="a bench.py config (its graph), or a graph JSON path")
    ap.add_argument("--traces", type=int, default=20000)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("-D", action="append", default=[], help="a compile-time define (e.g. TW_SCAN=2)")
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="wave_sim_")
    hdr = open(os.path.join(CSRC, "tree_walk.h")).read()
    for old, new in PATCHES:
        if hdr.count(old) != 1:
            sys.exit(f"tree_walk.h changed: anchor not found once: {old[:50]!r}")
        hdr = hdr.replace(old, new)
    open(os.path.join(tmp, "tree_walk.h"), "w").write(hdr)
    chk = open(os.path.join(ROOT, "tests", "cpp", "tree_walk_check.cpp")).read()
    open(os.path.join(tmp, "wave_sim.cpp"), "w").write(chk[:chk.index("int main(")] + MAIN)
    exe = os.path.join(tmp, "wave_sim")
    srcs = [os.path.join(tmp, "wave_sim.cpp")] + [os.path.join(CSRC, f) for f in
                                                   ("json.cpp", "gounits.cpp", "graph.cpp", "program.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O2", *[f"-D{d}" for d in a.D], "-I", tmp, "-I",
                    os.path.join(ROOT, "include"), "-I", CSRC, *srcs, "-o", exe], check=True)
    path = a.config
    if not os.path.exists(path):
        sys.path[:0] = [ROOT, os.path.join(ROOT, "istio-isotope_amd")]
        import bench
        g = bench.build_graph(a.config)
        path = os.path.join(tmp, "g.json")
        open(path, "w").write(g if isinstance(g, str) else g[0])
    out = subprocess.run([exe, path, str(a.mode), str(a.traces)], capture_output=True, text=True, check=True).stdout
    for line in out.splitlines():
        f = line.split()
        if f[0] == "site":
            print(f"  {SITES[int(f[1])]:<11} wave steps {float(f[3]):.3f}  lane-steps {float(f[5]):.3f}")
        else:
            print(line)


if __name__ == "__main__":
    main()
