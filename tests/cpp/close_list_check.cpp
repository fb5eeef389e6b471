// CPU check of the mode-B draw-stream close list (kernel kind 6, walk.hip
// walk_stream_cl; built by program.cpp): for random per-invocation error
// patterns, the chunked test `(bits & rmask) != 0 || last_err1 >= pre1` and
// the leaf counts must give the same per-site 500 counts, per-trace 500
// count and entry status as the direct definition (an invocation responds
// 500 iff an invocation of its subtree erred).  Test infrastructure only.
//   close_list_check <graph.json> <rounds> <error permille>
#include <cstdio>
#include <fstream>
#include <random>
#include <sstream>
#include <vector>

#include "graph.h"
#include "kernel_abi.h"
#include "program.h"

using namespace isim;

int main(int argc, char **argv) {
  if (argc < 4) return 2;
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
  p.error_mode = ISIM_MODE_B;
  Program prog;
  if (compile_program(g, entry, p, prog, err) != ISIM_OK) {
    std::fprintf(stderr, "compile: %s\n", err.c_str());
    return 2;
  }
  if (prog.stream_nodes == 0) {
    std::printf("no draw stream\n");
    return 3;
  }
  const uint32_t n_rec = (uint32_t)prog.stream.size();
  const uint32_t n_slots = (uint32_t)prog.n_slots;
  // direct definition: subtrees from the preorder stream and its close counts
  struct Sub {
    uint32_t pre, end, slot;
  };
  std::vector<Sub> calling;  // calling invocations other than the entry
  std::vector<uint32_t> open;
  for (uint32_t i = 0; i < prog.stream_nodes; ++i) {
    open.push_back(i);
    for (uint32_t k = (prog.stream[i].meta >> 24) & 0x7Fu; k > 0; --k) {
      const uint32_t q = open.back();
      open.pop_back();
      if (q != i && q != 0) calling.push_back({q, i, prog.stream[q].meta & 0xFFFFFFu});
    }
  }
  if (!open.empty()) return 4;
  if (calling.size() != prog.stream_closes.size()) {
    std::fprintf(stderr, "close count %zu != %zu\n", calling.size(), prog.stream_closes.size());
    return 1;
  }
  std::mt19937_64 rng(12345);
  const int rounds = std::atoi(argv[2]);
  const double pe = std::atof(argv[3]) / 1000.0;
  std::bernoulli_distribution draw(pe);
  for (int r = 0; r < rounds; ++r) {
    std::vector<uint8_t> e(n_rec, 0);
    for (uint32_t i = 0; i < prog.stream_nodes; ++i) e[i] = draw(rng) ? 1 : 0;
    // expected
    std::vector<uint64_t> want(n_slots, 0), got(n_slots, 0);
    std::vector<uint32_t> pref(n_rec + 1, 0);
    for (uint32_t i = 0; i < n_rec; ++i) pref[i + 1] = pref[i] + e[i];
    uint32_t want_errh = 0, got_errh = 0;
    for (const Sub &s : calling)
      if (pref[s.end + 1] > pref[s.pre]) {
        ++want[s.slot];
        ++want_errh;
      }
    for (uint32_t i = 0; i < prog.stream_nodes; ++i) {
      const uint32_t meta = prog.stream[i].meta, slot = meta & 0xFFFFFFu;
      if ((meta & 0x7F000000u) && slot < kSlotPad && e[i]) {
        ++want[slot];
        ++want_errh;
      }
    }
    const bool want_root = pref[n_rec] > 0;
    want_errh += want_root ? 1 : 0;
    // the kernel's chunked form
    uint32_t le = 0, cp = 0;
    const uint32_t n_chunks = (n_rec + kChunkRecords - 1) / kChunkRecords;
    for (uint32_t ch = 0; ch < n_chunks; ++ch) {
      const uint32_t cb = ch * kChunkRecords;
      const uint32_t n = std::min(kChunkRecords, n_rec - cb);
      uint32_t mb = 0;
      for (uint32_t i = cb; i < cb + n; ++i) {
        mb = 2 * mb + e[i];
        const uint32_t meta = prog.stream[i].meta, slot = meta & 0xFFFFFFu;
        if ((meta & 0x7F000000u) && slot < kSlotPad && e[i]) {
          ++got[slot];
          ++got_errh;
        }
      }
      for (; cp < prog.stream_close_end[ch]; ++cp) {
        const StreamClose &c = prog.stream_closes[cp];
        if ((mb & c.rmask) != 0 || le >= c.pre1) {
          ++got[prog.stream_close_slot[cp]];
          ++got_errh;
        }
      }
      if (mb) le = cb + n - (uint32_t)__builtin_ctz(mb);
    }
    const bool got_root = le != 0;
    got_errh += got_root ? 1 : 0;
    if (got != want || got_errh != want_errh || got_root != want_root) {
      std::fprintf(stderr, "round %d: mismatch (errh %u vs %u, root %d vs %d)\n", r, got_errh, want_errh,
                   (int)got_root, (int)want_root);
      return 1;
    }
  }
  std::printf("ok %u records, %zu closes, %d rounds\n", prog.stream_nodes, calling.size(), rounds);
  return 0;
}
