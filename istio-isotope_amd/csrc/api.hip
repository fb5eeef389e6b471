// C ABI of libisim (include/isim.h): graph load, handler creation, device
// program upload and the walk launch.  Host code; the kernel is in walk.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/isim.h"
#include "gounits.h"
#include "graph.h"
#include "k8s.h"
#include "marshal.h"
#include "des.h"
#include "kernel_abi.h"
#include "program.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

}  // namespace

namespace isim {
// error reporting of the other C-ABI translation units (multi.hip)
int set_error(int code, const std::string &msg) { return fail(code, msg); }
}  // namespace isim

namespace {

#define HIPCHK(expr)                                                                  \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      return fail(ISIM_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));     \
  } while (0)

struct DevState {
  void *d_prog = nullptr;  // Ins[] (interpreters) or Node[] (draw stream)
  uint32_t *d_mult = nullptr;  // draw stream: per-slot call multiplicity
  isim::StreamClose *d_closes = nullptr;  // mode-B draw stream (kind 6): close list
  uint32_t *d_close_slot = nullptr;       // per close: call-site slot
  uint32_t *d_close_end = nullptr;        // and its per-chunk ends
  uint32_t *d_mark_end = nullptr;         // mode-B draw stream (kind 8): per record its subtree's last record
  uint32_t *d_mark_slot = nullptr;        // and its call-site slot
  uint32_t mark_words = 0;                // kind 8: position marks per workgroup (records + the sentinel)
  uint32_t *d_dur = nullptr;   // dynamic walks: per-slot duration-table word (row | leaf bucket << 24)
  unsigned long long *d_work = nullptr;  // kWorkSlots sets of batch queues, zero between launches
  uint32_t *d_stage = nullptr;  // draw stream: kWorkSlots rows of n_slots u32 500 counts, zero between launches
  // draw-free static walks (no error draw anywhere): every trace walks alike
  bool draw_free = false;
  uint64_t *d_const_stats = nullptr;     // the stats of one trace (computed on first use)
  isim_trace_rec const_rec{};
  uint32_t work_next = 0;                // next queue (launches in flight use distinct queues)
  void *kernel = nullptr;
  uint64_t max_mult = 0;  // largest per-trace count of one per-site counter (calls through a site)
  uint32_t threads = 0;
  uint32_t lds_bytes = 0;
  uint32_t lds_counters = 0;
  uint32_t max_blocks = 0;  // resident workgroups for the whole device
  uint32_t per_cu = 0;
  uint32_t kind = 0;
  // DES (config 5): the plan uploaded on first use
  void *d_des_pos = nullptr;
  uint32_t *d_des_child = nullptr, *d_des_level = nullptr, *d_des_mult = nullptr;
  uint32_t *d_des_fast = nullptr, *d_des_sort = nullptr, *d_des_arr = nullptr, *d_des_zero = nullptr;
  uint32_t *d_des_pipe = nullptr;
  void *d_des_ext = nullptr, *d_des_steps = nullptr;
  // DES item engine (dynamic walks): per-position plan facts, BK rounds, the tree
  void *d_des_ipos = nullptr, *d_des_nodes = nullptr, *d_des_text = nullptr, *d_des_tstep = nullptr;
  uint32_t *d_des_sround = nullptr;
  isim::TreeExt *d_tree_ext = nullptr;  // kind 7: per position (the nodes are d_prog)
  isim::TreeStep *d_tree_step = nullptr;   // kind 7: per position, the rare step facts
  isim::TreeDynRow *d_tree_dyn = nullptr;  // kind 7: the LDS bucket tables' rows
  uint32_t *d_sum_row = nullptr;        // kind 7: per LDS sum index, its row
  uint32_t *d_slot_tc = nullptr;        // kind 7: per slot, the leaf callee's latency
  uint32_t *d_lds_slot = nullptr;       // kind 7, wide tree: per LDS counter its slot
  // kind 7: frames below the register stack, up to kSpillAreas areas (the
  // first allocated with the program, the others when a further stream first
  // needs one)
  uint32_t *d_spill[isim::kSpillAreas] = {};
  uint32_t spill_lanes = 0;
  size_t spill_words = 0;               // u32 words of one area
  hipEvent_t spill_ev[isim::kSpillAreas] = {};     // recorded after each area's latest launch
  hipStream_t spill_last[isim::kSpillAreas] = {};  // the stream of that launch
  bool spill_used[isim::kSpillAreas] = {};
  uint32_t spill_next = 0;
  hipMemPool_t des_pool = nullptr;      // the item engine's per-batch arrays (a private pool)
  bool des_ready = false;               // every DES upload above succeeded (des_prepare)
};

// the DES plan's device copies (des_prepare), freed together; the pool only
// after the device has drained the hipFreeAsync calls queued on user streams
void free_des(DevState &d) {
  for (void **q : {&d.d_des_pos, (void **)&d.d_des_child, (void **)&d.d_des_level, (void **)&d.d_des_arr,
                   &d.d_des_ext, &d.d_des_steps, (void **)&d.d_des_mult, (void **)&d.d_des_fast,
                   (void **)&d.d_des_sort, (void **)&d.d_des_zero, (void **)&d.d_des_pipe, &d.d_des_ipos,
                   (void **)&d.d_des_sround, &d.d_des_nodes, &d.d_des_text, &d.d_des_tstep}) {
    if (*q) (void)hipFree(*q);
    *q = nullptr;
  }
  if (d.des_pool) {
    (void)hipDeviceSynchronize();
    (void)hipMemPoolDestroy(d.des_pool);
    d.des_pool = nullptr;
  }
  d.des_ready = false;
}

void free_dev(DevState &d) {
  free_des(d);
  for (void *q : {(void *)d.d_prog, (void *)d.d_mult, (void *)d.d_closes, (void *)d.d_close_end,
                  (void *)d.d_close_slot, (void *)d.d_mark_end, (void *)d.d_mark_slot, (void *)d.d_dur, (void *)d.d_work, (void *)d.d_stage, (void *)d.d_const_stats,
                  (void *)d.d_tree_ext, (void *)d.d_tree_dyn, (void *)d.d_tree_step,
                  (void *)d.d_sum_row, (void *)d.d_slot_tc, (void *)d.d_lds_slot})
    if (q) (void)hipFree(q);
  for (uint32_t *q : d.d_spill)
    if (q) (void)hipFree(q);
  for (hipEvent_t e : d.spill_ev)
    if (e) (void)hipEventDestroy(e);
  d = DevState();
}

}  // namespace

struct isim_graph {
  isim::ServiceGraph g;
};

struct isim_handler {
  isim::Program prog;
  isim_params params{};
  std::mutex mu;
  std::mutex spill_mu;  // kind 7 spill areas: area choice, wait, launch, record
  std::map<int, DevState> dev;
  // the DES plan is built on first use (des_ensure): it unrolls the whole
  // invocation tree, which walks never need
  isim::ServiceGraph graph;
  std::mutex des_mu;
  bool des_built = false;
  int des_rc = ISIM_OK;
  std::string des_err;
  isim::DesPlan des;
  std::mutex report_mu;
  isim::DesItemsReport des_report{};  // the item engine's last batch (isim_des_last_batch)
  ~isim_handler() {
    for (auto &kv : dev) {
      int cur = 0;
      if (hipGetDevice(&cur) == hipSuccess && hipSetDevice(kv.first) == hipSuccess) {
        free_dev(kv.second);
        (void)hipSetDevice(cur);
      }
    }
  }
};

namespace {

// Kernel kinds 4-6 walk the draw stream (static walks).
bool is_stream(uint32_t kind) { return (kind >= 4 && kind <= 6) || kind == 8; }

// Rows of the device per-service duration table (dynamic walks only).
uint64_t svc_dur_rows(const isim_handler *h) {
  if (h->prog.static_walk || (h->params.flags & ISIM_FLAG_NO_SVC_DUR)) return 0;
  return h->prog.row_svc.size();
}

uint64_t stats_words(const isim_handler *h) {
  return ISIM_ST_SVC_DUR(h->prog.n_slots) + (uint64_t)ISIM_SVC_DUR_WORDS * svc_dur_rows(h);
}

#ifndef ISIM_DYN_MIN_GAIN
#define ISIM_DYN_MIN_GAIN 0  // resident waves a smaller workgroup / global counters must add to be chosen
#endif

// LDS layout of the walk kernel for a given workgroup size (walk.hip).
uint32_t lds_need(const isim::Program &p, uint32_t waves, bool counters) {
  uint32_t b = isim::kLdsAccBytes + isim::kHistWords * 4u;
  if (counters) b += 8u * (uint32_t)p.n_slots;
  b = (b + 15u) & ~15u;
  if (!p.static_walk) {
    uint32_t tt = p.time_bits == 32 ? 4u : 8u;
    b += waves * (uint32_t)p.max_frames * 64u * (2u * tt + 4u);
  }
  return b;
}

int build_device(isim_handler *h, int device, DevState &st);

int prepare_device(isim_handler *h, int device, DevState *&out) {
  std::lock_guard<std::mutex> lk(h->mu);
  auto it = h->dev.find(device);
  if (it != h->dev.end()) {
    out = &it->second;
    return ISIM_OK;
  }
  DevState st;
  const int rc = build_device(h, device, st);
  if (rc != ISIM_OK) {
    free_dev(st);  // one cleanup path for every allocation made before the failure
    return rc;
  }
  auto res = h->dev.emplace(device, st);
  out = &res.first->second;
  return ISIM_OK;
}

// Chooses the kernel and launch shape for `device` and uploads the program.
// On failure the caller frees whatever `st` holds.
int build_device(isim_handler *h, int device, DevState &st) {
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(ISIM_ENODEV, std::string("libisim is built for gfx950 only; device is ") + prop.gcnArchName);
  const isim::Program &p = h->prog;
  // HIP reports 64 KiB per block by default; a gfx950 workgroup may use all
  // 160 KiB of the CU's LDS once the kernel attribute is raised.
  const uint32_t lds_max = (uint32_t)std::max<size_t>(prop.sharedMemPerBlock, prop.maxSharedMemoryPerMultiProcessor);
  // Largest workgroup (waves) whose LDS fits, counters in LDS if possible.
  bool counters = true;
  uint32_t waves = 16;
  while (waves > 1 && lds_need(p, waves, counters) > lds_max) waves >>= 1;
  if (lds_need(p, waves, counters) > lds_max) {
    counters = false;
    waves = 16;
    while (waves > 1 && lds_need(p, waves, counters) > lds_max) waves >>= 1;
    if (lds_need(p, waves, counters) > lds_max)
      return fail(ISIM_EDEPTH, "call stack does not fit in LDS");
  }
  st.threads = waves * 64u;
  st.lds_bytes = lds_need(p, waves, counters);
  st.lds_counters = counters ? 1u : 0u;
  st.kind = p.stream_nodes ? 4u : (p.static_walk ? 0u : 2u) + (p.time_bits == 64 ? 1u : 0u);
  if ((h->params.flags & ISIM_FLAG_NO_STREAM) && st.kind == 4) st.kind = p.time_bits == 64 ? 1u : 0u;
  // mode B on the draw stream: the per-lane bit stack holds 32 stack positions
  // (ISIM_FLAG_BIT_STACK), else the close list (any depth)
  if (st.kind == 4 && h->params.error_mode == ISIM_MODE_B)
    st.kind = (h->params.flags & ISIM_FLAG_BIT_STACK) ? (p.max_depth <= 32 ? 5u : 4u) : 6u;
  // mode B by sparse ancestor marking (kind 8) when its per-position mark
  // table fits the LDS next to the histograms (ISIM_FLAG_CLOSE_LIST: kind 6)
  if (st.kind == 6 && !(h->params.flags & ISIM_FLAG_CLOSE_LIST)) {
    const uint32_t words = p.stream_nodes + 1u;
    const uint32_t need = isim::kLdsAccBytes + isim::kHistWords * 4u + 4u * words;
    if (need <= lds_max) {
      st.kind = 8;
      st.mark_words = words;
      counters = true;
      waves = 16;
      st.threads = waves * 64u;
      st.lds_bytes = need;
      st.lds_counters = 1;
    }
  }
  st.kernel = isim::walk_kernel((int)st.kind, h->params.error_mode == ISIM_MODE_B, counters);
  // dynamic walks: the lane tree walk (kind 7) when the unrolled tree was
  // built and its LDS layout placed (program.cpp place_tree); else the wave walk
  bool tree = false;
  if (!p.static_walk && p.has_tree() && !(h->params.flags & ISIM_FLAG_WAVE_WALK) &&
      p.tree_layout.bytes <= lds_max) {
    tree = true;
    st.kind = 7;
    st.kernel = isim::tree_kernel(h->params.error_mode == ISIM_MODE_B, p.tree_frames,
                                  p.tree_frames > isim::tree_reg_frames(p.tree_frames, p.tree_t64, p.tree_wide),
                                  p.tree_layout.nodes_lds != 0,
                                  (p.tree_flags & isim::kTreeAnyConc) != 0, (p.tree_flags & isim::kTreeAnyDraw) != 0,
                                  p.tree_layout.wg_per_cu == 2, p.tree_t64,
                                  p.tree_wide, p.tree_dag);
    if (!st.kernel) return fail(ISIM_EHIP, "no lane-tree-walk kernel for this tree");
    st.lds_bytes = p.tree_layout.bytes;
    st.lds_counters = 1;
    // the workgroup size with the most resident waves per CU (registers and
    // the LDS layout both bound it: two 768-thread workgroups = 24 waves when
    // the kernel fits 80 VGPRs and the layout half the LDS)
    HIPCHK(hipFuncSetAttribute((const void *)st.kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)st.lds_bytes));
    uint32_t best_t = isim::kWgThreads, best_res = 0;
    for (uint32_t t : {1024u, 768u, 512u}) {
      int pc = 0;
      HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, (const void *)st.kernel, (int)t, st.lds_bytes));
      if ((uint32_t)pc * t / 64u > best_res) {
        best_res = (uint32_t)pc * t / 64u;
        best_t = t;
      }
    }
    st.threads = best_t;
  }
  if (!p.static_walk && !tree) {
    // dynamic walks keep per-lane frame stacks in LDS (waves x frames x 64
    // lanes): the workgroup size with the most resident waves per CU, not the
    // largest that fits
    uint32_t best_w = waves, best_res = 0;
    bool best_c = counters;
    for (int c = counters ? 1 : 0; c >= 0; --c) {
      void *kern = isim::walk_kernel((int)st.kind, h->params.error_mode == ISIM_MODE_B, c != 0);
      for (uint32_t w = 16; w >= 1; w >>= 1) {
        const uint32_t need = lds_need(p, w, c != 0);
        if (need > lds_max) continue;
        HIPCHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)need));
        int pc = 0;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, (const void *)kern, (int)(w * 64u), need));
        const uint32_t res = (uint32_t)pc * w;
        if (res > best_res + ISIM_DYN_MIN_GAIN) {  // the LDS counter table wins ties
          best_res = res;
          best_w = w;
          best_c = c != 0;
        }
      }
    }
    waves = best_w;
    counters = best_c;
    st.kernel = isim::walk_kernel((int)st.kind, h->params.error_mode == ISIM_MODE_B, counters);
    st.threads = waves * 64u;
    st.lds_bytes = lds_need(p, waves, counters);
    st.lds_counters = counters ? 1u : 0u;
  }
  if (is_stream(st.kind)) {
    st.draw_free = true;
    for (const isim::Node &nd : p.stream) st.draw_free = st.draw_free && nd.thr == 0;
  }
  HIPCHK(hipFuncSetAttribute((const void *)st.kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)st.lds_bytes));
  int per_cu = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)st.kernel, (int)st.threads,
                                                      st.lds_bytes));
  if (per_cu < 1) return fail(ISIM_EHIP, "walk kernel cannot be resident (occupancy 0)");
  st.per_cu = (uint32_t)per_cu;
  st.max_blocks = (uint32_t)per_cu * (uint32_t)prop.multiProcessorCount;
  const void *src = st.kind == 8          ? (const void *)p.stream_mark.data()
                    : is_stream(st.kind) ? (const void *)p.stream.data()
                    : tree                ? (p.tree_wide ? (const void *)p.tree_nodes_w.data()
                                                         : (const void *)p.tree_nodes.data())
                                          : (const void *)p.code.data();
  const size_t bytes = is_stream(st.kind) ? p.stream.size() * sizeof(isim::Node)
                       : tree             ? (p.tree_wide ? p.tree_nodes_w.size() * sizeof(isim::TreeNodeW)
                                                         : p.tree_nodes.size() * sizeof(isim::TreeNode))
                                          : p.code.size() * sizeof(isim::Ins);
  // the draw-stream kernel prefetches group g+1 unconditionally: two zero
  // groups (32 B each) of tail padding keep those reads inside the buffer
  const size_t tail = is_stream(st.kind) ? 2 * 4 * sizeof(isim::Node) : 0;
  HIPCHK(hipMalloc(&st.d_prog, bytes + tail));
  HIPCHK(hipMemcpy(st.d_prog, src, bytes, hipMemcpyHostToDevice));
  if (tail) HIPCHK(hipMemset((char *)st.d_prog + bytes, 0, tail));
  if (tree) {
    auto up = [&](auto *&dst, const auto &v) -> int {
      using T = typename std::decay_t<decltype(v)>::value_type;
      HIPCHK(hipMalloc(&dst, std::max<size_t>(1, v.size()) * sizeof(T)));
      if (!v.empty()) HIPCHK(hipMemcpy(dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
      return ISIM_OK;
    };
    if (const int rc = up(st.d_tree_ext, p.tree_ext)) return rc;
    if (const int rc = up(st.d_tree_step, p.tree_step)) return rc;
    if (const int rc = up(st.d_sum_row, p.sum_row)) return rc;
    if (const int rc = up(st.d_slot_tc, p.slot_tc)) return rc;
    if (const int rc = up(st.d_lds_slot, p.tree_lds_slot)) return rc;
    HIPCHK(hipMalloc(&st.d_tree_dyn, std::max<size_t>(1, p.tree_dyn.size()) * sizeof(isim::TreeDynRow)));
    if (!p.tree_dyn.empty())
      HIPCHK(hipMemcpy(st.d_tree_dyn, p.tree_dyn.data(), p.tree_dyn.size() * sizeof(isim::TreeDynRow),
                       hipMemcpyHostToDevice));
    if (p.n_slots > 0) {  // per slot: callee row | static bucket (the kernel's duration flush)
      HIPCHK(hipMalloc(&st.d_dur, p.slot_tbkt.size() * sizeof(uint32_t)));
      HIPCHK(hipMemcpy(st.d_dur, p.slot_tbkt.data(), p.slot_tbkt.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
  }
  if (is_stream(st.kind) && p.n_slots > 0) {
    HIPCHK(hipMalloc(&st.d_mult, p.stream_mult.size() * sizeof(uint32_t)));
    HIPCHK(hipMemcpy(st.d_mult, p.stream_mult.data(), p.stream_mult.size() * sizeof(uint32_t),
                     hipMemcpyHostToDevice));
  }
  if (!tree && svc_dur_rows(h) && p.n_slots > 0) {
    HIPCHK(hipMalloc(&st.d_dur, p.slot_dur.size() * sizeof(uint32_t)));
    HIPCHK(hipMemcpy(st.d_dur, p.slot_dur.data(), p.slot_dur.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  }
  if (st.kind == 6) {
    // zero tail padding: the kernel prefetches blocks of 8 closes past the end
    auto upload = [&](void *&dst, const void *src, size_t bytes, size_t pad) -> int {
      HIPCHK(hipMalloc(&dst, bytes + pad));
      HIPCHK(hipMemset(dst, 0, bytes + pad));
      if (bytes) HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
      return ISIM_OK;
    };
    int rc = upload((void *&)st.d_closes, p.stream_closes.data(), p.stream_closes.size() * sizeof(isim::StreamClose),
                    isim::kClosePad * sizeof(isim::StreamClose));
    if (rc == ISIM_OK)
      rc = upload((void *&)st.d_close_slot, p.stream_close_slot.data(), p.stream_close_slot.size() * sizeof(uint32_t),
                  64 * sizeof(uint32_t));
    if (rc == ISIM_OK)
      rc = upload((void *&)st.d_close_end, p.stream_close_end.data(), p.stream_close_end.size() * sizeof(uint32_t),
                  2 * sizeof(uint32_t));
    if (rc != ISIM_OK) return rc;
  }
  if (st.kind == 8) {
    // the fold's inputs (per real record) and the launches' mark rows
    std::vector<uint32_t> slot(p.stream_nodes);
    for (uint32_t r = 0; r < p.stream_nodes; ++r) slot[r] = p.stream[r].meta & 0xFFFFFFu;
    HIPCHK(hipMalloc(&st.d_mark_end, p.stream_nodes * sizeof(uint32_t)));
    HIPCHK(hipMemcpy(st.d_mark_end, p.stream_end.data(), p.stream_nodes * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&st.d_mark_slot, p.stream_nodes * sizeof(uint32_t)));
    HIPCHK(hipMemcpy(st.d_mark_slot, slot.data(), p.stream_nodes * sizeof(uint32_t), hipMemcpyHostToDevice));
    const size_t bytes = (size_t)isim::kWorkSlots * st.mark_words * sizeof(uint32_t);
    HIPCHK(hipMalloc(&st.d_stage, bytes));
    HIPCHK(hipMemset(st.d_stage, 0, bytes));
    HIPCHK(hipFuncSetAttribute(isim::mark_fold_kernel(), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(st.mark_words * 4u)));
  }
  HIPCHK(hipMalloc(&st.d_work, (size_t)isim::kWorkWords * isim::kWorkSlots * sizeof(unsigned long long)));
  HIPCHK(hipMemset(st.d_work, 0, (size_t)isim::kWorkWords * isim::kWorkSlots * sizeof(unsigned long long)));
  // per-workgroup LDS site counters are u32: launch_walk splits a batch so
  // that no workgroup can count past 2^32 at one site (traces x calls
  // through the site per trace)
  st.max_mult = std::max<uint64_t>(1, p.hops_upper);
  if (tree) {
    st.max_mult = std::max<uint32_t>(1, p.tree_mult);
    const uint32_t regf = isim::tree_reg_frames(p.tree_frames, p.tree_t64, p.tree_wide);
    if (p.tree_frames > regf) {
      // the spill areas: frames below the register frames, one column per
      // lane of a full grid; a launch waits for the area's previous launch
      // (launch_walk_one)
      st.spill_lanes = st.max_blocks * st.threads;
      st.spill_words = (size_t)(p.tree_frames - regf) *
                       ((p.tree_t64 ? isim::kTreeSpillWords64 : isim::kTreeSpillWords) +
                        (p.tree_wide ? isim::kTreeSpillWide : 0u)) *
                       st.spill_lanes;
      HIPCHK(hipMalloc(&st.d_spill[0], st.spill_words * sizeof(uint32_t)));
      for (hipEvent_t &e : st.spill_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
  }
  if (is_stream(st.kind)) {
    st.max_mult = 1;
    for (uint32_t m : p.stream_mult) st.max_mult = std::max<uint64_t>(st.max_mult, m);
    if (st.kind != 8 && st.lds_counters && p.n_slots > 0 && p.n_slots <= isim::kStageMaxSlots) {
      const size_t bytes = (size_t)isim::kWorkSlots * p.n_slots * sizeof(uint32_t);
      HIPCHK(hipMalloc(&st.d_stage, bytes));
      HIPCHK(hipMemset(st.d_stage, 0, bytes));
    }
  }
  return ISIM_OK;
}

}  // namespace

static uint64_t max_launch_traces(const DevState *st);

extern "C" {

const char *isim_last_error(void) { return g_err.c_str(); }
int isim_abi_version(void) { return ISIM_ABI_VERSION; }

int isim_graph_unmarshal_json(const char *json, size_t len, isim_graph **out) {
  if (!json || !out) return fail(ISIM_EINVAL, "null argument");
  isim_graph *g = new (std::nothrow) isim_graph();
  if (!g) return fail(ISIM_ENOMEM, "out of memory");
  std::string err;
  if (!isim::unmarshal_service_graph(json, len, g->g, err)) {
    delete g;
    return fail(ISIM_EPARSE, err);
  }
  *out = g;
  return ISIM_OK;
}

void isim_graph_free(isim_graph *g) { delete g; }

int isim_graph_num_services(const isim_graph *g) { return g ? (int)g->g.services.size() : -1; }

int isim_graph_canonical_json(const isim_graph *g, char *buf, size_t cap, size_t *len) {
  if (!g) return fail(ISIM_EINVAL, "null graph");
  std::string s = isim::canonical_json(g->g);
  if (len) *len = s.size() + 1;
  if (buf && cap) {
    size_t n = std::min(cap - 1, s.size());
    std::memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return ISIM_OK;
}

static int emit(const std::string &s, char *buf, size_t cap, size_t *len) {
  if (len) *len = s.size() + 1;
  if (buf && cap) {
    size_t n = std::min(cap - 1, s.size());
    std::memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return ISIM_OK;
}

int isim_graph_marshal_json(const isim_graph *g, char *buf, size_t cap, size_t *len) {
  if (!g) return fail(ISIM_EINVAL, "null graph");
  return emit(isim::marshal_json(g->g), buf, cap, len);
}

int isim_graph_to_dot(const isim_graph *g, char *buf, size_t cap, size_t *len) {
  if (!g) return fail(ISIM_EINVAL, "null graph");
  return emit(isim::to_dot(g->g), buf, cap, len);
}

int isim_graph_to_k8s_manifests(const isim_graph *g, const isim_k8s_params *p, char *buf, size_t cap, size_t *len) {
  if (!g || !p) return fail(ISIM_EINVAL, "null argument");
  std::string out, err;
  const int rc = isim::k8s_manifests(g->g, *p, out, err);
  if (rc != ISIM_OK) return fail(rc, err);
  return emit(out, buf, cap, len);
}

int isim_graph_marshal_yaml(const isim_graph *g, char *buf, size_t cap, size_t *len) {
  if (!g) return fail(ISIM_EINVAL, "null graph");
  const std::string y = isim::graph_yaml(g->g);
  if (y.empty()) return fail(ISIM_EINVAL, "graph marshal failed");
  return emit(y, buf, cap, len);
}

int isim_graph_service_index(const isim_graph *g, const char *name) {
  if (!g || !name) return -1;
  return isim::service_index(g->g, name);
}

int isim_size_from_string(const char *s, uint64_t *out) {
  if (!s || !out) return fail(ISIM_EINVAL, "null argument");
  std::string err;
  if (!isim::size_from_string(s, *out, err)) return fail(ISIM_EPARSE, err);
  return ISIM_OK;
}

int isim_duration_parse(const char *s, int64_t *out_ns) {
  if (!s || !out_ns) return fail(ISIM_EINVAL, "null argument");
  std::string err;
  if (!isim::go_parse_duration(s, *out_ns, err)) return fail(ISIM_EPARSE, err);
  return ISIM_OK;
}

int isim_percentage_from_string(const char *s, double *out) {
  if (!s || !out) return fail(ISIM_EINVAL, "null argument");
  std::string err;
  if (!isim::pct_from_string(s, *out, err)) return fail(ISIM_EPARSE, err);
  return ISIM_OK;
}

int isim_handler_create(const isim_graph *g, const char *service_name, const isim_params *p,
                        isim_handler **out) {
  if (!g || !p || !out) return fail(ISIM_EINVAL, "null argument");
  int32_t entry = -1;
  if (service_name) {
    entry = isim::service_index(g->g, service_name);
    if (entry < 0) return fail(ISIM_ENOTFOUND, std::string("service with name ") + service_name + " does not exist");
  } else {
    for (size_t i = 0; i < g->g.services.size(); ++i)
      if (g->g.services[i].is_entrypoint) {
        entry = (int32_t)i;
        break;
      }
    if (entry < 0) return fail(ISIM_EINVAL, "no service has isEntrypoint: true");
  }
  isim_handler *h = new (std::nothrow) isim_handler();
  if (!h) return fail(ISIM_ENOMEM, "out of memory");
  h->params = *p;
  std::string err;
  int rc = isim::compile_program(g->g, entry, *p, h->prog, err);
  if (rc == ISIM_OK) h->graph = g->g;  // for the DES plan (des_ensure); the caller may free g
  if (rc != ISIM_OK) {
    delete h;
    return fail(rc, err);
  }
  *out = h;
  return ISIM_OK;
}

void isim_handler_free(isim_handler *h) { delete h; }

int isim_handler_info_get(const isim_handler *h, isim_handler_info *out) {
  if (!h || !out) return fail(ISIM_EINVAL, "null argument");
  const isim::Program &p = h->prog;
  out->n_services = p.n_services;
  out->n_sites = p.n_sites;
  out->n_slots = p.n_slots;
  out->entry = p.entry;
  out->max_depth = p.max_depth;
  out->static_walk = p.static_walk ? 1 : 0;
  out->time_bits = p.time_bits;
  out->program_len = (int32_t)p.code.size();
  out->max_latency_ns = p.max_latency;
  out->hops_upper = p.hops_upper;
  out->stats_words = stats_words(h);
  out->svc_dur_rows = (int32_t)svc_dur_rows(h);
  out->n_reachable = (int32_t)p.row_svc.size();
  out->draw_groups = 0;
  for (size_t g = 0; g + 3 < p.stream.size(); g += 4)
    out->draw_groups += (p.stream[g].thr | p.stream[g + 1].thr | p.stream[g + 2].thr | p.stream[g + 3].thr) != 0;
  return ISIM_OK;
}

int isim_handler_launch_info(isim_handler *h, int device, isim_launch_info *out) {
  if (!h || !out) return fail(ISIM_EINVAL, "null argument");
  int prev = 0;
  HIPCHK(hipGetDevice(&prev));
  HIPCHK(hipSetDevice(device));
  DevState *st = nullptr;
  int rc = prepare_device(h, device, st);
  (void)hipSetDevice(prev);
  if (rc != ISIM_OK) return rc;
  out->wg_threads = (int32_t)st->threads;
  out->lds_bytes = (int32_t)st->lds_bytes;
  out->lds_counters = (int32_t)st->lds_counters;
  out->blocks_per_cu = (int32_t)st->per_cu;
  out->max_blocks = (int32_t)st->max_blocks;
  out->kernel_kind = (int32_t)st->kind;
  out->fill = st->draw_free && !(h->params.flags & ISIM_FLAG_WALK_ALL) ? 1 : 0;
  out->tree_wide = st->kind == 7 && h->prog.tree_wide ? (h->prog.tree_dag ? 2 : 1) : 0;
  out->max_launch_traces = max_launch_traces(st);
  return ISIM_OK;
}

int isim_handler_slots(const isim_handler *h, int32_t *slot_site, int32_t *slot_callee) {
  if (!h) return fail(ISIM_EINVAL, "null handler");
  const isim::Program &p = h->prog;
  if (slot_site) std::copy(p.slot_site.begin(), p.slot_site.end(), slot_site);
  if (slot_callee) std::copy(p.slot_callee.begin(), p.slot_callee.end(), slot_callee);
  return ISIM_OK;
}

static int launch_walk_one(isim_handler *h, DevState *st, uint64_t trace_begin, uint64_t n_traces,
                           isim_trace_rec *d_records, uint64_t *d_stats, void *hip_stream);

// Per-workgroup LDS accumulators are u32: histogram counts (at most the
// launch's traces) and, with LDS site counters, per-site counts (at most
// traces x calls through the site per trace; a workgroup may claim any
// share of a launch's batches).  Launches are split so neither can wrap:
// below 2^31 traces, and below 2^32 / max_mult traces with LDS counters (a
// DAG whose shared callee is reached 2^22 times per trace: 1,023 traces per
// launch).  Global counters are u64 atomics and need no split.
static uint64_t max_launch_traces(const DevState *st) {
  uint64_t m = 1ull << 31;
  if (st->lds_counters) m = std::min<uint64_t>(m, std::max<uint64_t>(1, 0xFFFFFFFFull / st->max_mult));
  return m;
}

static int launch_walk(isim_handler *h, DevState *st, uint64_t trace_begin, uint64_t n_traces,
                       isim_trace_rec *d_records, uint64_t *d_stats, void *hip_stream) {
  const uint64_t kMaxLaunch = max_launch_traces(st);
  for (uint64_t done = 0; done < n_traces;) {
    const uint64_t n = std::min(n_traces - done, kMaxLaunch);
    const int rc = launch_walk_one(h, st, trace_begin + done, n, d_records ? d_records + done : nullptr, d_stats,
                                   hip_stream);
    if (rc != ISIM_OK) return rc;
    done += n;
  }
  return ISIM_OK;
}

static int launch_walk_one(isim_handler *h, DevState *st, uint64_t trace_begin, uint64_t n_traces,
                           isim_trace_rec *d_records, uint64_t *d_stats, void *hip_stream) {
  isim::KParams kp{};
  kp.trace_begin = trace_begin;
  kp.n_traces = n_traces;
  kp.seed_lo = (uint32_t)h->params.seed;
  kp.seed_hi = (uint32_t)(h->params.seed >> 32);
  kp.n_slots = (uint32_t)h->prog.n_slots;
  kp.max_frames = (uint32_t)h->prog.max_frames;
  kp.lds_counters = st->lds_counters;
  kp.n_nodes = h->prog.stream_nodes;
  kp.t_static = h->prog.max_latency;
  kp.svc_dur = svc_dur_rows(h) ? 1u : 0u;
  kp.root_dur = h->prog.root_dur;
  kp.closes = st->d_closes;
  kp.close_slot = st->d_close_slot;
  kp.close_end = st->d_close_end;
  kp.tree_ext = st->d_tree_ext;
  kp.tree_step = st->d_tree_step;
  kp.tree_dyn = st->d_tree_dyn;
  kp.sum_row = st->d_sum_row;
  kp.slot_tc = st->d_slot_tc;
  kp.spill_lanes = st->spill_lanes;
  kp.n_pos = h->prog.tree_positions();
  kp.n_rows = (uint32_t)h->prog.row_svc.size();
  kp.n_dyn = (uint32_t)h->prog.tree_dyn.size();
  kp.dyn_words = h->prog.tree_dyn_words;
  kp.tree_flags = h->prog.tree_flags;
  kp.lay = h->prog.tree_layout;
  kp.lds_slot = st->d_lds_slot;
  kp.n_lds_slots = (uint32_t)h->prog.tree_lds_slot.size();
  const uint64_t per_wave = is_stream(st->kind) ? isim::stream_traces_per_wave() : 64u;
  const uint64_t batches = (n_traces + per_wave - 1) / per_wave;
  const uint64_t waves = st->threads / 64;
  const uint64_t want = (batches + waves - 1) / waves;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(want, st->max_blocks);
  const uint32_t slot = __atomic_fetch_add(&st->work_next, 1u, __ATOMIC_RELAXED) % isim::kWorkSlots;
  kp.work = st->d_work + isim::kWorkWords * slot;
  // u32 staging of the 500 counts: the launch split (launch_walk) keeps n x max_mult below 2^32
  kp.stage = st->d_stage ? st->d_stage + (size_t)slot * (st->kind == 8 ? st->mark_words : h->prog.n_slots) : nullptr;
  kp.mark_words = st->mark_words;
  const void *prog = st->d_prog;
  const uint32_t *dur = st->d_dur;
  void *args[] = {&prog, &d_records, &d_stats, &dur, &kp};
  if (st->d_spill[0]) {
    // a spilling walk: the area its stream used last (else the next one,
    // round robin; allocated on first use), ordered after the area's previous
    // launch by an event; the wait, launch and record are one step under the
    // handler's lock.  Not graph-capturable: a captured launch
    // would keep its area in the graph, and nothing could order its replays
    // against the eager launches that later take the same area.
    const hipStream_t hs = (hipStream_t)hip_stream;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(hs, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone)
      return fail(ISIM_EINVAL, "a lane tree walk that spills frames (more nested calling invocations than its "
                               "register frames) cannot be captured into a HIP graph");
    std::lock_guard<std::mutex> lk(h->spill_mu);
    uint32_t a = isim::kSpillAreas;
    for (uint32_t i = 0; i < isim::kSpillAreas; ++i)
      if (st->spill_used[i] && st->spill_last[i] == hs) a = i;
    if (a == isim::kSpillAreas) a = st->spill_next++ % isim::kSpillAreas;
    if (!st->d_spill[a]) HIPCHK(hipMalloc(&st->d_spill[a], st->spill_words * sizeof(uint32_t)));
    if (st->spill_used[a]) HIPCHK(hipStreamWaitEvent(hs, st->spill_ev[a], 0));
    kp.spill = st->d_spill[a];
    HIPCHK(hipLaunchKernel(st->kernel, dim3(grid), dim3(st->threads), args, st->lds_bytes, hs));
    HIPCHK(hipEventRecord(st->spill_ev[a], hs));
    st->spill_last[a] = hs;
    st->spill_used[a] = true;
  } else {
    HIPCHK(hipLaunchKernel(st->kernel, dim3(grid), dim3(st->threads), args, st->lds_bytes, (hipStream_t)hip_stream));
  }
  if (st->kind == 8) {  // the launch's position marks into the per-site 500 counters
    uint32_t *row = kp.stage;
    uint32_t n = h->prog.stream_nodes, words = st->mark_words, n_slots = (uint32_t)h->prog.n_slots;
    const uint32_t *end = st->d_mark_end, *mslot = st->d_mark_slot;
    void *args3[] = {&row, &n, &words, &end, &mslot, &d_stats, &n_slots};
    HIPCHK(hipLaunchKernel(isim::mark_fold_kernel(), dim3(1), dim3(1024), args3, words * 4u, (hipStream_t)hip_stream));
  }
  if (is_stream(st->kind) && h->prog.n_slots > 0) {
    uint32_t n_slots = (uint32_t)h->prog.n_slots;
    const uint32_t *mult = st->d_mult;
    uint32_t *stage = st->kind == 8 ? nullptr : kp.stage;
    void *args2[] = {&mult, &n_slots, &n_traces, &d_stats, &stage};
    HIPCHK(hipLaunchKernel(isim::stream_calls_kernel(), dim3((n_slots + 255) / 256), dim3(256), args2, 0,
                           (hipStream_t)hip_stream));
  }
  return ISIM_OK;
}

// A draw-free static walk gives every trace the same record and statistics:
// walk ONE trace with the stream kernel (once per device), then a batch is
// a record fill plus n x that trace's statistics (bit-identical by
// construction).
static int prepare_constant(isim_handler *h, DevState *st) {
  std::lock_guard<std::mutex> lk(h->mu);
  if (st->d_const_stats) return ISIM_OK;
  const uint64_t words = stats_words(h);
  uint64_t *d_s1 = nullptr;
  isim_trace_rec *d_r1 = nullptr;
  hipStream_t s = nullptr;
  int rc = ISIM_OK;
  if (hipStreamCreate(&s) != hipSuccess || hipMalloc(&d_s1, words * 8) != hipSuccess ||
      hipMalloc(&d_r1, sizeof(isim_trace_rec)) != hipSuccess || hipMemsetAsync(d_s1, 0, words * 8, s) != hipSuccess)
    rc = fail(ISIM_EHIP, "constant-walk setup failed");
  if (rc == ISIM_OK) rc = launch_walk(h, st, 0, 1, d_r1, d_s1, s);
  if (rc == ISIM_OK && (hipMemcpyAsync(&st->const_rec, d_r1, sizeof(isim_trace_rec), hipMemcpyDeviceToHost, s) !=
                            hipSuccess ||
                        hipStreamSynchronize(s) != hipSuccess))
    rc = fail(ISIM_EHIP, "constant-walk setup failed");
  (void)hipFree(d_r1);
  if (s) (void)hipStreamDestroy(s);
  if (rc != ISIM_OK) {
    (void)hipFree(d_s1);
    return rc;
  }
  st->d_const_stats = d_s1;
  return ISIM_OK;
}

int isim_serve_device(isim_handler *h, uint64_t trace_begin, uint64_t n_traces, isim_trace_rec *d_records,
                      uint64_t *d_stats, void *hip_stream) {
  if (!h || !d_stats) return fail(ISIM_EINVAL, "null argument");
  if (n_traces == 0) return ISIM_OK;
  int device = 0;
  HIPCHK(hipGetDevice(&device));
  DevState *st = nullptr;
  int rc = prepare_device(h, device, st);
  if (rc != ISIM_OK) return rc;
  if (st->draw_free && !(h->params.flags & ISIM_FLAG_WALK_ALL)) {
    rc = prepare_constant(h, st);
    if (rc != ISIM_OK) return rc;
    const uint32_t words = (uint32_t)stats_words(h);
    uint64_t blocks = (n_traces + 1023) / 1024;
    blocks = std::max<uint64_t>(1, std::min<uint64_t>(blocks, 8192));
    const isim_trace_rec r = st->const_rec;
    const uint64_t *s1 = st->d_const_stats;
    void *args[] = {&d_records, &n_traces, (void *)&r, &s1, &d_stats, (void *)&words};
    HIPCHK(hipLaunchKernel(isim::fill_const_kernel(), dim3((uint32_t)blocks), dim3(256), args, 0,
                           (hipStream_t)hip_stream));
    return ISIM_OK;
  }
  return launch_walk(h, st, trace_begin, n_traces, d_records, d_stats, hip_stream);
}

int isim_serve(isim_handler *h, int device, uint64_t trace_begin, uint64_t n_traces, isim_trace_rec *h_records,
               uint64_t *h_stats) {
  if (!h) return fail(ISIM_EINVAL, "null handler");
  int prev = 0;
  HIPCHK(hipGetDevice(&prev));
  HIPCHK(hipSetDevice(device));
  const uint64_t words = stats_words(h);
  uint64_t *d_stats = nullptr;
  isim_trace_rec *d_rec = nullptr;
  int rc = ISIM_OK;
  hipStream_t s = nullptr;
  do {
    if (hipStreamCreate(&s) != hipSuccess) { rc = fail(ISIM_EHIP, "hipStreamCreate failed"); break; }
    if (hipMalloc(&d_stats, words * 8) != hipSuccess) { rc = fail(ISIM_EHIP, "hipMalloc(stats) failed"); break; }
    if (hipMemsetAsync(d_stats, 0, words * 8, s) != hipSuccess) { rc = fail(ISIM_EHIP, "hipMemset failed"); break; }
    if (h_records && n_traces) {
      if (hipMalloc(&d_rec, n_traces * sizeof(isim_trace_rec)) != hipSuccess) {
        rc = fail(ISIM_EHIP, "hipMalloc(records) failed");
        break;
      }
    }
    rc = isim_serve_device(h, trace_begin, n_traces, d_rec, d_stats, s);
    if (rc != ISIM_OK) break;
    if (const hipError_t e = hipStreamSynchronize(s); e != hipSuccess) {
      rc = fail(ISIM_EHIP, std::string("walk kernel failed: ") + hipGetErrorName(e) + ": " + hipGetErrorString(e));
      break;
    }
    if (h_stats && hipMemcpy(h_stats, d_stats, words * 8, hipMemcpyDeviceToHost) != hipSuccess) {
      rc = fail(ISIM_EHIP, "copy stats failed");
      break;
    }
    if (h_records && d_rec &&
        hipMemcpy(h_records, d_rec, n_traces * sizeof(isim_trace_rec), hipMemcpyDeviceToHost) != hipSuccess) {
      rc = fail(ISIM_EHIP, "copy records failed");
      break;
    }
  } while (0);
  if (d_rec) (void)hipFree(d_rec);
  if (d_stats) (void)hipFree(d_stats);
  if (s) (void)hipStreamDestroy(s);
  (void)hipSetDevice(prev);
  return rc;
}

int isim_stats_fold(const isim_handler *h, const uint64_t *stats, uint64_t *svc_calls, uint64_t *svc_errs,
                    uint64_t *site_calls) {
  if (!h || !stats) return fail(ISIM_EINVAL, "null argument");
  const isim::Program &p = h->prog;
  if (svc_calls) std::fill(svc_calls, svc_calls + p.n_services, 0);
  if (svc_errs) std::fill(svc_errs, svc_errs + p.n_services, 0);
  if (site_calls) std::fill(site_calls, site_calls + p.n_sites, 0);
  const uint64_t *calls = stats + ISIM_ST_SITES;
  const uint64_t *errs = calls + p.n_slots;
  for (int32_t s = 0; s < p.n_slots; ++s) {
    if (svc_calls) svc_calls[p.slot_callee[s]] += calls[s];
    if (svc_errs) svc_errs[p.slot_callee[s]] += errs[s];
    if (site_calls) site_calls[p.slot_site[s]] += calls[s];
  }
  // the client request into the entry is not a call site
  if (svc_calls) svc_calls[p.entry] += stats[ISIM_ST_N_TRACES];
  if (svc_errs) svc_errs[p.entry] += stats[ISIM_ST_N_500];
  return ISIM_OK;
}

int isim_stats_fold_durations(const isim_handler *h, const uint64_t *stats, uint64_t *svc_dur) {
  if (!h || !stats || !svc_dur) return fail(ISIM_EINVAL, "null argument");
  const isim::Program &p = h->prog;
  constexpr uint32_t W = ISIM_SVC_DUR_WORDS;
  std::fill(svc_dur, svc_dur + (size_t)p.n_services * W, 0);
  if (!p.static_walk) {
    if (!svc_dur_rows(h)) return fail(ISIM_EINVAL, "per-service durations disabled (ISIM_FLAG_NO_SVC_DUR)");
    const uint64_t *tab = stats + ISIM_ST_SVC_DUR(p.n_slots);
    for (size_t r = 0; r < p.row_svc.size(); ++r)
      std::copy(tab + r * W, tab + (r + 1) * W, svc_dur + (size_t)p.row_svc[r] * W);
    return ISIM_OK;
  }
  // static walk: every invocation of s lasts T(s); split by code with the counters
  std::vector<uint64_t> calls(p.n_services, 0), errs(p.n_services, 0);
  isim_stats_fold(h, stats, calls.data(), errs.data(), nullptr);
  for (int32_t s : p.row_svc) {
    const uint64_t T = p.svc_time[s];
    const uint32_t b = isim::prom_bucket_ns(T);
    uint64_t *row = svc_dur + (size_t)s * W;
    row[b] = calls[s] - errs[s];
    row[ISIM_N_PROM + b] = errs[s];
    row[2 * ISIM_N_PROM] = T * (calls[s] - errs[s]);
    row[2 * ISIM_N_PROM + 1] = T * errs[s];
  }
  return ISIM_OK;
}

}  // extern "C"

// ---- DES (BASELINE config 5) --------------------------------
namespace {

// Builds the DES plan on first use (host only); ISIM_OK or the reason the
// graph is outside the DES class.
int des_ensure(const isim_handler *hc) {
  isim_handler *h = const_cast<isim_handler *>(hc);
  std::lock_guard<std::mutex> lk(h->des_mu);
  if (!h->des_built) {
    h->des_rc = isim::build_des_plan(h->graph, h->prog, h->params.error_mode == ISIM_MODE_B, h->des, h->des_err);
    h->des_built = true;
  }
  return h->des_rc == ISIM_OK ? ISIM_OK : fail(h->des_rc, h->des_err);
}

int des_prepare(isim_handler *h, int device, DevState *&st) {
  int rc = des_ensure(h);
  if (rc != ISIM_OK) return rc;
  rc = prepare_device(h, device, st);
  if (rc != ISIM_OK) return rc;
  std::lock_guard<std::mutex> lk(h->mu);
  if (st->des_ready) return ISIM_OK;
  free_des(*st);  // the remains of an earlier attempt that failed part-way
  const isim::DesPlan &d = h->des;
  auto up = [&](void **dst, const void *src, size_t bytes) -> bool {
    if (hipMalloc(dst, bytes ? bytes : 8) != hipSuccess) return false;
    return !bytes || hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
  };
  if (!up(&st->d_des_pos, d.pos.data(), d.pos.size() * sizeof(isim::DesPos)) ||
      !up((void **)&st->d_des_child, d.child.data(), d.child.size() * 4) ||
      !up((void **)&st->d_des_level, d.fin_pos.data(), d.fin_pos.size() * 4) ||
      !up((void **)&st->d_des_arr, d.arr_ops.data(), d.arr_ops.size() * 4) ||
      !up(&st->d_des_ext, d.ext.data(), d.ext.size() * sizeof(isim::DesPosExt)) ||
      !up(&st->d_des_steps, d.steps.data(), d.steps.size() * sizeof(isim::DesStep)) ||
      !up((void **)&st->d_des_mult, d.slot_mult.data(), d.slot_mult.size() * 4) ||
      !up((void **)&st->d_des_fast, d.fast_pos.data(), d.fast_pos.size() * 4) ||
      !up((void **)&st->d_des_sort, d.sort_pos.data(), d.sort_pos.size() * 4) ||
      !up((void **)&st->d_des_zero, d.zero_pos.data(), d.zero_pos.size() * 4)) {
    free_des(*st);
    return fail(ISIM_EHIP, "DES plan upload failed");
  }
  std::vector<uint32_t> pipe(d.pipe_pos);
  pipe.insert(pipe.end(), d.pipe_dep.begin(), d.pipe_dep.end());
  if (!up((void **)&st->d_des_pipe, pipe.data(), pipe.size() * 4)) {
    free_des(*st);
    return fail(ISIM_EHIP, "DES plan upload failed");
  }
  if (d.items) {
    const isim::Program &p = h->prog;
    // the per-batch item arrays come from a pool of this handler's own (kept
    // between batches: a release threshold of ~0 on a pool nobody else uses)
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = device;
    uint64_t keep = ~0ull;
    if (hipMemPoolCreate(&st->des_pool, &props) != hipSuccess ||
        hipMemPoolSetAttribute(st->des_pool, hipMemPoolAttrReleaseThreshold, &keep) != hipSuccess) {
      free_des(*st);
      return fail(ISIM_EHIP, "DES item pool creation failed");
    }
    if (!up(&st->d_des_ipos, d.item_pos.data(), d.item_pos.size() * sizeof(isim::DesItemPos)) ||
        !up((void **)&st->d_des_sround, d.step_round.data(), d.step_round.size() * 4) ||
        !(p.tree_wide ? up(&st->d_des_nodes, p.tree_nodes_w.data(), p.tree_nodes_w.size() * sizeof(isim::TreeNodeW))
                      : up(&st->d_des_nodes, p.tree_nodes.data(), p.tree_nodes.size() * sizeof(isim::TreeNode))) ||
        !up(&st->d_des_text, p.tree_ext.data(), p.tree_ext.size() * sizeof(isim::TreeExt)) ||
        !up(&st->d_des_tstep, p.tree_step.data(), p.tree_step.size() * sizeof(isim::TreeStep))) {
      free_des(*st);
      return fail(ISIM_EHIP, "DES plan upload failed");
    }
  }
  st->des_ready = true;
  return ISIM_OK;
}

}  // namespace

extern "C" {

int isim_des_info_get(const isim_handler *h, isim_des_info *out) {
  if (!h || !out) return fail(ISIM_EINVAL, "null argument");
  std::memset(out, 0, sizeof(*out));
  if (const int drc = des_ensure(h)) return drc;
  out->n_positions = (int32_t)h->des.pos.size();
  out->n_levels = (int32_t)h->des.n_levels;
  out->max_width = (int32_t)h->des.max_width;
  out->table_rows = (int32_t)h->prog.row_svc.size();
  for (const auto &q : h->des.pos) out->n_fused += (q.flags & isim::kDesFlagFused) ? 1 : 0;
  out->cyclic = h->des.cyclic ? 1 : 0;
  uint32_t rr = 0, rw = 0;
  isim::des_row_traffic(h->des, rr, rw);
  out->row_reads = (int32_t)rr;
  out->row_writes = (int32_t)rw;
  out->items = h->des.items ? 1 : 0;
  return ISIM_OK;
}

int isim_des_last_batch(const isim_handler *h, isim_des_batch_stats *out) {
  if (!h || !out) return fail(ISIM_EINVAL, "null argument");
  isim_handler *hm = const_cast<isim_handler *>(h);
  std::lock_guard<std::mutex> lk(hm->report_mu);
  out->passes = h->des_report.passes;
  out->syncs = h->des_report.syncs;
  out->items = h->des_report.items;
  return ISIM_OK;
}

int isim_des_workspace_bytes(const isim_handler *h, uint64_t n_traces, uint64_t *bytes) {
  if (!h || !bytes) return fail(ISIM_EINVAL, "null argument");
  if (const int drc = des_ensure(h)) return drc;
  *bytes = h->des.items ? isim::des_items_workspace_bytes(n_traces)
                        : isim::des_workspace_bytes(h->des, n_traces, stats_words(h), h->prog.row_svc.size());
  return ISIM_OK;
}

int isim_serve_des_device(isim_handler *h, const isim_des_params *dp, uint64_t trace_begin, uint64_t n_traces,
                          isim_trace_rec *d_records, uint64_t *d_stats, uint64_t *d_des_table, void *d_workspace,
                          uint64_t workspace_bytes, void *hip_stream) {
  if (!h || !dp || !d_stats || !d_des_table) return fail(ISIM_EINVAL, "null argument");
  if (dp->mean_interarrival_ns == 0 || dp->mean_interarrival_ns > (1ull << 34))
    return fail(ISIM_EINVAL, "mean_interarrival_ns must be in [1, 2^34]");
  if (dp->reserved != 0 || (dp->flags & ~ISIM_DES_FLAG_WIDE) != 0)
    return fail(ISIM_EINVAL, "isim_des_params.flags must be 0 or ISIM_DES_FLAG_WIDE, reserved 0");
  if (n_traces == 0) return ISIM_OK;
  if (n_traces > (1ull << 31)) return fail(ISIM_EINVAL, "n_traces above 2^31 per DES batch");
  int device = 0;
  HIPCHK(hipGetDevice(&device));
  DevState *st = nullptr;
  int rc = des_prepare(h, device, st);
  if (rc != ISIM_OK) return rc;
  const isim::DesPlan &d = h->des;
  if (d.items) {
    // a dynamic walk: the item engine (des_items.hip); 64-bit times throughout
    if (!d_workspace || workspace_bytes < isim::des_items_workspace_bytes(n_traces))
      return fail(ISIM_EINVAL, "DES workspace smaller than isim_des_workspace_bytes()");
    isim::DesItemsLaunch L{};
    L.plan = &d;
    L.d_pos = st->d_des_pos;
    L.d_item_pos = st->d_des_ipos;
    L.d_steps = st->d_des_steps;
    L.d_step_round = st->d_des_sround;
    L.d_nodes = st->d_des_nodes;
    L.d_ext = st->d_des_text;
    L.d_tstep = st->d_des_tstep;
    L.tree_frames = h->prog.tree_frames;
    L.tree_t64 = h->prog.tree_t64 ? 1u : 0u;
    L.tree_flags = h->prog.tree_flags;
    L.n_nodes = h->prog.tree_positions();
    L.tree_wide = h->prog.tree_wide ? 1u : 0u;
    L.workspace = d_workspace;
    L.d_stats = d_stats;
    L.d_table = d_des_table;
    L.d_records = d_records;
    L.n_traces = n_traces;
    L.trace_begin = trace_begin;
    L.mean_ns = dp->mean_interarrival_ns;
    L.seed = h->params.seed;
    L.n_slots = (uint32_t)h->prog.n_slots;
    L.flags = h->params.flags;
    L.pool = st->des_pool;
    isim::DesItemsReport rep{};
    L.report = &rep;
    std::string e;
    const int irc = isim::des_items_launch(L, hip_stream, e);
    {
      std::lock_guard<std::mutex> lk(h->report_mu);
      h->des_report = rep;
    }
    if (irc == 2) return fail(ISIM_EINVAL, e);
    if (irc) return fail(ISIM_EHIP, e);
    return ISIM_OK;
  }
  if (n_traces * (uint64_t)std::max<uint32_t>(1, d.max_sort_pos) > 0xFFFFFFFFull)
    return fail(ISIM_EINVAL, "n_traces x positions of one service above 2^32 per DES batch");
  // the queue scans' keys a_t - t * hold are signed 64-bit (des.hip down passes)
  if ((long double)n_traces * (long double)d.max_hold +
          (long double)n_traces * dp->mean_interarrival_ns * 17.0L >= std::ldexp(1.0L, 62))
    return fail(ISIM_EINVAL, "DES batch too long for its worker hold times (n_traces x hold above 2^62 ns)");
  if (d.max_rep_bits) {
    // sort keys hold replica | arrival: the batch's arrival span (an exponential
    // gap is at most 24 ln 2 = 16.6 means) plus the static latency must fit
    const long double span = (long double)n_traces * dp->mean_interarrival_ns * 17.0L +
                             (long double)h->prog.max_latency;
    if (span >= std::ldexp(1.0L, 64 - (int)d.max_rep_bits - 1))
      return fail(ISIM_EINVAL, "DES batch too long for the sort keys of a replicated service (arrival span)");
  }
  const uint64_t words = stats_words(h);
  const uint32_t rows = (uint32_t)h->prog.row_svc.size();
  if (!d_workspace || workspace_bytes < isim::des_workspace_bytes(d, n_traces, words, rows))
    return fail(ISIM_EINVAL, "DES workspace smaller than isim_des_workspace_bytes()");
  isim::DesLaunch L{};
  L.plan = &d;
  L.d_pos = st->d_des_pos;
  L.d_ext = st->d_des_ext;
  L.d_steps = st->d_des_steps;
  L.d_child = st->d_des_child;
  L.d_fin_pos = st->d_des_level;
  L.d_arr_ops = st->d_des_arr;
  L.d_fast_pos = st->d_des_fast;
  L.d_zero_pos = st->d_des_zero;
  L.d_pipe = st->d_des_pipe;
  L.d_sort_pos = st->d_des_sort;
  L.d_mult = st->d_des_mult;
  L.d_stats = d_stats;
  L.d_table = d_des_table;
  L.d_records = d_records;
  L.n_traces = n_traces;
  L.trace_begin = trace_begin;
  L.mean_ns = dp->mean_interarrival_ns;
  L.seed = h->params.seed;
  L.stats_words = words;
  L.table_rows = rows;
  L.n_pos = (uint32_t)d.pos.size();
  L.n_slots = (uint32_t)h->prog.n_slots;
  L.modeb = h->params.error_mode == ISIM_MODE_B ? 1u : 0u;
  L.wide = (dp->flags & ISIM_DES_FLAG_WIDE) != 0;
  isim::des_carve(L, d_workspace);
  if (isim::des_launch(L, hip_stream) != 0) return fail(ISIM_EHIP, "DES kernel launch failed");
  return ISIM_OK;
}

int isim_serve_des(isim_handler *h, int device, const isim_des_params *dp, uint64_t trace_begin, uint64_t n_traces,
                   isim_trace_rec *h_records, uint64_t *h_stats, uint64_t *h_des_table) {
  if (!h || !dp) return fail(ISIM_EINVAL, "null argument");
  if (const int drc = des_ensure(h)) return drc;
  int prev = 0;
  HIPCHK(hipGetDevice(&prev));
  HIPCHK(hipSetDevice(device));
  const uint64_t words = stats_words(h);
  const uint64_t tab_words = (uint64_t)h->prog.row_svc.size() * ISIM_DES_ROW_WORDS;
  const uint64_t ws_bytes = h->des.items ? isim::des_items_workspace_bytes(n_traces)
                                         : isim::des_workspace_bytes(h->des, n_traces, words, h->prog.row_svc.size());
  uint64_t *d_stats = nullptr, *d_tab = nullptr;
  void *d_ws = nullptr;
  isim_trace_rec *d_rec = nullptr;
  hipStream_t s = nullptr;
  int rc = ISIM_OK;
  do {
    if (hipStreamCreate(&s) != hipSuccess) { rc = fail(ISIM_EHIP, "hipStreamCreate failed"); break; }
    if (hipMalloc(&d_stats, words * 8) != hipSuccess || hipMalloc(&d_tab, tab_words * 8 + 8) != hipSuccess ||
        hipMalloc(&d_ws, ws_bytes + 8) != hipSuccess) {
      rc = fail(ISIM_EHIP, "hipMalloc(DES buffers) failed");
      break;
    }
    if (h_records && n_traces && hipMalloc(&d_rec, n_traces * sizeof(isim_trace_rec)) != hipSuccess) {
      rc = fail(ISIM_EHIP, "hipMalloc(records) failed");
      break;
    }
    // 32-bit rows first; a batch they cannot hold (ISIM_ST_DES_RETRY) again with 64-bit rows
    isim_des_params p = *dp;
    for (int pass = 0; pass < 2; ++pass) {
      if (hipMemsetAsync(d_stats, 0, words * 8, s) != hipSuccess ||
          hipMemsetAsync(d_tab, 0, tab_words * 8 + 8, s) != hipSuccess) {
        rc = fail(ISIM_EHIP, "hipMemset failed");
        break;
      }
      rc = isim_serve_des_device(h, &p, trace_begin, n_traces, d_rec, d_stats, d_tab, d_ws, ws_bytes + 8, s);
      if (rc != ISIM_OK) break;
      uint64_t retry = 0;
      if (hipMemcpyAsync(&retry, d_stats + ISIM_ST_DES_RETRY, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess) {
        rc = fail(ISIM_EHIP, "DES retry check failed");
        break;
      }
      if (!retry) break;
      if (retry >= isim::kDesFaultUnit) {
        rc = fail(ISIM_EHIP, "DES batch failed: a queue pass's look-back gave up waiting for an earlier chunk "
                             "(device fault flag); the batch was not accumulated");
        break;
      }
      if ((p.flags & ISIM_DES_FLAG_WIDE) || h->des.items) {
        rc = fail(ISIM_EINVAL, "DES batch not accumulated with 64-bit rows: the cyclic schedule found no fixed point "
                               "within 256 passes (or arrivals beyond the sort keys)");
        break;
      }
      p.flags |= ISIM_DES_FLAG_WIDE;
    }
    if (rc != ISIM_OK) break;
    if (h_stats && hipMemcpyAsync(h_stats, d_stats, words * 8, hipMemcpyDeviceToHost, s) != hipSuccess) {
      rc = fail(ISIM_EHIP, "copy stats failed");
      break;
    }
    if (h_des_table && tab_words &&
        hipMemcpyAsync(h_des_table, d_tab, tab_words * 8, hipMemcpyDeviceToHost, s) != hipSuccess) {
      rc = fail(ISIM_EHIP, "copy DES table failed");
      break;
    }
    if (d_rec && hipMemcpyAsync(h_records, d_rec, n_traces * sizeof(isim_trace_rec), hipMemcpyDeviceToHost, s) !=
                     hipSuccess) {
      rc = fail(ISIM_EHIP, "copy records failed");
      break;
    }
    if (hipStreamSynchronize(s) != hipSuccess) rc = fail(ISIM_EHIP, "hipStreamSynchronize failed");
  } while (0);
  (void)hipFree(d_rec);
  (void)hipFree(d_ws);
  (void)hipFree(d_tab);
  (void)hipFree(d_stats);
  if (s) (void)hipStreamDestroy(s);
  (void)hipSetDevice(prev);
  return rc;
}

void isim_debug_set_spin_limit(uint32_t polls) { isim::des_set_spin_limit(polls); }

uint32_t isim_debug_spin_limit(void) { return isim::des_spin_limit(); }

int isim_des_fold(const isim_handler *h, const uint64_t *des_table, uint64_t *svc_rows) {
  if (!h || !des_table || !svc_rows) return fail(ISIM_EINVAL, "null argument");
  const isim::Program &p = h->prog;
  constexpr uint32_t W = ISIM_DES_ROW_WORDS;
  std::fill(svc_rows, svc_rows + (size_t)p.n_services * W, 0);
  for (size_t r = 0; r < p.row_svc.size(); ++r)
    std::copy(des_table + r * W, des_table + (r + 1) * W, svc_rows + (size_t)p.row_svc[r] * W);
  return ISIM_OK;
}

}  // extern "C"
