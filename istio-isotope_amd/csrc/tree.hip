// isim_tree — kernel kind 7: DYNAMIC walks (probabilistic calls, mode-B
// aborts) with one request trace per LANE over the unrolled tree of
// potential invocations ("lane tree walk").  The per-lane
// code is tree_walk.h (shared with the CPU check); this file holds the
// launch: LDS layout, batches, statistics.
//
// Why lanes, not the wave walk of kinds 2/3: a wave that walks its 64 traces
// in lock step visits the UNION of their call paths (config 4: ~167
// invocations and ~409 skip draws per 64 traces that each execute ~5.7
// invocations), every step a scalar program fetch plus global counter
// atomics.  Here each lane follows only its own path; the wave's cost is the
// longest of its 64 paths.  The tree nodes (16 B per position) are copied to
// LDS once per workgroup, so the per-lane dependent fetch of the next node is
// an LDS read, not an HBM/L2 gather; the rest of a position (TreeExt: hop
// cost, callee time, duration row) is read from HBM (L2-resident) only when
// the position executes.
//
// Statistics (isim.h stats words):
//   * per-slot executed calls / callee 500s: u32 LDS counters, one LDS
//     atomic per event, flushed once per workgroup (launches are split so a
//     counter cannot wrap: api.hip launch_walk, Program::tree_mult);
//   * per-service durations (RecordResponseSent, prometheus/handler.go:101-106):
//     code-200 sums in u64 LDS words; code-500 sums by global atomics (500s
//     are rare); bucket counts of a row whose duration bucket is static (the
//     host's lower and upper duration bounds share a bucket) follow from the
//     slot counters at the flush, other rows count each invocation with a
//     global atomic; the entry's row is the end-to-end histogram and sums of
//     the workgroup's traces;
//   * records, latency histograms and header sums as every walk (finish_batch).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "kernel_abi.h"
#include "tree_walk.h"
#include "walk_dev.h"

namespace isim {
namespace dev {

// LDS atomics through address-space-3 pointers: with generic pointers the
// compiler merged the code-200 LDS sum and the code-500 global sum into ONE
// flat_atomic_add_x2 on a selected pointer, which faulted on gfx950
// (hipErrorIllegalAddress) — keep every LDS atomic a ds_* instruction.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) unsigned long long lds_u64;
__device__ __forceinline__ void lds_add(uint32_t *p, uint32_t v) {
  __hip_atomic_fetch_add((lds_u32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_add(unsigned long long *p, unsigned long long v) {
  __hip_atomic_fetch_add((lds_u64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t lds_add_rtn(uint32_t *p, uint32_t v) {
  return __hip_atomic_fetch_add((lds_u32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Row of a duration-table word.  The empty asm hides the mask from the
// AMDGPU backend (ROCm 7.2 LLVM): with the mask's known bits it formed a u24
// multiply for the row offset, dropped the AND, and then selected
// v_mad_u64_u32, which multiplies all 32 bits — the atomic's address ran off
// by bucket x 9 GB (hipErrorIllegalAddress on rows with bucket > 0).
__device__ __forceinline__ uint32_t dur_row(uint32_t w) {
  uint32_t r = w & kTreeRowMask;
  asm volatile("" : "+v"(r));
  return r;
}

// The duration bucket of a u32 time (prometheus/handler.go:26-31, `le`) from
// the workgroup's LDS copy of kBucketTable (walk_dev.h): one ds_read_u8
// instead of an L1 gather, branch-free (entry 501 is the +Inf bucket).
__device__ __forceinline__ uint32_t lut_bucket(const uint8_t *lut, uint32_t t) {
  const uint32_t c = t < 500000001u ? t : 500000001u;
  return ((const __attribute__((address_space(3))) uint8_t *)lut)[(c + 999999u) / 1000000u];
}
__device__ __forceinline__ uint32_t lut_bucket(const uint8_t *lut, uint64_t t) {
  return lut_bucket(lut, (uint32_t)(t < 500000001ull ? t : 500000001ull));
}

// Node accessors of tree_walk.h: LDS (ds_read_b64) or global memory
// (global_load_dwordx2, L2-resident).
struct LdsNodes {
  const __attribute__((address_space(3))) unsigned long long *p;
  __device__ __forceinline__ tw::NodeW load(uint32_t i) const {
    const unsigned long long v = p[i];
    return tw::NodeW{(uint32_t)v, (uint32_t)(v >> 32)};
  }
};
struct GlobalNodes {
  static constexpr int kScan = 2;  // (tree_walk.h scan_of: scans from HBM)
  const unsigned long long *__restrict__ p;
  __device__ __forceinline__ tw::NodeW load(uint32_t i) const {
    const unsigned long long v = p[i];
    return tw::NodeW{(uint32_t)v, (uint32_t)(v >> 32)};
  }
};
// a wide tree's 16-byte nodes (global_load_dwordx4)
struct GlobalNodesW {
  static constexpr int kScan = 2;  // (tree_walk.h scan_of: scans from HBM)
  const uint4 *__restrict__ p;
  __device__ __forceinline__ tw::NodeW4 load(uint32_t i) const {
    const uint4 v = p[i];
    return tw::NodeW4{v.x, v.y, v.z, v.w};
  }
};
// the site graph's nodes (Program::tree_dag, tree_walk.h NodeD4): the same 16 bytes
struct GlobalNodesD {
  static constexpr int kScan = 2;  // (tree_walk.h scan_of: scans from HBM)
  const uint4 *__restrict__ p;
  __device__ __forceinline__ tw::NodeD4 load(uint32_t i) const {
    const uint4 v = p[i];
    return tw::NodeD4{v.x, v.y, v.z, v.w};
  }
};

// A wide tree's statistics (Program::tree_wide: call sites, rows or
// positions past 16 bits, or counters that do not fit in LDS): the hottest
// call sites (program.cpp, by expected calls per trace) count calls and
// callee 500s in guarded 16-bit LDS pairs as the 8-byte kernel does, their
// leaf callees' durations following from those counts at the flush; every
// other event is a global u64 atomic — a cold site's calls and 500s, each
// calling callee's duration bucket and sum in its row, a cold leaf callee's
// (static bucket and latency, from its slot).
__device__ __forceinline__ uint32_t wide_row(uint32_t w) {
  uint32_t r = w & (kTreeLeafSlot - 1u);
  asm volatile("" : "+v"(r));  // (as dur_row: keep the mask out of the address arithmetic)
  return r;
}
struct WideSink {
  const uint8_t *lut;
  uint64_t *svc_tab;
  uint32_t n_slots;
  unsigned long long *sites;
  const uint32_t *slot_tbkt, *slot_tc;
  uint32_t *cnt;               // LDS: per hot site calls | 500s << 16 (guarded 16-bit fields)
  const uint32_t *lds_slot;    // per LDS counter: its slot
  unsigned long long *sum200;  // LDS: the hot rows' code-200 duration sums
  uint32_t *dyn;               // LDS: the hot rows' code-200 bucket tables (header b_lo | width << 8, [width] u32)
  const uint32_t *sum_row;     // per hot row: its row
  // a leaf callee's durations, n of them (static bucket and latency)
  __device__ __forceinline__ void leaf_dur(uint32_t slot, bool st, unsigned long long n) {
    const uint32_t w = slot_tbkt[slot];
    unsigned long long *row = (unsigned long long *)(svc_tab + (uint64_t)wide_row(w) * ISIM_SVC_DUR_WORDS);
    atomicAdd(row + (st ? ISIM_N_PROM : 0u) + (w >> 24), n);
    const uint32_t tc = slot_tc[slot];
    if (tc) atomicAdd(row + 2 * ISIM_N_PROM + (st ? 1u : 0u), (unsigned long long)tc * n);
  }
  // a hot site's 16-bit field reached 2^15: 2^15 of its events to the stats
  // (and, a leaf callee's, their durations; a 500 moves from code 200 to 500)
  __device__ __forceinline__ void move(uint32_t li, bool err) {
    constexpr unsigned long long K = 0x8000ull;
    const uint32_t slot = lds_slot[li];
    atomicAdd(sites + (err ? n_slots : 0u) + slot, K);
    lds_add(cnt + li, err ? 0x80000000u : 0xFFFF8000u);  // the field less 2^15 (no borrow: it is >= 2^15)
    if (svc_tab && (slot_tbkt[slot] & kTreeLeafSlot)) {
      if (err) leaf_dur(slot, false, 0ull - K);
      leaf_dur(slot, err, K);
    }
  }
  __device__ __forceinline__ void count(uint32_t site, bool err) {
    if (site & tw::kSiteLds) {
      const uint32_t li = site & 0xFFFFu;
      const uint32_t old = lds_add_rtn(cnt + li, err ? 0x10000u : 1u);
      if (((old >> (err ? 16 : 0)) & 0xFFFFu) == 0x7FFFu) move(li, err);
    } else {
      atomicAdd(sites + (err ? n_slots : 0u) + site, 1ull);
    }
  }
  __device__ __forceinline__ void call(uint32_t site) { count(site, false); }
  __device__ __forceinline__ void resp_leaf(uint32_t site, bool st) {
    if (st) count(site, true);
    if (svc_tab && !(site & tw::kSiteLds)) leaf_dur(site, st, 1ull);  // (hot sites: at the flush)
  }
  template <typename TT>
  __device__ __forceinline__ void resp(uint32_t site, uint32_t roww, TT T, bool st) {
    if (st) count(site, true);
    if (!svc_tab) return;
    if (roww & 0x80000000u) {  // a hot row: sum index << 16 | its bucket table's LDS offset
      const uint32_t idx = (roww >> 16) & 0x7FFFu, place = roww & 0xFFFFu;
      if (st) {  // a 500 (errorRate-rare): bucket and sum in HBM (the LDS table holds code 200 only)
        unsigned long long *r = (unsigned long long *)(svc_tab + (uint64_t)wide_row(sum_row[idx]) *
                                                                      ISIM_SVC_DUR_WORDS);
        atomicAdd(r + ISIM_N_PROM + lut_bucket(lut, T), 1ull);
        atomicAdd(r + 2 * ISIM_N_PROM + 1, (unsigned long long)T);
        return;
      }
      const uint32_t hdr = dyn[place], lo = hdr & 0xFFu, w = hdr >> 8;
      uint32_t b = lut_bucket(lut, T) - lo;
      b = b < w ? b : w - 1;  // tmin <= T <= tmax keeps it in range; never write past the table
      lds_add(dyn + place + 1u + b, 1u);
      lds_add(sum200 + idx, (unsigned long long)T);
      return;
    }
    unsigned long long *r = (unsigned long long *)(svc_tab + (uint64_t)wide_row(roww) * ISIM_SVC_DUR_WORDS);
    atomicAdd(r + (st ? ISIM_N_PROM : 0u) + lut_bucket(lut, T), 1ull);
    atomicAdd(r + 2 * ISIM_N_PROM + (st ? 1u : 0u), (unsigned long long)T);
  }
};

struct TreeSink {
  uint32_t *cnt;                // LDS: per slot calls | 500s << 16 (cnt16), else [2][n_slots] u32
  const uint8_t *lut;           // LDS duration-bucket table
  void *sum200;                 // LDS [n_sum]: code-200 duration sums (u64; compact: u32, carries go to HBM)
  uint32_t *dyn;                // LDS bucket tables of the varying rows ([2][w] u32; compact: code 200, u16 pairs)
  bool compact;                 // kernel_abi.h TreeLayout.compact
  uint64_t *svc_tab;            // HBM duration table, or null (ISIM_FLAG_NO_SVC_DUR)
  const uint32_t *sum_row;      // per LDS sum index: its row (code-500 sums go to HBM)
  uint32_t n_slots;
  bool cnt16;
  unsigned long long *sites;    // stats: [2][n_slots] executed calls, callee 500s
  const uint32_t *slot_tbkt, *slot_tc;
  // A guarded 16-bit field reached 2^15: 2^15 of its events go to the stats
  // now, with what the flush derives from them (static duration buckets,
  // leaf-callee sums; for 500s, moved from code 200 to code 500)
  __device__ __forceinline__ void move(uint32_t slot, bool err) {
    constexpr unsigned long long K = 0x8000ull;
    atomicAdd(sites + (err ? n_slots : 0u) + slot, K);
    lds_add(cnt + slot, err ? 0x80000000u : 0xFFFF8000u);  // the field less 2^15 (no borrow: it is >= 2^15)
    if (!svc_tab) return;
    const uint32_t w = slot_tbkt[slot], bk = w >> 24;
    unsigned long long *row = (unsigned long long *)(svc_tab + (uint64_t)dur_row(w) * ISIM_SVC_DUR_WORDS);
    const unsigned long long tk = (w & kTreeLeafSlot) ? (unsigned long long)slot_tc[slot] * K : 0ull;
    if (bk != kTreeDynBucket) {
      atomicAdd(row + bk, err ? 0ull - K : K);
      if (err) atomicAdd(row + ISIM_N_PROM + bk, K);
    }
    if (tk) {
      atomicAdd(row + 2 * ISIM_N_PROM, err ? 0ull - tk : tk);
      if (err) atomicAdd(row + 2 * ISIM_N_PROM + 1, tk);
    }
  }
  __device__ __forceinline__ void count(uint32_t slot, bool err) {
    if (cnt16) {
      const uint32_t old = lds_add_rtn(cnt + slot, err ? 0x10000u : 1u);
      if (((old >> (err ? 16 : 0)) & 0xFFFFu) == 0x7FFFu) move(slot, err);
    } else {
      lds_add(cnt + (err ? n_slots : 0u) + slot, 1u);
    }
  }
#ifdef ISIM_TREE_DEBUG
  uint32_t n_pos, n_rows;
  unsigned long long *dbg;
  __device__ bool bad(uint32_t p, uint32_t f, uint32_t d, int frames) {
    uint32_t code = 0;
    if (p > n_pos) code |= 1;
    if (f >= n_pos) code |= 2;
    if (d >= (uint32_t)frames) code |= 4;
    if (code) atomicOr(dbg, (unsigned long long)code | ((unsigned long long)p << 8) | ((unsigned long long)f << 32));
    return code != 0;
  }
#endif
  __device__ __forceinline__ void call(uint32_t slot) {
#ifdef ISIM_TREE_DEBUG
    if (slot >= n_slots) { atomicOr(dbg, 16ull); return; }
#endif
    count(slot, false);
  }
  // a leaf callee: its duration is static (bucket and sums follow from the counters at the flush)
  __device__ __forceinline__ void resp_leaf(uint32_t slot, bool st) {
#ifdef TREE_NO_SINK
    return;
#endif
    if (st) count(slot, true);
  }
  // T: the callee's duration (u32, or u64 in the walks whose latency bound
  // reaches 2^32 ns: a duration of 2^32 ns or more adds to the row's sum in HBM)
  template <typename TT>
  __device__ __forceinline__ void resp(uint32_t slot, uint32_t roww, TT T, bool st) {
#ifdef TREE_NO_SINK
    return;
#endif
#ifdef ISIM_TREE_DEBUG
    if (slot >= n_slots) { atomicOr(dbg, 32ull); return; }
#endif
    if (st) count(slot, true);
    if (!svc_tab) return;
    const uint32_t idx = roww & 0xFFFFu, place = roww >> 16;
    if (place == kTreeGlobalDyn || place == kTreeGlobalStatic) {  // a cold row: sums (and varying buckets) by global atomics
      unsigned long long *r = (unsigned long long *)(svc_tab + (uint64_t)dur_row(idx) * ISIM_SVC_DUR_WORDS);
      if (place == kTreeGlobalDyn) atomicAdd(r + (st ? ISIM_N_PROM : 0u) + lut_bucket(lut, T), 1ull);
      atomicAdd(r + 2 * ISIM_N_PROM + (st ? 1u : 0u), (unsigned long long)T);
      return;
    }
    if (!compact) {  // a wide LDS row
      if (place != kTreeStaticRow) {  // the row's LDS bucket table: header b_lo | width << 8
        const uint32_t hdr = dyn[place], lo = hdr & 0xFFu, w = hdr >> 8;
        uint32_t b = lut_bucket(lut, T) - lo;
        b = b < w ? b : w - 1;  // tmin <= T <= tmax keeps it in range; never write past the table
        lds_add(dyn + place + 1u + (st ? w : 0u) + b, 1u);
      }
      if (st) {
        unsigned long long *r = (unsigned long long *)(svc_tab + (uint64_t)dur_row(sum_row[idx]) * ISIM_SVC_DUR_WORDS);
        atomicAdd(r + 2 * ISIM_N_PROM + 1, (unsigned long long)T);
      } else {
        lds_add((unsigned long long *)sum200 + idx, (unsigned long long)T);
      }
      return;
    }
    // a compact LDS row (round 5: 4-byte sums and u16 code-200 buckets, so
    // about twice the rows fit; 500s — errorRate-rare — go to HBM by atomics)
    if (st) {
      unsigned long long *r = (unsigned long long *)(svc_tab + (uint64_t)dur_row(sum_row[idx]) * ISIM_SVC_DUR_WORDS);
      if (place != kTreeStaticRow) atomicAdd(r + ISIM_N_PROM + lut_bucket(lut, T), 1ull);
      atomicAdd(r + 2 * ISIM_N_PROM + 1, (unsigned long long)T);
      return;
    }
    if (place != kTreeStaticRow) {  // the row's LDS bucket table: header b_lo | width << 8
      const uint32_t hdr = dyn[place], lo = hdr & 0xFFu, w = hdr >> 8;
      uint32_t b = lut_bucket(lut, T) - lo;
      b = b < w ? b : w - 1;  // tmin <= T <= tmax keeps it in range; never write past the table
      const uint32_t sh = (b & 1u) * 16u;
      uint32_t *wd = dyn + place + 1u + (b >> 1);
      const uint32_t old = lds_add_rtn(wd, 1u << sh);
      if (((old >> sh) & 0xFFFFu) == 0x7FFFu) bucket_move(wd, sh, sum_row[idx], lo + b);
    }
    if (sizeof(TT) == 8 && ((uint64_t)T >> 32)) {
      atomicAdd((unsigned long long *)(svc_tab + (uint64_t)dur_row(sum_row[idx]) * ISIM_SVC_DUR_WORDS) +
                    2 * ISIM_N_PROM,
                (unsigned long long)T);
      return;
    }
    const uint32_t t32 = (uint32_t)T;
    const uint32_t o = lds_add_rtn((uint32_t *)sum200 + idx, t32);
    if (o + t32 < o) sum_carry(sum_row[idx]);
  }
  // a u16 bucket field reached 2^15: 2^15 of its counts go to the row in HBM
  __device__ __forceinline__ void bucket_move(uint32_t *wd, uint32_t sh, uint32_t row, uint32_t bucket) {
    atomicAdd((unsigned long long *)(svc_tab + (uint64_t)dur_row(row) * ISIM_SVC_DUR_WORDS) + bucket, 0x8000ull);
    lds_add(wd, 0u - (0x8000u << sh));  // the field less 2^15 (no borrow: it is >= 2^15)
  }
  // the 32-bit LDS sum wrapped: 2^32 to the row's code-200 sum in HBM
  __device__ __forceinline__ void sum_carry(uint32_t row) {
    atomicAdd((unsigned long long *)(svc_tab + (uint64_t)dur_row(row) * ISIM_SVC_DUR_WORDS) + 2 * ISIM_N_PROM,
              1ull << 32);
  }
};

// WPE: waves per SIMD the register allocation must allow — 6 (80 VGPRs: two
// 768-thread workgroups per CU) when the LDS layout fits half the CU, else 4
// (one 1024-thread workgroup per CU: up to 128 VGPRs, no spills).
// T64: u64 time (a latency bound of 2^32 ns or more; tree_walk.h Lane TT).
// WIDE: a wide tree (16-byte nodes in global memory, WideSink); DAG (with
// WIDE): the site graph's nodes (one per call site, tree_walk.h NodeD4).
template <bool MODEB, int FRAMES, bool SPILL, bool NLDS, bool CONC, bool DRAW, int WPE, bool T64 = false,
          bool WIDE = false, bool DAG = false>
__global__ void __launch_bounds__(kWgThreads, WPE)
    isim_tree(const TreeNode *__restrict__ gnodes, isim_trace_rec *__restrict__ records,
              uint64_t *__restrict__ gstats, const uint32_t *__restrict__ slot_tbkt, KParams kp) {
  using TT = std::conditional_t<T64, uint64_t, uint32_t>;
  extern __shared__ __align__(16) unsigned char lds[];
  const uint32_t S = kp.n_slots, P = kp.n_pos;
  const TreeLayout &lay = kp.lay;
  Ctx c{};
  c.records = records;
  c.gstats = gstats;
  c.svc_tab = kp.svc_dur ? gstats + ISIM_ST_SVC_DUR(S) : nullptr;
  c.acc = reinterpret_cast<WgAcc *>(lds);
  c.hist = reinterpret_cast<uint32_t *>(lds + kLdsAccBytes);
  c.cnt = reinterpret_cast<uint32_t *>(lds + lay.off_cnt);
  c.n_slots = S;
  void *sum200 = lds + lay.off_sums;
  uint32_t *dyn = reinterpret_cast<uint32_t *>(lds + lay.off_dyn);
  const uint8_t *lut = lds + kLdsAccBytes + kHistWords * 4u;
  // zero the accumulators (everything before the nodes), copy the nodes in
  uint32_t *z = reinterpret_cast<uint32_t *>(lds);
  // (one write per word: the duration-bucket table's 128 words copied, the rest zeroed)
  {
    constexpr uint32_t l0 = (kLdsAccBytes + kHistWords * 4u) / 4u, l1 = l0 + kTreeLutBytes / 4u;
    const uint32_t *tab = reinterpret_cast<const uint32_t *>(kBucketTable.b);
    for (uint32_t i = threadIdx.x; i < lay.off_nodes / 4u; i += blockDim.x) z[i] = i >= l0 && i < l1 ? tab[i - l0] : 0u;
  }
  if constexpr (NLDS) {
    const uint2 *src = reinterpret_cast<const uint2 *>(gnodes);
    uint2 *dst = reinterpret_cast<uint2 *>(lds + lay.off_nodes);
    for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < kp.n_dyn; i += blockDim.x) {
    const TreeDynRow d = kp.tree_dyn[i];
    dyn[d.off] = d.b_lo | (d.width << 8);
  }
  __syncthreads();
  auto sink = [&]() {
    if constexpr (WIDE)
      return WideSink{lut,       c.svc_tab,  S,           reinterpret_cast<unsigned long long *>(gstats + ISIM_ST_SITES),
                      slot_tbkt, kp.slot_tc, c.cnt,       kp.lds_slot,
                      reinterpret_cast<unsigned long long *>(sum200), dyn, kp.sum_row};
    else
      return TreeSink{c.cnt, lut, sum200, dyn, lay.compact != 0, c.svc_tab, kp.sum_row, S, lay.cnt16 != 0,
                      reinterpret_cast<unsigned long long *>(gstats + ISIM_ST_SITES), slot_tbkt, kp.slot_tc};
  }();
#ifdef ISIM_TREE_DEBUG
  sink.n_pos = P;
  sink.n_rows = kp.n_rows;
  sink.dbg = reinterpret_cast<unsigned long long *>(gstats + ISIM_ST_DES_RETRY);
#endif
  using Nodes = std::conditional_t<WIDE, std::conditional_t<DAG, GlobalNodesD, GlobalNodesW>,
                                   std::conditional_t<NLDS, LdsNodes, GlobalNodes>>;
  Nodes nodes;
  if constexpr (WIDE)
    nodes.p = reinterpret_cast<const uint4 *>(gnodes);
  else if constexpr (NLDS)
    nodes.p = (const __attribute__((address_space(3))) unsigned long long *)(lds + lay.off_nodes);
  else
    nodes.p = reinterpret_cast<const unsigned long long *>(gnodes);
  const TreeExt *__restrict__ ext = kp.tree_ext;
  const TreeStep *__restrict__ stp = kp.tree_step;

  const uint32_t wave = threadIdx.x >> 6, waves = blockDim.x >> 6;
  const uint64_t n = kp.n_traces;
  const uint64_t n_batches = (n + 63) / 64;
  const uint64_t stride = (uint64_t)gridDim.x * waves;
  // batches of 64 trace ids: the first wave-stride statically, then claimed
  // from the launch's per-XCD queues (walk.hip isim_walk).  A lane whose
  // trace has responded takes the next id of its wave's batch at once (trace
  // lengths vary widely: the wave would otherwise wait for its longest
  // trace), so records and histograms are per lane, the sums per lane until
  // the wave runs dry.
  const uint32_t nq = gridDim.x < kWorkQueues ? gridDim.x : kWorkQueues;
  const uint32_t q = blockIdx.x % nq;
  unsigned long long *queue = kp.work + q * kWorkLine;
  auto claim = [&]() -> uint64_t {
    unsigned long long v = 0;
    if (lane_id() == 0) v = atomicAdd(queue, 1ull);
    const uint64_t cc = (uint64_t)rfl((uint32_t)(v >> 32)) << 32 | rfl((uint32_t)v);
    return stride + cc * nq + q;
  };
  uint64_t b = (uint64_t)blockIdx.x * waves + wave;
  bool dry = b >= n_batches;
  uint64_t nxt = dry ? 0 : b * 64, lim = dry ? 0 : (b * 64 + 64 < n ? b * 64 + 64 : n);
  const uint64_t lt = ((uint64_t)1 << lane_id()) - 1;  // lanes below this one
  tw::Lane<FRAMES, MODEB, CONC, SPILL, DRAW, TT, WIDE> L;
  if constexpr (SPILL) {
    L.sp = kp.spill + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    L.sp_stride = kp.spill_lanes;
  }
  bool active = false;  // the lane holds a trace whose record is not yet written
  uint32_t idx = 0;     // launches hold fewer than 2^31 traces (api.hip max_launch_traces)
  // per-lane sums in 32 bits (a latency sum that wraps carries 2^32 into the
  // workgroup's u64 accumulator at once); trace and 500 counts follow from
  // the histograms at the flush
  // (u64 time: u64 per-lane sums, no carries)
  TT a_lat = 0, a_lat500 = 0, a_max = 0, a_min = ~(TT)0;
  uint32_t a_hops = 0, a_err = 0;
  while (true) {
    // responded traces: record, histograms, sums
    const uint64_t fin = ballot(active && L.done);
    if (fin) {
      const bool mine = lane_in(fin);
      const TT lat = L.lat;
      const bool is500 = L.root500;
      if (mine) {
        uint4 r;
        r.x = (uint32_t)lat;
        r.y = T64 ? (uint32_t)((uint64_t)lat >> 32) : 0u;
        r.z = L.hops();
        r.w = (is500 ? 0x80000000u : 0u) | L.errs();
        if (c.records) *reinterpret_cast<uint4 *>(c.records + idx) = r;
        const TT nl = a_lat + lat;
        if (!T64 && nl < a_lat) lds_add(&c.acc->sum_latency, 1ull << 32);
        a_lat = nl;
        if (is500) {
          const TT n5 = a_lat500 + lat;
          if (!T64 && n5 < a_lat500) lds_add(&c.acc->sum_latency500, 1ull << 32);
          a_lat500 = n5;
        }
        a_hops += L.hops();
        a_err += L.errs();
        a_max = lat > a_max ? lat : a_max;
        a_min = lat < a_min ? lat : a_min;
        active = false;
      }
#ifndef TREE_NO_HIST
      // the latency histograms: one LDS atomic per responding lane (their
      // buckets mostly differ, so a wave-aggregated add would loop per bucket)
      if (mine) {
        lds_add(c.hist + (is500 ? ISIM_N_PROM : 0u) + lut_bucket(lut, lat), 1u);
        const uint32_t l2 = lat == 0 ? 0u : 64u - (uint32_t)__builtin_clzll((uint64_t)lat);
        lds_add(c.hist + 2 * ISIM_N_PROM + (is500 ? ISIM_N_LOG2 : 0u) + l2, 1u);
      }
#endif
    }
    // idle lanes take the next trace ids of the wave's batch, claiming batches as it runs dry
    uint64_t idle = ballot(!active);
    while (idle && !dry) {
      if (nxt >= lim) {
        b = claim();
        if (b >= n_batches) {
          dry = true;
          break;
        }
        nxt = b * 64;
        lim = nxt + 64 < n ? nxt + 64 : n;
      }
      const uint64_t avail = lim - nxt;
      const uint32_t rank = popc(idle & lt);
      const bool take = lane_in(idle) && rank < avail;
      if (take) {
        idx = nxt + rank;
        active = true;
        L.start(kp.trace_begin + idx);
      }
      const uint64_t took = ballot(take);
      nxt += popc(took);
      idle &= ~took;
    }
    if (!ballot(active)) break;  // every trace of the wave's batches has responded
    if (active && !L.done) L.step(nodes, ext, stp, sink, kp.seed_lo, kp.seed_hi);
  }
  // the wave's sums into the workgroup accumulators
  {
    const uint64_t s_lat = wave_sum64(a_lat), s_hops = wave_sum64(a_hops), s_err = wave_sum64(a_err);
    const uint64_t s_500 = wave_sum64(a_lat500);
    const uint64_t mx = wave_max64(a_max), nmn = wave_max64(T64 ? ~(uint64_t)a_min : ~(uint64_t)(uint32_t)a_min);
    if (lane_id() == 0) {
      lds_add(&c.acc->sum_latency, (unsigned long long)s_lat);
      lds_add(&c.acc->sum_hops, (unsigned long long)s_hops);
      lds_add(&c.acc->sum_err, (unsigned long long)s_err);
      lds_add(&c.acc->sum_latency500, (unsigned long long)s_500);
      atomicMax(&c.acc->max, (unsigned long long)mx);
      atomicMax(&c.acc->notmin, (unsigned long long)nmn);
    }
  }
  // (the wave count recomputed from the scalar launch sizes: kept from the
  // prologue it was one VGPR pair spilled to scratch across the loop)
  const uint64_t nwaves = (uint64_t)__builtin_amdgcn_readfirstlane(gridDim.x) * (blockDim.x >> 6);
  if (lane_id() == 0 && atomicAdd(kp.work + kWorkQueues * kWorkLine, 1ull) == nwaves - 1) {
    for (uint32_t i = 0; i <= kWorkQueues; ++i) atomicExch(kp.work + i * kWorkLine, 0ull);
  }
  __syncthreads();
  // the workgroup's trace and 500 counts: its end-to-end histogram
  if (threadIdx.x < 64) {
    uint32_t n2 = 0, n5 = 0;
    if (threadIdx.x < ISIM_N_PROM) {
      n2 = c.hist[threadIdx.x];
      n5 = c.hist[ISIM_N_PROM + threadIdx.x];
    }
    const uint64_t t2 = wave_sum64(n2), t5 = wave_sum64(n5);
    if (threadIdx.x == 0) {
      c.acc->ntr = t2 + t5;
      c.acc->n500 = t5;
    }
  }
  __syncthreads();
  // ---- flush the workgroup's accumulators (coalesced over slots / rows)
  unsigned long long *st = reinterpret_cast<unsigned long long *>(gstats);
  for (uint32_t i = threadIdx.x; i < kHistWords; i += blockDim.x)
    if (c.hist[i]) atomicAdd(st + ISIM_ST_PROM + i, (unsigned long long)c.hist[i]);
  // per-slot calls and 500s (their guarded 16-bit fields or the two u32 tables)
  if constexpr (!WIDE) {
  auto calls_of = [&](uint32_t s) -> uint32_t { return lay.cnt16 ? (c.cnt[s] & 0xFFFFu) : c.cnt[s]; };
  auto errs_of = [&](uint32_t s) -> uint32_t { return lay.cnt16 ? (c.cnt[s] >> 16) : c.cnt[S + s]; };
  for (uint32_t i = threadIdx.x; i < 2u * S; i += blockDim.x) {
    const uint32_t v = i < S ? calls_of(i) : errs_of(i - S);
    if (v) atomicAdd(st + ISIM_ST_SITES + i, (unsigned long long)v);
  }
  if (c.svc_tab) {
    unsigned long long *tab = reinterpret_cast<unsigned long long *>(c.svc_tab);
    for (uint32_t s = threadIdx.x; s < S; s += blockDim.x) {
      const uint32_t w = slot_tbkt[s], bk = w >> 24;
      const uint32_t calls = calls_of(s), errs = errs_of(s);
      if (calls == 0 && errs == 0) continue;
      // code-200 events = calls - 500s, in u64 wrap-around arithmetic: with the
      // guarded 16-bit fields the two remainders are independent (the moved
      // 2^15 steps already counted their share), so it may be "negative"
      const unsigned long long ok = (unsigned long long)calls - (unsigned long long)errs;
      unsigned long long *row = tab + (uint64_t)dur_row(w) * ISIM_SVC_DUR_WORDS;
      if (bk != kTreeDynBucket) {
        if (ok) atomicAdd(row + bk, ok);
        if (errs) atomicAdd(row + ISIM_N_PROM + bk, (unsigned long long)errs);
      }
      if (w & kTreeLeafSlot) {  // a leaf callee lasts its latency every time
        const unsigned long long tc = kp.slot_tc[s];
        if (ok && tc) atomicAdd(row + 2 * ISIM_N_PROM, tc * ok);
        if (errs && tc) atomicAdd(row + 2 * ISIM_N_PROM + 1, tc * errs);
      }
    }
    for (uint32_t r = threadIdx.x; r < lay.n_sum; r += blockDim.x) {
      const unsigned long long v =
          lay.compact ? (unsigned long long)((uint32_t *)sum200)[r] : ((unsigned long long *)sum200)[r];
      if (v) atomicAdd(tab + (uint64_t)dur_row(kp.sum_row[r]) * ISIM_SVC_DUR_WORDS + 2 * ISIM_N_PROM, v);
    }
  }
  } else {  // a wide tree: the hot sites' LDS counters (the cold ones counted in HBM as they came)
    unsigned long long *tab = reinterpret_cast<unsigned long long *>(c.svc_tab);
    for (uint32_t i = threadIdx.x; i < kp.n_lds_slots; i += blockDim.x) {
      const uint32_t v = c.cnt[i], calls = v & 0xFFFFu, errs = v >> 16;
      if (!v) continue;
      const uint32_t s = kp.lds_slot[i];
      if (calls) atomicAdd(st + ISIM_ST_SITES + s, (unsigned long long)calls);
      if (errs) atomicAdd(st + ISIM_ST_SITES + S + s, (unsigned long long)errs);
      const uint32_t w = slot_tbkt[s];
      if (!tab || !(w & kTreeLeafSlot)) continue;  // (a calling callee's durations came per response)
      // code-200 events = calls - 500s, in u64 wrap-around arithmetic (the guarded fields, as above)
      const unsigned long long ok = (unsigned long long)calls - (unsigned long long)errs;
      unsigned long long *row = tab + (uint64_t)wide_row(w) * ISIM_SVC_DUR_WORDS;
      const uint32_t bk = w >> 24;
      const unsigned long long tc = kp.slot_tc[s];
      if (ok) atomicAdd(row + bk, ok);
      if (errs) atomicAdd(row + ISIM_N_PROM + bk, (unsigned long long)errs);
      if (ok && tc) atomicAdd(row + 2 * ISIM_N_PROM, tc * ok);
      if (errs && tc) atomicAdd(row + 2 * ISIM_N_PROM + 1, tc * errs);
    }
    for (uint32_t r = threadIdx.x; r < lay.n_sum && tab; r += blockDim.x) {  // the hot rows' code-200 sums
      const unsigned long long v = ((unsigned long long *)sum200)[r];
      if (v) atomicAdd(tab + (uint64_t)wide_row(kp.sum_row[r]) * ISIM_SVC_DUR_WORDS + 2 * ISIM_N_PROM, v);
    }
  }  // !WIDE
  if (c.svc_tab) {
    unsigned long long *tab = reinterpret_cast<unsigned long long *>(c.svc_tab);
    // the varying LDS rows' bucket tables: one thread per (row, word)
    for (uint32_t i = threadIdx.x; i < kp.dyn_words; i += blockDim.x) {
      const uint32_t v = dyn[i];
      if (!v) continue;
      // the table holding word i: the last entry whose header is at or before it
      uint32_t lo = 0, hi = kp.n_dyn;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (kp.tree_dyn[mid].off <= i) lo = mid;
        else hi = mid;
      }
      const TreeDynRow d = kp.tree_dyn[lo];
      if (i == d.off) continue;  // the header
      unsigned long long *row = tab + (uint64_t)(WIDE ? wide_row(d.row) : dur_row(d.row)) * ISIM_SVC_DUR_WORDS;
      if (lay.compact) {  // code-200 u16 pairs
        const uint32_t b = d.b_lo + 2u * (i - d.off - 1u);
        if (v & 0xFFFFu) atomicAdd(row + b, (unsigned long long)(v & 0xFFFFu));
        if (v >> 16) atomicAdd(row + b + 1u, (unsigned long long)(v >> 16));
      } else if (WIDE) {  // [width] u32, code 200 (a wide tree's 500s went to HBM)
        atomicAdd(row + d.b_lo + (i - d.off - 1u), (unsigned long long)v);
      } else {  // [code][width] u32
        const uint32_t j = i - d.off - 1, code = j >= d.width ? 1u : 0u, b = d.b_lo + j - code * d.width;
        atomicAdd(row + code * ISIM_N_PROM + b, (unsigned long long)v);
      }
    }
  }
  if (c.svc_tab) {
    unsigned long long *tab = reinterpret_cast<unsigned long long *>(c.svc_tab);
    // the entry's row: its invocations are the traces (end-to-end histogram and sums)
    unsigned long long *root = tab + (uint64_t)(kp.root_dur & kDurRowMask) * ISIM_SVC_DUR_WORDS;
    for (uint32_t i = threadIdx.x; i < 2u * ISIM_N_PROM; i += blockDim.x)
      if (c.hist[i]) atomicAdd(root + i, (unsigned long long)c.hist[i]);
    if (threadIdx.x == 0 && c.acc->ntr) {
      const unsigned long long s5 = c.acc->sum_latency500, s2 = c.acc->sum_latency - s5;
      if (s2) atomicAdd(root + 2 * ISIM_N_PROM, s2);
      if (s5) atomicAdd(root + 2 * ISIM_N_PROM + 1, s5);
    }
  }
  if (threadIdx.x == 0 && c.acc->ntr) {
    atomicAdd(st + ISIM_ST_N_TRACES, c.acc->ntr);
    atomicAdd(st + ISIM_ST_SUM_LATENCY, c.acc->sum_latency);
    atomicAdd(st + ISIM_ST_SUM_HOPS, c.acc->sum_hops);
    atomicAdd(st + ISIM_ST_SUM_ERR_HOPS, c.acc->sum_err);
    atomicAdd(st + ISIM_ST_N_500, c.acc->n500);
    atomicMax(st + ISIM_ST_NOT_MIN_LATENCY, c.acc->notmin);
    atomicMax(st + ISIM_ST_MAX_LATENCY, c.acc->max);
  }
}

}  // namespace dev

// The variants of one (mode, concurrency) pair: this file is compiled once
// per pair (Makefile: tree_m<MODEB>c<CONC>.o) so the 144 kernels build in
// parallel.  Register-stack depths: the smallest of 4, 6, 8, 12, 16 that
// holds the graph's frames, else 8 registers + a global spill; nodes in LDS
// when the layout holds them; the error-block cache only with error draws.
#ifndef TREE_MODEB
#define TREE_MODEB 0
#endif
#ifndef TREE_CONC
#define TREE_CONC 0
#endif
// waves per SIMD of the two-workgroups-per-CU kernels (timing experiments: 8)
#ifndef TREE_WPE2
#define TREE_WPE2 6
#endif
template <bool NLDS, bool DRAW>
static void *tree_pick(uint32_t frames, bool spill, bool occ2, bool t64, bool wide, bool dag) {
  using namespace dev;
  constexpr bool M = TREE_MODEB != 0, C = TREE_CONC != 0;
  if (wide) {  // a wide tree: nodes in global memory; tree_wide_reg_frames register frames (+ the spill)
    if constexpr (!NLDS) {
      if (dag) {  // the site graph (always wide)
        if (t64) return spill ? (void *)&isim_tree<M, 4, true, false, C, DRAW, 4, true, true, true>
                              : (void *)&isim_tree<M, 4, false, false, C, DRAW, 4, true, true, true>;
        return spill ? (void *)&isim_tree<M, 6, true, false, C, DRAW, 4, false, true, true>
                     : (void *)&isim_tree<M, 6, false, false, C, DRAW, 4, false, true, true>;
      }
      if (t64) return spill ? (void *)&isim_tree<M, 4, true, false, C, DRAW, 4, true, true>
                            : (void *)&isim_tree<M, 4, false, false, C, DRAW, 4, true, true>;
      return spill ? (void *)&isim_tree<M, 6, true, false, C, DRAW, 4, false, true>
                   : (void *)&isim_tree<M, 6, false, false, C, DRAW, 4, false, true>;
    }
    return nullptr;
  }
  if (t64) {  // u64 time: register stacks of 8 or 16 frames, or 8 + the spill; 4 waves per SIMD
    if (spill) return (void *)&isim_tree<M, 8, true, NLDS, C, DRAW, 4, true>;
    if (frames <= 8) return (void *)&isim_tree<M, 8, false, NLDS, C, DRAW, 4, true>;
    return (void *)&isim_tree<M, 16, false, NLDS, C, DRAW, 4, true>;
  }
  if (occ2 && !spill && frames <= 8) {
    if (frames <= 4) return (void *)&isim_tree<M, 4, false, NLDS, C, DRAW, TREE_WPE2>;
    if (frames <= 6) return (void *)&isim_tree<M, 6, false, NLDS, C, DRAW, TREE_WPE2>;
    return (void *)&isim_tree<M, 8, false, NLDS, C, DRAW, TREE_WPE2>;
  }
  if (spill) return (void *)&isim_tree<M, 8, true, NLDS, C, DRAW, 4>;
  if (frames <= 4) return (void *)&isim_tree<M, 4, false, NLDS, C, DRAW, 4>;
  if (frames <= 6) return (void *)&isim_tree<M, 6, false, NLDS, C, DRAW, 4>;
  if (frames <= 8) return (void *)&isim_tree<M, 8, false, NLDS, C, DRAW, 4>;
  if (frames <= 12) return (void *)&isim_tree<M, 12, false, NLDS, C, DRAW, 4>;
  return (void *)&isim_tree<M, 16, false, NLDS, C, DRAW, 4>;
}

#define TREE_CAT2(a, b, c) a##b##c
#define TREE_CAT(a, b, c) TREE_CAT2(a, b, c)
void *TREE_CAT(tree_kernel_m, TREE_MODEB, TREE_CAT(c, TREE_CONC, ))(uint32_t frames, bool spill, bool nodes_lds,
                                                                      bool draw, bool occ2, bool t64, bool wide,
                                                                      bool dag) {
  if (nodes_lds && !wide)
    return draw ? tree_pick<true, true>(frames, spill, occ2, t64, false, false)
                : tree_pick<true, false>(frames, spill, occ2, t64, false, false);
  return draw ? tree_pick<false, true>(frames, spill, occ2, t64, wide, dag)
              : tree_pick<false, false>(frames, spill, occ2, t64, wide, dag);
}

}  // namespace isim
