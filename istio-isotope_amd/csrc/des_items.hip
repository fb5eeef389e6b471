// DES item engine: the exact per-replica worker-pool DES of
// a DYNAMIC walk — probabilistic calls (shouldSkipRequest, isotope/service/
// pkg/srv/executable.go:84-90), and in mode B (EXT) scripts that a failed
// call step ends (handler.go:66-75 with the 500 propagated) — on the GPU.
//
// The static engine (des.hip) keeps one row per (position, trace): every
// invocation executes in every trace.  Here a trace executes a few of the
// tree's potential invocations (config 4's mesh: 5.7 of 3,280), so the unit
// is the ITEM — one executed invocation — and the work is proportional to
// the items, not the positions:
//   1. arrivals    A_t = prefix sum of the exponential gaps (des.h Q24 log)
//   2. pre-walk    the lane tree walk (tree_walk.h Lane, one trace per lane,
//                  waves refilling from a batch counter, no error draws)
//                  counts each trace's executed invocations, a scan gives
//                  the item offsets, a second walk writes each item's
//                  position, caller and contention-free duration (hop id =
//                  item index within the trace: executed invocations in
//                  preorder); the own errors are drawn per item afterwards;
//                  then the items are RENUMBERED position-major (a stable
//                  radix sort by position), so every later pass reads them
//                  nearly in sequence
//   3. buckets     the items sorted (stable radix sort) by their position's
//                  queue round and by (finish group, position) (des_plan.cpp's
//                  schedule over the tree's positions); step-begin ops by round
//   4. rounds      step begins (BK per item and call step), queues (a round
//                  whose positions arrive in trace order with one replica is
//                  already in FIFO order; otherwise ONE stable radix sort by
//                  row | replica | arrival — two when the bits do not fit —,
//                  ties in (trace, hop) order as the oracle's event heap pops
//                  them — then one segmented max-plus scan: S = max(a,
//                  S_prev + hold)), finishes (deepest group first: F from the
//                  start or last BK and the callees' maxima, which each callee
//                  folds into its caller's per-step slot with a 64-bit atomic
//                  max); statistics summed in LDS per 4,096-item chunk; a
//                  cyclic schedule runs quiet passes to its fixed point first
//   5. finalize    records and latency statistics per trace.
// Reference anchors: as des.hip (handler.go:37-79, executable.go:94-179,
// svc/service.go:30-31, prometheus/handler.go:87-106).  Parity: bit-exact
// against oracle/des_oracle.c (its pre-walk, semantics v1 §2.3).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>
#include <rocprim/device/device_scan_by_key.hpp>

#include "des.h"
#include "kernel_abi.h"
#include "tree_walk.h"

namespace isim {
namespace dit {

constexpr uint32_t kT = 256;
constexpr uint32_t kNone = 0xFFFFFFFFu;

__constant__ int32_t c_ln[257] = {
#include "des_ln_table.inc"
};
// service_request_duration_seconds edges (prometheus/handler.go:26-31), ns
__constant__ uint64_t c_edges[32] = {
    7000000ull,   8000000ull,   9000000ull,   10000000ull,  11000000ull,  12000000ull,  14000000ull,
    16000000ull,  18000000ull,  20000000ull,  25000000ull,  30000000ull,  35000000ull,  40000000ull,
    45000000ull,  50000000ull,  60000000ull,  70000000ull,  80000000ull,  90000000ull,  100000000ull,
    120000000ull, 140000000ull, 160000000ull, 180000000ull, 200000000ull, 250000000ull, 300000000ull,
    350000000ull, 400000000ull, 450000000ull, 500000000ull};

// The same bucket from a workgroup's LDS table by ceil(t / 1 ms) (every edge
// is a whole number of milliseconds; entry 501 is +Inf): one ds_read_u8
// instead of five dependent constant loads per item.
constexpr uint32_t kLutEntries = 502;
__device__ __forceinline__ void lut_init(uint8_t *lut) {
  for (uint32_t i = threadIdx.x; i < kLutEntries; i += blockDim.x) {
    uint32_t b = 0;
    while (b < 32 && (uint64_t)i * 1000000ull > c_edges[b]) ++b;
    lut[i] = (uint8_t)b;
  }
  __syncthreads();
}
__device__ __forceinline__ uint32_t lut_bucket(const uint8_t *lut, uint64_t t) {
  const uint64_t c = t < 500000001ull ? t : 500000001ull;
  return lut[(uint32_t)((c + 999999ull) / 1000000ull)];
}

__device__ __forceinline__ uint32_t prom_bucket(uint64_t t) {
  uint32_t lo = 0, hi = 32;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (t <= c_edges[mid]) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// word 0 of Philox4x32-10 (t, w2, w3) under the handler's seed
__device__ __forceinline__ uint32_t draw0(uint64_t t, uint32_t w2, uint32_t w3, uint32_t k0, uint32_t k1) {
  uint32_t a = (uint32_t)t, b = (uint32_t)(t >> 32), c = w2, d = w3;
  tw::philox10(a, b, c, d, k0, k1);
  return a;
}

// -ln(w / 2^24) in Q24, w = (u >> 8) + 1 (des.h des_exp_q24_host)
__device__ __forceinline__ uint64_t exp_q24(uint32_t u) {
  const uint32_t w = (u >> 8) + 1u;
  const int e = 31 - __builtin_clz(w);
  const uint32_t f = (w << (24 - e)) & 0xFFFFFFu;
  const uint32_t idx = f >> 16, rem = f & 0xFFFFu;
  const int64_t lnm = c_ln[idx] + ((((int64_t)c_ln[idx + 1] - c_ln[idx]) * (int64_t)rem) >> 16);
  return (uint64_t)(24 * kLn2Q24 - ((int64_t)e * kLn2Q24 + lnm));
}

struct K {
  // plan
  const DesPos *pos;
  const DesItemPos *ip;
  const DesStep *steps;
  const uint32_t *step_round;
  // tree (pre-walk)
  const unsigned long long *nodes;
  uint32_t n_nodes;
  const TreeExt *ext;
  const TreeStep *tstep;
  uint32_t *spill;
  // per trace
  uint64_t *gap, *A, *cnt, *tend;  // cnt: hops; tend: inclusive item offsets
  uint32_t *terr;                  // status_err
  // per item
  uint32_t *ipos, *ipar, *itr, *ihop;
  uint8_t *iown;
  uint32_t *troot;                 // per trace: its entry item (items are renumbered position-major)
  // the pre-walk's items in trace order, before the renumbering: one 16-byte
  // record each (one line touched per item, not one per field) — x: position
  // (k_own replaces it with the hop), y: duration without contention
  // (saturated), z: caller hop (k_own: the caller's new index; kNone: the
  // entry), w: trace | status << 31
  uint4 *erec;
  uint64_t *IA, *IS, *IF, *acc, *bk;
  const uint64_t *acc_prev;        // cyclic schedules: the previous pass's callee maxima
  const uint64_t *row_hold;        // per duration-table row: the service's worker hold
  uint32_t aw, bw;                 // acc / bk slots per item
  uint64_t M;
  // outputs
  unsigned long long *stats, *table;
  isim_trace_rec *records;
  uint64_t n, trace_begin, mean_ns;
  uint32_t k0, k1, n_slots;
  // cyclic schedules (des_plan.cpp): passes to a fixed point; a quiet pass
  // records no statistics and flags any stored value it changes
  uint32_t quiet;
  uint32_t *changed;
  uint32_t first;                  // the first quiet pass: acc_prev holds contention-free relative maxima
  // incremental quiet passes (round 5): traces in chunks of 2^cshift; a pass
  // recomputes the step begins, arrivals and finishes of the items whose
  // chunk had a value change in the previous pass (dcur; null: every item),
  // and marks the chunks whose values it changes (dnext).  Queue scans stay
  // whole-round (a change moves later traces of the queue: their chunks are
  // marked as their starts change)
  // Round 6: the same marks per TRACE as well (dcur_t / dnext_t, n bytes):
  // after the first passes about 1 % of the items change per pass, spread
  // over enough traces that nearly every 256-trace chunk stays marked; a
  // chunk mark now only pre-filters, an item is recomputed when its own
  // trace changed (the invariant holds per trace: every dependence between
  // traces goes through the whole-round queue scans, which mark the traces
  // whose starts they change)
  const uint8_t *dcur;
  uint8_t *dnext;
  const uint8_t *dcur_t;
  uint8_t *dnext_t;
  uint32_t cshift;
  uint16_t *irep;                  // per item: its replica (drawn once per batch)
  // mode B: the walks draw the errors (a failed step ends its script); per
  // item the call step it failed at (kNone: it did not fail)
  uint32_t modeb;
  uint32_t *ifst;
  // a look-back that gave up after spin_limit polls (des_spin_limit) sets
  // *fault: the batch is not accumulated and des_items_launch fails
  uint32_t *fault;
  uint32_t spin_limit;
};

// a quiet pass flags a change with ONE atomic per wave, and none once the
// flag is set (millions of lanes changing values in the first passes would
// otherwise serialise on the flag's address)
__device__ __forceinline__ void store_tracked(const K &k, uint64_t *p, uint64_t v, uint32_t item) {
  if (k.changed) {
    const bool diff = *p != v;
    if (diff && k.dnext) {
      const uint32_t t = k.itr[item];
      k.dnext[t >> k.cshift] = 1;
      k.dnext_t[t] = 1;
    }
    const unsigned long long m = __ballot(diff);
    if (m && (threadIdx.x & 63u) == (uint32_t)__ffsll((long long)m) - 1u) {
      if (__hip_atomic_load(k.changed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) atomicOr(k.changed, 1u);
    }
  }
  *p = v;
}

__device__ __forceinline__ uint64_t gid() { return (uint64_t)blockIdx.x * kT + threadIdx.x; }
// the item is recomputed in this pass (its trace changed in the previous one;
// the chunk map first: it is small and cached)
__device__ __forceinline__ bool live(const K &k, uint32_t i) {
  if (!k.dcur) return true;
  const uint32_t t = k.itr[i];
  return k.dcur[t >> k.cshift] && k.dcur_t[t];
}
__device__ __forceinline__ uint64_t nthreads() { return (uint64_t)gridDim.x * kT; }
__device__ __forceinline__ uint64_t item_off(const K &k, uint64_t t) { return t ? k.tend[t - 1] : 0; }

// ---- 1. the exponential inter-arrival gaps (summed by a rocPRIM scan)
__global__ void __launch_bounds__(kT) k_gaps(K k) {
  for (uint64_t t = gid(); t < k.n; t += nthreads())
    k.gap[t] = (k.mean_ns * exp_q24(draw0(k.trace_begin + t, 0u, 0x80000001u, k.k0, k.k1))) >> 24;
}

// ---- 2. the pre-walk
struct GNodes {
  const unsigned long long *__restrict__ p;
  __device__ __forceinline__ tw::NodeW load(uint32_t i) const {
    const unsigned long long v = p[i];
    return tw::NodeW{(uint32_t)v, (uint32_t)(v >> 32)};
  }
};
// a wide tree's 16-byte nodes
struct GNodesW {
  const uint4 *__restrict__ p;
  __device__ __forceinline__ tw::NodeW4 load(uint32_t i) const {
    const uint4 v = p[i];
    return tw::NodeW4{v.x, v.y, v.z, v.w};
  }
};
struct CountSink {
  __device__ __forceinline__ void call(uint32_t) {}
  __device__ __forceinline__ void resp_leaf(uint32_t, bool) {}
  template <typename TT>
  __device__ __forceinline__ void resp(uint32_t, uint32_t, TT, bool) {}
};
// records of the current trace go to rec[base + hop], each written once,
// whole, when its invocation closes (tree_walk.h close_rec): position, its
// duration without contention (a lower bound is all k_relmax needs: u64
// durations saturate at 2^32 - 1; the entry's is 0), caller hop, trace and
// in mode B the response status in bit 31 (mode A draws the own errors
// afterwards, k_own).  Before: the record at the open and the duration and
// status at the close — two scattered stores per item.
template <bool MB>
struct EmitSink : CountSink {
  static constexpr bool kCloseRec = true;
  uint4 *rec;
  uint64_t base;
  uint32_t t;
  template <typename TT>
  __device__ __forceinline__ void rec_close(uint32_t p, uint32_t hop, uint32_t caller, TT T, bool st) {
    rec[base + hop] = uint4{p, (uint64_t)T > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)T,
                            caller == tw::kNoCaller ? kNone : caller, t | (MB && st ? 0x80000000u : 0u)};
  }
};

// One trace per lane; a lane whose trace has responded takes the next trace
// id of its wave's batch of 64, the wave claiming batches from a global
// counter as it runs dry (the kind-7 kernel's refill, tree.hip): the waves
// stay full instead of waiting for their longest trace.
// the tree's nodes in LDS when they fit (one ds_read_b64 per visit instead of
// an L2 round trip; kind 7's LdsNodes)
struct LNodes {
  const __attribute__((address_space(3))) unsigned long long *p;
  __device__ __forceinline__ tw::NodeW load(uint32_t i) const {
    const unsigned long long v = p[i];
    return tw::NodeW{(uint32_t)v, (uint32_t)(v >> 32)};
  }
};

template <int FR, bool SPILL, bool EMIT, bool T64, bool MB, bool W, class Nodes>
__device__ __forceinline__ void prewalk_body(const K &k, unsigned long long *work, const Nodes &nodes) {
  // mode A: no error draws in the walk (DRAW = false): an invocation's own
  // error changes no skip, so the walks only need the skip residues; the
  // errors are drawn per item afterwards (k_own), fully parallel.  Mode B:
  // the errors decide which steps run, so the walk draws them (MODEB, DRAW)
  tw::Lane<FR, MB, true, SPILL, MB, std::conditional_t<T64, uint64_t, uint32_t>, W> L;
  if constexpr (SPILL) {
    L.sp = k.spill + ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x);
    L.sp_stride = gridDim.x * blockDim.x;
  }
  const uint32_t lane = threadIdx.x & 63u;
  const unsigned long long lt = (1ull << lane) - 1ull;
  uint64_t nxt = 0, lim = 0;
  bool dry = false, active = false;
  uint32_t t = 0;
  EmitSink<MB> s;
  s.rec = k.erec;
  s.base = 0;
  s.t = 0;
  CountSink cs;
  while (true) {
    if (active && L.done) {
      if constexpr (!EMIT) k.cnt[t] = L.hops();
      active = false;
    }
    unsigned long long idle = __ballot(!active);
    while (idle && !dry) {
      if (nxt >= lim) {
        unsigned long long b = 0;
        if (lane == 0) b = atomicAdd(work, 1ull);
        b = __shfl(b, 0, 64);
        if (b * 64 >= k.n) {
          dry = true;
          break;
        }
        nxt = b * 64;
        lim = nxt + 64 < k.n ? nxt + 64 : k.n;
      }
      const uint32_t rank = (uint32_t)__popcll(idle & lt);
      const bool take = ((idle >> lane) & 1ull) && rank < lim - nxt;
      if (take) {
        t = (uint32_t)(nxt + rank);
        active = true;
        L.start(k.trace_begin + t);
        if constexpr (EMIT) {
          s.base = item_off(k, t);
          s.t = t;
        }
      }
      const unsigned long long took = __ballot(take);
      nxt += (uint64_t)__popcll(took);
      idle &= ~took;
    }
    if (!__ballot(active)) break;
    if (active && !L.done) {
      if constexpr (EMIT) L.step(nodes, k.ext, k.tstep, s, k.k0, k.k1);
      else L.step(nodes, k.ext, k.tstep, cs, k.k0, k.k1);
    }
  }
}

// (W: a wide tree — 16-byte nodes in global memory)
template <int FR, bool SPILL, bool EMIT, bool LDSN, bool T64, bool MB, bool W = false>
__global__ void __launch_bounds__(LDSN ? 1024 : kT) k_prewalk(K k, unsigned long long *work) {
  if constexpr (W) {
    prewalk_body<FR, SPILL, EMIT, T64, MB, true>(k, work, GNodesW{(const uint4 *)k.nodes});
  } else if constexpr (LDSN) {
    extern __shared__ unsigned long long s_nodes[];
    for (uint32_t i = threadIdx.x; i < k.n_nodes; i += blockDim.x) s_nodes[i] = k.nodes[i];
    __syncthreads();
    prewalk_body<FR, SPILL, EMIT, T64, MB, false>(
        k, work, LNodes{(const __attribute__((address_space(3))) unsigned long long *)s_nodes});
  } else {
    prewalk_body<FR, SPILL, EMIT, T64, MB, false>(k, work, GNodes{k.nodes});
  }
}

// ---- 2a. own errors (RecordRequestReceived's status in mode A): word
// (hop & 3) of Philox (t, hop >> 2, 0, 0) against the callee's threshold, as
// the walk draws it (tree_walk.h own_error); the trace's 500 count by atomics
// (errors are rare), its entry status below.  Mode B: the walk wrote each
// item's status (EmitSink::dur), only counted here.  Runs in trace order
// after the renumbering's inverse (inv) is known: the caller hop becomes the
// caller's NEW index here, where the caller's inv entry is a near read (same
// trace), so k_perm_apply gathers nothing but the record
__global__ void __launch_bounds__(kT) k_own(K k, const uint32_t *inv) {
  for (uint64_t i = gid(); i < k.M; i += nthreads()) {
    const uint4 r = k.erec[i];
    const uint32_t t = r.w & 0x7FFFFFFFu;
    const uint32_t hop = (uint32_t)(i - item_off(k, t));  // (a near read: t advances with i)
    const DesPos P = k.pos[r.x];
    bool own = k.modeb ? (r.w >> 31) != 0 : (P.flags & kDesFlagAlways) != 0;
    if (!k.modeb && !own && P.thr) {
      uint32_t a = (uint32_t)(k.trace_begin + t), b = (uint32_t)((k.trace_begin + t) >> 32), c = hop >> 2, d = 0;
      tw::philox10(a, b, c, d, k.k0, k.k1);
      own = tw::word4(hop & 3u, a, b, c, d) < P.thr;
    }
    k.erec[i] = uint4{hop, r.y, r.z == kNone ? kNone : inv[i - hop + r.z], t | (own ? 0x80000000u : 0u)};
    if (own) atomicAdd(k.terr + t, 1u);
  }
}
__global__ void __launch_bounds__(kT) k_root500(K k) {
  for (uint64_t t = gid(); t < k.n; t += nthreads())
    if (k.erec[item_off(k, t)].w >> 31) k.terr[t] |= 0x80000000u;
}

// ---- 2b. renumbering: items in (position, trace) order (a stable radix
// sort of the trace-ordered items by position) so that the passes, which
// visit a position's items together (queues by service, finishes by
// position), read the per-item arrays nearly in sequence
// (the sort reads its keys from the records: an item's position)
struct PosOf {
  __host__ __device__ uint32_t operator()(const uint4 &r) const { return r.x; }
};
// inv[old] = new
__global__ void __launch_bounds__(kT) k_perm_inv(K k, const uint32_t *perm, uint32_t *inv) {
  for (uint64_t j = gid(); j < k.M; j += nthreads()) inv[perm[j]] = (uint32_t)j;
}
__global__ void __launch_bounds__(kT) k_perm_apply(K k, const uint32_t *perm) {
  for (uint64_t j = gid(); j < k.M; j += nthreads()) {
    const uint4 r = k.erec[perm[j]];
    k.itr[j] = r.w & 0x7FFFFFFFu;
    k.iown[j] = (uint8_t)(r.w >> 31);
    k.ihop[j] = r.x;  // the hop (k_own)
    k.ipar[j] = r.z;  // the caller's new index (k_own)
  }
}
// mode B: an item with a callee that responded 500 failed at that callee's
// call step — the last it ran, so the smallest such step (statuses in iown)
__global__ void __launch_bounds__(kT) k_fail(K k) {
  for (uint64_t j = gid(); j < k.M; j += nthreads()) {
    const uint32_t par = k.ipar[j];
    if (par != kNone && k.iown[j]) atomicMin(k.ifst + par, (uint32_t)k.ip[k.ipos[j]].kstep);
  }
}

// cyclic schedules: the first quiet pass starts its cut step begins from the
// contention-free callee durations instead of zero (a lower bound of every
// callee's finish: F(c) >= begin(step) + H(c) + T(c)), so the passes only
// have to settle the queueing, not the whole chain of cut links.  Per
// (caller, call step): max over its callees of H + T, relative to the
// step's begin
__global__ void __launch_bounds__(kT) k_relmax(K k, const uint32_t *perm, unsigned long long *rel) {
  for (uint64_t j = gid(); j < k.M; j += nthreads()) {
    const uint32_t par = k.ipar[j];
    if (par == kNone) continue;
    const uint32_t v = k.ipos[j];
    const DesItemPos p = k.ip[v];
    const DesItemPos pp = k.ip[k.ipos[par]];
    if (pp.nsteps < 2) continue;  // no step begins: nothing reads it
    // off = H, except in the first call step: pre + H relative to the start (the step begins at start + pre)
    const uint64_t h = k.pos[v].off - (p.kstep == 0 ? k.steps[pp.bk_first].add : 0ull);
    atomicMax(rel + (uint64_t)par * k.aw + p.kstep, (unsigned long long)(h + k.erec[perm[j]].y));
  }
}

// a pass's callee maxima: for the items it recomputes, the maxima of the last
// pass that computed them move to `prev` (a cut step begin reads them) and
// the current ones restart from zero (a start can move down when a queue's
// order changes, so maxima are never carried over); the other items keep
// both (their finishes are not recomputed: the maxima they built stay valid)
__global__ void __launch_bounds__(kT) k_acc_init(K k, uint64_t *prev, uint64_t *cur) {
  for (uint64_t i = gid(); i < k.M; i += nthreads()) {
    if (!live(k, (uint32_t)i)) continue;
    for (uint32_t s = 0; s < k.aw; ++s) {
      if (prev) prev[i * k.aw + s] = cur[i * k.aw + s];
      cur[i * k.aw + s] = 0ull;
    }
  }
}

__global__ void __launch_bounds__(kT) k_roots(K k, const uint32_t *inv) {
  for (uint64_t t = gid(); t < k.n; t += nthreads()) k.troot[t] = inv[item_off(k, t)];
}

// ---- 3. bucket keys: the position's queue round and finish group
// (finish groups keyed with the position below them, so a group's items come
// position by position: k_fin sums runs), and the step-begin ops of the
// multi-step items: (round, item << 16 | step), appended one atomic per wave
__global__ void __launch_bounds__(kT) k_bucket_keys(K k, uint32_t *sk, unsigned long long *sv, uint32_t *n_ops) {
  const uint32_t lane = threadIdx.x & 63u;
  for (uint64_t i0 = gid() - lane; i0 < k.M; i0 += nthreads()) {  // whole waves stay in the loop
    const uint64_t i = i0 + lane;
    uint32_t nst = 0;
    DesItemPos p{};
    if (i < k.M) {
      p = k.ip[k.ipos[i]];
      nst = p.nsteps >= 2 ? p.nsteps : 0u;
    }
    // wave prefix sum of the op counts
    uint32_t incl = nst;
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t x = __shfl_up(incl, d, 64);
      if (lane >= d) incl += x;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    if (!total) continue;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(n_ops, total);
    base = __shfl(base, 0, 64);
    for (uint32_t s2 = 0; s2 < nst; ++s2) {
      const uint32_t o = base + incl - nst + s2;
      sk[o] = k.step_round[p.bk_first + s2] & ~kDesStepCut;
      // (item, step) and, in the top 16 bits, the item's trace chunk (k_steps'
      // liveness test without a gather)
      sv[o] = ((unsigned long long)(k.itr[i] >> k.cshift) << 48) | ((unsigned long long)i << 16) | s2;
    }
  }
}

// off[b] = first index of key b in the sorted keys >> shift (b = 0..nb)
__global__ void __launch_bounds__(kT) k_bounds(const uint32_t *keys, uint64_t m, uint32_t nb, uint32_t shift,
                                               uint32_t *off) {
  for (uint64_t i = gid(); i <= m; i += nthreads()) {
    const uint32_t lo = i == 0 ? 0u : (keys[i - 1] >> shift) + 1u;  // keys (keys[i-1], keys[i]] start here
    const uint32_t hi = i == m ? nb : (keys[i] >> shift);
    for (uint32_t b = lo; b <= hi && b <= nb; ++b) off[b] = (uint32_t)i;
  }
}

// The rounds' and finish groups' item lists from the position-major ids: a
// position's items are one contiguous range [poff[v], poff[v + 1]) in trace
// order, so each list is its positions' ranges, concatenated in position
// order (the host places them: qdst / fdst) — no sort of the items
__global__ void __launch_bounds__(kT) k_scatter_ids(K k, const uint32_t *poff, const uint32_t *qdst,
                                                    const uint32_t *fdst, uint32_t *qids, uint32_t *fids) {
  for (uint64_t j = gid(); j < k.M; j += nthreads()) {
    const uint32_t v = k.ipos[j];
    const uint32_t rel = (uint32_t)j - poff[v];
    qids[qdst[v] + rel] = (uint32_t)j;
    fids[fdst[v] + rel] = (uint32_t)j;
  }
}

// ---- 4a. step begins of round r (calls after calls, des.h DesStep)
__global__ void __launch_bounds__(kT) k_steps(K k, const unsigned long long *ops, uint64_t m) {
  for (uint64_t j = gid(); j < m; j += nthreads()) {
    const unsigned long long op = ops[j];
    if (k.dcur && !k.dcur[op >> 48]) continue;  // not recomputed in this pass (its chunk)
    const uint64_t i = (op >> 16) & 0xFFFFFFFFull;
    if (k.dcur && !k.dcur_t[k.itr[i]]) continue;  // (its trace)
    const uint32_t s = (uint32_t)(op & 0xFFFFu);
    if (k.ifst && s > k.ifst[i]) continue;  // mode B: the script failed at an earlier step
    const DesItemPos p = k.ip[k.ipos[i]];
    const uint32_t b = p.bk_first + s;
    const uint32_t sr = k.step_round[b];
    const DesStep st = k.steps[b];
    uint64_t v;
    if (s == 0) {
      v = k.IS[i];
    } else {
      v = k.bk[i * k.bw + (s - 1)] + st.smax;
      // a cut step's callees finish later in the pass: their maxima of the
      // previous one (the first pass: the contention-free lower bound)
      uint64_t c;
      if (!(sr & kDesStepCut)) c = k.acc[i * k.aw + (s - 1)];
      else if (k.first) c = k.bk[i * k.bw + (s - 1)] + k.acc_prev[i * k.aw + (s - 1)];
      else c = k.acc_prev[i * k.aw + (s - 1)];
      v = c > v ? c : v;
    }
    store_tracked(k, k.bk + i * k.bw + s, v + st.add, (uint32_t)i);
  }
}

// FIFO of one worker as a max-plus map x -> max(x + B, C) on "free at x"
// (des.hip SegMP without the segment flag: rocPRIM's scan by key segments)
struct MP {
  uint64_t B, C;
};
struct MPThen {
  __device__ __forceinline__ MP operator()(const MP &a, const MP &b) const {
    const uint64_t c = a.C + b.B;
    return MP{a.B + b.B, c > b.C ? c : b.C};
  }
};

// ---- 4b. queues of round r: each item's arrival and replica, and the
// round's arrival range (mm[0..1]: one 64-bit atomic min / max per
// workgroup); in a quiet pass of a cyclic schedule mm[2] flags an arrival
// that differs from the previous pass's (none: the round's queues are as
// they were and the pass skips them); mm[3]: k_ordchk's flag.  The words
// alternate between two slots by launch; this launch empties the other slot
// for the next one.
// an item's arrival: its trace's, or its caller's start / step begin + off
__device__ __forceinline__ uint64_t item_arrival(const K &k, uint32_t i, uint32_t v, uint64_t off) {
  const uint32_t par = k.ipar[i];
  if (par == kNone) return k.A[k.itr[i]];
  const uint32_t ks = k.ip[v].kstep;
  return (ks == 0 ? k.IS[par] : k.bk[(uint64_t)par * k.bw + ks]) + off;
}
__device__ __forceinline__ void qarr_reset(unsigned long long *mm_next) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // vector atomics: no scalar-cache stores
    atomicExch(mm_next, ~0ull);
    atomicExch(mm_next + 1, 0ull);
    atomicExch(mm_next + 2, 0ull);
    atomicExch(mm_next + 3, 0ull);
  }
}
// the workgroup's range into mm[0..1]: one min / max per workgroup, and only
// when it improves on the current range (thousands of workgroups on one
// address otherwise serialise)
__device__ __forceinline__ void qarr_range(unsigned long long lo, unsigned long long hi, unsigned long long *mm) {
  for (uint32_t d = 32; d > 0; d >>= 1) {
    const unsigned long long x = __shfl_xor(lo, d, 64), y = __shfl_xor(hi, d, 64);
    lo = x < lo ? x : lo;
    hi = y > hi ? y : hi;
  }
  __shared__ unsigned long long s_lo[kT / 64], s_hi[kT / 64];
  if ((threadIdx.x & 63u) == 0) {
    s_lo[threadIdx.x >> 6] = lo;
    s_hi[threadIdx.x >> 6] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t w = 1; w < kT / 64; ++w) {
      lo = s_lo[w] < lo ? s_lo[w] : lo;
      hi = s_hi[w] > hi ? s_hi[w] : hi;
    }
    if (lo <= hi) {
      if (lo < __hip_atomic_load(mm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(mm, lo);
      if (hi > __hip_atomic_load(mm + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(mm + 1, hi);
    }
  }
}
// a quiet pass: flag an arrival that differs from the previous pass's (one atomic per wave at most)
__device__ __forceinline__ void qarr_changed(const K &k, bool diff, unsigned long long *mm) {
  const unsigned long long dm = __ballot(diff);
  if (dm && (threadIdx.x & 63u) == (uint32_t)__ffsll((long long)dm) - 1u &&
      __hip_atomic_load(mm + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0ull)
    atomicOr(mm + 2, 1ull);
}
__global__ void __launch_bounds__(kT) k_qarr(K k, const uint32_t *ids, uint64_t m, unsigned long long *mm,
                                             unsigned long long *mm_next) {
  qarr_reset(mm_next);
  unsigned long long lo = ~0ull, hi = 0;
  for (uint64_t j = gid(); j < m; j += nthreads()) {
    const uint32_t i = ids[j];
    if (!live(k, i)) continue;  // its arrival is the previous pass's (the host keeps the round's range)
    const uint32_t v = k.ipos[i];
    const uint64_t a = item_arrival(k, i, v, k.pos[v].off);
    if (k.changed) qarr_changed(k, k.IA[i] != a, mm);
    k.IA[i] = a;
    lo = a < lo ? a : lo;
    hi = a > hi ? a : hi;
  }
  qarr_range(lo, hi, mm);
}

// each item's replica (the oracle's draw at its hop), once per batch
__global__ void __launch_bounds__(kT) k_reps(K k) {
  for (uint64_t i = gid(); i < k.M; i += nthreads()) {
    const DesPos P = k.pos[k.ipos[i]];
    uint32_t rep = 0;
    if (P.reps > 1) rep = draw0(k.trace_begin + k.itr[i], k.ihop[i], 0x80000002u, k.k0, k.k1) % P.reps;
    k.irep[i] = (uint16_t)rep;
  }
}

// ONE sort key when the bits fit: row | replica | arrival - amin (equal keys
// are put in (trace, hop) order afterwards: k_tiefix)
// (the value is the list index j: a cyclic schedule keeps each round's sorted
// order for the next pass, k_ordchk)
__global__ void __launch_bounds__(kT) k_qkey1(K k, const uint32_t *ids, uint64_t m, uint64_t amin, uint32_t rb,
                                              uint32_t ab, uint64_t *key, uint32_t *val) {
  for (uint64_t j = gid(); j < m; j += nthreads()) {
    const uint32_t i = ids[j];
    const uint64_t row = k.pos[k.ipos[i]].row;
    key[j] = (((row << rb) | k.irep[i]) << ab) | (k.IA[i] - amin);
    val[j] = (uint32_t)j;
  }
}

// the previous pass's sorted order of a round (list indices j) against this
// pass's (row, replica, arrival): when (row, replica, arrival, j) strictly
// increases along it, it IS the stable sort of the round's queue keys, and
// the sort is skipped (k_qscan reads it); any inversion raises mm[3]
// (k_ordchk) and the host sorts (des_items_launch)
// the oracle's tie order of equal (row, replica, arrival): (trace, hop) —
// the event heap pops the earlier trace first (des_oracle.c).  The rounds'
// lists are position-major, so a stable sort alone would break such ties by
// position (a service reached from several positions, arrivals that meet
// exactly: starts chained by a hold equal to a hop cost, for one)
__device__ __forceinline__ uint64_t tie_key(const K &k, uint32_t i) {
  return ((uint64_t)k.itr[i] << 32) | k.ihop[i];
}
// runs of equal keys in a sorted round, re-ordered by (trace, hop): the run's
// first thread sorts it — insertion sort (runs are mostly short, or long
// and already in order), bounded on runs past kTieInsert by 8 moves per item,
// then heapsort, so that one lane's work stays O(r log r) when many items
// meet one service at one instant out of order (a wide fan-out to one
// replica, near-zero gaps).  Tie keys are unique
// (one item per (trace, hop)), so the order is the same either way.  LIST:
// the values are list indices into ids (k_qkey1), else item ids (k_qkey2)
constexpr uint64_t kTieInsert = 32;
template <bool LIST>
__global__ void __launch_bounds__(kT) k_tiefix(K k, const uint64_t *key, uint32_t *val, uint64_t m,
                                               const uint32_t *ids) {
  auto tk = [&](uint32_t v) { return tie_key(k, LIST ? ids[v] : v); };
  for (uint64_t j = gid(); j + 1 < m; j += nthreads()) {
    const uint64_t kj = key[j];
    if (key[j + 1] != kj || (j > 0 && key[j - 1] == kj)) continue;  // the first of a run of ties only
    uint64_t e = j + 2;
    while (e < m && key[e] == kj) ++e;
    // insertion sort: the stable radix sort leaves a run in its list order,
    // usually (trace, hop) order already, so this is O(run) — with a budget
    // of moves on a long run; past it (a wide fan-out meeting one service at
    // one instant) a heapsort, O(run log run).  (Heapsort alone
    // on every run past 32 items made c5p 26x slower: its long runs are
    // already in order.)
    const uint64_t budget = e - j <= kTieInsert ? ~0ull : 8u * (e - j);
    uint64_t moves = 0;
    for (uint64_t x = j + 1; x < e && moves <= budget; ++x) {
      const uint32_t v = val[x];
      const uint64_t t = tk(v);
      uint64_t y = x;
      while (y > j && tk(val[y - 1]) > t && ++moves <= budget) {
        val[y] = val[y - 1];
        --y;
      }
      val[y] = v;  // (the run stays a permutation when the budget runs out)
    }
    if (moves <= budget) continue;
    // heapsort of val[j, e) by tie key (a max-heap, then the max moved to the end)
    uint32_t *a = val + j;
    const uint64_t r = e - j;
    auto sift = [&](uint64_t root, uint64_t len) {
      const uint32_t v = a[root];
      const uint64_t t = tk(v);
      for (;;) {
        uint64_t c = 2 * root + 1;
        if (c >= len) break;
        uint64_t tc = tk(a[c]);
        if (c + 1 < len) {
          const uint64_t t1 = tk(a[c + 1]);
          if (t1 > tc) {
            ++c;
            tc = t1;
          }
        }
        if (tc <= t) break;
        a[root] = a[c];
        root = c;
      }
      a[root] = v;
    };
    for (uint64_t x = r / 2; x-- > 0;) sift(x, r);
    for (uint64_t len = r - 1; len > 0; --len) {
      const uint32_t top = a[0];
      a[0] = a[len];
      a[len] = top;
      sift(0, len);
    }
  }
}
// the kept order against this pass's arrivals (k_qarr's, in list order):
// any inversion raises mm[3] (this slot's, emptied by the launch before)
__global__ void __launch_bounds__(kT) k_ordchk(K k, const uint32_t *ids, const uint32_t *ord, const uint16_t *ordc,
                                               uint64_t m, unsigned long long *mm) {
  auto tuple = [&](uint32_t i, uint64_t &h, uint64_t &a) {
    h = ((uint64_t)k.pos[k.ipos[i]].row << 32) | k.irep[i];
    a = k.IA[i];
  };
  for (uint64_t jj = gid(); jj < m; jj += nthreads()) {
    bool inv = false;
    // a pair of items neither of which this pass recomputes kept its keys:
    // its order stands (ordc: their trace chunks, stored with the order)
    if (jj > 0 && (!k.dcur || k.dcur[ordc[jj]] || k.dcur[ordc[jj - 1]])) {
      const uint32_t i = ids[ord[jj]], ip = ids[ord[jj - 1]];
      uint64_t h, a, hp, ap;
      tuple(i, h, a);
      tuple(ip, hp, ap);
      inv = hp > h || (hp == h && (ap > a || (ap == a && tie_key(k, ip) > tie_key(k, i))));
    }
    const unsigned long long bm = __ballot(inv);
    if (bm && (threadIdx.x & 63u) == (uint32_t)__ffsll((long long)bm) - 1u &&
        __hip_atomic_load(mm + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0ull)
      atomicOr(mm + 3, 1ull);
  }
}

// a sort round's order kept for the next pass: the list indices and the
// items' trace chunks
__global__ void __launch_bounds__(kT) k_keep_ord(K k, const uint32_t *js, const uint32_t *ids, uint64_t m,
                                                 uint32_t *ord, uint16_t *ordc) {
  for (uint64_t jj = gid(); jj < m; jj += nthreads()) {
    const uint32_t j = js[jj];
    ord[jj] = j;
    ordc[jj] = (uint16_t)(k.itr[ids[j]] >> k.cshift);
  }
}

// k_pairs1's outputs along a kept order
__global__ void __launch_bounds__(kT) k_pairs1o(K k, uint64_t m, const uint32_t *ord, const uint32_t *ids,
                                                uint32_t rb, uint32_t *segk, uint32_t *rowk,
                                                MP *mp, uint32_t *sid) {
  for (uint64_t jj = gid(); jj < m; jj += nthreads()) {
    const uint32_t j = ord[jj];
    const uint32_t i = ids[j];
    const uint32_t row = k.pos[k.ipos[i]].row;
    const uint64_t hold = k.row_hold[row];
    segk[jj] = (row << rb) | k.irep[i];
    rowk[jj] = row;
    mp[jj] = MP{hold, k.IA[i] + hold};
    sid[jj] = i;
  }
}

// the segment key (row | replica), row, map (hold, a + hold) and item of
// each position of the sorted order
__global__ void __launch_bounds__(kT) k_pairs1(K k, uint64_t m, const uint64_t *key, const uint32_t *js,
                                               const uint32_t *ids, uint32_t rb, uint32_t ab, uint64_t amin,
                                               uint32_t *segk, uint32_t *rowk, MP *mp, uint32_t *sid) {
  const uint64_t amask = (1ull << ab) - 1ull;
  for (uint64_t j = gid(); j < m; j += nthreads()) {
    const uint64_t kk = key[j];
    const uint32_t row = (uint32_t)(kk >> (ab + rb));
    const uint64_t hold = k.row_hold[row];
    segk[j] = (uint32_t)(kk >> ab);
    rowk[j] = row;
    mp[j] = MP{hold, (kk & amask) + amin + hold};
    sid[j] = ids[js[j]];
  }
}

// a round whose positions need no sort (DesPlan::round_nosort): its items in
// their (position, trace) order are each position's FIFO already; the
// segment key is the position.  A zero-hold position (its arrivals need not
// come in trace order) starts each item at its own arrival (des_oracle.c: an
// invocation holding its worker for 0 starts when it arrives): every item is
// a segment of its own, keys alternating by list index above any position
__global__ void __launch_bounds__(kT) k_pairs0(K k, const uint32_t *ids, uint64_t m, uint32_t *segk, uint32_t *rowk,
                                               MP *mp, uint32_t *sid) {
  for (uint64_t j = gid(); j < m; j += nthreads()) {
    const uint32_t i = ids[j];
    const uint32_t v = k.ipos[i];
    const uint32_t row = k.pos[v].row;
    const uint64_t hold = k.row_hold[row];
    segk[j] = hold ? v : 0x80000000u | (uint32_t)(j & 1u);
    rowk[j] = row;
    mp[j] = MP{hold, k.IA[i] + hold};
    sid[j] = i;
  }
}

// TWO stable sorts otherwise: replica | arrival - amin first, then the row
__global__ void __launch_bounds__(kT) k_qkey2(K k, const uint32_t *ids, uint64_t m, uint64_t amin, uint32_t rb,
                                              uint64_t *key, uint32_t *val,
                                              uint32_t *ovf) {
  for (uint64_t j = gid(); j < m; j += nthreads()) {
    const uint32_t i = ids[j];
    const uint64_t a = k.IA[i] - amin;
    if (rb && (a >> (64 - rb))) atomicOr(ovf, 1u);
    key[j] = rb ? ((uint64_t)k.irep[i] << (64 - rb)) | a : a;
    val[j] = i;
  }
}

// the service's duration-table row of each item, in the arrival order
__global__ void __launch_bounds__(kT) k_rkeys(K k, const uint32_t *items, uint64_t m, uint32_t *rk, uint32_t *rv) {
  for (uint64_t j = gid(); j < m; j += nthreads()) {
    rk[j] = k.pos[k.ipos[items[j]]].row;
    rv[j] = (uint32_t)j;
  }
}

__global__ void __launch_bounds__(kT) k_pairs2(K k, uint64_t m, const uint32_t *rkb, const uint32_t *rvb,
                                               const uint64_t *key, const uint32_t *items, uint32_t rb, uint32_t *segk,
                                               MP *mp, uint32_t *sid) {
  for (uint64_t j = gid(); j < m; j += nthreads()) {
    const uint32_t j1 = rvb[j];
    const uint32_t i = items[j1];
    const uint32_t rep = rb ? (uint32_t)(key[j1] >> (64 - rb)) : 0u;
    const uint64_t hold = k.row_hold[rkb[j]];
    segk[j] = (rkb[j] << 16) | rep;
    mp[j] = MP{hold, k.IA[i] + hold};
    sid[j] = i;
  }
}

// start times; the queue figures per table row (runs of one row within a
// thread's span are summed before the atomics)
constexpr uint32_t kQSpan = 16;
__global__ void __launch_bounds__(kT) k_qout(K k, uint64_t m, const uint32_t *rkb, const uint32_t *sid,
                                             const MP *in, const MP *inc, uint32_t span) {
  // the chunk's first row's queue figures in LDS (a chunk of 4,096 items is
  // mostly one row: one global atomic per figure and chunk, not per lane run)
  __shared__ unsigned long long s_n, s_sw, s_mw, s_sh;
  __shared__ uint32_t s_row;
  // a workgroup takes kT x span consecutive sorted items (uniform trip
  // count: its barriers), a wave 64 x span, lane l the items l, l + 64, ...
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t kChunk = (uint64_t)kT * span;
  for (uint64_t c0 = (uint64_t)blockIdx.x * kChunk; c0 < m; c0 += (uint64_t)gridDim.x * kChunk) {
    if (!k.quiet) {
      if (threadIdx.x == 0) {
        s_n = s_sw = s_mw = s_sh = 0;
        s_row = rkb[c0];
      }
      __syncthreads();
    }
    const uint32_t hrow = k.quiet ? kNone : s_row;
    const uint64_t j0 = c0 + (uint64_t)wave * 64 * span;
    uint32_t row = kNone;
    unsigned long long n = 0, sw = 0, mw = 0, sh = 0;
    auto flush = [&]() {
      if (row == kNone || !n) return;
      if (row == hrow) {
        atomicAdd(&s_n, n);
        if (sw) atomicAdd(&s_sw, sw);
        if (mw) atomicMax(&s_mw, mw);
        if (sh) atomicAdd(&s_sh, sh);
        return;
      }
      unsigned long long *tr = k.table + (uint64_t)row * ISIM_DES_ROW_WORDS;
      atomicAdd(tr + ISIM_DES_COUNT, n);
      if (sw) atomicAdd(tr + ISIM_DES_SUM_WAIT, sw);
      if (mw) atomicMax(tr + ISIM_DES_MAX_WAIT, mw);
      if (sh) atomicAdd(tr + ISIM_DES_SUM_HOLD, sh);
    };
    for (uint64_t j = j0 + lane; j < j0 + 64 * span && j < m; j += 64) {
      const uint32_t i = sid[j];
      const uint32_t r = rkb[j];
      const uint64_t hold = k.row_hold[r];
      const uint64_t S = inc[j].C - hold;
      const uint64_t a = in[j].C - hold;
      store_tracked(k, k.IS + i, S, i);
      if (r != row) {
        if (!k.quiet) flush();
        row = r;
        n = sw = mw = sh = 0;
      }
      const uint64_t w = S - a;
      n += 1;
      sw += w;
      mw = w > mw ? w : mw;
      sh += hold;
    }
    if (!k.quiet) {
      flush();
      __syncthreads();
      if (threadIdx.x == 0 && s_n) {
        unsigned long long *tr = k.table + (uint64_t)hrow * ISIM_DES_ROW_WORDS;
        atomicAdd(tr + ISIM_DES_COUNT, s_n);
        if (s_sw) atomicAdd(tr + ISIM_DES_SUM_WAIT, s_sw);
        if (s_mw) atomicMax(tr + ISIM_DES_MAX_WAIT, s_mw);
        if (s_sh) atomicAdd(tr + ISIM_DES_SUM_HOLD, s_sh);
      }
      __syncthreads();  // the LDS figures are reset for the next chunk
    }
  }
}

// ---- 4b'. the scan and k_qout in one pass.  The FIFO of one replica with a
// constant hold h (a segment: a run of one (row, replica) in the round's
// order; a zero-hold item is a segment of its own) starts its j-th item at
//   S_j = max over the segment's items i <= j of a_i + (j - i) h
//       = j h + max(a_i - i h),
// a segmented prefix maximum of the keys a_i - i h (i, j: list indices; the
// offset cancels within a segment; the host keeps j h below 2^62).  A
// workgroup takes a tile of kT x IPT items by ticket; tiles are chained by a
// decoupled look-back (des.hip chain_body's hand-off: sc1 stores drained
// before the flag store, sc1 loads).  The flag word carries the launch's
// epoch, so the states are cleared once per batch, not per launch.
struct QState {
  uint64_t agg, inc;  // the max after the tile's last segment start (flag >= 1); with the prefix (flag 2)
  uint32_t flag, pad[3];
};
static_assert(sizeof(QState) == 32, "QState is 32 bytes");
constexpr uint32_t kQAgg = 1, kQInc = 2, kQEpochShift = 2;
constexpr int64_t kQMin = INT64_MIN;
__device__ __forceinline__ int64_t qmax(int64_t a, int64_t b) { return a > b ? a : b; }

// Where a round's queue order comes from (the kernel reads it directly, so
// no k_pairs* arrays are written and read back, except for kQArrays):
//   kQArrays  k_pairs2's arrays (segment key, row, item, (hold, a + hold))
//   kQList    a round that needs no sort: its list in (position, trace)
//             order; segment = the position (a zero-hold item alone); the
//             arrival computed here as k_qarr would (no k_qarr launched)
//   kQKept    a cyclic schedule's kept order that still sorts the round
//             (list indices; k_ordchk checked it)
//   kQSorted  the round's sorted keys row | replica | arrival - amin with
//             their list indices
constexpr int kQArrays = 0, kQList = 1, kQKept = 2, kQSorted = 3;
struct QSrc {
  const uint32_t *list;  // the round's item list
  const uint32_t *ord;   // kQKept
  const uint64_t *key;   // kQSorted
  const uint32_t *val;   // kQSorted
  uint64_t amin;         // kQSorted
  uint32_t rb, ab;       // replica bits; kQSorted: arrival bits
  const uint32_t *segk, *rowk, *sid;  // kQArrays
  const MP *mp;                       // kQArrays
};

// item j of the order: its segment key (hold-free: kQList treats zero holds
// itself), and with FULL its item, row, hold and arrival
template <int SRC, bool FULL>
__device__ __forceinline__ uint64_t qitem(const K &k, const QSrc &q, uint64_t j, uint32_t &i, uint32_t &row,
                                          uint64_t &h, uint64_t &a) {
  uint64_t sk;
  if constexpr (SRC == kQArrays) {
    sk = q.segk[j];
    if (FULL) {
      i = q.sid[j];
      row = q.rowk[j];
      const MP p = q.mp[j];
      h = p.B;
      a = p.C - p.B;
    }
  } else if constexpr (SRC == kQSorted) {
    const uint64_t kk = q.key[j];
    sk = kk >> q.ab;
    if (FULL) {
      i = q.list[q.val[j]];
      row = (uint32_t)(kk >> (q.ab + q.rb));
      h = k.row_hold[row];
      a = (kk & ((1ull << q.ab) - 1ull)) + q.amin;
    }
  } else {
    i = q.list[SRC == kQKept ? q.ord[j] : (uint32_t)j];
    const uint32_t v = k.ipos[i];
    if (SRC == kQList) {
      sk = v;
    } else {
      row = k.pos[v].row;
      sk = ((uint64_t)row << q.rb) | k.irep[i];
    }
    if (FULL) {
      const DesPos P = k.pos[v];
      row = P.row;
      h = k.row_hold[row];
      if (SRC == kQKept || !live(k, i)) {
        a = k.IA[i];  // (kQList: an item a quiet pass does not recompute keeps its own)
      } else {
        a = item_arrival(k, i, v, P.off);
        k.IA[i] = a;
      }
    }
  }
  return sk;
}

template <uint32_t IPT, int SRC>
__global__ void __launch_bounds__(kT) k_qscan(K k, uint64_t m, QSrc q, QState *qs, uint32_t *ticket, uint32_t tbase,
                                              uint32_t epoch) {
  constexpr uint32_t NW = kT / 64;
  __shared__ uint32_t s_tile, s_row;
  __shared__ int64_t w_v[NW], s_cin;
  __shared__ uint32_t w_f[NW];
  __shared__ unsigned long long s_n, s_sw, s_mw, s_sh;
  if (threadIdx.x == 0) {
    const uint32_t t = atomicAdd(ticket, 1u) - tbase;
    s_tile = t;
    const uint64_t j0 = (uint64_t)t * kT * IPT;
    if constexpr (SRC == kQArrays) s_row = q.rowk[j0];
    else if constexpr (SRC == kQSorted) s_row = (uint32_t)(q.key[j0] >> (q.ab + q.rb));
    else s_row = k.pos[k.ipos[q.list[SRC == kQKept ? q.ord[j0] : (uint32_t)j0]]].row;
    s_n = s_sw = s_mw = s_sh = 0;
  }
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t w0 = (uint64_t)tile * kT * IPT + (uint64_t)wave * 64 * IPT;
  // the wave's rows of 64 items: a segmented max over the lanes, then over
  // the rows (cf, cv: the wave's items so far)
  int64_t v[IPT];
  bool f[IPT];
  uint64_t a[IPT], h[IPT];
  uint32_t it[IPT], rw[IPT];
  bool cf = false;
  int64_t cv = kQMin;
#pragma unroll
  for (uint32_t r = 0; r < IPT; ++r) {
    const uint64_t j = w0 + r * 64 + lane;
    bool s = false;
    int64_t x = kQMin;
    a[r] = h[r] = 0;
    it[r] = rw[r] = 0;
    // the previous item's segment: the lane below's, lane 0 reads it
    uint64_t sk = ~0ull, ps = ~0ull;
    if (j < m) {
      sk = qitem<SRC, true>(k, q, j, it[r], rw[r], h[r], a[r]);
      if (lane == 0 && j > 0) {
        uint32_t i1, r1;
        uint64_t h1, a1;
        ps = qitem<SRC, false>(k, q, j - 1, i1, r1, h1, a1);
      }
    }
    const uint64_t up = __shfl_up(sk, 1, 64);
    if (lane > 0) ps = up;
    if (j < m) {
      s = j == 0 || ps != sk || (SRC == kQList && h[r] == 0);
      x = (int64_t)(a[r] - j * h[r]);
    }
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const int64_t ox = __shfl_up(x, d, 64);
      const int os = __shfl_up((int)s, d, 64);
      if (lane >= d) {
        if (!s) x = qmax(x, ox);
        s = s || os;
      }
    }
    v[r] = s ? x : qmax(cv, x);
    f[r] = s || cf;
    cv = __shfl(v[r], 63, 64);
    cf = __shfl((int)f[r], 63, 64);
  }
  if (lane == 0) {
    w_v[wave] = cv;
    w_f[wave] = cf;
  }
  __syncthreads();
  if (wave == 0) {
    bool bf = false;
    int64_t bv = kQMin;
    for (uint32_t w = 0; w < NW; ++w) {
      bv = w_f[w] ? w_v[w] : qmax(bv, w_v[w]);
      bf = bf || w_f[w];
    }
    QState *me = qs + tile;
    const uint32_t ep = epoch << kQEpochShift;
    if (lane == 0 && (bf || tile > 0)) {  // a tile with a segment start knows its prefix already
      __hip_atomic_store(&me->agg, (uint64_t)bv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (bf) __hip_atomic_store(&me->inc, (uint64_t)bv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&me->flag, ep | (bf ? kQAgg | kQInc : kQAgg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the open segment's max before the tile, unless its first item starts one
    int64_t cin = kQMin;
    if (tile > 0 && !__shfl((int)f[0], 0, 64)) {
      int64_t top = (int64_t)tile - 1;
      uint32_t spins = 0;
      for (;;) {
        if (spins >= k.spin_limit) {  // never expected (tickets order the tiles): fail the batch
          if (lane == 0) atomicOr(k.fault, 1u);
          break;
        }
        const int64_t jt = top - (int64_t)lane;  // lane 0: the nearest tile
        uint32_t fl = kQInc;                    // before tile 0: an empty prefix
        if (jt >= 0) {
          fl = __hip_atomic_load(&qs[jt].flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          fl = (fl >> kQEpochShift) == epoch ? fl & (kQAgg | kQInc) : 0u;
        }
        const uint64_t m0 = __ballot(fl == 0), mi = __ballot((fl & kQInc) != 0);
        const uint32_t fi = mi ? (uint32_t)__builtin_ctzll(mi) : 64u;
        const uint64_t upto = fi >= 63 ? ~0ull : ((1ull << (fi + 1)) - 1);
        if (m0 & upto) {  // a tile this one needs has not published yet
          __builtin_amdgcn_s_sleep(1);
          ++spins;
          continue;
        }
        int64_t x = kQMin;
        if (jt >= 0 && lane <= fi)
          x = (int64_t)__hip_atomic_load(lane == fi ? &qs[jt].inc : &qs[jt].agg, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        for (uint32_t d = 32; d > 0; d >>= 1) x = qmax(x, __shfl_xor(x, d, 64));
        cin = qmax(cin, x);
        if (fi < 64) break;
        top -= 64;
      }
    }
    if (lane == 0) {
      if (!bf && tile > 0) {
        __hip_atomic_store(&me->inc, (uint64_t)qmax(cin, bv), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&me->flag, ep | kQAgg | kQInc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      s_cin = cin;
    }
  }
  __syncthreads();
  int64_t c = s_cin;
  for (uint32_t w = 0; w < wave; ++w) c = w_f[w] ? w_v[w] : qmax(c, w_v[w]);
  // starts; the queue figures as k_qout sums them
  const uint32_t hrow = k.quiet ? kNone : s_row;
  uint32_t row = kNone;
  unsigned long long n = 0, sw = 0, mw = 0, sh = 0;
  auto flush = [&]() {
    if (row == kNone || !n) return;
    if (row == hrow) {
      atomicAdd(&s_n, n);
      if (sw) atomicAdd(&s_sw, sw);
      if (mw) atomicMax(&s_mw, mw);
      if (sh) atomicAdd(&s_sh, sh);
      return;
    }
    unsigned long long *tr = k.table + (uint64_t)row * ISIM_DES_ROW_WORDS;
    atomicAdd(tr + ISIM_DES_COUNT, n);
    if (sw) atomicAdd(tr + ISIM_DES_SUM_WAIT, sw);
    if (mw) atomicMax(tr + ISIM_DES_MAX_WAIT, mw);
    if (sh) atomicAdd(tr + ISIM_DES_SUM_HOLD, sh);
  };
#pragma unroll
  for (uint32_t r = 0; r < IPT; ++r) {
    const uint64_t j = w0 + r * 64 + lane;
    if (j >= m) break;
    const uint64_t S = (uint64_t)(f[r] ? v[r] : qmax(c, v[r])) + j * h[r];
    const uint32_t i = it[r];
    store_tracked(k, k.IS + i, S, i);
    if (k.quiet) continue;
    const uint32_t rj = rw[r];
    if (rj != row) {
      flush();
      row = rj;
      n = sw = mw = sh = 0;
    }
    const uint64_t w = S - a[r];
    n += 1;
    sw += w;
    mw = w > mw ? w : mw;
    sh += h[r];
  }
  if (k.quiet) return;
  flush();
  __syncthreads();
  if (threadIdx.x == 0 && s_n) {
    unsigned long long *tr = k.table + (uint64_t)hrow * ISIM_DES_ROW_WORDS;
    atomicAdd(tr + ISIM_DES_COUNT, s_n);
    if (s_sw) atomicAdd(tr + ISIM_DES_SUM_WAIT, s_sw);
    if (s_mw) atomicMax(tr + ISIM_DES_MAX_WAIT, s_mw);
    if (s_sh) atomicAdd(tr + ISIM_DES_SUM_HOLD, s_sh);
  }
}

// ---- 4c. finishes of one group (its items position by position): per
// item the finish and its callee maximum into the caller's slot; the
// statistics summed over a thread's run of one position (and one bucket for
// the histogram) before the atomics
__global__ void __launch_bounds__(kT) k_fin(K k, const uint32_t *ids, uint64_t m, uint32_t span) {
  __shared__ uint8_t lut[kLutEntries];
  // the duration histogram of the chunk's first row (a chunk of 4,096 sorted
  // items is mostly one position): LDS atomics, one global add per bucket
  __shared__ uint32_t hist[2 * ISIM_N_PROM];
  __shared__ uint32_t s_row, s_pos;
  // and the chunk's first position's duration sums and site counts
  __shared__ unsigned long long f_d0, f_d1, f_n, f_n5;
  if (!k.quiet) lut_init(lut);
  // a workgroup takes kT x span consecutive sorted items (uniform trip
  // count: its barriers), a wave 64 x span of them, lane l the items
  // l, l + 64, ...: coalesced loads, and a lane's items mostly share a
  // position, so its runs sum before the atomics
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t kChunk = (uint64_t)kT * span;
  for (uint64_t c0 = (uint64_t)blockIdx.x * kChunk; c0 < m; c0 += (uint64_t)gridDim.x * kChunk) {
    if (!k.quiet) {
      for (uint32_t x = threadIdx.x; x < 2 * ISIM_N_PROM; x += kT) hist[x] = 0;
      if (threadIdx.x == 0) {
        s_pos = k.ipos[ids[c0]];
        s_row = k.pos[s_pos].row;
        f_d0 = f_d1 = f_n = f_n5 = 0;
      }
      __syncthreads();
    }
    const uint32_t hrow = k.quiet ? kNone : s_row, hpos = k.quiet ? kNone : s_pos;
    const uint64_t j0 = c0 + (uint64_t)wave * 64 * span;
    uint32_t v_run = kNone, b_run = kNone;
    DesPos P{};
    DesItemPos p{};
    unsigned long long n = 0, n5 = 0, d0 = 0, d1 = 0, nb = 0;
    auto flush_bucket = [&]() {
      if (!k.quiet && nb) {
        if (P.row == hrow) atomicAdd(&hist[b_run], (uint32_t)nb);
        else atomicAdd(k.table + (uint64_t)P.row * ISIM_DES_ROW_WORDS + b_run, nb);
      }
      nb = 0;
    };
    auto flush = [&]() {
      flush_bucket();
      if (k.quiet || v_run == kNone || !n) return;
      if (v_run == hpos) {
        atomicAdd(&f_n, n);
        if (n5) atomicAdd(&f_n5, n5);
        if (d0) atomicAdd(&f_d0, d0);
        if (d1) atomicAdd(&f_d1, d1);
        return;
      }
      unsigned long long *tr = k.table + (uint64_t)P.row * ISIM_DES_ROW_WORDS;
      if (d0) atomicAdd(tr + 2 * ISIM_N_PROM, d0);
      if (d1) atomicAdd(tr + 2 * ISIM_N_PROM + 1, d1);
      if (P.parent != kDesNoParent) {
        atomicAdd(k.stats + ISIM_ST_SITES + P.slot, n);
        if (n5) atomicAdd(k.stats + ISIM_ST_SITES + k.n_slots + P.slot, n5);
      }
    };
    for (uint64_t j = j0 + lane; j < j0 + 64 * span && j < m; j += 64) {
      const uint32_t i = ids[j];
      if (k.quiet && !live(k, i)) continue;
      const uint32_t v = k.ipos[i];
      if (v != v_run) {
        flush();
        v_run = v;
        P = k.pos[v];
        p = k.ip[v];
        n = n5 = d0 = d1 = 0;
        b_run = kNone;
      }
      uint64_t F;
      const uint32_t fst = k.ifst ? k.ifst[i] : kNone;
      if (P.flags & kDesFlagLeaf) {
        F = k.IS[i] + P.floor;
      } else if (fst != kNone) {
        // mode B, failed at call step fst: that step's end (its begin plus its
        // longest sleep, or its callees' finishes), no later command
        const uint64_t b0 = p.nsteps >= 2 ? k.bk[(uint64_t)i * k.bw + fst] : k.IS[i];
        const uint64_t sm = p.nsteps >= 2 && fst + 1u < p.nsteps ? k.steps[p.bk_first + fst + 1].smax : P.floor;
        const uint64_t c = k.acc[(uint64_t)i * k.aw + fst];
        F = c > b0 + sm ? c : b0 + sm;
      } else {
        const uint32_t last = p.nsteps >= 2 ? p.nsteps - 1u : 0u;
        F = (p.nsteps >= 2 ? k.bk[(uint64_t)i * k.bw + last] : k.IS[i]) + P.floor;
        const uint64_t c = k.acc[(uint64_t)i * k.aw + last];
        F = (c > F ? c : F) + P.post;
      }
      store_tracked(k, k.IF + i, F, i);
      const uint32_t par = k.ipar[i];
      if (par != kNone)
        atomicMax((unsigned long long *)(k.acc + (uint64_t)par * k.aw + p.kstep), (unsigned long long)F);
      if (k.quiet) continue;
      const uint32_t own = k.iown[i];
      const uint64_t dur = F - k.IA[i];
      const uint32_t b = own * ISIM_N_PROM + lut_bucket(lut, dur);
      if (b != b_run) {
        flush_bucket();
        b_run = b;
      }
      nb += 1;
      n += 1;
      n5 += own;
      if (own) d1 += dur;
      else d0 += dur;
    }
    flush();
    if (!k.quiet) {
      __syncthreads();
      for (uint32_t x = threadIdx.x; x < 2 * ISIM_N_PROM; x += kT)
        if (hist[x]) atomicAdd(k.table + (uint64_t)hrow * ISIM_DES_ROW_WORDS + x, (unsigned long long)hist[x]);
      if (threadIdx.x == 0 && f_n) {
        unsigned long long *tr = k.table + (uint64_t)hrow * ISIM_DES_ROW_WORDS;
        if (f_d0) atomicAdd(tr + 2 * ISIM_N_PROM, f_d0);
        if (f_d1) atomicAdd(tr + 2 * ISIM_N_PROM + 1, f_d1);
        const DesPos P0 = k.pos[hpos];
        if (P0.parent != kDesNoParent) {
          atomicAdd(k.stats + ISIM_ST_SITES + P0.slot, f_n);
          if (f_n5) atomicAdd(k.stats + ISIM_ST_SITES + k.n_slots + P0.slot, f_n5);
        }
      }
      __syncthreads();  // the LDS figures are reset for the next chunk
    }
  }
}

// ---- 5. records and the latency statistics
__global__ void __launch_bounds__(kT) k_final(K k) {
  if (*k.fault) return;  // a failed batch writes no record and accumulates nothing
  __shared__ uint32_t hp[2 * ISIM_N_PROM], hl[2 * ISIM_N_LOG2];
  __shared__ unsigned long long red[6][kT / 64];
  for (uint32_t i = threadIdx.x; i < 2 * ISIM_N_PROM; i += kT) hp[i] = 0;
  for (uint32_t i = threadIdx.x; i < 2 * ISIM_N_LOG2; i += kT) hl[i] = 0;
  __syncthreads();
  unsigned long long sl = 0, sh = 0, se = 0, n5 = 0, mn = ~0ull, mx = 0;
  for (uint64_t t = gid(); t < k.n; t += nthreads()) {
    const uint64_t root = k.troot[t];
    const uint64_t L = k.IF[root] - k.A[t];
    const uint32_t hops = (uint32_t)(k.tend[t] - item_off(k, t));
    const uint32_t s_e = k.terr[t];
    const uint32_t st = s_e >> 31, e = s_e & 0x7FFFFFFFu;
    if (k.records) {
      isim_trace_rec r;
      r.latency_ns = L;
      r.hops = hops;
      r.status_err = s_e;
      k.records[t] = r;
    }
    sl += L;
    sh += hops;
    se += e;
    n5 += st;
    mn = L < mn ? L : mn;
    mx = L > mx ? L : mx;
    atomicAdd(&hp[st * ISIM_N_PROM + prom_bucket(L)], 1u);
    atomicAdd(&hl[st * ISIM_N_LOG2 + (L ? 64u - (uint32_t)__builtin_clzll(L) : 0u)], 1u);
  }
  for (uint32_t d = 32; d > 0; d >>= 1) {
    sl += __shfl_xor(sl, d, 64);
    sh += __shfl_xor(sh, d, 64);
    se += __shfl_xor(se, d, 64);
    n5 += __shfl_xor(n5, d, 64);
    const unsigned long long a = __shfl_xor(mn, d, 64), b = __shfl_xor(mx, d, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  if ((threadIdx.x & 63u) == 0) {
    const uint32_t w = threadIdx.x >> 6;
    red[0][w] = sl;
    red[1][w] = sh;
    red[2][w] = se;
    red[3][w] = n5;
    red[4][w] = mn;
    red[5][w] = mx;
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 2 * ISIM_N_PROM; i += kT)
    if (hp[i]) atomicAdd(k.stats + ISIM_ST_PROM + i, (unsigned long long)hp[i]);
  for (uint32_t i = threadIdx.x; i < 2 * ISIM_N_LOG2; i += kT)
    if (hl[i]) atomicAdd(k.stats + ISIM_ST_LOG2 + i, (unsigned long long)hl[i]);
  if (threadIdx.x == 0) {
    for (uint32_t w = 1; w < kT / 64; ++w) {
      for (uint32_t q = 0; q < 4; ++q) red[q][0] += red[q][w];
      red[4][0] = red[4][w] < red[4][0] ? red[4][w] : red[4][0];
      red[5][0] = red[5][w] > red[5][0] ? red[5][w] : red[5][0];
    }
    if (blockIdx.x == 0) atomicAdd(k.stats + ISIM_ST_N_TRACES, (unsigned long long)k.n);
    atomicAdd(k.stats + ISIM_ST_SUM_LATENCY, red[0][0]);
    atomicAdd(k.stats + ISIM_ST_SUM_HOPS, red[1][0]);
    atomicAdd(k.stats + ISIM_ST_SUM_ERR_HOPS, red[2][0]);
    atomicAdd(k.stats + ISIM_ST_N_500, red[3][0]);
    if (red[4][0] != ~0ull) atomicMax(k.stats + ISIM_ST_NOT_MIN_LATENCY, ~red[4][0]);
    atomicMax(k.stats + ISIM_ST_MAX_LATENCY, red[5][0]);
  }
}

__global__ void k_flag_retry(unsigned long long *stats, const uint32_t *ovf) {
  if (ovf[2]) atomicAdd(stats + ISIM_ST_DES_RETRY, (unsigned long long)kDesFaultUnit);  // a fault: an error
  else if (ovf[0] || ovf[1]) atomicAdd(stats + ISIM_ST_DES_RETRY, 1ull);
}

}  // namespace dit

namespace {

uint64_t al256(uint64_t b) { return (b + 255) & ~255ull; }
uint32_t grid_for(uint64_t m, uint32_t cap = 8192) {
  const uint64_t g = (m + dit::kT - 1) / dit::kT;
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(g, cap));
}
uint32_t bits_for(uint64_t v) {  // bits of the largest key v
  uint32_t b = 0;
  while (b < 64 && (v >> b)) ++b;
  return std::max<uint32_t>(b, 1);
}
size_t scan_u64_bytes(uint64_t n) {
  size_t b = 0;
  (void)rocprim::inclusive_scan(nullptr, b, (const uint64_t *)nullptr, (uint64_t *)nullptr, (size_t)n,
                                rocprim::plus<uint64_t>());
  return b;
}
constexpr uint32_t kPrewalkBlocks = 2048;  // pre-walk grid (waves refill from a global batch counter)
constexpr uint32_t kMaxPasses = 256;       // fixed-point passes of a cyclic schedule (des.hip)
// incremental quiet passes: chunks of 256 traces, or larger so that a chunk
// id fits 16 bits (step ops and kept orders carry it)
uint32_t chunk_shift(uint64_t n) { return std::max<uint32_t>(8u, bits_for(n) > 16u ? bits_for(n) - 16u : 0u); }

}  // namespace

// per trace: gaps, arrivals, hops, item ends (u64), status_err (u32), scan temp
uint64_t des_items_workspace_bytes(uint64_t n) {
  return 4 * al256(n * 8) + al256(n * 4) + al256(16) + al256(scan_u64_bytes(n)) + 256;
}

int des_items_launch(const DesItemsLaunch &L, void *stream_, std::string &err) {
  using namespace dit;
  hipStream_t s = (hipStream_t)stream_;
  const DesPlan &pl = *L.plan;
  const uint64_t n = L.n_traces;
  char *ws = (char *)L.workspace;
  auto take = [&](uint64_t bytes) {
    char *p = ws;
    ws += al256(bytes);
    return (void *)p;
  };
  K k{};
  k.pos = (const DesPos *)L.d_pos;
  k.ip = (const DesItemPos *)L.d_item_pos;
  k.steps = (const DesStep *)L.d_steps;
  k.step_round = L.d_step_round;
  k.nodes = (const unsigned long long *)L.d_nodes;
  k.ext = (const TreeExt *)L.d_ext;
  k.tstep = (const TreeStep *)L.d_tstep;
  k.gap = (uint64_t *)take(n * 8);
  k.A = (uint64_t *)take(n * 8);
  k.cnt = (uint64_t *)take(n * 8);
  k.tend = (uint64_t *)take(n * 8);
  k.terr = (uint32_t *)take(n * 4);
  // the refill counters of the two pre-walks
  unsigned long long *work = (unsigned long long *)take(16);
  const size_t scan_bytes = scan_u64_bytes(n);
  void *scan_tmp = take(scan_bytes);
  k.stats = (unsigned long long *)L.d_stats;
  k.table = (unsigned long long *)L.d_table;
  k.records = L.d_records;
  k.n = n;
  k.trace_begin = L.trace_begin;
  k.mean_ns = L.mean_ns;
  k.k0 = (uint32_t)L.seed;
  k.k1 = (uint32_t)(L.seed >> 32);
  k.n_slots = L.n_slots;
  k.modeb = pl.modeb ? 1u : 0u;
  uint32_t max_reps = 1, max_row = 0;
  for (const DesPos &q : pl.pos) {
    max_reps = std::max(max_reps, q.reps);
    max_row = std::max(max_row, q.row);
  }
  const uint32_t rep_bits = max_reps > 1 ? bits_for(max_reps - 1) : 0u;
  k.aw = pl.item_acc;
  k.bw = pl.item_bk;
  auto fail = [&](const char *what) {
    err = std::string("DES items: ") + what;
    return 1;
  };
  // the batch's report (isim_des_last_batch): host synchronisations, passes, items
  DesItemsReport rep{};
  auto sync_s = [&]() {
    ++rep.syncs;
    return hipStreamSynchronize(s);
  };
  struct ReportOut {
    const DesItemsReport &r;
    DesItemsReport *out;
    ~ReportOut() {
      if (out) *out = r;
    }
  } report_out{rep, L.report};
  // 1. arrivals
  hipLaunchKernelGGL(k_gaps, dim3(grid_for(n)), dim3(kT), 0, s, k);
  size_t b = scan_bytes;
  if (rocprim::inclusive_scan(scan_tmp, b, k.gap, k.A, (size_t)n, rocprim::plus<uint64_t>(), s) != hipSuccess)
    return fail("arrival scan");
  // 2. pre-walk: count, offsets, emit
  const uint32_t fr = L.tree_frames;
  const bool spill = fr > 16;
  // per-batch buffers come from the handler's private pool (L.pool: never the
  // device's default pool, whose attributes belong to the application) and go
  // back to it on every return
  struct PoolBuf {
    void *p = nullptr;
    hipStream_t s;
    ~PoolBuf() {
      if (p) (void)hipFreeAsync(p, s);
    }
  } spill_mem{nullptr, s}, item_mem{nullptr, s};
  auto pool_alloc = [&](PoolBuf &b, uint64_t bytes) {
    return hipMallocFromPoolAsync(&b.p, bytes, (hipMemPool_t)L.pool, s) == hipSuccess;
  };
  uint32_t *spill_buf = nullptr;
  const uint64_t pw_threads = (uint64_t)kPrewalkBlocks * kT;
  if (spill) {
    const uint64_t words = (uint64_t)(fr - 8 + 1) *
                           ((L.tree_t64 ? kTreeSpillWords64 : kTreeSpillWords) + (L.tree_wide ? kTreeSpillWide : 0u)) *
                           pw_threads;
    if (!pool_alloc(spill_mem, words * 4)) return fail("spill allocation");
    spill_buf = (uint32_t *)spill_mem.p;
  }
  k.spill = spill_buf;
  // the nodes in LDS (1024-thread workgroups, one per CU at these register
  // counts) when they fit in 96 KB
  k.n_nodes = L.n_nodes;
  const uint32_t lds_nodes = L.n_nodes * 8u;
  const bool ldsn = !L.tree_wide && lds_nodes <= 96u * 1024u ;
  auto launch = [&](auto kern, unsigned long long *w) {
    if (ldsn) {
      (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_nodes);
      hipLaunchKernelGGL(kern, dim3(kPrewalkBlocks / 4), dim3(1024), lds_nodes, s, k, w);
    } else {
      hipLaunchKernelGGL(kern, dim3(kPrewalkBlocks), dim3(kT), 0, s, k, w);
    }
  };
  // the variant: register frames (8 + spill, 16, 8), nodes in LDS, time width
  // (and the error mode: mode B walks draw errors)
  auto pw = [&](auto fr_c, auto spill_c, auto t64_c, auto mb_c, bool emit) {
    constexpr int FRc = decltype(fr_c)::value;
    constexpr bool SP = decltype(spill_c)::value, T6 = decltype(t64_c)::value, MB = decltype(mb_c)::value;
    unsigned long long *w = work + (emit ? 1 : 0);
    if (L.tree_wide) {
      if (emit) launch(k_prewalk<FRc, SP, true, false, T6, MB, true>, w);
      else launch(k_prewalk<FRc, SP, false, false, T6, MB, true>, w);
    } else if (ldsn) {
      if (emit) launch(k_prewalk<FRc, SP, true, true, T6, MB>, w);
      else launch(k_prewalk<FRc, SP, false, true, T6, MB>, w);
    } else {
      if (emit) launch(k_prewalk<FRc, SP, true, false, T6, MB>, w);
      else launch(k_prewalk<FRc, SP, false, false, T6, MB>, w);
    }
  };
  auto prewalk_t = [&](auto t64_c, auto mb_c, bool emit) {
    if (spill) pw(std::integral_constant<int, 8>{}, std::true_type{}, t64_c, mb_c, emit);
    else if (fr > 8) pw(std::integral_constant<int, 16>{}, std::false_type{}, t64_c, mb_c, emit);
    else pw(std::integral_constant<int, 8>{}, std::false_type{}, t64_c, mb_c, emit);
  };
  auto prewalk_m = [&](auto mb_c, bool emit) {
    if (L.tree_t64) prewalk_t(std::true_type{}, mb_c, emit);
    else prewalk_t(std::false_type{}, mb_c, emit);
  };
  auto prewalk = [&](bool emit) {
    if (pl.modeb) prewalk_m(std::true_type{}, emit);
    else prewalk_m(std::false_type{}, emit);
  };
  if (hipMemsetAsync(work, 0, 16, s) != hipSuccess) return fail("memset");
  prewalk(false);
  b = scan_bytes;
  if (rocprim::inclusive_scan(scan_tmp, b, k.cnt, k.tend, (size_t)n, rocprim::plus<uint64_t>(), s) != hipSuccess)
    return fail("item offset scan");
  uint64_t M = 0;
  if (hipMemcpyAsync(&M, k.tend + (n - 1), 8, hipMemcpyDeviceToHost, s) != hipSuccess || sync_s() != hipSuccess)
    return fail("item count read-back");
  if (M >= 0xFFFFFFFFull) {
    err = "DES items: a batch of more than 2^32 - 1 executed invocations (use smaller batches)";
    return 2;
  }
  k.M = M;
  rep.items = M;
  rep.passes = 1;
  // the per-item arrays and the rounds' sort buffers, one allocation
  const uint32_t R = pl.rounds();
  const uint32_t G = (uint32_t)pl.fin_off.size() - 1;
  size_t sort32_bytes = 0, sort64_bytes = 0, sbk_bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, sort32_bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                  (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)M, 0, 32);
  (void)rocprim::radix_sort_pairs(nullptr, sort64_bytes, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                  (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)M, 0, 64);
  (void)rocprim::inclusive_scan_by_key(nullptr, sbk_bytes, (const uint32_t *)nullptr, (const MP *)nullptr,
                                       (MP *)nullptr, (size_t)M, MPThen(), rocprim::equal_to<uint32_t>());
  size_t sop_bytes = 0;
  if (pl.item_bk)
    (void)rocprim::radix_sort_pairs(nullptr, sop_bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                    (const unsigned long long *)nullptr, (unsigned long long *)nullptr,
                                    (size_t)(M * pl.item_bk), 0, 32);
  size_t perm_bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, perm_bytes, rocprim::make_transform_iterator((const uint4 *)nullptr, PosOf()),
                                  (uint32_t *)nullptr, rocprim::make_counting_iterator<uint32_t>(0u),
                                  (uint32_t *)nullptr, (size_t)M, 0, 32);
  const size_t tmp_bytes =
      std::max({sort32_bytes, sort64_bytes, sbk_bytes, sop_bytes, perm_bytes});
  // per duration-table row: the service's worker hold (the queue kernels read no item's position)
  std::vector<uint64_t> row_hold(std::max<size_t>(1, max_row + 1), 0);
  for (const DesPos &q : pl.pos) row_hold[q.row] = q.hold;
  const size_t rows_n = row_hold.size();
  const uint64_t parts[] = {
      M * 4, M * 4, M * 4, M,                                  // ipos ipar itr iown
      M * 8, M * 8, M * 8,                                     // IA IS IF
      M * 8 * k.aw, M * 8 * std::max<uint32_t>(1, k.bw),       // acc bk
      pl.cyclic ? M * 8 * k.aw : 8,                            // acc of the previous pass
      k.bw ? M * k.bw * 4 : 4, k.bw ? M * k.bw * 8 : 8,        // step ops: rounds, (item, step)
      4, pl.cyclic ? M * 4 : 4, 4, 4, M * 4, M * 4,            // (spare) ord (spare spare) qids fids
      M * 8, M * 8, M * 4, M * 4,                              // round: key a/b, val a/b
      M * 4, M * 4, M * 4, M * 4, M * 16, M * 16, M * 4,      // rk a/b, rv a/b, mp in/out, sid
      4, 4, 16,                                                // (k_qscan ticket, spare); ovf: key overflow, no fixed
                                                               // point, look-back fault, step-op count
      96,                                                      // two arrival-range slots; change flag, count
      k.bw ? M * k.bw * 4 : 4, k.bw ? M * k.bw * 8 : 8,        // step ops sorted
      (uint64_t)(R + 1) * 4, (uint64_t)rows_n * 8,              // step-op offsets; hold per row
      M * 4, n * 4, M * 16, 4, 4, 8, M * 4,                    // ihop troot; erec (3 spare); inverse
      (uint64_t)(pl.pos.size() + 1) * 4, (uint64_t)pl.pos.size() * 4, (uint64_t)pl.pos.size() * 4,  // poff qdst fdst
      tmp_bytes,
      M * 2, (n >> chunk_shift(n)) + 1, (n >> chunk_shift(n)) + 1,  // replicas; the two chunk-change maps
      pl.cyclic ? M * 2 : 2,                                    // kept orders' trace chunks
      pl.modeb ? M * 4 : 4,                                     // mode B: failed call step per item
      n + 1, n + 1};                                            // the two per-trace change maps
  uint64_t total = 0;
  for (uint64_t q : parts) total += al256(q ? q : 1);
  if (!pool_alloc(item_mem, total)) return fail("item allocation");
  char *at = (char *)item_mem.p;
  auto carve = [&](uint64_t bytes) {
    char *p = at;
    at += al256(bytes ? bytes : 1);
    return (void *)p;
  };
  k.ipos = (uint32_t *)carve(parts[0]);
  k.ipar = (uint32_t *)carve(parts[1]);
  k.itr = (uint32_t *)carve(parts[2]);
  k.iown = (uint8_t *)carve(parts[3]);
  k.IA = (uint64_t *)carve(parts[4]);
  k.IS = (uint64_t *)carve(parts[5]);
  k.IF = (uint64_t *)carve(parts[6]);
  k.acc = (uint64_t *)carve(parts[7]);
  k.bk = (uint64_t *)carve(parts[8]);
  uint64_t *acc_b = (uint64_t *)carve(parts[9]);
  uint32_t *op_k = (uint32_t *)carve(parts[10]);
  unsigned long long *op_v = (unsigned long long *)carve(parts[11]);
  (void)carve(parts[12]);
  uint32_t *ord = (uint32_t *)carve(parts[13]);  // per sort round: the last sorted order (list indices)
  (void)carve(parts[14]);
  (void)carve(parts[15]);
  uint32_t *qids = (uint32_t *)carve(parts[16]), *fids = (uint32_t *)carve(parts[17]);
  uint64_t *key_a = (uint64_t *)carve(parts[18]), *key_b = (uint64_t *)carve(parts[19]);
  uint32_t *val_a = (uint32_t *)carve(parts[20]), *val_b = (uint32_t *)carve(parts[21]);
  uint32_t *rk_a = (uint32_t *)carve(parts[22]), *rk_b = (uint32_t *)carve(parts[23]);
  uint32_t *rv_a = (uint32_t *)carve(parts[24]), *rv_b = (uint32_t *)carve(parts[25]);
  MP *mp_in = (MP *)carve(parts[26]), *mp_out = (MP *)carve(parts[27]);
  uint32_t *sid = (uint32_t *)carve(parts[28]);
  uint32_t *qticket = (uint32_t *)carve(parts[29]);  // k_qscan's tile tickets (its states: mp_out)
  (void)carve(parts[30]);
  uint32_t *ovf = (uint32_t *)carve(parts[31]);
  k.fault = ovf + 2;
  k.spin_limit = des_spin_limit();
  uint64_t *mm = (uint64_t *)carve(parts[32]);
  uint32_t *chg = (uint32_t *)(mm + 8);  // [0] a quiet pass changed a value, [1] (spare)
  uint32_t *op_k2 = (uint32_t *)carve(parts[33]);
  unsigned long long *op_v2 = (unsigned long long *)carve(parts[34]);
  uint32_t *d_soff = (uint32_t *)carve(parts[35]);
  uint64_t *d_row_hold = (uint64_t *)carve(parts[36]);
  k.ihop = (uint32_t *)carve(parts[37]);
  k.troot = (uint32_t *)carve(parts[38]);
  k.erec = (uint4 *)carve(parts[39]);
  (void)carve(parts[40]);
  (void)carve(parts[41]);
  (void)carve(parts[42]);
  uint32_t *inv = (uint32_t *)carve(parts[43]);
  uint32_t *d_poff = (uint32_t *)carve(parts[44]);
  uint32_t *d_qdst = (uint32_t *)carve(parts[45]);
  uint32_t *d_fdst = (uint32_t *)carve(parts[46]);
  void *tmp = carve(parts[47]);
  k.irep = (uint16_t *)carve(parts[48]);
  k.cshift = chunk_shift(n);
  const uint64_t n_chunks = (n >> k.cshift) + 1;
  uint8_t *chg_a = (uint8_t *)carve(parts[49]), *chg_b = (uint8_t *)carve(parts[50]);
  uint16_t *ordc = (uint16_t *)carve(parts[51]);
  uint32_t *ifst = (uint32_t *)carve(parts[52]);
  k.ifst = pl.modeb ? ifst : nullptr;
  uint8_t *chg_ta = (uint8_t *)carve(parts[53]), *chg_tb = (uint8_t *)carve(parts[54]);
  // the rounds' queues by k_qscan (its keys a - j h need j h < 2^62), else
  // rocPRIM's scan by key over the maps and k_qout (ISIM_FLAG_DES_SCAN_BY_KEY:
  // always, an independent check of k_qscan)
  uint64_t max_hold = 0;
  for (uint64_t hv : row_hold) max_hold = std::max(max_hold, hv);
  const bool qscan = !(L.flags & ISIM_FLAG_DES_SCAN_BY_KEY) &&
                     (max_hold == 0 || M <= (1ull << 62) / max_hold);
  QState *qstate = (QState *)mp_out;  // mp_out's bytes: >= 32 B per 512 items
  uint32_t qepoch = 0, qtbase = 0;
  int rc = 0;
  std::vector<uint32_t> qoff(R + 1), foff(G + 1);
  do {
    static const uint64_t mm_empty[8] = {~0ull, 0ull, 0ull, 0ull, ~0ull, 0ull, 0ull, 0ull};
    if (hipMemsetAsync(ovf, 0, 16, s) != hipSuccess ||
        hipMemcpyAsync(mm, mm_empty, 64, hipMemcpyHostToDevice, s) != hipSuccess) {
      rc = fail("memset");
      break;
    }
    prewalk(true);
    if (hipMemsetAsync(k.terr, 0, n * 4, s) != hipSuccess) {
      rc = fail("memset");
      break;
    }
    // 2b. renumber position-major: ipos = the sorted keys, the rest gathered
    // (keys read from the records, values counted: no key / index arrays)
    {
      size_t tb0 = tmp_bytes;
      if (rocprim::radix_sort_pairs(tmp, tb0, rocprim::make_transform_iterator((const uint4 *)k.erec, PosOf()),
                                    k.ipos, rocprim::make_counting_iterator<uint32_t>(0u), qids, (size_t)M, 0,
                                    bits_for(std::max<size_t>(1, pl.pos.size()) - 1), s) != hipSuccess) {
        rc = fail("position sort");
        break;
      }
    }
    hipLaunchKernelGGL(k_perm_inv, dim3(grid_for(M)), dim3(kT), 0, s, k, qids, inv);
    hipLaunchKernelGGL(k_own, dim3(grid_for(M)), dim3(kT), 0, s, k, (const uint32_t *)inv);
    hipLaunchKernelGGL(k_root500, dim3(grid_for(n)), dim3(kT), 0, s, k);
    hipLaunchKernelGGL(k_perm_apply, dim3(grid_for(M)), dim3(kT), 0, s, k, qids);
    if (pl.modeb) {
      if (hipMemsetAsync(ifst, 0xFF, M * 4, s) != hipSuccess) {
        rc = fail("memset");
        break;
      }
      hipLaunchKernelGGL(k_fail, dim3(grid_for(M)), dim3(kT), 0, s, k);
    }
    hipLaunchKernelGGL(k_roots, dim3(grid_for(n)), dim3(kT), 0, s, k, inv);
    hipLaunchKernelGGL(k_reps, dim3(grid_for(M)), dim3(kT), 0, s, k);
    if (pl.cyclic) {  // the first pass's cut step begins: contention-free callee maxima (k_relmax)
      if (hipMemsetAsync(k.acc, 0, M * 8 * k.aw, s) != hipSuccess) {
        rc = fail("memset");
        break;
      }
      hipLaunchKernelGGL(k_relmax, dim3(grid_for(M)), dim3(kT), 0, s, k, qids, (unsigned long long *)k.acc);
    }
    // 3. buckets
    if (hipMemcpyAsync(d_row_hold, row_hold.data(), rows_n * 8, hipMemcpyHostToDevice, s) != hipSuccess) {
      rc = fail("hold table upload");
      break;
    }
    k.row_hold = d_row_hold;
    // the step-begin ops; each position's item range (k.ipos is sorted)
    hipLaunchKernelGGL(k_bucket_keys, dim3(grid_for(M)), dim3(kT), 0, s, k, op_k, op_v, ovf + 3);
    const uint32_t NP = (uint32_t)pl.pos.size();
    hipLaunchKernelGGL(k_bounds, dim3(grid_for(M + 1)), dim3(kT), 0, s, (const uint32_t *)k.ipos, M, NP, 0u, d_poff);
    uint32_t n_ops = 0;
    std::vector<uint32_t> poff(NP + 1);
    if (hipMemcpyAsync(&n_ops, ovf + 3, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(poff.data(), d_poff, (NP + 1) * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        sync_s() != hipSuccess) {
      rc = fail("bucket read-back");
      break;
    }
    // the rounds' and groups' lists: positions in increasing order within each
    std::vector<uint32_t> qdst(NP), fdst(NP);
    {
      std::vector<uint64_t> qn(R + 1, 0), fn(G + 1, 0);
      for (uint32_t v = 0; v < NP; ++v) {
        qn[pl.item_pos[v].qround + 1] += poff[v + 1] - poff[v];
        fn[pl.item_pos[v].fgroup + 1] += poff[v + 1] - poff[v];
      }
      for (uint32_t r = 0; r < R; ++r) qn[r + 1] += qn[r];
      for (uint32_t g = 0; g < G; ++g) fn[g + 1] += fn[g];
      for (uint32_t r = 0; r <= R; ++r) qoff[r] = (uint32_t)qn[r];
      for (uint32_t g = 0; g <= G; ++g) foff[g] = (uint32_t)fn[g];
      for (uint32_t v = 0; v < NP; ++v) {
        const uint32_t c = poff[v + 1] - poff[v];
        qdst[v] = (uint32_t)qn[pl.item_pos[v].qround];
        qn[pl.item_pos[v].qround] += c;
        fdst[v] = (uint32_t)fn[pl.item_pos[v].fgroup];
        fn[pl.item_pos[v].fgroup] += c;
      }
    }
    if (hipMemcpyAsync(d_qdst, qdst.data(), NP * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d_fdst, fdst.data(), NP * 4, hipMemcpyHostToDevice, s) != hipSuccess) {
      rc = fail("list upload");
      break;
    }
    hipLaunchKernelGGL(k_scatter_ids, dim3(grid_for(M)), dim3(kT), 0, s, k, d_poff, d_qdst, d_fdst, qids, fids);
    size_t tb = tmp_bytes;
    std::vector<uint32_t> soff(R + 1, 0);
    if (n_ops) {
      if (rocprim::radix_sort_pairs(tmp, tb, op_k, op_k2, op_v, op_v2, (size_t)n_ops, 0, bits_for(R), s) != hipSuccess) {
        rc = fail("step-op sort");
        break;
      }
      hipLaunchKernelGGL(k_bounds, dim3(grid_for(n_ops + 1)), dim3(kT), 0, s, op_k2, (uint64_t)n_ops, R, 0u, d_soff);
      if (hipMemcpyAsync(soff.data(), d_soff, (R + 1) * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
          sync_s() != hipSuccess) {
        rc = fail("step-op offsets read-back");
        break;
      }
    }
    const uint32_t row_bits = bits_for(max_row);
    // ISIM_FLAG_DES_TWO_SORTS: always the two-sort queue path (an independent check)
    const bool two_sorts = (L.flags & ISIM_FLAG_DES_TWO_SORTS) != 0;
    constexpr uint32_t stats_span = kQSpan;
    // 4. rounds; a cyclic schedule: quiet passes from zero (a lower bound of
    // every time: the iteration only raises values) until no stored value
    // changes, then the pass that records the statistics (des.hip des_launch)
    // callee maxima: restarted from zero for every item a pass recomputes (a
    // start can move down when the order of a queue changes, so maxima are
    // never carried over); a cut step begin reads the last computed ones
    // (k_acc_init moves them to acc_prev).  After the first pass a quiet pass
    // recomputes only the items of the trace chunks the previous pass
    // changed (k.dcur)
    uint32_t qn = 0;       // k_qarr launches: the arrival-range slot alternates
    // ISIM_FLAG_DES_SORT_ALL: never reuse a kept order (an independent check)
    const bool keep_ord = pl.cyclic && !(L.flags & ISIM_FLAG_DES_SORT_ALL);
    std::vector<uint8_t> have_ord(R, 0);
    std::vector<uint64_t> rlo(R, ~0ull), rhi(R, 0);  // per sort round: its arrival range over the passes
    // k_qscan's states (their epochs: 1, 2, ... per launch) and ticket
    if (qscan && (hipMemsetAsync(qstate, 0, al256((M + 511) / 512 * sizeof(QState)), s) != hipSuccess ||
                  hipMemsetAsync(qticket, 0, 4, s) != hipSuccess)) {
      rc = fail("memset");
      break;
    }
    auto pass = [&](K &kk) {
    hipLaunchKernelGGL(k_acc_init, dim3(grid_for(M)), dim3(kT), 0, s, kk, pl.cyclic ? acc_b : nullptr, kk.acc);
    // items per lane of k_qout / k_fin: runs of one row / position summed
    // before the statistics atomics; a quiet pass records none, and one item
    // per lane gives its finish groups (~0.8 M items on c4d) 16x the waves
    const uint32_t span = kk.quiet ? 1u : stats_span;
    for (uint32_t r = 0; r < R && !rc; ++r) {
      if (soff[r + 1] > soff[r])
        hipLaunchKernelGGL(k_steps, dim3(grid_for(soff[r + 1] - soff[r])), dim3(kT), 0, s, kk, op_v2 + soff[r],
                           (uint64_t)(soff[r + 1] - soff[r]));
      const uint64_t m = qoff[r + 1] - qoff[r];
      if (m) {
        const bool nosort = pl.round_nosort[r] && !two_sorts;
        // (a no-sort round reads no arrival range back; k_qscan computes its arrivals)
        uint64_t *slot = mm + 4 * (qn & 1u), *slot_next = mm + 4 * ((qn + 1) & 1u);
        const bool chk = !nosort && have_ord[r];
        if (!(nosort && qscan)) {
          ++qn;
          hipLaunchKernelGGL(k_qarr, dim3(grid_for(m)), dim3(kT), 0, s, kk, qids + qoff[r], m,
                             (unsigned long long *)slot, (unsigned long long *)slot_next);
          if (chk)  // (its flag in the same slot: one read-back)
            hipLaunchKernelGGL(k_ordchk, dim3(grid_for(m)), dim3(kT), 0, s, kk, (const uint32_t *)(qids + qoff[r]),
                               (const uint32_t *)(ord + qoff[r]), (const uint16_t *)(ordc + qoff[r]), m,
                               (unsigned long long *)slot);
        }
        // a quiet pass after the first: a round whose arrivals all equal the
        // previous pass's keeps its starts (its queues are skipped)
        // (sort rounds only: they read the range back anyway; a sort-free
        // round would pay a stream synchronisation for the check)
        const bool may_skip = kk.quiet && !kk.first && !nosort;
        // range, change flag, kept-order flag (k_ordchk)
        uint64_t hmm[4] = {0, 0, 1, 1};
        if ((!nosort || may_skip) &&
            (hipMemcpyAsync(hmm, slot, 32, hipMemcpyDeviceToHost, s) != hipSuccess || sync_s() != hipSuccess)) {
          rc = fail("arrival range read-back");
          break;
        }
        const bool bad = hmm[3] != 0;
        if (may_skip && !hmm[2]) {
          goto finishes;
        }
        if (!nosort) {
          // the round's arrival range over the passes: the items a pass does
          // not recompute keep their arrivals (a superset range is a valid key)
          rlo[r] = std::min<uint64_t>(rlo[r], hmm[0]);
          rhi[r] = std::max<uint64_t>(rhi[r], hmm[1]);
          hmm[0] = rlo[r];
          hmm[1] = rhi[r];
        }
        const uint32_t ab = bits_for(hmm[1] - hmm[0]);
        tb = tmp_bytes;
        // k_qscan's source of the round's order (k_pairs* only for the two-sort path)
        QSrc qsrc{qids + qoff[r], ord + qoff[r], key_b, val_b, hmm[0], rep_bits, ab, rk_a, rk_b, sid, mp_in};
        int qsk = kQArrays;
        if (chk && !bad) {  // the kept order holds: no sort
          qsk = kQKept;
          if (!qscan)
            hipLaunchKernelGGL(k_pairs1o, dim3(grid_for(m)), dim3(kT), 0, s, kk, m, (const uint32_t *)(ord + qoff[r]),
                               (const uint32_t *)(qids + qoff[r]), rep_bits, rk_a, rk_b, mp_in, sid);
        } else if (nosort) {
          qsk = kQList;
          if (!qscan)  // k_qscan reads the list itself
            hipLaunchKernelGGL(k_pairs0, dim3(grid_for(m)), dim3(kT), 0, s, kk, qids + qoff[r], m, rk_a, rk_b,
                               mp_in, sid);
        } else if (!two_sorts && row_bits + rep_bits + ab <= 64) {
          hipLaunchKernelGGL(k_qkey1, dim3(grid_for(m)), dim3(kT), 0, s, kk, qids + qoff[r], m, hmm[0], rep_bits, ab,
                             key_a, val_a);
          if (rocprim::radix_sort_pairs(tmp, tb, key_a, key_b, val_a, val_b, (size_t)m, 0, row_bits + rep_bits + ab,
                                        s) != hipSuccess) {
            rc = fail("queue sort");
            break;
          }
          hipLaunchKernelGGL(k_tiefix<true>, dim3(grid_for(m)), dim3(kT), 0, s, kk, (const uint64_t *)key_b, val_b, m,
                             (const uint32_t *)(qids + qoff[r]));
          if (keep_ord) {  // the next pass checks this order first
            hipLaunchKernelGGL(k_keep_ord, dim3(grid_for(m)), dim3(kT), 0, s, kk, (const uint32_t *)val_b,
                               (const uint32_t *)(qids + qoff[r]), m, ord + qoff[r], ordc + qoff[r]);
            have_ord[r] = 1;
          }
          qsk = kQSorted;
          if (!qscan)
            hipLaunchKernelGGL(k_pairs1, dim3(grid_for(m)), dim3(kT), 0, s, kk, m, key_b, val_b,
                               (const uint32_t *)(qids + qoff[r]), rep_bits, ab, hmm[0], rk_a, rk_b, mp_in, sid);
        } else {
          hipLaunchKernelGGL(k_qkey2, dim3(grid_for(m)), dim3(kT), 0, s, kk, qids + qoff[r], m, hmm[0], rep_bits,
                             key_a, val_a, ovf);
          if (rocprim::radix_sort_pairs(tmp, tb, key_a, key_b, val_a, val_b, (size_t)m, 0, 64, s) != hipSuccess) {
            rc = fail("arrival sort");
            break;
          }
          // ties of (replica, arrival) by (trace, hop); the stable row sort keeps them
          hipLaunchKernelGGL(k_tiefix<false>, dim3(grid_for(m)), dim3(kT), 0, s, kk, (const uint64_t *)key_b, val_b, m,
                             (const uint32_t *)nullptr);
          hipLaunchKernelGGL(k_rkeys, dim3(grid_for(m)), dim3(kT), 0, s, kk, val_b, m, rk_a, rv_a);
          tb = tmp_bytes;
          if (rocprim::radix_sort_pairs(tmp, tb, rk_a, rk_b, rv_a, rv_b, (size_t)m, 0, row_bits, s) != hipSuccess) {
            rc = fail("service sort");
            break;
          }
          hipLaunchKernelGGL(k_pairs2, dim3(grid_for(m)), dim3(kT), 0, s, kk, m, rk_b, rv_b, key_b, val_b, rep_bits,
                             rk_a, mp_in, sid);
        }
        if (qscan) {
          // 8 items per lane on a large round, 2 otherwise (more tiles to spread)
          const bool big = m >= 2048ull * 512;
          const uint32_t tiles = (uint32_t)((m + (big ? 2047 : 511)) / (big ? 2048 : 512));
          if (qtbase > 0xFFFFFFFFu - tiles) {  // the ticket counter restarts
            if (hipMemsetAsync(qticket, 0, 4, s) != hipSuccess) {
              rc = fail("memset");
              break;
            }
            qtbase = 0;
          }
          ++qepoch;
          static void (*const qs_k[2][4])(K, uint64_t, QSrc, QState *, uint32_t *, uint32_t, uint32_t) = {
              {k_qscan<2, kQArrays>, k_qscan<2, kQList>, k_qscan<2, kQKept>, k_qscan<2, kQSorted>},
              {k_qscan<8, kQArrays>, k_qscan<8, kQList>, k_qscan<8, kQKept>, k_qscan<8, kQSorted>}};
          hipLaunchKernelGGL(qs_k[big][qsk], dim3(tiles), dim3(kT), 0, s, kk, m, qsrc, qstate, qticket, qtbase,
                             qepoch);
          qtbase += tiles;
        } else {
          tb = tmp_bytes;
          if (rocprim::inclusive_scan_by_key(tmp, tb, rk_a, mp_in, mp_out, (size_t)m, MPThen(),
                                             rocprim::equal_to<uint32_t>(), s) != hipSuccess) {
            rc = fail("queue scan");
            break;
          }
          hipLaunchKernelGGL(k_qout, dim3(grid_for((m + span - 1) / span)), dim3(kT), 0, s, kk, m, rk_b, sid,
                             mp_in, mp_out, span);
        }
      }
    finishes:
      for (uint32_t gi = pl.fin_round_off[r]; gi < pl.fin_round_off[r + 1]; ++gi) {
        const uint64_t mg = foff[gi + 1] - foff[gi];
        if (mg) hipLaunchKernelGGL(k_fin, dim3(grid_for((mg + span - 1) / span)), dim3(kT), 0, s, kk,
                                   fids + foff[gi], mg, span);  // grid_for(ceil(mg / span)) blocks of kT: >= the chunks
      }
    }
    };
    if (pl.cyclic) {
      if (hipMemsetAsync(k.IS, 0, M * 8, s) != hipSuccess || hipMemsetAsync(k.IF, 0, M * 8, s) != hipSuccess ||
          (k.bw && hipMemsetAsync(k.bk, 0, M * 8 * k.bw, s) != hipSuccess)) {
        rc = fail("memset");
        break;
      }
      K kq = k;
      kq.quiet = 1;
      kq.acc_prev = acc_b;
      kq.changed = chg;
      uint32_t p = 0;
      for (; p < kMaxPasses && !rc; ++p) {
        uint32_t changed[2] = {1, 0};
        if (hipMemsetAsync(kq.changed, 0, 8, s) != hipSuccess || hipMemsetAsync(chg_b, 0, n_chunks, s) != hipSuccess ||
            hipMemsetAsync(chg_tb, 0, n, s) != hipSuccess) {
          rc = fail("memset");
          break;
        }
        kq.first = p == 0 ? 1u : 0u;
        // the first pass recomputes everything; later ones the chunks the
        // previous pass changed
        kq.dcur = p == 0 ? nullptr : chg_a;
        kq.dnext = chg_b;
        kq.dcur_t = chg_ta;
        kq.dnext_t = chg_tb;
        pass(kq);
        if (rc) break;
        std::swap(chg_a, chg_b);
        std::swap(chg_ta, chg_tb);
        if (hipMemcpyAsync(changed, kq.changed, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
            sync_s() != hipSuccess) {
          rc = fail("fixed-point read-back");
          break;
        }
        rep.passes = p + 2;  // the quiet passes so far and the recording pass
        if (!changed[0]) break;
      }
      if (!rc && p == kMaxPasses) {
        static const uint32_t one = 1;
        if (hipMemcpyAsync(ovf + 1, &one, 4, hipMemcpyHostToDevice, s) != hipSuccess) rc = fail("flag");
      }
      if (rc) break;
    }
    k.acc_prev = acc_b;
    pass(k);  // dcur null: every item
    if (rc) break;
    // 5. records and statistics
    hipLaunchKernelGGL(k_final, dim3(grid_for(n, 1024)), dim3(kT), 0, s, k);
    hipLaunchKernelGGL(k_flag_retry, dim3(1), dim3(1), 0, s, k.stats, ovf);
    if (hipGetLastError() != hipSuccess) {
      rc = fail("kernel launch");
      break;
    }
    // a look-back that gave up (k_qscan) fails the batch loudly: nothing was
    // accumulated (k_final) and the call returns the error
    uint32_t fault = 0;
    if (hipMemcpyAsync(&fault, ovf + 2, 4, hipMemcpyDeviceToHost, s) != hipSuccess || sync_s() != hipSuccess) {
      rc = fail("fault read-back");
      break;
    }
    if (fault)
      rc = fail("a queue scan's look-back gave up waiting for an earlier tile (k_qscan): the batch was not "
                "accumulated");
  } while (0);
  return rc;
}

}  // namespace isim
