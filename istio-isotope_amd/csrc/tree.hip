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

// Row of a duration-table word (row | bucket << 24).  The empty asm hides the
// 24-bit mask from the AMDGPU backend (ROCm 7.2 LLVM): with the mask's known
// bits it formed a u24 multiply for the row offset, dropped the AND, and then
// selected v_mad_u64_u32, which multiplies all 32 bits — the atomic's address
// ran off by bucket x 9 GB (hipErrorIllegalAddress on rows with bucket > 0).
__device__ __forceinline__ uint32_t dur_row(uint32_t w) {
  uint32_t r = w & kDurRowMask;
  asm volatile("" : "+v"(r));
  return r;
}

struct TreeSink {
  uint32_t *cnt;                // LDS [2][n_slots]: executed calls, callee 500s
  unsigned long long *sum200;   // LDS [n_rows]
  uint32_t *dyn;                // LDS bucket tables of the varying rows
  uint64_t *svc_tab;            // HBM duration table, or null (ISIM_FLAG_NO_SVC_DUR)
  uint32_t n_slots;
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
    lds_add(cnt + slot, 1u);
  }
  __device__ __forceinline__ void resp(uint32_t slot, uint32_t roww, uint32_t T, bool st) {
#ifdef TREE_NO_SINK
    return;
#endif
#ifdef ISIM_TREE_DEBUG
    if (slot >= n_slots || (roww & kDurRowMask) >= n_rows) { atomicOr(dbg, 32ull); return; }
#endif
    if (st) lds_add(cnt + n_slots + slot, 1u);
    if (!svc_tab) return;
    const uint32_t row = roww & 0xFFFFu, off = roww >> 16;
    if (off != kTreeStaticRow) {  // the row's LDS bucket table: header b_lo | width << 8
      const uint32_t hdr = dyn[off], lo = hdr & 0xFFu, w = hdr >> 8;
      uint32_t b = prom_bucket(T) - lo;
      b = b < w ? b : w - 1;  // tmin <= T <= tmax keeps it in range; never write past the table
      lds_add(dyn + off + 1u + (st ? w : 0u) + b, 1u);
    }
    if (st) {
      unsigned long long *r = (unsigned long long *)(svc_tab + (uint64_t)dur_row(row) * ISIM_SVC_DUR_WORDS);
      atomicAdd(r + 2 * ISIM_N_PROM + 1, (unsigned long long)T);
    } else {
      lds_add(sum200 + row, (unsigned long long)T);
    }
  }
};

template <bool MODEB, int FRAMES, bool EXTL, bool CONC>
__global__ void __launch_bounds__(kWgThreads, 1)
    isim_tree(const TreeNode *__restrict__ gnodes, isim_trace_rec *__restrict__ records,
              uint64_t *__restrict__ gstats, const uint32_t *__restrict__ slot_tbkt, KParams kp) {
  extern __shared__ __align__(16) unsigned char lds[];
  const uint32_t S = kp.n_slots, R = kp.n_rows, P = kp.n_pos;
  Ctx c{};
  c.records = records;
  c.gstats = gstats;
  c.svc_tab = kp.svc_dur ? gstats + ISIM_ST_SVC_DUR(S) : nullptr;
  c.acc = reinterpret_cast<WgAcc *>(lds);
  c.hist = reinterpret_cast<uint32_t *>(lds + kLdsAccBytes);
  c.cnt = c.hist + kHistWords;
  c.n_slots = S;
  const uint32_t off = tree_lds_nodes_offset(S, R, kp.dyn_words);
  unsigned long long *sum200 = reinterpret_cast<unsigned long long *>(lds + tree_lds_sums_offset(S));
  uint32_t *dyn = reinterpret_cast<uint32_t *>(lds + tree_lds_dyn_offset(S, R));
  TreeNode *nodes = reinterpret_cast<TreeNode *>(lds + off);
  TreeExt *lext = reinterpret_cast<TreeExt *>(lds + off + 16u * P);
  // zero the accumulators (everything before the nodes), copy the tree in
  uint32_t *z = reinterpret_cast<uint32_t *>(lds);
  for (uint32_t i = threadIdx.x; i < off / 4u; i += blockDim.x) z[i] = 0;
  {
    const uint4 *src = reinterpret_cast<const uint4 *>(gnodes);
    uint4 *dst = reinterpret_cast<uint4 *>(nodes);
    for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) dst[i] = src[i];
    if constexpr (EXTL) {
      const uint4 *xs = reinterpret_cast<const uint4 *>(kp.tree_ext);
      uint4 *xd = reinterpret_cast<uint4 *>(lext);
      for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) xd[i] = xs[i];
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < kp.n_dyn; i += blockDim.x) {
    const TreeDynRow d = kp.tree_dyn[i];
    dyn[d.off] = d.b_lo | (d.width << 8);
  }
  __syncthreads();
  TreeSink sink{c.cnt, sum200, dyn, c.svc_tab, S};
#ifdef ISIM_TREE_DEBUG
  sink.n_pos = P;
  sink.n_rows = R;
  sink.dbg = reinterpret_cast<unsigned long long *>(gstats + ISIM_ST_DES_RETRY);
#endif
  const TreeExt *__restrict__ ext = EXTL ? lext : kp.tree_ext;

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
  tw::Lane<FRAMES, MODEB, CONC> L;
  bool active = false;  // the lane holds a trace whose record is not yet written
  uint64_t idx = 0;
  uint64_t a_lat = 0, a_hops = 0, a_err = 0, a_lat500 = 0, a_max = 0, a_notmin = 0;
  uint32_t a_n500 = 0, a_ntr = 0;
  while (true) {
    // responded traces: record, histograms, sums
    const uint64_t fin = ballot(active && L.done);
    if (fin) {
      const bool mine = lane_in(fin);
      const uint64_t lat = L.lat;
      const bool is500 = L.root500;
      if (mine) {
        uint4 r;
        r.x = (uint32_t)lat;
        r.y = 0u;
        r.z = L.hopn;
        r.w = (is500 ? 0x80000000u : 0u) | L.errh;
        if (c.records) *reinterpret_cast<uint4 *>(c.records + idx) = r;
        a_lat += lat;
        a_hops += L.hopn;
        a_err += L.errh;
        a_n500 += is500 ? 1u : 0u;
        a_lat500 += is500 ? lat : 0u;
        a_ntr += 1;
        a_max = lat > a_max ? lat : a_max;
        a_notmin = ~lat > a_notmin ? ~lat : a_notmin;
        active = false;
      }
#ifndef TREE_NO_HIST
      // the latency histograms: one LDS atomic per responding lane (their
      // buckets mostly differ, so a wave-aggregated add would loop per bucket)
      if (mine) {
        lds_add(c.hist + (is500 ? ISIM_N_PROM : 0u) + prom_bucket(lat), 1u);
        const uint32_t l2 = lat == 0 ? 0u : 64u - (uint32_t)__builtin_clzll(lat);
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
    if (active && !L.done) L.step(nodes, ext, sink, kp.seed_lo, kp.seed_hi);
  }
  // the wave's sums into the workgroup accumulators
  {
    const uint64_t s_lat = wave_sum64(a_lat), s_hops = wave_sum64(a_hops), s_err = wave_sum64(a_err);
    const uint64_t s_500 = wave_sum64(a_lat500), s_n500 = wave_sum64(a_n500), s_ntr = wave_sum64(a_ntr);
    const uint64_t mx = wave_max64(a_max), nmn = wave_max64(a_notmin);
    if (lane_id() == 0 && s_ntr) {
      atomicAdd(&c.acc->sum_latency, (unsigned long long)s_lat);
      atomicAdd(&c.acc->sum_hops, (unsigned long long)s_hops);
      atomicAdd(&c.acc->sum_err, (unsigned long long)s_err);
      atomicAdd(&c.acc->n500, (unsigned long long)s_n500);
      atomicAdd(&c.acc->ntr, (unsigned long long)s_ntr);
      atomicAdd(&c.acc->sum_latency500, (unsigned long long)s_500);
      atomicMax(&c.acc->max, (unsigned long long)mx);
      atomicMax(&c.acc->notmin, (unsigned long long)nmn);
    }
  }
  if (lane_id() == 0 && atomicAdd(kp.work + kWorkQueues * kWorkLine, 1ull) == stride - 1) {
    for (uint32_t i = 0; i <= kWorkQueues; ++i) atomicExch(kp.work + i * kWorkLine, 0ull);
  }
  __syncthreads();
  // ---- flush the workgroup's accumulators (coalesced over slots / rows)
  unsigned long long *st = reinterpret_cast<unsigned long long *>(gstats);
  for (uint32_t i = threadIdx.x; i < kHistWords; i += blockDim.x)
    if (c.hist[i]) atomicAdd(st + ISIM_ST_PROM + i, (unsigned long long)c.hist[i]);
  for (uint32_t i = threadIdx.x; i < 2u * S; i += blockDim.x)
    if (c.cnt[i]) atomicAdd(st + ISIM_ST_SITES + i, (unsigned long long)c.cnt[i]);
  if (c.svc_tab) {
    unsigned long long *tab = reinterpret_cast<unsigned long long *>(c.svc_tab);
    for (uint32_t s = threadIdx.x; s < S; s += blockDim.x) {
      const uint32_t w = slot_tbkt[s], bk = w >> 24;
      const uint32_t calls = c.cnt[s], errs = c.cnt[S + s];
      if (bk == kTreeDynBucket || calls == 0) continue;
      unsigned long long *row = tab + (uint64_t)dur_row(w) * ISIM_SVC_DUR_WORDS;
      if (calls != errs) atomicAdd(row + bk, (unsigned long long)(calls - errs));
      if (errs) atomicAdd(row + ISIM_N_PROM + bk, (unsigned long long)errs);
    }
    for (uint32_t r = threadIdx.x; r < R; r += blockDim.x)
      if (sum200[r]) atomicAdd(tab + (uint64_t)r * ISIM_SVC_DUR_WORDS + 2 * ISIM_N_PROM, sum200[r]);
    // the varying rows' bucket tables: one thread per (row, word)
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
      const uint32_t j = i - d.off - 1, code = j >= d.width ? 1u : 0u, b = d.b_lo + j - code * d.width;
      atomicAdd(tab + (uint64_t)dur_row(d.row) * ISIM_SVC_DUR_WORDS + code * ISIM_N_PROM + b, (unsigned long long)v);
    }
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

// Register-stack depths compiled: the smallest that holds the graph's frames;
// TreeExt in LDS when it fits (ext_lds), else read from HBM; walks without
// concurrent steps keep no step maxima (CONC = false).
template <bool EXTL, bool CONC>
static void *tree_pick(bool modeb, uint32_t frames) {
  using namespace dev;
  if (frames <= 4) return modeb ? (void *)&isim_tree<true, 4, EXTL, CONC> : (void *)&isim_tree<false, 4, EXTL, CONC>;
  if (frames <= 8) return modeb ? (void *)&isim_tree<true, 8, EXTL, CONC> : (void *)&isim_tree<false, 8, EXTL, CONC>;
  return modeb ? (void *)&isim_tree<true, 16, EXTL, CONC> : (void *)&isim_tree<false, 16, EXTL, CONC>;
}

void *tree_kernel(bool modeb, uint32_t frames, bool ext_lds, bool conc) {
  if (conc) return ext_lds ? tree_pick<true, true>(modeb, frames) : tree_pick<false, true>(modeb, frames);
  return ext_lds ? tree_pick<true, false>(modeb, frames) : tree_pick<false, false>(modeb, frames);
}

}  // namespace isim
