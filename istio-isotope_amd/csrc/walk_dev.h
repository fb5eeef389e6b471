// Device helpers shared by the walk kernels (walk.hip) and the lane tree
// walk (tree.hip): Philox4x32-10, lane masks, VGPR-lane stacks, histogram
// and counter accumulation, the per-batch epilogue.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernel_abi.h"

namespace isim {
namespace dev {

constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;

struct Ins2 {
  Ins a, b;
};

// a ^ b ^ c in one gfx950 v_bitop3_b32 (LUT 0x96) instead of two v_xor_b32
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ void round1(uint32_t &c0, uint32_t &c1, uint32_t &c2, uint32_t &c3, uint32_t k0,
                                       uint32_t k1) {
  const uint64_t p0 = (uint64_t)M0 * c0;
  const uint64_t p1 = (uint64_t)M1 * c2;
  const uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1, k0);
  const uint32_t n2 = xor3((uint32_t)(p0 >> 32), c3, k1);
  c0 = n0;
  c1 = (uint32_t)p1;
  c2 = n2;
  c3 = (uint32_t)p0;
}

// Philox4x32-10, generic (all counter words per lane).
__device__ __forceinline__ void philox10(uint32_t &c0, uint32_t &c1, uint32_t &c2, uint32_t &c3, uint32_t k0,
                                         uint32_t k1) {
  asm volatile("" : "+s"(k0), "+s"(k1));  // do not hoist the key schedule into 20 SGPRs
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    round1(c0, c1, c2, c3, k0, k1);
    k0 += W0;
    k1 += W1;
  }
}

__device__ __forceinline__ uint64_t ballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }
__device__ __forceinline__ bool lane_in(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ uint32_t popc(uint64_t m) { return (uint32_t)__builtin_popcountll(m); }
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
// v_writelane_b32: no clang builtin on this toolchain, so bind the LLVM
// intrinsic directly (value and lane index are wave-uniform).
__device__ int llvm_writelane(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t wrl(uint32_t v, uint32_t l, uint32_t old) {
  return (uint32_t)llvm_writelane((int)v, (int)l, (int)old);
}
__device__ __forceinline__ uint64_t u64of(uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); }

// A wave-uniform value kept in VGPR lanes (lane d = frame d).
template <typename T>
struct LaneStack;
template <>
struct LaneStack<uint32_t> {
  uint32_t v = 0;
  __device__ __forceinline__ void put(uint32_t d, uint32_t x) { v = wrl(x, d, v); }
  __device__ __forceinline__ uint32_t get(uint32_t d) const { return rdl(v, d); }
};
template <>
struct LaneStack<uint64_t> {
  uint32_t lo = 0, hi = 0;
  __device__ __forceinline__ void put(uint32_t d, uint64_t x) {
    lo = wrl((uint32_t)x, d, lo);
    hi = wrl((uint32_t)(x >> 32), d, hi);
  }
  __device__ __forceinline__ uint64_t get(uint32_t d) const { return u64of(rdl(lo, d), rdl(hi, d)); }
};

// Per-site counter add of a wave-uniform amount by one lane (LDS table, or
// global atomics when the table does not fit).
__device__ __forceinline__ void count(uint64_t *__restrict__ gstats, uint32_t *cnt, uint32_t idx, uint32_t v) {
  if (v == 0) return;
  if (lane_id() == 0) {
    if (cnt) atomicAdd(cnt + idx, v);
    else atomicAdd((unsigned long long *)(gstats + ISIM_ST_SITES + idx), (unsigned long long)v);
  }
}

// service_request_duration_seconds buckets (srv/prometheus/handler.go:26-31):
// bucket = first i with t <= edge_i ms  <=>  ceil(t / 1ms) <= edge_i.
// A 512-byte table of buckets by m = ceil(t / 1 ms) (0..500), built at
// compile time; per-lane lookups hit L1 (the LDS of the lane tree walk is
// full): 7 VALU per duration instead of a 32-compare chain.
struct alignas(16) BucketTable {
  uint8_t b[512];
  constexpr BucketTable() : b() {
    const uint32_t e[32] = {7, 8, 9, 10, 11, 12, 14, 16, 18, 20, 25, 30, 35, 40, 45, 50,
                            60, 70, 80, 90, 100, 120, 140, 160, 180, 200, 250, 300, 350, 400, 450, 500};
    for (uint32_t m = 0; m < 512; ++m) {
      uint32_t k = 0;
      for (uint32_t i = 0; i < 32; ++i) k += e[i] < m ? 1u : 0u;
      b[m] = (uint8_t)k;
    }
  }
};
__device__ constexpr BucketTable kBucketTable{};
__device__ __forceinline__ uint32_t prom_bucket(uint64_t t) {
  if (t > 500000000ull) return 32;
  return kBucketTable.b[((uint32_t)t + 999999u) / 1000000u];  // ceil(t / 1ms) <= 500
}

// Wave-aggregated LDS histogram add: one ds_add per distinct key.
__device__ __forceinline__ void hist_add(uint32_t *h, uint32_t key, uint64_t lanes) {
  while (lanes) {
    const uint32_t leader = (uint32_t)__builtin_ctzll(lanes);
    const uint32_t k = rdl(key, leader);
    const uint64_t m = ballot(key == k) & lanes;
    if (lane_id() == leader) atomicAdd(h + k, popc(m));
    lanes &= ~m;
  }
}

// Wave-aggregated global histogram add (u64 words): one atomic per distinct key.
__device__ __forceinline__ void hist_add_global(uint64_t *h, uint32_t key, uint64_t lanes) {
  while (lanes) {
    const uint32_t leader = (uint32_t)__builtin_ctzll(lanes);
    const uint32_t k = rdl(key, leader);
    const uint64_t m = ballot(key == k) & lanes;
    if (lane_id() == leader) atomicAdd((unsigned long long *)(h + k), (unsigned long long)popc(m));
    lanes &= ~m;
  }
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint64_t wave_max64(uint64_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint64_t w = __shfl_xor(v, o, 64);
    v = w > v ? w : v;
  }
  return v;
}

// Workgroup-shared accumulators (LDS).
struct WgAcc {
  unsigned long long sum_latency, sum_hops, sum_err, n500, ntr, notmin, max;
  unsigned long long sum_latency500;  // tree walk (kind 7): the entry's 500 duration sum
};
static_assert(sizeof(WgAcc) <= kLdsAccBytes, "WgAcc must fit its LDS slot");

struct Ctx {
  const Ins *__restrict__ prog;
  isim_trace_rec *__restrict__ records;
  uint64_t *__restrict__ gstats;
  const uint32_t *__restrict__ dur;  // dynamic walks: per-slot duration-table words, or null
  uint64_t *svc_tab;                 // dynamic walks: per-service duration table (HBM), or null
  uint32_t root_dur;
  uint32_t *cnt;   // LDS per-site counters or null
  uint32_t *hist;  // LDS histograms
  WgAcc *acc;      // LDS accumulators
  uint32_t n_slots;
  uint32_t k0, k1;
};

// Per-batch epilogue: record, histograms, sums (SUM500: also the latency sum
// of the traces whose entry responded 500).
template <bool SUM500 = false>
__device__ __forceinline__ void finish_batch(const Ctx &c, uint64_t idx, bool valid, uint64_t all, uint64_t lat,
                                             uint32_t hops, uint64_t root_st, uint32_t errh) {
  const bool is500 = lane_in(root_st);
  if (c.records != nullptr && valid) {
    uint4 r;
    r.x = (uint32_t)lat;
    r.y = (uint32_t)(lat >> 32);
    r.z = hops;
    r.w = (is500 ? 0x80000000u : 0u) | errh;
    *reinterpret_cast<uint4 *>(c.records + idx) = r;
  }
  hist_add(c.hist, (is500 ? ISIM_N_PROM : 0u) + prom_bucket(lat), all);
  const uint32_t l2 = lat == 0 ? 0u : 64u - (uint32_t)__builtin_clzll(lat);
  hist_add(c.hist + 2 * ISIM_N_PROM, (is500 ? ISIM_N_LOG2 : 0u) + l2, all);
  const uint64_t s_lat = wave_sum64(valid ? lat : 0);
  const uint64_t s_hops = wave_sum64(valid ? (uint64_t)hops : 0);
  const uint64_t s_err = wave_sum64(valid ? (uint64_t)errh : 0);
  const uint64_t mx = wave_max64(valid ? lat : 0);
  const uint64_t nmn = wave_max64(valid ? ~lat : 0);
  const uint64_t s500 = SUM500 && (root_st & all) ? wave_sum64(valid && is500 ? lat : 0) : 0;
  if (lane_id() == 0) {
    if (SUM500 && s500) atomicAdd(&c.acc->sum_latency500, (unsigned long long)s500);
    atomicAdd(&c.acc->sum_latency, (unsigned long long)s_lat);
    atomicAdd(&c.acc->sum_hops, (unsigned long long)s_hops);
    atomicAdd(&c.acc->sum_err, (unsigned long long)s_err);
    atomicAdd(&c.acc->n500, (unsigned long long)popc(root_st & all));
    atomicAdd(&c.acc->ntr, (unsigned long long)popc(all));
    atomicMax(&c.acc->max, (unsigned long long)mx);
    atomicMax(&c.acc->notmin, (unsigned long long)nmn);
  }
}

}  // namespace dev
}  // namespace isim
