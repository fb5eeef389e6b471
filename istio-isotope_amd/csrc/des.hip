// Per-replica worker-pool DES on gfx950: exact,
// level-synchronous over a batch of N traces.
//
//   arrivals   A[t] = sum of exponential inter-arrival times (Philox draw,
//              integer inverse CDF) — a block scan + a scan of block sums
//   down pass  per queue round: the replica queue of a position's service is
//              FIFO over its arrivals a(v,t) = S(parent,t) + off(v), which are
//              in trace order, so the start times are one
//              max-plus scan over t:  fin_t = max(fin_{t-1}, a_t) + hold,
//              S_t = fin_t - hold (per replica for replicated services).
//              Wide groups: one workgroup per position; narrow groups: chunks
//              of a position chained by a decoupled look-back.  Leaves finish
//              here (F = S + script time, status, duration).
//   up pass    finish groups from the deepest, (position, trace-range)
//              blocks: F = max(S + floor, max_c F(c)) + post, status (own
//              Philox draw; mode B ORs the children's), duration F - a(v,t)
//              into the per-service histogram.
//   finalize   latency F(entry), records and the stats header.
//
// Rows W[position][trace] (and the step-begin rows BK) hold times RELATIVE to
// the arrival of the trace's GROUP, G_t = A[t & ~63] (64 consecutive traces,
// round 3): every value of trace t lies in [A_t - G_t, A_t - G_t + latency_t].
// A queue scan then needs no per-trace arrival time (its keys are G + row +
// off - t hold, the wave's groups' bases are 4 scalars), and within one wave
// the keys relative to the wave's first key fit 32 bits (down1_chunk_n32).
// Narrow rows are u32 (status in bit 31), so a batch whose latencies plus 63
// inter-arrival gaps stay below 2^31 ns (2.1 s) moves 4 B per value; a value that does not fit sets
// the overflow flag, the batch's statistics (staged in the workspace) are
// then dropped and ISIM_ST_DES_RETRY counts it, to be rerun with u64 rows
// (ISIM_DES_FLAG_WIDE; isim_serve_des does that itself).  Bytes per
// (position, trace), narrow: queue pass 4 R + 4 W, up pass 4 R (S) + 4 R
// (arrival row) + 4 R per child + 4 W.
#include <atomic>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <rocprim/device/device_radix_sort.hpp>

#include "des.h"
#ifndef ISIM_DES_N32_FOLD
#define ISIM_DES_N32_FOLD 1  // 32-bit queue finish: waits summed in pairs, duration sums derived, 500s under one branch
#endif
#ifndef ISIM_NT_ROWS
#define ISIM_NT_ROWS 1  // row stores of fused leaves and finishes nontemporal: keep L2 for the A_t re-reads
#endif
#include "kernel_abi.h"

namespace isim {
void *stream_calls_kernel();
namespace dev {

constexpr uint32_t kDesPer = 8;                   // traces per thread in the arrivals
constexpr uint32_t kDesThreads = 1024;
constexpr uint32_t kDesOvfFault = 4u;  // ovf bit: a look-back gave up (the batch fails)
constexpr uint32_t kDesChunk = kDesPer * kDesThreads;  // 8192 traces per arrivals chunk
constexpr uint32_t kPer = 4;                           // consecutive traces per thread in the row passes
constexpr uint32_t kDownChunk = kPer * kDesThreads;    // traces per down-pass chunk
#ifndef ISIM_DES_CHAIN_BELOW
#define ISIM_DES_CHAIN_BELOW 256  // positions per launch below which the chained scan is used
#endif
constexpr uint32_t kDesUpThreads = 256;

// sort keys of a service with `reps` replicas: replica << shift | arrival,
// shift = 64 - bits(reps - 1) (arrivals below 2^shift ns: >= 2^48 ns for up
// to 65536 replicas; the host checks the batch's arrival span)
__device__ __forceinline__ uint32_t rep_bits(uint32_t reps) { return reps > 1 ? 32u - __builtin_clz(reps - 1u) : 0u; }
#ifndef ISIM_DES_DOWN_THREADS
#define ISIM_DES_DOWN_THREADS 256  // round 3: 512 -> 256 threads per queue-pass workgroup, 36.9 -> 36.4 ms per c5 step
#endif
constexpr uint32_t kDownThreads = ISIM_DES_DOWN_THREADS;  // one-workgroup-per-position queue pass
#ifndef ISIM_DES_MIX
#define ISIM_DES_MIX 1  // fused and other single-replica positions of a round in one queue launch
#endif
#ifndef ISIM_DES_FIN_BLOCKS
#define ISIM_DES_FIN_BLOCKS 512  // des_finalize workgroups (each flushes the stats header by atomics; 2048 -> 512: -0.05 ms)
#endif
#ifndef ISIM_DES_MAX_SPLITS
#define ISIM_DES_MAX_SPLITS 256u  // (position x trace-range) blocks per position (uncapped -> 256: 35.5 -> 34.8 ms per c5 step)
#endif
#ifndef ISIM_DES_SPLIT_TARGET
#define ISIM_DES_SPLIT_TARGET 8192  // (position x trace-range) blocks per up / step-begin launch
#endif
#ifndef ISIM_DES_PIPE
#define ISIM_DES_PIPE 1  // runs of single-replica queue rounds in one pipelined launch
#endif
#ifndef ISIM_DES_DOWN_WAVES
#define ISIM_DES_DOWN_WAVES 6  // waves per SIMD the one-workgroup-per-position pass is compiled for
#endif

__constant__ int32_t c_ln[257] = {
#include "des_ln_table.inc"
};

__device__ __forceinline__ uint32_t des_xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Philox4x32-10 (Random123), counter (t_lo, t_hi, w2, w3), key (k0, k1)
__device__ __forceinline__ void des_round(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
  const uint32_t n0 = des_xor3((uint32_t)(p1 >> 32), c[1], k0);
  const uint32_t n2 = des_xor3((uint32_t)(p0 >> 32), c[3], k1);
  c[0] = n0;
  c[1] = (uint32_t)p1;
  c[2] = n2;
  c[3] = (uint32_t)p0;
}
__device__ __forceinline__ void des_philox(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    des_round(c, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__device__ __forceinline__ uint32_t des_draw(uint64_t t, uint32_t w2, uint32_t w3, uint32_t word, uint32_t k0,
                                             uint32_t k1) {
  uint32_t c[4] = {(uint32_t)t, (uint32_t)(t >> 32), w2, w3};
  des_philox(c, k0, k1);
  return word == 0 ? c[0] : word == 1 ? c[1] : word == 2 ? c[2] : c[3];
}

// -ln(w / 2^24) in Q24, w = (u >> 8) + 1 (des.h / DESIGN §10.2)
__device__ __forceinline__ uint64_t des_exp_q24(uint32_t u) {
  const uint32_t w = (u >> 8) + 1u;
  const int e = 31 - __builtin_clz(w);
  const uint32_t f = (w << (24 - e)) & 0xFFFFFFu;
  const uint32_t idx = f >> 16, rem = f & 0xFFFFu;
  const int64_t lnm = c_ln[idx] + ((((int64_t)c_ln[idx + 1] - c_ln[idx]) * (int64_t)rem) >> 16);
  return (uint64_t)(24 * kLn2Q24 - ((int64_t)e * kLn2Q24 + lnm));
}

// Prometheus duration bucket (prometheus/handler.go:26-35): the first edge
// >= t.  The edges are whole milliseconds in six arithmetic runs (7..12 by 1,
// 14..20 by 2, 25..50 by 5, 60..100 by 10, 120..200 by 20, 250..500 by 50), so
// with m = ceil(t / 1 ms) (t <= e ms  <=>  m <= e) the bucket is the run's
// base + ceil((m - run start) / step).  The kernels look m up in a 501-byte
// LDS table built from this formula (des_bucket_lut: 7 VALU per duration
// instead of 57).
__host__ __device__ constexpr uint32_t des_prom_bucket_m(uint32_t m) {
  const uint32_t lo = m <= 12 ? 7 : m <= 20 ? 12 : m <= 50 ? 20 : m <= 100 ? 50 : m <= 200 ? 100 : 200;
  const uint32_t base = m <= 12 ? 0 : m <= 20 ? 5 : m <= 50 ? 9 : m <= 100 ? 15 : m <= 200 ? 20 : 25;
  const uint32_t d = m <= 12 ? 1 : m <= 20 ? 2 : m <= 50 ? 5 : m <= 100 ? 10 : m <= 200 ? 20 : 50;
  // ceil(65536 / d): exact quotients for numerators below 2^9
  const uint32_t M = m <= 12 ? 65536 : m <= 20 ? 32768 : m <= 50 ? 13108 : m <= 100 ? 6554 : m <= 200 ? 3277 : 1311;
  const uint32_t n = m > lo ? m - lo : 0;
  return base + (((n + d - 1) * M) >> 16);
}
constexpr uint32_t kBucketLut = 502;  // m = ceil(t / 1 ms) in 0..500; 501: above 500 ms (+Inf)
constexpr uint32_t kBucketLutWords = 128;
struct DesBucketLut {
  uint32_t w[kBucketLutWords];  // byte m of the table: the bucket of m (m <= 501), little-endian
  constexpr DesBucketLut() : w() {
    for (uint32_t m = 0; m < 4 * kBucketLutWords; ++m)
      w[m / 4] |= (m < kBucketLut ? des_prom_bucket_m(m) : 32u) << (8 * (m % 4));
  }
};
__device__ constexpr DesBucketLut kDesBucketLut{};
// copies the table into the workgroup's LDS (the caller's barrier publishes
// it): one 4-byte word per thread instead of computing 502 entries
__device__ __forceinline__ void des_bucket_lut_init(uint8_t *lut) {
  for (uint32_t i = threadIdx.x; i < kBucketLutWords; i += blockDim.x)
    reinterpret_cast<uint32_t *>(lut)[i] = kDesBucketLut.w[i];
}
__device__ __forceinline__ uint32_t des_prom_bucket32(const uint8_t *lut, uint32_t t) {
  const uint32_t c = t < 500000001u ? t : 500000001u;  // v_min_u32
  return lut[(c + 999999u) / 1000000u];
}
__device__ __forceinline__ uint32_t des_prom_bucket(const uint8_t *lut, uint64_t t) {
  const uint32_t c = (uint32_t)(t < 500000001ull ? t : 500000001ull);  // branch-free: entry 501 is the +Inf bucket
  return lut[(c + 999999u) / 1000000u];
}

struct ChainState;

struct DesK {
  const DesPos *pos;
  const DesPosExt *ext;
  const DesStep *steps;
  const uint32_t *child;
  const uint32_t *level_pos;  // the positions of the launch (fast queue or finish group)
  const uint32_t *arr_ops;    // BK rows of the launch (step begins)
  void *BK;                   // [steps][ld] row type T
  void *W;                    // [n_pos][ld] row type T: starts S
  void *WF;                   // [n_pos][ld] row type T: finishes F | status (separate rows, so a
                              // fixed-point pass reads last pass's F while S is being rewritten)
  uint64_t *A;                // [N] absolute arrival times
  uint32_t *E;                // [N] per-trace 500 count
  uint64_t *blk;
  uint64_t *stats;            // narrow rows: the staging copy (des_commit)
  uint64_t *table;            // [rows][ISIM_DES_ROW_WORDS] (staged likewise)
  isim_trace_rec *records;
  uint32_t *ovf;              // bit 0: a 32-bit row value reached 2^31; bit 1: no fixed point;
                              // kDesOvfFault: a look-back gave up (the batch is dropped as a fault)
  uint32_t spin_limit;        // look-back polls before that fault (des_spin_limit)
  uint32_t *changed;          // fixed-point passes: set when a stored row value changes (null: no tracking)
  uint32_t quiet;             // fixed-point passes before the last: no statistics
  const uint32_t *stbits;     // own error status of (position, trace): bit t%32 of word [v][t/32]
  uint32_t st_wpr;            // words per status row
  uint64_t N, trace_begin, mean_ns;
  uint64_t ld;                // row stride in traces: N rounded up to 16 (64-B aligned rows)
  uint32_t k0, k1;
  uint32_t n_pos, n_slots;
  uint32_t level_begin, splits;
  uint32_t modeb, n_blk;
  // sort path: the service being queued and its sorted arrivals
  const uint32_t *sort_pos;
  DesSortSvc svc;
  const uint64_t *skeys;
  const uint32_t *svals;
  uint64_t *keys;
  uint32_t *vals;
  // chained down pass
  ChainState *chain;
  uint32_t *chain_ticket;     // this launch's ticket counter
  uint32_t n_chunks;
  // pipelined down pass
  const uint32_t *pipe_dep;   // per level_pos entry: the position it waits on (kDesNone: none)
  uint32_t *prog;             // [n_pos] chunks of a position's start row published (zeroed per pass)
};

// ---- rows: u32 (narrow) or u64, times relative to A_t, status in the top bit
template <typename T>
struct Row {
  static constexpr uint32_t kTop = 8 * sizeof(T) - 1;
  static constexpr uint64_t kSt = 1ull << kTop;
  static constexpr uint64_t kMask = kSt - 1;
  // narrow rows hold values below 2^31 (the status bit stays free)
  __device__ static bool fits(uint64_t v) { return sizeof(T) == 8 || v < kSt; }
};

template <typename T>
__device__ __forceinline__ T *row(void *base, uint64_t ld, uint32_t r) {
  return reinterpret_cast<T *>(base) + (uint64_t)r * ld;
}

// four consecutive values at a 16-B aligned index
template <typename T>
__device__ __forceinline__ void load4(const T *p, uint64_t (&x)[kPer]) {
  if constexpr (sizeof(T) == 4) {
    const uint4 v = *reinterpret_cast<const uint4 *>(p);
    x[0] = v.x;
    x[1] = v.y;
    x[2] = v.z;
    x[3] = v.w;
  } else {
    const ulonglong2 a = reinterpret_cast<const ulonglong2 *>(p)[0];
    const ulonglong2 b = reinterpret_cast<const ulonglong2 *>(p)[1];
    x[0] = a.x;
    x[1] = a.y;
    x[2] = b.x;
    x[3] = b.y;
  }
}
template <typename T>
__device__ __forceinline__ void store4(T *p, const uint64_t (&x)[kPer]) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<uint4 *>(p) = make_uint4((uint32_t)x[0], (uint32_t)x[1], (uint32_t)x[2], (uint32_t)x[3]);
  } else {
    reinterpret_cast<ulonglong2 *>(p)[0] = make_ulonglong2(x[0], x[1]);
    reinterpret_cast<ulonglong2 *>(p)[1] = make_ulonglong2(x[2], x[3]);
  }
}
// values [base, base+4) of a row, zero past n (vector load when whole)
template <typename T>
__device__ __forceinline__ void load4n(const T *p, uint64_t base, uint64_t n, uint64_t (&x)[kPer]) {
  if (base + kPer <= n) {
    load4<T>(p + base, x);
  } else {
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) x[i] = base + i < n ? (uint64_t)p[base + i] : 0;
  }
}
template <typename T>
__device__ __forceinline__ void store4t(T *p, uint64_t base, uint64_t n, const T (&x)[kPer]) {
  if (base + kPer <= n) {
    if constexpr (sizeof(T) == 4) {
#if ISIM_NT_ROWS
      typedef uint32_t v4u __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(v4u{x[0], x[1], x[2], x[3]}, reinterpret_cast<v4u *>(p + base));
#else
      *reinterpret_cast<uint4 *>(p + base) = make_uint4(x[0], x[1], x[2], x[3]);
#endif
    } else {
      reinterpret_cast<ulonglong2 *>(p + base)[0] = make_ulonglong2(x[0], x[1]);
      reinterpret_cast<ulonglong2 *>(p + base)[1] = make_ulonglong2(x[2], x[3]);
    }
  } else {
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i)
      if (base + i < n) p[base + i] = x[i];
  }
}
template <typename T>
__device__ __forceinline__ void store4n(T *p, uint64_t base, uint64_t n, const uint64_t (&x)[kPer]) {
  if (base + kPer <= n) {
    store4<T>(p + base, x);
  } else {
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i)
      if (base + i < n) p[base + i] = (T)x[i];
  }
}
// the same in the row type (no widening: 4 VGPRs per u32 row)
template <typename T>
__device__ __forceinline__ void load4t(const T *p, uint64_t base, uint64_t n, T (&x)[kPer]) {
  if (base + kPer <= n) {
    if constexpr (sizeof(T) == 4) {
      const uint4 v = *reinterpret_cast<const uint4 *>(p + base);
      x[0] = v.x;
      x[1] = v.y;
      x[2] = v.z;
      x[3] = v.w;
    } else {
      const ulonglong2 a = reinterpret_cast<const ulonglong2 *>(p + base)[0];
      const ulonglong2 b = reinterpret_cast<const ulonglong2 *>(p + base)[1];
      x[0] = a.x;
      x[1] = a.y;
      x[2] = b.x;
      x[3] = b.y;
    }
  } else {
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) x[i] = base + i < n ? p[base + i] : (T)0;
  }
}
__device__ __forceinline__ void load4a(const uint64_t *p, uint64_t base, uint64_t n, uint64_t (&x)[kPer]);

// stores of row values; in fixed-point passes a changed value is flagged
template <typename T>
__device__ __forceinline__ void track4(const DesK &k, const T *p, uint64_t base, uint64_t n, const T (&x)[kPer]) {
  if (!k.changed) return;
  T o[kPer];
  load4t<T>(p, base, n, o);
  bool d = false;
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) d |= base + i < n && o[i] != x[i];
  if (d) atomicOr(k.changed, 1u);
}
template <typename T>
__device__ __forceinline__ void track1(const DesK &k, const T *p, T x) {
  if (k.changed && *p != x) atomicOr(k.changed, 1u);
}

__device__ __forceinline__ void load4a(const uint64_t *p, uint64_t base, uint64_t n, uint64_t (&x)[kPer]) {
  load4n<uint64_t>(p, base, n, x);
}

__device__ __forceinline__ void flag_overflow(const DesK &k, bool bad) {
  if (bad) atomicOr(k.ovf, 1u);
}

// the time every row value of trace t is relative to: its group's first arrival
constexpr uint32_t kN32 = kDesN32Per;            // consecutive traces per thread in the 32-bit-key queue chunks
// pipe_body's callers and callees hand chunks off by chunk INDEX (st_flag /
// the wait on a chunk), and the 32-bit and 64-bit branches step through
// chunks of kN32 and kPer traces per thread: the indices only name the same
// traces while both sizes agree.
static_assert(kN32 == kPer, "32-bit and 64-bit queue chunks must cover the same traces");
constexpr uint64_t kDesGrp = kDesGroupTraces;     // a trace group = one DPP row of the 32-bit-key queue pass
constexpr uint64_t kN32HoldMax = kDesN32HoldMax;  // (t - t_g) h < 2^31
__device__ __forceinline__ uint64_t des_gbase(const DesK &k, uint64_t t) { return k.A[t & ~(kDesGrp - 1)]; }

// relative arrival of position v (pp = pos[v]) for trace t
template <typename T>
__device__ __forceinline__ uint64_t des_arrival(const DesK &k, uint32_t v, const DesPos &pp, uint64_t t) {
  if (pp.parent == kDesNoParent) return k.A[t] - des_gbase(k, t);
  const uint32_t b = k.ext[v].bk_in;
  const T *r = b == kDesNone ? row<T>(k.W, k.ld, pp.parent) : row<T>(k.BK, k.ld, b);
  return (uint64_t)r[t] + pp.off;
}

// the row a position's arrivals are read from (null: the entry, arrival 0)
template <typename T>
__device__ __forceinline__ const T *arrival_row(const DesK &k, uint32_t v, const DesPos &pp) {
  if (pp.parent == kDesNoParent) return nullptr;
  const uint32_t b = k.ext[v].bk_in;
  return b == kDesNone ? row<T>(k.W, k.ld, pp.parent) : row<T>(k.BK, k.ld, b);
}

// (B, C) represents x -> max(x + B, C); `then` composes a after b.
struct MaxPlus {
  uint64_t B, C;
};
__device__ __forceinline__ MaxPlus mp_then(MaxPlus first, MaxPlus second) {
  const uint64_t c = first.C + second.B;
  return {first.B + second.B, c > second.C ? c : second.C};
}

// Inclusive block scan of MaxPlus over kDesThreads threads (wave shuffles +
// one LDS pass over the 16 wave totals).
template <uint32_t NT = kDesThreads>
__device__ __forceinline__ MaxPlus mp_block_scan(MaxPlus v, MaxPlus *wtot) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    MaxPlus o;
    o.B = __shfl_up(v.B, d, 64);
    o.C = __shfl_up(v.C, d, 64);
    if (lane >= d) v = mp_then(o, v);
  }
  if (lane == 63) wtot[wave] = v;
  __syncthreads();
  if (wave == 0) {
    MaxPlus w = lane < NT / 64 ? wtot[lane] : MaxPlus{0, 0};
#pragma unroll
    for (uint32_t d = 1; d < NT / 64; d <<= 1) {
      MaxPlus o;
      o.B = __shfl_up(w.B, d, 64);
      o.C = __shfl_up(w.C, d, 64);
      if (lane >= d) w = mp_then(o, w);
    }
    if (lane < NT / 64) wtot[lane] = w;
  }
  __syncthreads();
  if (wave > 0) v = mp_then(wtot[wave - 1], v);
  __syncthreads();  // wtot is reused by the next call
  return v;
}

__device__ __forceinline__ uint64_t block_scan_add(uint64_t v, uint64_t *wtot, uint64_t &total) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  if (lane == 63) wtot[wave] = v;
  __syncthreads();
  if (wave == 0) {
    uint64_t w = lane < kDesThreads / 64 ? wtot[lane] : 0;
#pragma unroll
    for (uint32_t d = 1; d < kDesThreads / 64; d <<= 1) {
      const uint64_t o = __shfl_up(w, d, 64);
      if (lane >= d) w += o;
    }
    if (lane < kDesThreads / 64) wtot[lane] = w;
  }
  __syncthreads();
  if (wave > 0) v += wtot[wave - 1];
  total = wtot[kDesThreads / 64 - 1];
  __syncthreads();
  return v;  // inclusive
}

// ---- single-replica queues in closed form.  A FIFO worker with hold h fed
// arrivals a_t in trace order starts trace t at
//   S_t = max(S_{t-1} + h, a_t) = t h + max_{s <= t} (a_s - s h)
// (an idle worker at time 0 contributes 0), so the queue is ONE running max
// of the signed keys a_t - t h: a wave max-scan by DPP row shifts and row
// broadcasts, wave totals through LDS, the carry across chunks a running max
// (the host bounds n_traces x hold below 2^62, api.hip).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ int64_t dpp_i64(int64_t old, int64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)old, (int)(uint32_t)v, CTRL, ROW_MASK,
                                                           0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)((uint64_t)old >> 32),
                                                           (int)(uint32_t)((uint64_t)v >> 32), CTRL, ROW_MASK, 0xF,
                                                           false);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int64_t max_i64(int64_t a, int64_t b) { return a > b ? a : b; }
constexpr int64_t kKeyMin = INT64_MIN;
// a lane's value moved by a full-mask DPP control, 0 where the source lane
// does not exist (bound_ctrl: no register to preset)
template <int CTRL>
__device__ __forceinline__ int64_t dpp0_i64(int64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xF, 0xF, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)((uint64_t)v >> 32), CTRL, 0xF, 0xF, true);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
// inclusive max-scan over the wave's 64 lanes of max(0, v): every prefix the
// queues need is at least 0 (the idle start), so lanes past an edge read 0
__device__ __forceinline__ int64_t wave_max_scan(int64_t v) {
  v = max_i64(v, dpp0_i64<0x111>(v));              // row_shr:1
  v = max_i64(v, dpp0_i64<0x112>(v));              // row_shr:2
  v = max_i64(v, dpp0_i64<0x114>(v));              // row_shr:4
  v = max_i64(v, dpp0_i64<0x118>(v));              // row_shr:8
  v = max_i64(v, dpp_i64<0x142, 0xA>(v, v));       // row_bcast:15 into rows 1, 3 (rows 0, 2 keep v)
  v = max_i64(v, dpp_i64<0x143, 0xC>(v, v));       // row_bcast:31 into rows 2, 3
  return v;
}
// the previous lane's value (lane 0: 0)
__device__ __forceinline__ int64_t wave_shr1(int64_t v) { return dpp0_i64<0x138>(v); }
__device__ __forceinline__ int64_t read_lane(int64_t v, uint32_t l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), (int)l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
// the block's wave totals (LDS, NW <= 16): pre = max(carry, totals of the
// waves before `wave`), carry = max(carry, all totals); both wave-uniform
template <uint32_t NW>
__device__ __forceinline__ void fold_totals(const int64_t *wtot, uint32_t wave, int64_t &carry, int64_t &pre) {
  static_assert(NW >= 2 && NW <= 16, "one DPP row of wave totals");
  const uint32_t lane = threadIdx.x & 63u;
  int64_t v = lane < NW ? wtot[lane] : 0;  // totals are >= 0 (wave_max_scan)
  v = max_i64(v, dpp0_i64<0x111>(v));
  v = max_i64(v, dpp0_i64<0x112>(v));
  v = max_i64(v, dpp0_i64<0x114>(v));
  if constexpr (NW > 8) v = max_i64(v, dpp0_i64<0x118>(v));
  const int64_t before = wave ? read_lane(v, wave - 1) : kKeyMin;
  pre = max_i64(carry, before);
  carry = max_i64(carry, read_lane(v, NW - 1));
}
// the keys a_t - t h of this thread's (up to) 4 traces from `base`
// (kKeyMin past N) and their largest
template <bool FULL>
__device__ __forceinline__ int64_t queue_keys(const uint64_t (&a)[kPer], uint64_t base, uint64_t N, uint64_t hold,
                                              int64_t (&key)[kPer]) {
  int64_t kt = kKeyMin;
  uint64_t th = base * hold;
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    key[i] = FULL || base + i < N ? (int64_t)(a[i] - th) : kKeyMin;
    kt = max_i64(kt, key[i]);
    th += hold;
  }
  return kt;
}

// ---- arrivals: per chunk inclusive prefix of the inter-arrival times
__global__ void __launch_bounds__(kDesThreads) des_arrivals(DesK k) {
  __shared__ uint64_t wtot[kDesThreads / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kDesChunk + (uint64_t)threadIdx.x * kDesPer;
  uint64_t x[kDesPer], s = 0;
#pragma unroll
  for (uint32_t i = 0; i < kDesPer; ++i) {
    const uint64_t t = base + i;
    x[i] = 0;
    if (t < k.N) {
      const uint32_t u = des_draw(k.trace_begin + t, 0u, 0x80000001u, 0, k.k0, k.k1);
      x[i] = (k.mean_ns * des_exp_q24(u)) >> 24;
    }
    s += x[i];
  }
  uint64_t total;
  uint64_t run = block_scan_add(s, wtot, total) - s;
#pragma unroll
  for (uint32_t i = 0; i < kDesPer; ++i) {
    run += x[i];
    if (base + i < k.N) k.A[base + i] = run;
  }
  if (threadIdx.x == 0) k.blk[blockIdx.x] = total;
}

// exclusive scan of the chunk totals (one workgroup)
__global__ void __launch_bounds__(kDesThreads) des_scan_blocks(DesK k) {
  __shared__ uint64_t wtot[kDesThreads / 64];
  uint64_t carry = 0;
  for (uint32_t b0 = 0; b0 < k.n_blk; b0 += kDesThreads) {
    const uint32_t b = b0 + threadIdx.x;
    const uint64_t v = b < k.n_blk ? k.blk[b] : 0;
    uint64_t total;
    const uint64_t inc = block_scan_add(v, wtot, total);
    if (b < k.n_blk) k.blk[b] = carry + inc - v;
    carry += total;
  }
}

__global__ void __launch_bounds__(kDesThreads) des_add_blocks(DesK k) {
  const uint64_t off = k.blk[blockIdx.x];
  const uint64_t base = (uint64_t)blockIdx.x * kDesChunk;
  for (uint32_t i = threadIdx.x; i < kDesChunk; i += kDesThreads)
    if (base + i < k.N) k.A[base + i] += off;
}

// hist[bin[i]] += 1 for the (up to) 4 bins of every lane (kNoBin: none).
// The durations of one position mostly share a bin: the wave counts the bins
// equal to its first lane's first bin with ballots and adds them with one LDS
// atomic; the rest go one atomic each.  Call with the wave converged.
constexpr uint32_t kNoBin = 0xFFFFFFFFu;
// FULL: every bin is set (whole quads of traces below N)
template <bool FULL = false>
__device__ __forceinline__ void hist_add4(uint32_t *hist, const uint32_t (&bin)[4]) {
  const uint32_t first =
      FULL ? bin[0] : bin[0] != kNoBin ? bin[0] : bin[1] != kNoBin ? bin[1] : bin[2] != kNoBin ? bin[2] : bin[3];
  const uint64_t any = __ballot(first != kNoBin);
  if (!any) return;
  const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)first, (int)__builtin_ctzll(any));
  uint32_t n = 0;
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) {
    n += (uint32_t)__builtin_popcountll(__ballot(bin[i] == b0));
    if ((FULL || bin[i] != kNoBin) && bin[i] != b0) atomicAdd(&hist[bin[i]], 1u);
  }
  if ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(any)) atomicAdd(&hist[b0], n);
}

// m = 2 m + (this lane in mask): one v_addc_co_u32 with the mask as carry-in
__device__ __forceinline__ void des_shift_in(uint32_t &m, uint64_t mask) {
  uint64_t co;
  asm("v_addc_co_u32 %0, %1, %0, %0, %2" : "+v"(m), "=s"(co) : "s"(mask));
}

// own error statuses of traces [base, base+4) of position v (base % 4 == 0),
// bit i.  The status pass zeroes the bits past N inside a row, but a partial
// last chunk also asks for quads far past N — up to a chunk beyond the row's
// 16-word padding, i.e. into the NEXT position's row.  Those quads read
// nothing (round 3: this was the cause of the "hoisted 500-count atomics gave
// wrong batches" variant of round 2 — without the per-trace N guard its
// atomics counted the next row's bits into E[t >= N], past the end of E).
__device__ __forceinline__ uint32_t des_status4(const DesK &k, uint32_t v, uint64_t base) {
  if (base >= k.N) return 0u;
  return (k.stbits[(uint64_t)v * k.st_wpr + (base >> 5)] >> (base & 31u)) & 0xFu;
}

// ---- status pass: the own error status of every (position, trace).  The
// four positions 4g..4g+3 share Philox block (t, g, 0, 0) (word j for
// position 4g+j, as in the walks), so one block per (group, trace) instead of
// one per (position, trace).  One thread: a group x 32 consecutive traces.
__global__ void __launch_bounds__(256) des_status(DesK k) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint32_t ng = (k.n_pos + 3) / 4;
  const uint64_t g = tid / k.st_wpr, w = tid - g * k.st_wpr;
  if (g >= ng) return;
  uint32_t thr[4], always[4], live[4];
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    const uint32_t v = (uint32_t)g * 4 + j;
    live[j] = v < k.n_pos;
    const DesPos &P = k.pos[live[j] ? v : 0];
    thr[j] = live[j] ? P.thr : 0u;
    always[j] = live[j] && (P.flags & kDesFlagAlways);
  }
  uint32_t bits[4] = {0, 0, 0, 0};
  const uint32_t any = thr[0] | thr[1] | thr[2] | thr[3];
  auto put = [&](const uint32_t (&c)[4], uint32_t b) {
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) bits[j] |= (uint32_t)(always[j] || (thr[j] && c[j] < thr[j])) << b;
  };
  // whole waves of one group and one trace-id high word (the usual case):
  // counter words 1-3 are wave-uniform, so rounds 1-2 fold into scalar math
  // (as walk.hip philox_lockstep), and each trace's bit is shifted in from
  // the compare's lane mask (one v_addc_co_u32)
  const uint64_t t0 = k.trace_begin + w * 32;
  const uint32_t gu = __builtin_amdgcn_readfirstlane((uint32_t)g);
  const uint32_t hiu = __builtin_amdgcn_readfirstlane((uint32_t)(t0 >> 32));
  const bool lane_ok = any && w * 32 + 32 <= k.N && (uint32_t)g == gu && (uint32_t)(t0 >> 32) == hiu &&
                       (uint32_t)((t0 + 31) >> 32) == hiu;
  if (__ballot(!lane_ok) == 0) {
    uint32_t lim[4], en[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {  // wave-uniform: bit = en && c <= lim
      const uint32_t a = __builtin_amdgcn_readfirstlane(always[j]), t = __builtin_amdgcn_readfirstlane(thr[j]);
      en[j] = a | (t != 0u);
      lim[j] = a ? 0xFFFFFFFFu : t - 1u;
    }
    constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
    const uint64_t q1 = (uint64_t)M1 * gu;                           // scalar
    const uint32_t u0 = (uint32_t)(q1 >> 32) ^ hiu ^ k.k0;           // uniform
    const uint64_t q0 = (uint64_t)M0 * u0;                           // scalar (round 2)
    uint32_t uk0 = (uint32_t)q1 ^ (k.k0 + W0), uk1 = (uint32_t)(q0 >> 32) ^ (k.k1 + W1);
    asm volatile("" : "+s"(uk0), "+s"(uk1));
    uint32_t lo[4] = {0, 0, 0, 0}, hi[4] = {0, 0, 0, 0};
    for (int b = 15; b >= 0; --b) {  // traces b and b + 16, shifted in from the top bit down
      uint32_t c[2][4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint32_t tl = (uint32_t)t0 + (uint32_t)b + 16u * u;
        const uint64_t p0 = (uint64_t)M0 * tl;
        const uint64_t p1 = (uint64_t)M1 * ((uint32_t)(p0 >> 32) ^ k.k1);
        c[u][0] = (uint32_t)(p1 >> 32) ^ uk0;
        c[u][1] = (uint32_t)p1;
        c[u][2] = (uint32_t)p0 ^ uk1;
        c[u][3] = (uint32_t)q0;
      }
      uint32_t k0 = k.k0 + 2u * W0, k1 = k.k1 + 2u * W1;
#pragma unroll
      for (int r = 2; r < 10; ++r) {
        asm volatile("" : "+s"(k0), "+s"(k1));
        des_round(c[0], k0, k1);
        des_round(c[1], k0, k1);
        k0 += W0;
        k1 += W1;
      }
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        des_shift_in(lo[j], en[j] ? __ballot(c[0][j] <= lim[j]) : 0ull);
        des_shift_in(hi[j], en[j] ? __ballot(c[1][j] <= lim[j]) : 0ull);
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) bits[j] = lo[j] | (hi[j] << 16);
  } else if (any && w * 32 + 32 <= k.N) {
    // two independent Philox chains per step (ILP)
    for (uint32_t b = 0; b < 16; ++b) {
      const uint64_t t0 = k.trace_begin + w * 32 + b, t1 = t0 + 16;
      uint32_t c0[4] = {(uint32_t)t0, (uint32_t)(t0 >> 32), (uint32_t)g, 0u};
      uint32_t c1[4] = {(uint32_t)t1, (uint32_t)(t1 >> 32), (uint32_t)g, 0u};
      uint32_t k0 = k.k0, k1 = k.k1;
#pragma unroll
      for (int r = 0; r < 10; ++r) {
        des_round(c0, k0, k1);
        des_round(c1, k0, k1);
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
      }
      put(c0, b);
      put(c1, b + 16);
    }
  } else {
    for (uint32_t b = 0; b < 32; ++b) {
      const uint64_t t = w * 32 + b;
      if (t >= k.N) break;
      if (any) {
        uint32_t c[4] = {(uint32_t)(k.trace_begin + t), (uint32_t)((k.trace_begin + t) >> 32), (uint32_t)g, 0u};
        des_philox(c, k.k0, k.k1);
        put(c, b);
      } else {
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) bits[j] |= always[j] << b;
      }
    }
  }
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j)
    if (live[j]) const_cast<uint32_t *>(k.stbits)[(g * 4 + j) * k.st_wpr + w] = bits[j];
}

// per-service duration statistics of a workgroup: LDS histogram + sums -> the
// service's table row, 500s -> the call site's callee-500 counter
template <uint32_t NT>
__device__ __forceinline__ void des_flush_durations(const DesK &k, const DesPos &P, const uint32_t *hist,
                                                    uint64_t d0, uint64_t d1, uint64_t n5, uint64_t *red) {
#pragma unroll
  for (uint32_t d = 32; d > 0; d >>= 1) {
    d0 += __shfl_xor(d0, d, 64);
    d1 += __shfl_xor(d1, d, 64);
    n5 += __shfl_xor(n5, d, 64);
  }
  constexpr uint32_t W = NT / 64;
  if ((threadIdx.x & 63u) == 0) {
    red[threadIdx.x >> 6] = d0;
    red[W + (threadIdx.x >> 6)] = d1;
    red[2 * W + (threadIdx.x >> 6)] = n5;
  }
  __syncthreads();
  unsigned long long *trow = (unsigned long long *)(k.table + (uint64_t)P.row * ISIM_DES_ROW_WORDS);
  for (uint32_t i = threadIdx.x; i < 2 * ISIM_N_PROM; i += NT)
    if (hist[i]) atomicAdd(trow + i, (unsigned long long)hist[i]);
  if (threadIdx.x == 0) {
    uint64_t s0 = 0, s1 = 0, e = 0;
#pragma unroll 2
    for (uint32_t i = 0; i < W; ++i) {
      s0 += red[i];
      s1 += red[W + i];
      e += red[2 * W + i];
    }
    if (s0) atomicAdd(trow + 2 * ISIM_N_PROM, (unsigned long long)s0);
    if (s1) atomicAdd(trow + 2 * ISIM_N_PROM + 1, (unsigned long long)s1);
    if (e && P.slot != kSlotRoot)
      atomicAdd((unsigned long long *)(k.stats + ISIM_ST_SITES + k.n_slots + P.slot), (unsigned long long)e);
  }
}

// queue statistics of a workgroup -> the service's table row
template <uint32_t NT>
__device__ __forceinline__ void des_flush_waits(const DesK &k, uint32_t trow_idx, uint64_t wsum, uint64_t wmax,
                                                uint64_t count, uint64_t hold_sum, uint64_t *red) {
#pragma unroll
  for (uint32_t d = 32; d > 0; d >>= 1) {
    wsum += __shfl_xor(wsum, d, 64);
    const uint64_t o = __shfl_xor(wmax, d, 64);
    wmax = o > wmax ? o : wmax;
  }
  if ((threadIdx.x & 63u) == 0) {
    red[threadIdx.x >> 6] = wsum;
    red[NT / 64 + (threadIdx.x >> 6)] = wmax;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t s = 0, m = 0;
#pragma unroll 2
    for (uint32_t i = 0; i < NT / 64; ++i) {
      s += red[i];
      m = red[NT / 64 + i] > m ? red[NT / 64 + i] : m;
    }
    unsigned long long *trow = (unsigned long long *)(k.table + (uint64_t)trow_idx * ISIM_DES_ROW_WORDS);
    if (count) atomicAdd(trow + ISIM_DES_COUNT, (unsigned long long)count);
    if (hold_sum) atomicAdd(trow + ISIM_DES_SUM_HOLD, (unsigned long long)hold_sum);
    if (s) atomicAdd(trow + ISIM_DES_SUM_WAIT, (unsigned long long)s);
    if (m) atomicMax(trow + ISIM_DES_MAX_WAIT, (unsigned long long)m);
  }
}

// The queue of one chunk of 4 traces per thread, once the carry into the
// thread is known: S = max(x, a) per trace (absolute), the stored value
// (S or, fused, F | status, relative to A_t), waits and durations.
template <typename T, bool FUSED>
__device__ __forceinline__ void queue_finish(const DesK &k, const DesPos &P, uint64_t base, uint64_t N,
                                             uint64_t x, const uint64_t (&a)[kPer], const T (&r)[kPer],
                                             uint64_t off, uint32_t mask, uint32_t stm, T (&out)[kPer], uint32_t *hist,
                                             const uint8_t *lut,
                                             uint64_t &wsum, uint64_t &wmax, uint64_t &d0, uint64_t &d1,
                                             uint64_t &n5, bool &bad) {
  uint32_t bin[kPer] = {kNoBin, kNoBin, kNoBin, kNoBin};
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    if (base + i < N && ((mask >> i) & 1u)) {
      const uint64_t S = x > a[i] ? x : a[i];
      const uint64_t w = S - a[i];
      wsum += w;
      wmax = w > wmax ? w : wmax;
      x = S + P.hold;
      uint64_t val = w + (uint64_t)r[i] + off;  // S - A_t (off is 0 for the entry: r = 0)
      if constexpr (FUSED) {
        const uint64_t F = val + P.floor;
        const uint32_t st = (stm >> i) & 1u;
        const uint64_t dur = w + P.floor;  // F - a
        if (st && !k.quiet) atomicAdd(k.E + base + i, 1u);
        n5 += st;
        d1 += st ? dur : 0;  // selects, not a branch: keeps d0/d1 in registers
        d0 += st ? 0 : dur;
        bin[i] = st * ISIM_N_PROM + des_prom_bucket(lut, dur);
        bad |= !Row<T>::fits(F);
        val = F | ((uint64_t)st << Row<T>::kTop);
      } else {
        bad |= !Row<T>::fits(val);
      }
      out[i] = (T)val;
    }
  }
  if constexpr (FUSED) hist_add4(hist, bin);
}

// agent-scope relaxed accesses: sc1 loads and stores (L1 bypassed)
__device__ __forceinline__ uint64_t ld_relaxed(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_flag(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_flag(uint32_t *p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Rows handed between workgroups inside a launch (des_down_pipe), the sc1
// form of the guide's Guideline 16: the producer's 16-B stores are sc1
// (write-through), drained by every storing wave before the barrier behind
// which one lane stores the flag (sc1); the consumer polls the flag with sc1
// loads and reads every handed-off byte with sc1 loads (L1 bypassed), so no
// release or acquire fence.  A buffer resource per chunk keeps the offsets
// 32-bit; the last (partial) chunk goes value by value.
typedef uint32_t des_v4u __attribute__((ext_vector_type(4)));
constexpr int kRsrcWord3 = 0x00020000;  // gfx9 raw buffer: 32-bit data format, no swizzle
constexpr int kSc1 = 16;                // cache-policy aux bit of the buffer builtins
template <typename T, bool FULL>
__device__ __forceinline__ void load_row_sc1(const T *p, uint64_t c0, uint64_t base, uint64_t N, T (&x)[kPer]) {
  if constexpr (FULL) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<T *>(p + c0), (short)0, (int)(sizeof(T) * kPer * kDownThreads),
                                          kRsrcWord3);
    const uint32_t vo = (uint32_t)(base - c0) * (uint32_t)sizeof(T);
    if constexpr (sizeof(T) == 4) {
      const des_v4u w = __builtin_amdgcn_raw_buffer_load_b128(r, vo, 0, kSc1);
      x[0] = w.x;
      x[1] = w.y;
      x[2] = w.z;
      x[3] = w.w;
    } else {
      const des_v4u w0 = __builtin_amdgcn_raw_buffer_load_b128(r, vo, 0, kSc1);
      const des_v4u w1 = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 16, 0, kSc1);
      x[0] = (T)w0.x | ((T)w0.y << (4 * sizeof(T)));
      x[1] = (T)w0.z | ((T)w0.w << (4 * sizeof(T)));
      x[2] = (T)w1.x | ((T)w1.y << (4 * sizeof(T)));
      x[3] = (T)w1.z | ((T)w1.w << (4 * sizeof(T)));
    }
  } else {
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i)
      x[i] = base + i < N ? __hip_atomic_load(p + base + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (T)0;
  }
}
template <typename T, bool FULL>
__device__ __forceinline__ void store_row_sc1(T *p, uint64_t c0, uint64_t base, uint64_t N, const T (&x)[kPer]) {
  if constexpr (FULL) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(p + c0, (short)0, (int)(sizeof(T) * kPer * kDownThreads), kRsrcWord3);
    const uint32_t vo = (uint32_t)(base - c0) * (uint32_t)sizeof(T);
    if constexpr (sizeof(T) == 4) {
      const des_v4u w = {x[0], x[1], x[2], x[3]};
      __builtin_amdgcn_raw_buffer_store_b128(w, r, vo, 0, kSc1);
    } else {
      const des_v4u w0 = {(uint32_t)x[0], (uint32_t)((uint64_t)x[0] >> 32), (uint32_t)x[1],
                          (uint32_t)((uint64_t)x[1] >> 32)};
      const des_v4u w1 = {(uint32_t)x[2], (uint32_t)((uint64_t)x[2] >> 32), (uint32_t)x[3],
                          (uint32_t)((uint64_t)x[3] >> 32)};
      __builtin_amdgcn_raw_buffer_store_b128(w0, r, vo, 0, kSc1);
      __builtin_amdgcn_raw_buffer_store_b128(w1, r, vo + 16, 0, kSc1);
    }
  } else {
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i)
      if (base + i < N) __hip_atomic_store(p + base + i, x[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Single-replica queues (closed form): from the thread's exclusive prefix p
// the running max of the keys gives the wait of each trace, S_t - a_t =
// p_t - key_t; the stored value (S or, fused, F | status, relative to A_t),
// waits and durations as queue_finish.
struct QAcc {
  uint64_t wsum = 0, wmax = 0, dsum = 0, d1 = 0, n5 = 0;  // d0 = dsum - d1
  uint32_t wmax32 = 0;  // 32-bit rows: the largest wait (< 2^31 unless `bad`), folded into wmax by max_wait()
  bool bad = false;
  __device__ uint64_t max_wait() const { return wmax > wmax32 ? wmax : wmax32; }
};
template <typename T, bool FUSED, bool FULL>
__device__ __forceinline__ void queue_finish1(const DesK &k, const DesPos &P, uint64_t base, uint64_t N, int64_t p,
                                              const int64_t (&key)[kPer], const T (&r)[kPer], uint64_t off,
                                              uint32_t stm, T (&out)[kPer], uint32_t *hist, const uint8_t *lut,
                                              QAcc &q) {
  uint32_t bin[kPer] = {kNoBin, kNoBin, kNoBin, kNoBin};
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    if (FULL || base + i < N) {
      p = max_i64(p, key[i]);
      if constexpr (sizeof(T) == 4) {
        // 32-bit rows: a stored value below 2^31 needs a wait below 2^31, so
        // the wait, the duration and their maxima are 32-bit (a larger wait
        // marks the batch bad: it is rerun with 64-bit rows)
        const uint64_t w64 = (uint64_t)(p - key[i]);
        const uint32_t w = (uint32_t)w64;
        q.bad |= w64 >= Row<T>::kSt;
        q.wsum += w;
        q.wmax32 = w > q.wmax32 ? w : q.wmax32;
        uint64_t val = (uint64_t)w + (uint64_t)r[i] + off;  // S - A_t (off is 0 for the entry: r = 0)
        if constexpr (FUSED) {
          const uint64_t F = val + P.floor;
          const uint32_t st = (stm >> i) & 1u;
          const uint32_t dur = w + (uint32_t)P.floor;  // F - a; exact whenever F fits
#ifndef DES_HOIST_500
          if (st && !k.quiet) atomicAdd(k.E + base + i, 1u);
#endif
          q.n5 += st;
          q.dsum += dur;
          q.d1 += st ? dur : 0u;
          bin[i] = st * ISIM_N_PROM + des_prom_bucket32(lut, dur);
          q.bad |= !Row<T>::fits(F);
          val = F | ((uint64_t)st << Row<T>::kTop);
        } else {
          q.bad |= !Row<T>::fits(val);
        }
        out[i] = (T)val;
        continue;
      }
      const uint64_t w = (uint64_t)(p - key[i]);
      q.wsum += w;
      q.wmax = w > q.wmax ? w : q.wmax;
      uint64_t val = w + (uint64_t)r[i] + off;  // S - A_t (off is 0 for the entry: r = 0)
      if constexpr (FUSED) {
        const uint64_t F = val + P.floor;
        const uint32_t st = (stm >> i) & 1u;
        const uint64_t dur = w + P.floor;  // F - a
        // (per trace; DES_HOIST_500 builds the variant with the atomics under
        // one wave-uniform test — correct since des_status4's N guard, no faster)
#ifndef DES_HOIST_500
        if (st && !k.quiet) atomicAdd(k.E + base + i, 1u);
#endif
        q.n5 += st;
        q.dsum += dur;
        q.d1 += st ? dur : 0;  // a select, not a branch
        bin[i] = st * ISIM_N_PROM + des_prom_bucket(lut, dur);
        q.bad |= !Row<T>::fits(F);
        val = F | ((uint64_t)st << Row<T>::kTop);
      } else {
        q.bad |= !Row<T>::fits(val);
      }
      out[i] = (T)val;
    }
  }
  if constexpr (FUSED) {
#ifdef DES_HOIST_500
    // per-trace 500 counts: one wave-uniform test, the atomics only where a 500 is
    if (!k.quiet && __ballot(stm != 0u)) {
#pragma unroll
      for (uint32_t i = 0; i < kPer; ++i)
        if ((stm >> i) & 1u) atomicAdd(k.E + base + i, 1u);
    }
#endif
    hist_add4<FULL>(hist, bin);
  }
}

// this thread's 4 traces (one group: base % 4 == 0): absolute arrivals a =
// G + relative arrival, and the relative arrivals' row values r (S relative
// = wait + r + off); the entry's relative arrival is A_t - G.  Returns true
// when an entry value does not fit the row type (the batch is redone wide).
template <typename T, bool FULL = false>
__device__ __forceinline__ bool load_arrivals(const DesK &k, const T *par, uint64_t off, uint64_t base,
                                              uint64_t N, uint64_t (&a)[kPer], T (&r)[kPer]) {
  const uint64_t n = FULL ? base + kPer : N;  // whole: one vector access each
  const uint64_t g = FULL || base < N ? des_gbase(k, base) : 0;
  if (par) {
    load4t<T>(par, base, n, r);
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) a[i] = g + (uint64_t)r[i] + off;
    return false;
  }
  load4n<uint64_t>(k.A, base, n, a);
  bool bad = false;
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    const uint64_t d = FULL || base + i < N ? a[i] - g : 0;
    r[i] = (T)d;
    bad |= !Row<T>::fits(d);
  }
  return bad;
}

// ---- queue pass, one workgroup per position (wide groups; replicated
// services: per-replica scans, the routing draw per trace)
// single-replica services: the closed form, one barrier per chunk (the wave
// totals double-buffered; every thread folds them into its prefix and into the
// carry itself)
// One chunk of kPer x kDownThreads traces from c0 (FULL: all below N).
// Pipelined pass (des_down_pipe): HAND_IN, the caller's start row is written
// in this launch, read with sc1 loads; HAND_OUT, this start row is read in
// this launch: sc1 stores, and at the chunk's barrier (every wave drained its
// previous chunk's stores first) one lane publishes the chunks done so far.
template <typename T, bool FUSED, bool FULL, bool HAND_IN = false, bool HAND_OUT = false>
__device__ __forceinline__ void down1_chunk(const DesK &k, const DesPos &P, uint32_t v, const T *par, uint64_t off,
                                            T *out, uint64_t c0, int64_t *wtot, int64_t &carry, uint32_t *hist,
                                            const uint8_t *lut, QAcc &q, uint32_t chunk = 0) {
  constexpr uint32_t NW = kDownThreads / 64;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t N = k.N;
  uint64_t base = c0 + (uint64_t)threadIdx.x * kPer;
  // opaque to loop strength reduction, which otherwise keeps a dozen 64-bit
  // induction variables ((base + i) * hold, ...) live across the chunk loop
  __asm__ volatile("" : "+v"(base));
  uint64_t a[kPer];
  T ar[kPer];
  if constexpr (HAND_IN) {
    const uint64_t g = FULL || base < N ? des_gbase(k, base) : 0;
    load_row_sc1<T, FULL>(par, c0, base, N, ar);
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) a[i] = g + (uint64_t)ar[i] + off;
  } else {
    q.bad |= load_arrivals<T, FULL>(k, par, off, base, N, a, ar);
  }
  const uint32_t stm = FUSED ? des_status4(k, v, base) : 0u;
  int64_t key[kPer];
  const int64_t inc = wave_max_scan(queue_keys<FULL>(a, base, N, P.hold, key));
  const int64_t exc = wave_shr1(inc);
  if (lane == 63) wtot[wave] = inc;
  if constexpr (HAND_OUT) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the previous chunk's stores
  __syncthreads();
  if constexpr (HAND_OUT)
    if (threadIdx.x == 0 && chunk > 0) st_flag(k.prog + v, chunk);
  // lanes 0..NW-1 scan the wave totals: the waves before this one and all
  int64_t pre;
  fold_totals<NW>(wtot, wave, carry, pre);
  T o[kPer] = {0, 0, 0, 0};
  queue_finish1<T, FUSED, FULL>(k, P, base, N, max_i64(pre, exc), key, ar, off, stm, o, hist, lut, q);
  if constexpr (FUSED) track4<T>(k, out, base, N, o);  // a fused leaf's row is final (F)
  if constexpr (HAND_OUT) {
    store_row_sc1<T, FULL>(out, c0, base, N, o);
  } else {
    store4t<T>(out, base, FULL ? base + kPer : N, o);
  }
}

// ---- 32-bit queue keys (round 3; narrow rows, whole chunks, every position
// but the entry).  A wave's 256 traces are 4 groups of 64, one DPP row (16
// lanes x 4 traces) each.  With x_t = row + off the group-relative arrival
// and the group's base kb = G - t_g h (G its first arrival, t_g its first
// trace), the keys relative to kb,
//   key_t - kb = x_t - (t - t_g) h,
// lie in (-64 h, x_t]: 32-bit whenever x_t < 2^31 (a larger one overflows
// the start row anyway: the batch is redone wide) and 64 h < 2^31 (the
// caller's check).  A row scan by DPP gives each trace its prefix within the
// group; the group totals (64-bit absolute) combine across the wave's rows
// by two row broadcasts, across the waves through LDS (fold_totals) and
// across chunks in the carry.  A prefix below every key is clamped to
// INT32_MIN (exact: keys exceed -2^31); one at or above 2^31 puts the
// group's first start at or above 2^31 (a row overflow: the batch is redone).
__device__ __forceinline__ int32_t max_i32(int32_t a, int32_t b) { return a > b ? a : b; }
template <int CTRL>
__device__ __forceinline__ int32_t dpp_max32(int32_t v) {
  return max_i32(v, __builtin_amdgcn_update_dpp((int)INT32_MIN, v, CTRL, 0xF, 0xF, false));
}
// inclusive max-scan within each DPP row (INT32_MIN where a source lane does not exist)
__device__ __forceinline__ int32_t row_max_scan32(int32_t v) {
  v = dpp_max32<0x111>(v);  // row_shr:1
  v = dpp_max32<0x112>(v);  // row_shr:2
  v = dpp_max32<0x114>(v);  // row_shr:4
  v = dpp_max32<0x118>(v);  // row_shr:8
  return v;
}

// the finish of one thread's KP traces with 32-bit keys from the prefix p
// (FULL: all below N; else the traces past N are left out)
template <bool FUSED, bool FULL, uint32_t KP>
__device__ __forceinline__ void queue_finish_n32(const DesK &k, uint64_t base, int32_t p, const int32_t (&key)[KP],
                                                 const uint32_t (&x)[KP], uint32_t floor32, uint32_t stm,
                                                 uint32_t (&out)[KP], uint32_t *hist, const uint8_t *lut, QAcc &q) {
  static_assert(KP % 2 == 0, "waits are summed in pairs");
  uint32_t bin[KP], wv[KP], big = 0, cnt = 0;
#pragma unroll
  for (uint32_t i = 0; i < KP; ++i) {
    out[i] = 0;
    bin[i] = kNoBin;
    wv[i] = 0;
    if (!FULL && base + i >= k.N) continue;
    if constexpr (!FULL) ++cnt;
    p = max_i32(p, key[i]);
    const uint32_t w = (uint32_t)p - (uint32_t)key[i];  // the wait S - a (< 2^32: exact)
#if !ISIM_DES_N32_FOLD
    q.wsum += w;
#endif
    wv[i] = w;
    q.wmax32 = w > q.wmax32 ? w : q.wmax32;
    uint32_t val = w + x[i];  // S - G (no wrap unless the batch is redone)
    big |= w | val;           // a wait or start at or above 2^31: redone with 64-bit rows
    if constexpr (FUSED) {
      const uint32_t F = val + floor32;
      const uint32_t st = (stm >> i) & 1u;
      const uint32_t dur = w + floor32;  // F - a
#if !ISIM_DES_N32_FOLD
      if (st && !k.quiet) atomicAdd(k.E + base + i, 1u);
      q.n5 += st;
      q.dsum += dur;
      q.d1 += st ? dur : 0u;
#endif
      bin[i] = st * ISIM_N_PROM + des_prom_bucket32(lut, dur);
      big |= F;
      val = F | (st << 31);
    }
    out[i] = val;
  }
#if ISIM_DES_N32_FOLD
  // the sums once per call: a pair of waits fits 32 bits (each is below 2^31,
  // or `big` redoes the batch with 64-bit rows and these statistics are not
  // committed); the durations' sum is the waits' plus n x floor; the 500s
  // (rare: stm is almost always 0 wave-wide) under one branch
  uint64_t ws = 0;
#pragma unroll
  for (uint32_t h = 0; h < KP; h += 2) ws += (uint64_t)(wv[h] + wv[h + 1]);
  q.wsum += ws;
  if constexpr (FUSED) {
    q.dsum += ws + (uint64_t)(FULL ? KP : cnt) * floor32;
    if (stm) {
#pragma unroll
      for (uint32_t i = 0; i < KP; ++i)
        if ((stm >> i) & 1u) {
          if (!k.quiet) atomicAdd(k.E + base + i, 1u);
          q.n5 += 1;
          q.d1 += wv[i] + floor32;
        }
    }
  }
#endif
  q.bad |= (big >> 31) != 0u;
  if constexpr (FUSED) {
#pragma unroll
    for (uint32_t h = 0; h < KP; h += 4) {
      const uint32_t b4[4] = {bin[h], bin[h + 1], bin[h + 2], bin[h + 3]};
      hist_add4<FULL>(hist, b4);
    }
  }
}

// a narrow row's KP values [base, base + KP) of a chunk of kN32 x
// kDownThreads traces from c0 (16-B accesses; SC1: the pipelined pass's
// hand-off form, sc1 buffer accesses; past N: per value)
template <bool SC1, bool FULL, uint32_t KP>
__device__ __forceinline__ void load_rowk(const uint32_t *p, uint64_t c0, uint64_t base, uint64_t N, uint32_t (&x)[KP]) {
  if constexpr (FULL) {
    if constexpr (SC1) {
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint32_t *>(p + c0), (short)0, (int)(4 * KP * kDownThreads), kRsrcWord3);
      const uint32_t vo = (uint32_t)(base - c0) * 4u;
#pragma unroll
      for (uint32_t h = 0; h < KP; h += 4) {
        const des_v4u w = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 4 * h, 0, kSc1);
        x[h] = w.x;
        x[h + 1] = w.y;
        x[h + 2] = w.z;
        x[h + 3] = w.w;
      }
    } else {
#pragma unroll
      for (uint32_t h = 0; h < KP; h += 4) {
        const uint4 v = *reinterpret_cast<const uint4 *>(p + base + h);
        x[h] = v.x;
        x[h + 1] = v.y;
        x[h + 2] = v.z;
        x[h + 3] = v.w;
      }
    }
  } else {
#pragma unroll
    for (uint32_t i = 0; i < KP; ++i)
      x[i] = base + i < N ? (SC1 ? __hip_atomic_load(p + base + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                 : p[base + i])
                          : 0u;
  }
}
template <bool SC1, bool FULL, uint32_t KP>
__device__ __forceinline__ void store_rowk(uint32_t *p, uint64_t c0, uint64_t base, uint64_t N, const uint32_t (&x)[KP]) {
  if constexpr (FULL) {
    if constexpr (SC1) {
      const __amdgpu_buffer_rsrc_t r =
          __builtin_amdgcn_make_buffer_rsrc(p + c0, (short)0, (int)(4 * KP * kDownThreads), kRsrcWord3);
      const uint32_t vo = (uint32_t)(base - c0) * 4u;
#pragma unroll
      for (uint32_t h = 0; h < KP; h += 4) {
        const des_v4u w = {x[h], x[h + 1], x[h + 2], x[h + 3]};
        __builtin_amdgcn_raw_buffer_store_b128(w, r, vo + 4 * h, 0, kSc1);
      }
    } else {
#pragma unroll
      for (uint32_t h = 0; h < KP; h += 4) {
#if ISIM_NT_ROWS
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(v4u{x[h], x[h + 1], x[h + 2], x[h + 3]}, reinterpret_cast<v4u *>(p + base + h));
#else
        *reinterpret_cast<uint4 *>(p + base + h) = make_uint4(x[h], x[h + 1], x[h + 2], x[h + 3]);
#endif
      }
    }
  } else {
#pragma unroll
    for (uint32_t i = 0; i < KP; ++i)
      if (base + i < N) {
        if constexpr (SC1) __hip_atomic_store(p + base + i, x[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else p[base + i] = x[i];
      }
  }
}

// down1_chunk for narrow rows (FULL: a whole chunk; ENTRY: the entry, whose
// group-relative arrival is A_t - G; else the caller's row `par`), kN32
// consecutive traces per thread: a DPP row (16 lanes) holds one trace group;
// `jh0` = (t - t_g) h of the thread's first trace (the caller's per-position
// constant).  The same results as down1_chunk<uint32_t, FUSED, FULL, ...>.
template <bool FUSED, bool HAND_IN, bool HAND_OUT, bool FULL = true, bool ENTRY = false>
__device__ __forceinline__ void down1_chunk_n32(const DesK &k, const DesPos &P, uint32_t v, const uint32_t *par,
                                                uint32_t *out, uint64_t c0, int64_t *wtot, int64_t &carry,
                                                uint32_t *hist, const uint8_t *lut, QAcc &q, uint32_t chunk,
                                                uint32_t jh0) {
  constexpr uint32_t NW = kDownThreads / 64, KP = kN32;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t N = k.N;
  uint64_t base = c0 + (uint64_t)threadIdx.x * KP;
  __asm__ volatile("" : "+v"(base));  // (down1_chunk)
  const uint64_t tg = base & ~(kDesGrp - 1);
  const uint64_t g = FULL || tg < N ? k.A[tg] : 0;  // every lane of a group with a trace below N
  uint32_t x[KP], xo = 0;
  if constexpr (ENTRY) {
    uint64_t d = 0;
#pragma unroll
    for (uint32_t i = 0; i < KP; ++i) {
      const uint64_t r = FULL || base + i < N ? k.A[base + i] - g : 0;
      d |= r;
      x[i] = (uint32_t)r;
    }
    q.bad |= (d >> 31) != 0;
  } else {
    uint32_t ar[KP];
    load_rowk<HAND_IN, FULL, KP>(par, c0, base, N, ar);
    const uint32_t off32 = (uint32_t)P.off;
#pragma unroll
    for (uint32_t i = 0; i < KP; ++i) x[i] = ar[i] + off32;
  }
  // own error statuses, bit i (base % KP == 0: one status word, nothing past N)
  const uint32_t stm = FUSED && base < N ? (k.stbits[(uint64_t)v * k.st_wpr + (base >> 5)] >> (base & 31u)) &
                                               ((1u << KP) - 1u)
                                         : 0u;
  const uint32_t hold32 = (uint32_t)P.hold;
  int32_t key[KP], kt = INT32_MIN;
#pragma unroll
  for (uint32_t i = 0; i < KP; ++i) {
    xo |= x[i];
    key[i] = FULL || base + i < N ? (int32_t)(x[i] - (jh0 + i * hold32)) : INT32_MIN;
    kt = max_i32(kt, key[i]);
  }
  q.bad |= (xo >> 31) != 0u;  // an arrival at or above 2^31: its start row overflows
  const int32_t inc = row_max_scan32(kt);
  const int32_t exc = __builtin_amdgcn_update_dpp((int)INT32_MIN, inc, 0x111, 0xF, 0xF, false);  // row_shr:1
  // the group totals, absolute, at lane 15 of each row; their inclusive prefix
  // over the wave's rows at lanes 15/31/47/63, and each row's exclusive one
  // (a group past N: kb = -t_g h, its total INT32_MIN relative — below any key)
  const int64_t kb = (int64_t)(g - tg * P.hold);
  int64_t s = kb + (int64_t)inc;
  s = max_i64(s, dpp_i64<0x142, 0xA>(s, s));  // row_bcast:15 into rows 1, 3
  s = max_i64(s, dpp_i64<0x143, 0xC>(s, s));  // row_bcast:31 into rows 2, 3
  int64_t e = dpp_i64<0x142, 0xA>(kKeyMin, s);  // rows 1, 3: lane 15 / 47
  e = dpp_i64<0x143, 0x4>(e, s);                // row 2: lane 31
  if (lane == 63) wtot[wave] = max_i64(0, s);
  if constexpr (HAND_OUT) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the previous chunk's stores
  __syncthreads();
  if constexpr (HAND_OUT)
    if (threadIdx.x == 0 && chunk > 0) st_flag(k.prog + v, chunk);
  int64_t pre;
  fold_totals<NW>(wtot, wave, carry, pre);
  const int64_t pr = max_i64(pre, e) - kb;  // the group's prefix, relative
  q.bad |= (FULL || base < N) && pr > (int64_t)INT32_MAX;
  const int32_t p0 = pr < (int64_t)INT32_MIN ? INT32_MIN : pr > (int64_t)INT32_MAX ? INT32_MAX : (int32_t)pr;
  uint32_t o[KP];
  queue_finish_n32<FUSED, FULL, KP>(k, base, max_i32(p0, exc), key, x, (uint32_t)P.floor, stm, o, hist, lut, q);
  if constexpr (FUSED) {
    if (k.changed) {  // a fused leaf's row is final (F)
#pragma unroll
      for (uint32_t h = 0; h < KP; h += 4) {
        const uint32_t o4[4] = {o[h], o[h + 1], o[h + 2], o[h + 3]};
        track4<uint32_t>(k, out, base + h, N, o4);
      }
    }
  }
  store_rowk<HAND_OUT, FULL, KP>(out, c0, base, N, o);
}

// whether a position's whole chunks take the 32-bit keys, and the thread's (t - t_g) h
template <typename T, bool FUSED>
__device__ __forceinline__ bool n32_ok(const DesPos &P, const void *par, uint32_t &jh0) {
  jh0 = (threadIdx.x & 15u) * kN32 * (uint32_t)P.hold;
  return sizeof(T) == 4 && par != nullptr && P.hold < kN32HoldMax && P.off < (1ull << 30) &&
         (!FUSED || P.floor < (1ull << 30));
}

template <typename T, bool FUSED>
__device__ __forceinline__ void down1_body(const DesK &k, uint32_t v) {
  constexpr uint32_t NW = kDownThreads / 64;
  __shared__ int64_t wtot[2][NW];
  __shared__ uint64_t red[3 * NW];
  __shared__ uint32_t hist[2 * ISIM_N_PROM];
  __shared__ __attribute__((aligned(4))) uint8_t lut[4 * kBucketLutWords];
  const DesPos P = k.pos[v];
  if constexpr (FUSED) {
    for (uint32_t i = threadIdx.x; i < 2 * ISIM_N_PROM; i += kDownThreads) hist[i] = 0;
    des_bucket_lut_init(lut);
    __syncthreads();
  }
  const uint64_t N = k.N;
  const T *par = arrival_row<T>(k, v, P);
  const uint64_t off = par ? P.off : 0;
  T *out = row<T>(FUSED ? k.WF : k.W, k.ld, v);  // a fused leaf stores its finish
  QAcc q;
  int64_t carry = 0;  // max key of the chunks before (0: the idle start)
  uint32_t buf = 0;
  constexpr uint64_t CH = (uint64_t)kPer * kDownThreads;
  uint64_t c0 = 0;
  uint32_t jh0;
  if (n32_ok<T, FUSED>(P, par, jh0)) {
    if constexpr (sizeof(T) == 4) {
      constexpr uint64_t CH32 = (uint64_t)kN32 * kDownThreads;
#pragma unroll 1
      for (; c0 + CH32 <= N; c0 += CH32) {
        down1_chunk_n32<FUSED, false, false>(k, P, v, par, out, c0, wtot[buf], carry, hist, lut, q, 0, jh0);
        buf ^= 1u;
      }
    }
  }
#pragma unroll 1
  for (; c0 + CH <= N; c0 += CH) {
    down1_chunk<T, FUSED, true>(k, P, v, par, off, out, c0, wtot[buf], carry, hist, lut, q);
    buf ^= 1u;
  }
  if (c0 < N) down1_chunk<T, FUSED, false>(k, P, v, par, off, out, c0, wtot[buf], carry, hist, lut, q);
  flag_overflow(k, q.bad);
  if (k.quiet) return;
  des_flush_waits<kDownThreads>(k, P.row, q.wsum, q.max_wait(), N, N * P.hold, red);
  if constexpr (FUSED) {
    __syncthreads();
    des_flush_durations<kDownThreads>(k, P, hist, q.dsum - q.d1, q.d1, q.n5, red);
  }
}

// replicated services: per-replica max-plus scans
template <typename T, bool MULTI, bool FUSED>
__device__ __forceinline__ void downr_body(const DesK &k, uint32_t v) {
  __shared__ MaxPlus wtot[kDownThreads / 64];
  __shared__ uint64_t carry[kDesMaxReplicas];
  __shared__ uint64_t red[3 * kDownThreads / 64];
  __shared__ MaxPlus xs[kDownThreads];
  __shared__ uint32_t hist[2 * ISIM_N_PROM];
  __shared__ __attribute__((aligned(4))) uint8_t lut[4 * kBucketLutWords];
  const DesPos P = k.pos[v];
  const uint32_t reps = MULTI ? P.reps : 1u;
  if (threadIdx.x < reps) carry[threadIdx.x] = 0;
  if constexpr (FUSED) {
    for (uint32_t i = threadIdx.x; i < 2 * ISIM_N_PROM; i += kDownThreads) hist[i] = 0;
    des_bucket_lut_init(lut);
  }
  __syncthreads();
  const uint64_t N = k.N;
  const T *par = arrival_row<T>(k, v, P);
  const uint64_t off = par ? P.off : 0;
  T *out = row<T>(FUSED ? k.WF : k.W, k.ld, v);  // a fused leaf stores its finish
  uint64_t wsum = 0, wmax = 0, d0 = 0, d1 = 0, n5 = 0;
  bool bad = false;
  for (uint64_t c0 = 0; c0 < N; c0 += (uint64_t)kPer * kDownThreads) {
    const uint64_t base = c0 + (uint64_t)threadIdx.x * kPer;
    uint64_t a[kPer];
    T o[kPer] = {0, 0, 0, 0};
    T ar[kPer];
    bad |= load_arrivals<T>(k, par, off, base, N, a, ar);
    uint32_t rr[kPer];
    const uint32_t stm = FUSED ? des_status4(k, v, base) : 0u;  // fused leaves: own error statuses, bit i
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) {
      if constexpr (MULTI)
        rr[i] = base + i < N ? des_draw(k.trace_begin + base + i, v, 0x80000002u, 0, k.k0, k.k1) % reps : 0u;
      else
        rr[i] = 0u;
    }
    for (uint32_t r = 0; r < reps; ++r) {
      MaxPlus f{0, 0};
      uint32_t mask = 0;
#pragma unroll
      for (uint32_t i = 0; i < kPer; ++i)
        if (base + i < N && rr[i] == r) {
          f = mp_then(f, MaxPlus{P.hold, a[i] + P.hold});
          mask |= 1u << i;
        }
      const MaxPlus inc = mp_block_scan<kDownThreads>(f, wtot);
      // exclusive prefix = the previous thread's inclusive one
      xs[threadIdx.x] = inc;
      __syncthreads();
      const MaxPlus pre = threadIdx.x ? xs[threadIdx.x - 1] : MaxPlus{0, 0};
      const uint64_t cin = carry[r];
      const uint64_t x = cin + pre.B > pre.C ? cin + pre.B : pre.C;
      queue_finish<T, FUSED>(k, P, base, N, x, a, ar, off, mask, stm, o, hist, lut, wsum, wmax, d0, d1, n5, bad);
      __syncthreads();  // every thread has read carry[r]
      if (threadIdx.x == kDownThreads - 1) {
        uint64_t xe = x;
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i)
          if ((mask >> i) & 1u) xe = (xe > a[i] ? xe : a[i]) + P.hold;
        carry[r] = xe;
      }
      __syncthreads();
    }
    if constexpr (FUSED) track4<T>(k, out, base, N, o);  // a fused leaf's row is final (F)
    store4t<T>(out, base, N, o);
  }
  flag_overflow(k, bad);
  if (k.quiet) return;
  des_flush_waits<kDownThreads>(k, P.row, wsum, wmax, N, N * P.hold, red);
  if constexpr (FUSED) {
    __syncthreads();
    des_flush_durations<kDownThreads>(k, P, hist, d0, d1, n5, red);
  }
}

template <typename T, bool MULTI, bool FUSED>
__device__ __forceinline__ void down_body(const DesK &k, uint32_t v) {
  if constexpr (MULTI) downr_body<T, true, FUSED>(k, v);
  else down1_body<T, FUSED>(k, v);
}

template <typename T, bool MULTI, bool FUSED>
__global__ void __launch_bounds__(kDownThreads, ISIM_DES_DOWN_WAVES) des_down(DesK k) {
  down_body<T, MULTI, FUSED>(k, k.level_pos[k.level_begin + blockIdx.x]);
}

// single-replica positions of a round, fused leaves and others in ONE launch
// (better packing of the last wave of workgroups than two launches)
template <typename T>
__global__ void __launch_bounds__(kDownThreads, ISIM_DES_DOWN_WAVES) des_down_mix(DesK k) {
  const uint32_t v = k.level_pos[k.level_begin + blockIdx.x];
  if (k.pos[v].flags & kDesFlagFused) down_body<T, false, true>(k, v);
  else down_body<T, false, false>(k, v);
}

// ---- queue pass, single-replica services of narrow groups: one workgroup
// per (position, chunk of kDownChunk traces), chunks of a position chained by
// a decoupled look-back over their max-plus maps.  Workgroups take tickets in
// launch order (position-major, chunk-minor), so every chunk they wait on
// has started.
struct ChainState {
  uint64_t B, C;   // B: the chunk's largest key a_t - t h, as int64 (flag >= 1); C unused
  uint64_t P;      // the largest key up to and including the chunk (flag 2)
  uint32_t flag, pad;
};
static_assert(sizeof(ChainState) == 32, "ChainState is 32 bytes");

// the ticket of a chained-scan workgroup: (position, chunk) in launch order
__device__ __forceinline__ uint32_t chain_ticket(const DesK &k) {
  __shared__ uint32_t s_ticket;
  if (threadIdx.x == 0) s_ticket = atomicAdd(k.chain_ticket, 1u);
  __syncthreads();
  return s_ticket;
}

template <typename T, bool FUSED>
__device__ __forceinline__ void chain_body(const DesK &k, uint32_t v, uint32_t chunk) {
  constexpr uint32_t NW = kDesThreads / 64;
  __shared__ int64_t wtot[NW];
  __shared__ uint64_t red[3 * kDesThreads / 64];
  __shared__ uint32_t hist[2 * ISIM_N_PROM];
  __shared__ __attribute__((aligned(4))) uint8_t lut[4 * kBucketLutWords];
  __shared__ int64_t s_carry;
  if constexpr (FUSED) {
    for (uint32_t i = threadIdx.x; i < 2 * ISIM_N_PROM; i += kDesThreads) hist[i] = 0;
    des_bucket_lut_init(lut);
  }
  const DesPos P = k.pos[v];
  const uint64_t N = k.N;
  const T *par = arrival_row<T>(k, v, P);
  const uint64_t off = par ? P.off : 0;
  T *out = row<T>(FUSED ? k.WF : k.W, k.ld, v);  // a fused leaf stores its finish
  ChainState *cs = k.chain + (uint64_t)v * k.n_chunks;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t base = (uint64_t)chunk * kDownChunk + (uint64_t)threadIdx.x * kPer;
  uint64_t a[kPer];
  T ar[kPer];
  const bool in_bad = load_arrivals<T>(k, par, off, base, N, a, ar);
  const uint32_t stm = FUSED && base < N ? des_status4(k, v, base) : 0u;
  int64_t key[kPer];
  const int64_t inc = wave_max_scan(queue_keys<false>(a, base, N, P.hold, key));
  const int64_t exc = wave_shr1(inc);
  if (lane == 63) wtot[wave] = inc;
  __syncthreads();
  if (threadIdx.x < 64) {
    // wave 0: publish this chunk's largest key, then look back (64 chunks
    // per step) for the largest key before it.  Hand-offs between workgroups
    // (other XCDs included) use sc1 stores drained before the flag store and
    // sc1 loads (no L2 writeback / invalidate).
    int64_t agg = kKeyMin, unused;
    fold_totals<NW>(wtot, 0, agg, unused);
    if (chunk > 0 && lane == 0) {
      st_relaxed(&cs[chunk].B, (uint64_t)agg);
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
      st_flag(&cs[chunk].flag, 1u);
    }
    int64_t cin = 0;  // chunk 0 starts from an idle worker
    if (chunk > 0) {
      int64_t run = kKeyMin;  // the windows already passed
      int64_t top = (int64_t)chunk - 1;
      uint32_t spins = 0;
      for (;;) {
        if (spins >= k.spin_limit) {  // never expected (tickets order the chunks): fail the batch
          if (lane == 0) atomicOr(k.ovf, kDesOvfFault);
          break;
        }
        const int64_t j = top - (int64_t)lane;  // lane 0 = the nearest chunk
        const uint32_t fl = j >= 0 ? ld_flag(&cs[j].flag) : 2u;  // j < 0: the idle start, prefix 0
        const uint64_t m0 = __ballot(fl == 0), m2 = __ballot(fl == 2);
        const uint32_t f2 = m2 ? (uint32_t)__builtin_ctzll(m2) : 64u;
        const uint64_t below = f2 >= 64 ? ~0ull : ((1ull << f2) - 1);
        if (m0 & below) {  // a chunk this one needs has not published yet
          __builtin_amdgcn_s_sleep(1);
          ++spins;
          continue;
        }
        // chunks nearer than the first inclusive prefix give their own key,
        // that chunk its prefix (the order does not matter for a max)
        int64_t m = kKeyMin;
        if (lane < f2 && j >= 0) m = (int64_t)ld_relaxed(&cs[j].B);
        if (lane == f2) m = j >= 0 ? (int64_t)ld_relaxed(&cs[j].P) : 0;
        run = max_i64(run, read_lane(wave_max_scan(m), 63));
        if (f2 < 64) {
          cin = run;
          break;
        }
        top -= 64;
      }
    }
    if (lane == 0) {
      st_relaxed(&cs[chunk].P, (uint64_t)max_i64(cin, agg));
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
      st_flag(&cs[chunk].flag, 2u);
      s_carry = cin;
    }
  }
  __syncthreads();
  int64_t cin = s_carry, pre;
  fold_totals<NW>(wtot, wave, cin, pre);
  T o[kPer] = {0, 0, 0, 0};
  QAcc q;
  q.bad = in_bad;
  queue_finish1<T, FUSED, false>(k, P, base, N, max_i64(pre, exc), key, ar, off, stm, o, hist, lut, q);
  if constexpr (FUSED) track4<T>(k, out, base, N, o);  // a fused leaf's row is final (F)
  store4t<T>(out, base, N, o);
  flag_overflow(k, q.bad);
  if (k.quiet) return;
  des_flush_waits<kDesThreads>(k, P.row, q.wsum, q.max_wait(), chunk == 0 ? N : 0, chunk == 0 ? N * P.hold : 0, red);
  if constexpr (FUSED) {
    __syncthreads();
    des_flush_durations<kDesThreads>(k, P, hist, q.dsum - q.d1, q.d1, q.n5, red);
  }
}

template <typename T, bool FUSED>
__global__ void __launch_bounds__(kDesThreads, 8) des_down_chain(DesK k) {
  const uint32_t ticket = chain_ticket(k);
  chain_body<T, FUSED>(k, k.level_pos[k.level_begin + ticket / k.n_chunks], ticket % k.n_chunks);
}

template <typename T>
__global__ void __launch_bounds__(kDesThreads, 8) des_down_chain_mix(DesK k) {
  const uint32_t ticket = chain_ticket(k);
  const uint32_t v = k.level_pos[k.level_begin + ticket / k.n_chunks];
  if (k.pos[v].flags & kDesFlagFused) chain_body<T, true>(k, v, ticket % k.n_chunks);
  else chain_body<T, false>(k, v, ticket % k.n_chunks);
}

// ---- pipelined queue pass: the single-replica positions of
// consecutive rounds in ONE launch, one workgroup per position, tickets in the
// plan's round order.  A position whose arrivals are its caller's start row
// waits chunk by chunk for the caller to publish them (the caller's ticket is
// earlier, so it is resident and progressing): no level boundaries, no tail
// of one level in front of the next.
// N32: every chunk takes the 32-bit keys (narrow rows; the host checked the
// segment's holds and offsets, DesPlan::pipe_n32): the launch holds no 64-bit
// key code, so it runs at more waves per SIMD
template <typename T, bool FUSED, bool HAND_IN, bool N32 = false>
__device__ __forceinline__ void pipe_body(const DesK &k, uint32_t v, uint32_t dep) {
  constexpr uint32_t NW = kDownThreads / 64;
  constexpr bool HAND_OUT = !FUSED;  // non-leaves: their callees may read the start row in this launch
  __shared__ int64_t wtot[2][NW];
  __shared__ uint64_t red[3 * NW];
  __shared__ uint32_t hist[2 * ISIM_N_PROM];
  __shared__ __attribute__((aligned(4))) uint8_t lut[4 * kBucketLutWords];
  __shared__ uint32_t s_known;
  const DesPos P = k.pos[v];
  if constexpr (FUSED) {
    for (uint32_t i = threadIdx.x; i < 2 * ISIM_N_PROM; i += kDownThreads) hist[i] = 0;
    des_bucket_lut_init(lut);
    __syncthreads();
  }
  const uint64_t N = k.N;
  const T *par = arrival_row<T>(k, v, P);
  const uint64_t off = par ? P.off : 0;
  T *out = row<T>(FUSED ? k.WF : k.W, k.ld, v);  // a fused leaf stores its finish
  QAcc q;
  int64_t carry = 0;
  uint32_t buf = 0, known = 0, chunk = 0;
  // the caller's chunks [0, chunk] published (one lane polls, the barrier
  // shares the count; bounded: a timeout drops the batch, never expected)
  auto wait = [&]() {
    if constexpr (HAND_IN) {
      if (known <= chunk) {
        if (threadIdx.x == 0) {
          uint32_t pv, spins = 0;
          while ((pv = ld_flag(k.prog + dep)) <= chunk) {
            if (spins++ >= k.spin_limit) {  // never expected: fail the batch
              atomicOr(k.ovf, kDesOvfFault);
              pv = 0xFFFFFFFFu;
              break;
            }
            __builtin_amdgcn_s_sleep(2);
          }
          s_known = pv;
        }
        __syncthreads();
        known = s_known;
      }
    }
  };
  constexpr uint64_t CH = (uint64_t)kPer * kDownThreads;
  uint64_t c0 = 0;
  if constexpr (N32 && sizeof(T) == 4) {
    const uint32_t jh0 = (threadIdx.x & 15u) * kN32 * (uint32_t)P.hold;
    constexpr uint64_t CH32 = (uint64_t)kN32 * kDownThreads;
    auto chunks = [&](auto entry_t) {
      constexpr bool ENTRY = decltype(entry_t)::value;
#pragma unroll 1
      for (; c0 + CH32 <= N; c0 += CH32, ++chunk) {
        wait();
        down1_chunk_n32<FUSED, HAND_IN, HAND_OUT, true, ENTRY>(k, P, v, par, out, c0, wtot[buf], carry, hist, lut, q,
                                                               chunk, jh0);
        buf ^= 1u;
      }
      if (c0 < N) {
        wait();
        down1_chunk_n32<FUSED, HAND_IN, HAND_OUT, false, ENTRY>(k, P, v, par, out, c0, wtot[buf], carry, hist, lut, q,
                                                                chunk, jh0);
        ++chunk;
      }
    };
    if (par) chunks(std::false_type{});
    else chunks(std::true_type{});
  } else {
    // (no 32-bit chunks here: a caller and its callees must count chunks of
    // one size, and this launch has positions the 32-bit keys do not fit)
#pragma unroll 1
    for (; c0 + CH <= N; c0 += CH, ++chunk) {
      wait();
      down1_chunk<T, FUSED, true, HAND_IN, HAND_OUT>(k, P, v, par, off, out, c0, wtot[buf], carry, hist, lut, q, chunk);
      buf ^= 1u;
    }
    if (c0 < N) {
      wait();
      down1_chunk<T, FUSED, false, HAND_IN, HAND_OUT>(k, P, v, par, off, out, c0, wtot[buf], carry, hist, lut, q, chunk);
      ++chunk;
    }
  }
  if constexpr (HAND_OUT) {
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's last stores
    __syncthreads();
    if (threadIdx.x == 0) st_flag(k.prog + v, chunk);
  }
  flag_overflow(k, q.bad);
  if (k.quiet) return;
  des_flush_waits<kDownThreads>(k, P.row, q.wsum, q.max_wait(), N, N * P.hold, red);
  if constexpr (FUSED) {
    __syncthreads();
    des_flush_durations<kDownThreads>(k, P, hist, q.dsum - q.d1, q.d1, q.n5, red);
  }
}

#ifndef ISIM_DES_PIPE32_WAVES
#define ISIM_DES_PIPE32_WAVES 6  // waves per SIMD of the 32-bit-key pipelined pass
#endif
template <typename T, bool N32>
__global__ void __launch_bounds__(kDownThreads, N32 ? ISIM_DES_PIPE32_WAVES : ISIM_DES_DOWN_WAVES)
    des_down_pipe(DesK k) {
  const uint32_t t = chain_ticket(k);
  const uint32_t v = k.level_pos[k.level_begin + t], dep = k.pipe_dep[k.level_begin + t];
  if (k.pos[v].flags & kDesFlagFused) {
    if (dep != kDesNone) pipe_body<T, true, true, N32>(k, v, dep);
    else pipe_body<T, true, false, N32>(k, v, dep);
  } else {
    if (dep != kDesNone) pipe_body<T, false, true, N32>(k, v, dep);
    else pipe_body<T, false, false, N32>(k, v, dep);
  }
}

// One thread's 4 consecutive traces of the up pass (FULL: all below te, so
// every row access is one vector load).  Every load of the quad is issued
// before any arithmetic (start, arrival and step-begin rows, the status word,
// the first kUpCB children's finish rows: one memory round trip, not five);
// children past kUpCB (hubs) follow in batches.  `ch`: the child positions,
// staged in LDS by the workgroup when they fit.
#ifndef ISIM_DES_UP_CB
#define ISIM_DES_UP_CB 2  // round 3: 3 -> 2 (with the 256-thread queue pass: 36.4 -> 36.1 ms per c5 step)
#endif
#ifndef ISIM_DES_UP_WAVES
#define ISIM_DES_UP_WAVES 6  // waves per SIMD the up pass is compiled for (80 VGPRs: no spills)
#endif
template <typename T>
constexpr uint32_t kUpCB = sizeof(T) == 4 ? ISIM_DES_UP_CB : 2;  // children rows in flight with the rest
constexpr uint32_t kUpChildLds = kDesUpChildLds;  // child ids staged in LDS per workgroup
// Per-block state of the durations a caller records for its flagged callees
// (kDesFlagParentDur): per callee (index j < kDesDurKids) the histogram, the
// start sum S(caller) over the traces where the callee responded 500 and
// their count; the callee's own block adds its finish sums by status, the
// caller's subtracts the arrivals S(caller) + off (Σ over all its traces: ss).
struct UpKids {
  uint32_t nd;                // flagged callees
  const uint32_t *dch;        // [j]: the callee's position
  const uint64_t *doff;       // [j]: the callee's off
  uint32_t *dhist;            // [j][2 * ISIM_N_PROM]
  unsigned long long *ds5;    // [j]
  uint32_t *dn5;              // [j]
};

// OWN: the block records its position's durations (its arrival row is read);
// else they are 0 (the entry: des_finalize) or its caller's (PDUR sums: the
// finishes by status).  DK: the block records its flagged callees' durations.
// NS: the finish needs no start row (kDesFlagNoStart, no callee durations here)
template <typename T, bool FULL, bool OWN, bool DK, bool NS = false>
__device__ __forceinline__ void up_quad(const DesK &k, const DesPos &P, uint32_t v, uint64_t b0, uint64_t te,
                                        T *fin, const T *arow, uint64_t off, bool leaf, bool pdur,
                                        const T *mrow, uint32_t c_max_from, const uint32_t *ch,
                                        const uint32_t (&id0)[kUpCB<T>], uint32_t *hist, const uint8_t *lut,
                                        const UpKids &dk, uint64_t &ss,
                                        uint64_t &dsum0, uint64_t &dsum1, uint64_t &n500, bool &bad) {
  __asm__ volatile("" : "+v"(b0));  // opaque to loop strength reduction (down1_chunk)
  const uint64_t n = FULL ? b0 + kPer : te;
  const uint32_t cnt = leaf ? 0u : P.child_cnt;
  T ar[kPer], mr[kPer];
  T f0[kUpCB<T>][kPer];
  // 1. the loads (no branch around the row loads: a branch that merges
  // loaded values makes the compiler wait for them inside it)
  if constexpr (OWN) load4t<T>(arow, b0, n, ar);
  if constexpr (NS) {
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) mr[i] = 0;
  } else {
    load4t<T>(mrow, b0, n, mr);
  }
  const uint32_t stm = des_status4(k, v, b0);
#pragma unroll
  for (uint32_t j = 0; j < kUpCB<T>; ++j)
    if (j < cnt) load4t<T>(row<T>(k.WF, k.ld, id0[j]), b0, n, f0[j]);
  // 2. the arithmetic
  uint64_t a[kPer], m[kPer];
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    a[i] = OWN ? (uint64_t)ar[i] + off : 0;
    m[i] = NS ? 0 : (uint64_t)mr[i] + P.floor;  // NS: max_c F(c) >= S + floor
    if constexpr (DK) ss += FULL || b0 + i < te ? (uint64_t)mr[i] : 0;  // S(caller): no step begins (plan)
  }
  uint32_t sto = 0;  // children's 500s, bit i
  if (cnt) {
    T cm[kPer] = {0, 0, 0, 0};
    auto take = [&](const T (&f)[kPer], bool in_max) {
#pragma unroll
      for (uint32_t i = 0; i < kPer; ++i) {
        const T tc = f[i] & (T)Row<T>::kMask;
        if (in_max) cm[i] = tc > cm[i] ? tc : cm[i];
        sto |= (uint32_t)(f[i] >> Row<T>::kTop) << i;
      }
    };
#pragma unroll
    for (uint32_t j = 0; j < kUpCB<T>; ++j)
      if (j < cnt) take(f0[j], j >= c_max_from);
    for (uint32_t c = kUpCB<T>; c < cnt; c += kUpCB<T>) {
      T f[kUpCB<T>][kPer];
#pragma unroll
      for (uint32_t j = 0; j < kUpCB<T>; ++j)
        if (c + j < cnt) load4t<T>(row<T>(k.WF, k.ld, ch[c + j]), b0, n, f[j]);
#pragma unroll
      for (uint32_t j = 0; j < kUpCB<T>; ++j)
        if (c + j < cnt) take(f[j], c + j >= c_max_from);
    }
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) m[i] = (uint64_t)cm[i] > m[i] ? (uint64_t)cm[i] : m[i];
  }
  uint64_t o[kPer];
  uint32_t bin[kPer] = {kNoBin, kNoBin, kNoBin, kNoBin};
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    const uint64_t t = b0 + i;
    o[i] = 0;
    if (FULL || t < te) {
      const uint64_t F = leaf ? m[i] : m[i] + P.post;
      const uint32_t own = (stm >> i) & 1u;
      const uint32_t st = k.modeb ? (own | ((sto >> i) & 1u)) : own;
      // OWN: the duration; a caller-recorded position: its finish (the
      // caller subtracts the arrival); the entry: 0 (des_finalize)
      const uint64_t dur = OWN ? F - a[i] : pdur ? F : 0;
      bad |= !Row<T>::fits(F);
      o[i] = F | ((uint64_t)st << Row<T>::kTop);
      if (st && !k.quiet) atomicAdd(k.E + t, 1u);
      n500 += st;
      dsum1 += st ? dur : 0;
      dsum0 += st ? 0 : dur;
      if constexpr (OWN) bin[i] = st * ISIM_N_PROM + des_prom_bucket(lut, dur);
    }
  }
  if constexpr (OWN) hist_add4<FULL>(hist, bin);
  if (k.changed) {
    T ot[kPer];
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) ot[i] = (T)o[i];
    track4<T>(k, fin, b0, n, ot);
  }
  store4n<T>(fin, b0, n, o);
  if constexpr (DK) {
    // the flagged callees' durations F(c) - (S + off(c)): their finish rows
    // again (just read above: cache hits), after the quad's own work so the
    // children loop keeps its registers
    for (uint32_t j = 0; j < dk.nd; ++j) {
      T f[kPer];
      load4t<T>(row<T>(k.WF, k.ld, dk.dch[j]), b0, n, f);
      const uint64_t offc = dk.doff[j];
      uint32_t cb[kPer] = {kNoBin, kNoBin, kNoBin, kNoBin};
#pragma unroll
      for (uint32_t i = 0; i < kPer; ++i) {
        if (FULL || b0 + i < te) {
          const uint64_t dur = (uint64_t)(f[i] & (T)Row<T>::kMask) - ((uint64_t)mr[i] + offc);
          const uint32_t st = (uint32_t)(f[i] >> Row<T>::kTop);
          cb[i] = st * ISIM_N_PROM + des_prom_bucket(lut, dur);
          if (st) {
            atomicAdd(dk.ds5 + j, (unsigned long long)mr[i]);
            atomicAdd(dk.dn5 + j, 1u);
          }
        }
      }
      hist_add4<FULL>(dk.dhist + j * 2 * ISIM_N_PROM, cb);
    }
  }
}

// up_quad for narrow rows in 32-bit arithmetic (round 3): every value below
// 2^31 + 2^30 (row values < 2^31, the host-checked off / floor / post
// < 2^30: DesPlan::up_n32), so no 64-bit time in the quad — fewer VGPRs,
// more waves of loads in flight.  The same results as up_quad<uint32_t, ...>.
template <bool FULL, bool OWN, bool DK, bool NS>
__device__ __forceinline__ void up_quad32(const DesK &k, const DesPos &P, uint32_t v, uint64_t b0, uint64_t te,
                                          uint32_t *fin, const uint32_t *arow, uint32_t off32, bool leaf, bool pdur,
                                          const uint32_t *mrow, const uint32_t *ch, const uint32_t (&id0)[kUpCB<uint32_t>],
                                          uint32_t *hist, const uint8_t *lut, const UpKids &dk, uint64_t &ss,
                                          uint64_t &dsum0, uint64_t &dsum1, uint32_t &n500, bool &bad) {
  using T = uint32_t;
  __asm__ volatile("" : "+v"(b0));  // opaque to loop strength reduction (down1_chunk)
  const uint64_t n = FULL ? b0 + kPer : te;
  const uint32_t cnt = leaf ? 0u : P.child_cnt;
  T ar[kPer], mr[kPer];
  T f0[kUpCB<T>][kPer];
  if constexpr (OWN) load4t<T>(arow, b0, n, ar);
  if constexpr (NS) {
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) mr[i] = 0;
  } else {
    load4t<T>(mrow, b0, n, mr);
  }
  const uint32_t stm = des_status4(k, v, b0);
#pragma unroll
  for (uint32_t j = 0; j < kUpCB<T>; ++j)
    if (j < cnt) load4t<T>(row<T>(k.WF, k.ld, id0[j]), b0, n, f0[j]);
  const uint32_t floor32 = (uint32_t)P.floor, post32 = leaf ? 0u : (uint32_t)P.post;
  uint32_t m[kPer];
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    m[i] = NS ? 0u : mr[i] + floor32;  // NS: max_c F(c) >= S + floor
    if constexpr (DK) ss += FULL || b0 + i < te ? (uint64_t)mr[i] : 0;
  }
  uint32_t sto = 0;  // children's 500s, bit i
  auto take = [&](const T (&f)[kPer]) {
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) {
      const T tc = f[i] & 0x7FFFFFFFu;
      m[i] = tc > m[i] ? tc : m[i];
      sto |= (f[i] >> 31) << i;
    }
  };
#pragma unroll
  for (uint32_t j = 0; j < kUpCB<T>; ++j)
    if (j < cnt) take(f0[j]);
  for (uint32_t c = kUpCB<T>; c < cnt; c += kUpCB<T>) {
    T f[kUpCB<T>][kPer];
#pragma unroll
    for (uint32_t j = 0; j < kUpCB<T>; ++j)
      if (c + j < cnt) load4t<T>(row<T>(k.WF, k.ld, ch[c + j]), b0, n, f[j]);
#pragma unroll
    for (uint32_t j = 0; j < kUpCB<T>; ++j)
      if (c + j < cnt) take(f[j]);
  }
  T o[kPer];
  uint32_t bin[kPer] = {kNoBin, kNoBin, kNoBin, kNoBin}, big = 0;
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    const uint64_t t = b0 + i;
    o[i] = 0;
    if (FULL || t < te) {
      const uint32_t F = m[i] + post32;
      const uint32_t own = (stm >> i) & 1u;
      const uint32_t st = k.modeb ? (own | ((sto >> i) & 1u)) : own;
      // OWN: the duration; a caller-recorded position: its finish (the
      // caller subtracts the arrival); the entry: 0 (des_finalize)
      const uint32_t dur = OWN ? F - (ar[i] + off32) : pdur ? F : 0u;
      big |= F;
      o[i] = F | (st << 31);
      if (st && !k.quiet) atomicAdd(k.E + t, 1u);
      n500 += st;
      dsum1 += st ? dur : 0u;
      dsum0 += st ? 0u : dur;
      if constexpr (OWN) bin[i] = st * ISIM_N_PROM + des_prom_bucket32(lut, dur);
    }
  }
  bad |= (big >> 31) != 0u;
  if constexpr (OWN) hist_add4<FULL>(hist, bin);
  if (k.changed) track4<T>(k, fin, b0, n, o);
  if constexpr (FULL) store4t<T>(fin, b0, n, o);
  else {
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i)
      if (b0 + i < te) fin[b0 + i] = o[i];
  }
  if constexpr (DK) {
    // the flagged callees' durations F(c) - (S + off(c)) (up_quad)
    for (uint32_t j = 0; j < dk.nd; ++j) {
      T f[kPer];
      load4t<T>(row<T>(k.WF, k.ld, dk.dch[j]), b0, n, f);
      const uint32_t offc = (uint32_t)dk.doff[j];
      uint32_t cb[kPer] = {kNoBin, kNoBin, kNoBin, kNoBin};
#pragma unroll
      for (uint32_t i = 0; i < kPer; ++i) {
        if (FULL || b0 + i < te) {
          const uint32_t dur = (f[i] & 0x7FFFFFFFu) - (mr[i] + offc);
          const uint32_t st = f[i] >> 31;
          cb[i] = st * ISIM_N_PROM + des_prom_bucket32(lut, dur);
          if (st) {
            atomicAdd(dk.ds5 + j, (unsigned long long)mr[i]);
            atomicAdd(dk.dn5 + j, 1u);
          }
        }
      }
      hist_add4<FULL>(dk.dhist + j * 2 * ISIM_N_PROM, cb);
    }
  }
}

// ---- up pass: finish times, statuses, per-service durations.
// (position, trace-range) blocks; 4 consecutive traces per thread.
#ifndef ISIM_DES_UP32_WAVES
#define ISIM_DES_UP32_WAVES 7  // 69 VGPRs: no spills at 7 (35.6 -> 35.4 ms per c5 step), 8 spill
#endif
// N32: narrow rows and every finish constant below 2^30 (DesPlan::up_n32): up_quad32
template <typename T, bool N32>
__global__ void __launch_bounds__(kDesUpThreads, N32 ? ISIM_DES_UP32_WAVES : ISIM_DES_UP_WAVES) des_up(DesK k) {
  __shared__ uint32_t hist[2 * ISIM_N_PROM];
  __shared__ uint64_t red[3 * kDesUpThreads / 64];
  __shared__ __attribute__((aligned(4))) uint8_t lut[4 * kBucketLutWords];
  __shared__ uint64_t s_doff[kDesDurKids];
  __shared__ uint32_t s_dch[kDesDurKids], s_nd;
  __shared__ uint32_t dhist[kDesDurKids * 2 * ISIM_N_PROM];
  __shared__ unsigned long long ds5[kDesDurKids];
  __shared__ uint32_t dn5[kDesDurKids];
  for (uint32_t i = threadIdx.x; i < 2 * ISIM_N_PROM; i += kDesUpThreads) hist[i] = 0;
  des_bucket_lut_init(lut);
  if (threadIdx.x == 0) s_nd = 0;
  const uint32_t v = k.level_pos[k.level_begin + blockIdx.y];
  const DesPos P = k.pos[v];
  const uint64_t N = k.N;
  // trace range: split boundaries on multiples of 16 (aligned vector accesses)
  const uint64_t tb = blockIdx.x ? (N * blockIdx.x / k.splits) & ~15ull : 0;
  const uint64_t te = blockIdx.x + 1 == k.splits ? N : (N * (blockIdx.x + 1) / k.splits) & ~15ull;
  const T *mine = row<T>(k.W, k.ld, v);
  T *fin = row<T>(k.WF, k.ld, v);
  const DesPosExt X = k.ext[v];
  const T *par = arrival_row<T>(k, v, P);
  const uint64_t off = par ? P.off : 0;
  const bool leaf = P.flags & kDesFlagLeaf;
  const bool pdur = (P.flags & kDesFlagParentDur) != 0;
  const bool own = par && !pdur;  // the block records the position's durations
  // several call steps: F = max(BK_last + floor, max F(last step's callees)) + post
  const T *base_t = X.bk_last == kDesNone ? nullptr : row<T>(k.BK, k.ld, X.bk_last);
  const uint32_t c_max_from = X.bk_last == kDesNone ? 0u : X.last_child;
  uint64_t dsum0 = 0, dsum1 = 0, n500 = 0, ss = 0;
  uint32_t n500_32 = 0;
  bool bad = false;
  // rows read: the arrival row when the block records the durations, and the
  // row F's floor starts from (the last step's begin, or S)
  const T *arow = par;
  const T *mrow = base_t ? base_t : mine;
  // the child positions: in LDS when they fit (read by every quad; LDS
  // addressing known to the compiler, not flat), else from global memory;
  // with them, which are flagged callees (the plan flags only callees of
  // callers with at most kUpChildLds children)
  __shared__ uint32_t s_ch[kUpChildLds];
  const uint32_t cnt = leaf ? 0u : P.child_cnt;
  const uint32_t *gch = k.child + P.child_off;
  __syncthreads();  // s_nd
  UpKids dk{0, s_dch, s_doff, dhist, ds5, dn5};
  auto run = [&](const uint32_t *ch, auto own_t, auto dk_t, auto ns_t) {
    constexpr bool OWN = decltype(own_t)::value, DK = decltype(dk_t)::value, NS = decltype(ns_t)::value;
    // the first children's positions in (uniform) registers for the whole
    // range: their row loads issue with the others, no id load in front
    uint32_t id0[kUpCB<T>];
#pragma unroll
    for (uint32_t j = 0; j < kUpCB<T>; ++j) id0[j] = j < cnt ? ch[j] : 0u;
    for (uint64_t b0 = tb + (uint64_t)threadIdx.x * kPer; b0 < te; b0 += (uint64_t)kPer * kDesUpThreads) {
      if constexpr (N32 && sizeof(T) == 4) {
        if (b0 + kPer <= te)
          up_quad32<true, OWN, DK, NS>(k, P, v, b0, te, fin, arow, (uint32_t)off, leaf, pdur, mrow, ch, id0, hist, lut,
                                       dk, ss, dsum0, dsum1, n500_32, bad);
        else
          up_quad32<false, OWN, DK, NS>(k, P, v, b0, te, fin, arow, (uint32_t)off, leaf, pdur, mrow, ch, id0, hist, lut,
                                        dk, ss, dsum0, dsum1, n500_32, bad);
      } else {
        if (b0 + kPer <= te)
          up_quad<T, true, OWN, DK, NS>(k, P, v, b0, te, fin, arow, off, leaf, pdur, mrow, c_max_from, ch, id0, hist,
                                        lut, dk, ss, dsum0, dsum1, n500, bad);
        else
          up_quad<T, false, OWN, DK, NS>(k, P, v, b0, te, fin, arow, off, leaf, pdur, mrow, c_max_from, ch, id0, hist,
                                         lut, dk, ss, dsum0, dsum1, n500, bad);
      }
    }
  };
  using tt = std::true_type;
  using ff = std::false_type;
  uint32_t nd = 0;
  if (cnt <= kUpChildLds) {
    for (uint32_t i = threadIdx.x; i < cnt; i += kDesUpThreads) {
      const uint32_t c = gch[i];
      s_ch[i] = c;
      const uint32_t f = k.pos[c].flags;
      if (f & kDesFlagParentDur) {
        const uint32_t j = (f >> kDesDurShift) & 0xFFu;
        s_doff[j] = k.pos[c].off;
        s_dch[j] = c;
        atomicMax(&s_nd, j + 1);
      }
    }
    __syncthreads();
    nd = s_nd;
    dk.nd = nd;
    for (uint32_t i = threadIdx.x; i < nd * 2 * ISIM_N_PROM; i += kDesUpThreads) dhist[i] = 0;
    if (threadIdx.x < nd) {
      ds5[threadIdx.x] = 0;
      dn5[threadIdx.x] = 0;
    }
    __syncthreads();
    const bool ns = (P.flags & kDesFlagNoStart) != 0;
    if (nd) {
      if (own) run(s_ch, tt{}, tt{}, ff{});
      else run(s_ch, ff{}, tt{}, ff{});
    } else if (ns) {
      if (own) run(s_ch, tt{}, ff{}, tt{});
      else run(s_ch, ff{}, ff{}, tt{});
    } else {
      if (own) run(s_ch, tt{}, ff{}, ff{});
      else run(s_ch, ff{}, ff{}, ff{});
    }
  } else {
    if (own) run(gch, tt{}, ff{}, ff{});
    else run(gch, ff{}, ff{}, ff{});
  }
  n500 += n500_32;
  flag_overflow(k, bad);
  if (k.quiet) return;
  if (nd) {
    // the flagged callees' histograms, and their duration sums less the
    // arrivals: Σ (S + off) over this block's traces, by the callee's status
#pragma unroll
    for (uint32_t d = 32; d > 0; d >>= 1) ss += __shfl_xor(ss, d, 64);
    if ((threadIdx.x & 63u) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    uint64_t sall = 0;
#pragma unroll
    for (uint32_t w = 0; w < kDesUpThreads / 64; ++w) sall += red[w];
    for (uint32_t i = threadIdx.x; i < nd * 2 * ISIM_N_PROM; i += kDesUpThreads) {
      const uint32_t j = i / (2 * ISIM_N_PROM), b = i - j * (2 * ISIM_N_PROM);
      if (dhist[i])
        atomicAdd((unsigned long long *)(k.table + (uint64_t)k.pos[s_dch[j]].row * ISIM_DES_ROW_WORDS + b),
                  (unsigned long long)dhist[i]);
    }
    if (threadIdx.x < nd) {
      const uint32_t j = threadIdx.x;
      const uint64_t s5 = ds5[j], n5 = dn5[j], offc = s_doff[j];
      const uint64_t a1 = s5 + n5 * offc, a0 = (sall - s5) + ((te - tb) - n5) * offc;
      unsigned long long *trow =
          (unsigned long long *)(k.table + (uint64_t)k.pos[s_dch[j]].row * ISIM_DES_ROW_WORDS);
      if (a0) atomicAdd(trow + 2 * ISIM_N_PROM, (unsigned long long)(0 - a0));
      if (a1) atomicAdd(trow + 2 * ISIM_N_PROM + 1, (unsigned long long)(0 - a1));
    }
    __syncthreads();  // red is reused below
  }
  des_flush_durations<kDesUpThreads>(k, P, hist, dsum0, dsum1, n500, red);
}

// ---- finalize: records and the latency statistics
template <typename T>
__global__ void __launch_bounds__(kDesUpThreads) des_finalize(DesK k) {
  __shared__ uint32_t hp[2 * ISIM_N_PROM], hl[2 * ISIM_N_LOG2];
  __shared__ uint64_t red[6 * kDesUpThreads / 64];
  __shared__ __attribute__((aligned(4))) uint8_t lut[4 * kBucketLutWords];
  for (uint32_t i = threadIdx.x; i < 2 * ISIM_N_PROM; i += kDesUpThreads) hp[i] = 0;
  for (uint32_t i = threadIdx.x; i < 2 * ISIM_N_LOG2; i += kDesUpThreads) hl[i] = 0;
  des_bucket_lut_init(lut);
  __syncthreads();
  const uint64_t N = k.N;
  // an overflowed narrow batch is dropped (des_commit): records untouched
  const bool keep = *k.ovf == 0;
  const T *F0 = row<T>(k.WF, k.ld, 0);  // position 0: the entry
  uint64_t sl = 0, s5 = 0, se = 0, n5 = 0, mn = ~0ull, mx = 0;
  for (uint64_t t = (uint64_t)blockIdx.x * kDesUpThreads + threadIdx.x; t < N;
       t += (uint64_t)gridDim.x * kDesUpThreads) {
    const uint64_t F = F0[t];
    const uint32_t st = (uint32_t)(F >> Row<T>::kTop);
    const uint64_t L = (F & Row<T>::kMask) - (k.A[t] - des_gbase(k, t));  // the latency
    const uint32_t e = k.E[t];
    if (k.records && keep) {
      isim_trace_rec r;
      r.latency_ns = L;
      r.hops = k.n_pos;
      r.status_err = (st << 31) | e;
      k.records[t] = r;
    }
    sl += L;
    s5 += st ? L : 0;
    se += e;
    n5 += st;
    mn = L < mn ? L : mn;
    mx = L > mx ? L : mx;
    atomicAdd(&hp[st * ISIM_N_PROM + des_prom_bucket(lut, L)], 1u);
    atomicAdd(&hl[st * ISIM_N_LOG2 + (L ? 64u - (uint32_t)__builtin_clzll(L) : 0u)], 1u);
  }
#pragma unroll
  for (uint32_t d = 32; d > 0; d >>= 1) {
    sl += __shfl_xor(sl, d, 64);
    s5 += __shfl_xor(s5, d, 64);
    se += __shfl_xor(se, d, 64);
    n5 += __shfl_xor(n5, d, 64);
    const uint64_t a = __shfl_xor(mn, d, 64), b = __shfl_xor(mx, d, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  constexpr uint32_t W = kDesUpThreads / 64;
  if ((threadIdx.x & 63u) == 0) {
    const uint32_t w = threadIdx.x >> 6;
    red[w] = sl;
    red[W + w] = se;
    red[2 * W + w] = n5;
    red[3 * W + w] = mn;
    red[4 * W + w] = mx;
    red[5 * W + w] = s5;
  }
  __syncthreads();
  unsigned long long *st = (unsigned long long *)k.stats;
  // the entry's invocation durations (RecordResponseSent) are the latencies;
  // des_up leaves them here unless the entry finished in its queue pass
  const bool entry_dur = !(k.pos[0].flags & kDesFlagFused);
  unsigned long long *trow = (unsigned long long *)(k.table + (uint64_t)k.pos[0].row * ISIM_DES_ROW_WORDS);
  for (uint32_t i = threadIdx.x; i < 2 * ISIM_N_PROM; i += kDesUpThreads)
    if (hp[i]) {
      atomicAdd(st + ISIM_ST_PROM + i, (unsigned long long)hp[i]);
      if (entry_dur) atomicAdd(trow + i, (unsigned long long)hp[i]);
    }
  for (uint32_t i = threadIdx.x; i < 2 * ISIM_N_LOG2; i += kDesUpThreads)
    if (hl[i]) atomicAdd(st + ISIM_ST_LOG2 + i, (unsigned long long)hl[i]);
  if (threadIdx.x == 0) {
    for (uint32_t i = 1; i < W; ++i) {
      red[0] += red[i];
      red[W] += red[W + i];
      red[2 * W] += red[2 * W + i];
      red[3 * W] = red[3 * W + i] < red[3 * W] ? red[3 * W + i] : red[3 * W];
      red[4 * W] = red[4 * W + i] > red[4 * W] ? red[4 * W + i] : red[4 * W];
      red[5 * W] += red[5 * W + i];
    }
    if (entry_dur) {
      if (red[0] - red[5 * W]) atomicAdd(trow + 2 * ISIM_N_PROM, (unsigned long long)(red[0] - red[5 * W]));
      if (red[5 * W]) atomicAdd(trow + 2 * ISIM_N_PROM + 1, (unsigned long long)red[5 * W]);
    }
    if (blockIdx.x == 0) {
      atomicAdd(st + ISIM_ST_N_TRACES, (unsigned long long)N);
      atomicAdd(st + ISIM_ST_SUM_HOPS, (unsigned long long)(N * k.n_pos));
    }
    atomicAdd(st + ISIM_ST_SUM_LATENCY, (unsigned long long)red[0]);
    atomicAdd(st + ISIM_ST_SUM_ERR_HOPS, (unsigned long long)red[W]);
    atomicAdd(st + ISIM_ST_N_500, (unsigned long long)red[2 * W]);
    if (red[3 * W] != ~0ull) atomicMax(st + ISIM_ST_NOT_MIN_LATENCY, (unsigned long long)~red[3 * W]);
    atomicMax(st + ISIM_ST_MAX_LATENCY, (unsigned long long)red[4 * W]);
  }
}

// ---- sort path: arrivals of all positions of one service,
// item i = t * P + j (j = the position's rank in hop order), keyed by
// (replica | absolute arrival), so a stable sort groups each replica's
// queue contiguously with ties in (t, hop) order
template <typename T>
__global__ void __launch_bounds__(kDesUpThreads) des_sort_keys(DesK k) {
  const uint32_t P = k.svc.pos_cnt;
  const uint64_t M = k.N * P;
  for (uint64_t i = (uint64_t)blockIdx.x * kDesUpThreads + threadIdx.x; i < M;
       i += (uint64_t)gridDim.x * kDesUpThreads) {
    const uint64_t t = i / P;
    const uint32_t v = k.sort_pos[k.svc.pos_off + (uint32_t)(i - t * P)];
    const uint64_t a = des_gbase(k, t) + des_arrival<T>(k, v, k.pos[v], t);
    const uint32_t rb = rep_bits(k.svc.reps);
    uint64_t key = a;
    if (rb) {
      const uint64_t r = des_draw(k.trace_begin + t, v, 0x80000002u, 0, k.k0, k.k1) % k.svc.reps;
      key = r << (64 - rb) | a;
      if (a >> (64 - rb)) atomicOr(k.ovf, 1u);  // never within the host's arrival-span check
    }
    k.keys[i] = key;
    k.vals[i] = (uint32_t)i;
  }
}

// FIFO scan of one sort-path service over its sorted arrivals (one
// workgroup): the replicas' queues are contiguous segments, scanned as one
// SEGMENTED max-plus scan (a segment starts with an idle worker, x = 0)
struct SegMP {
  uint64_t B, C;
  uint32_t f;  // the span contains a segment start: its input is replaced by 0
};
__device__ __forceinline__ SegMP smp_then(SegMP first, SegMP second) {
  if (second.f) return second;
  const MaxPlus m = mp_then(MaxPlus{first.B, first.C}, MaxPlus{second.B, second.C});
  return {m.B, m.C, first.f};
}
__device__ __forceinline__ uint64_t smp_apply(SegMP m, uint64_t x) {
  const uint64_t xi = m.f ? 0 : x;
  return xi + m.B > m.C ? xi + m.B : m.C;
}

template <typename T>
__global__ void __launch_bounds__(kDesThreads) des_down_sorted(DesK k) {
  __shared__ SegMP wtot[kDesThreads / 64];
  __shared__ uint64_t red[2 * kDesThreads / 64];
  __shared__ SegMP xs[kDesThreads];
  __shared__ uint64_t s_carry;
  const DesSortSvc sv = k.svc;
  const uint32_t P = sv.pos_cnt;
  const uint64_t M = k.N * P;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t rb = rep_bits(sv.reps), shift = 64 - rb;
  const uint64_t amask = rb ? (1ull << shift) - 1 : ~0ull;
  uint64_t wsum = 0, wmax = 0;
  bool bad = false;
  for (uint64_t c0 = 0; c0 < M; c0 += kDownChunk) {
    const uint64_t base = c0 + (uint64_t)threadIdx.x * kPer;
    uint64_t a[kPer], tt[kPer];
    uint32_t vv[kPer], st[kPer];
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) {
      const uint64_t q = base + i;
      a[i] = 0;
      tt[i] = 0;
      vv[i] = 0;
      st[i] = 0;
      if (q < M) {
        const uint64_t key = k.skeys[q];
        a[i] = key & amask;
        st[i] = q == 0 || (rb && (k.skeys[q - 1] >> shift) != (key >> shift));  // a replica's first item
        const uint32_t idx = k.svals[q];
        tt[i] = idx / P;
        vv[i] = k.sort_pos[sv.pos_off + (idx - (uint32_t)tt[i] * P)];
      }
    }
    SegMP f{0, 0, 0};
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i)
      if (base + i < M) f = smp_then(f, SegMP{sv.hold, a[i] + sv.hold, st[i]});
    // inclusive block scan of the segmented maps
    SegMP v = f;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      SegMP o;
      o.B = __shfl_up(v.B, d, 64);
      o.C = __shfl_up(v.C, d, 64);
      o.f = __shfl_up(v.f, d, 64);
      if (lane >= d) v = smp_then(o, v);
    }
    if (lane == 63) wtot[wave] = v;
    __syncthreads();
    if (wave == 0) {
      SegMP w = lane < kDesThreads / 64 ? wtot[lane] : SegMP{0, 0, 0};
#pragma unroll
      for (uint32_t d = 1; d < kDesThreads / 64; d <<= 1) {
        SegMP o;
        o.B = __shfl_up(w.B, d, 64);
        o.C = __shfl_up(w.C, d, 64);
        o.f = __shfl_up(w.f, d, 64);
        if (lane >= d) w = smp_then(o, w);
      }
      if (lane < kDesThreads / 64) wtot[lane] = w;
    }
    __syncthreads();
    if (wave > 0) v = smp_then(wtot[wave - 1], v);
    xs[threadIdx.x] = v;
    __syncthreads();
    const SegMP pre = threadIdx.x ? xs[threadIdx.x - 1] : SegMP{0, 0, 0};
    uint64_t x = smp_apply(pre, s_carry);
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) {
      if (base + i < M) {
        if (st[i]) x = 0;  // the replica's worker is idle before its first invocation
        const uint64_t S = x > a[i] ? x : a[i];
        const uint64_t rel = S - des_gbase(k, tt[i]);
        bad |= !Row<T>::fits(rel);
        row<T>(k.W, k.ld, vv[i])[tt[i]] = (T)rel;
        const uint64_t w = S - a[i];
        wsum += w;
        wmax = w > wmax ? w : wmax;
        x = S + sv.hold;
      }
    }
    __syncthreads();  // every thread has read s_carry
    if (threadIdx.x == kDesThreads - 1) s_carry = smp_apply(xs[kDesThreads - 1], s_carry);
    __syncthreads();
  }
  flag_overflow(k, bad);
  if (k.quiet) return;
  des_flush_waits<kDesThreads>(k, sv.row, wsum, wmax, M, M * sv.hold, red);
}

// ---- step begins (calls after calls): BK rows of one round
template <typename T>
__global__ void __launch_bounds__(kDesUpThreads) des_arrive(DesK k) {
  const uint32_t b = k.arr_ops[k.level_begin + blockIdx.y];
  const DesStep st = k.steps[b];
  const uint64_t N = k.N;
  const uint64_t tb = N * blockIdx.x / k.splits, te = N * (blockIdx.x + 1) / k.splits;
  T *out = row<T>(k.BK, k.ld, b);
  bool bad = false;
  for (uint64_t t = tb + threadIdx.x; t < te; t += kDesUpThreads) {
    uint64_t v;
    if (st.prev == kDesNone) {
      v = row<T>(k.W, k.ld, st.pos)[t];  // the position's start
    } else {
      v = (uint64_t)row<T>(k.BK, k.ld, st.prev)[t] + st.smax;
      for (uint32_t j = 0; j < st.child_cnt; ++j) {
        const uint64_t f = row<T>(k.WF, k.ld, k.child[st.child_off + j])[t] & Row<T>::kMask;
        v = f > v ? f : v;
      }
    }
    v += st.add;
    bad |= !Row<T>::fits(v);
    track1<T>(k, out + t, (T)v);
    out[t] = (T)v;
  }
  flag_overflow(k, bad);
}

// ---- zero-hold services: no queue, start = arrival (relative), per
// (position, trace-range) block; the queue statistics: N invocations, no wait
template <typename T>
__global__ void __launch_bounds__(kDesUpThreads) des_zero(DesK k) {
  const uint32_t v = k.level_pos[k.level_begin + blockIdx.y];
  const DesPos P = k.pos[v];
  const uint64_t N = k.N;
  const uint64_t tb = N * blockIdx.x / k.splits, te = N * (blockIdx.x + 1) / k.splits;
  const T *par = arrival_row<T>(k, v, P);
  const uint64_t off = par ? P.off : 0;
  T *out = row<T>(k.W, k.ld, v);
  bool bad = false;
  for (uint64_t t = tb + threadIdx.x; t < te; t += kDesUpThreads) {
    const uint64_t a = par ? (uint64_t)par[t] + off : k.A[t] - des_gbase(k, t);
    bad |= !Row<T>::fits(a);
    out[t] = (T)a;
  }
  flag_overflow(k, bad);
  if (threadIdx.x == 0 && te > tb && !k.quiet)
    atomicAdd((unsigned long long *)(k.table + (uint64_t)P.row * ISIM_DES_ROW_WORDS + ISIM_DES_COUNT),
              (unsigned long long)(te - tb));
}

// ---- narrow rows: merge the staged statistics into the caller's buffers,
// or count the batch in ISIM_ST_DES_RETRY when a value overflowed
__global__ void __launch_bounds__(256) des_commit(const uint64_t *__restrict__ stage, uint64_t *stats,
                                                  uint64_t *table, uint64_t stats_words, uint64_t table_words,
                                                  const uint32_t *ovf) {
  if (const uint32_t o = *ovf) {
    // dropped: a retry (narrow rows overflowed, no fixed point) or a fault
    // (a look-back gave up: counted in the word's high half, an error)
    if (blockIdx.x == 0 && threadIdx.x == 0)
      atomicAdd((unsigned long long *)(stats + ISIM_ST_DES_RETRY),
                (unsigned long long)((o & kDesOvfFault) ? kDesFaultUnit : 1ull));
    return;
  }
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < stats_words + table_words;
       i += (uint64_t)gridDim.x * 256) {
    const uint64_t x = stage[i];
    if (!x) continue;
    if (i < stats_words) {
      unsigned long long *p = (unsigned long long *)(stats + i);
      if (i == ISIM_ST_NOT_MIN_LATENCY || i == ISIM_ST_MAX_LATENCY) atomicMax(p, (unsigned long long)x);
      else atomicAdd(p, (unsigned long long)x);
    } else {
      const uint64_t j = i - stats_words;
      unsigned long long *p = (unsigned long long *)(table + j);
      if (j % ISIM_DES_ROW_WORDS == ISIM_DES_MAX_WAIT) atomicMax(p, (unsigned long long)x);
      else atomicAdd(p, (unsigned long long)x);
    }
  }
}

}  // namespace dev

static size_t sort_temp_bytes(uint64_t m) {
  size_t bytes = 0;
  if (m == 0) return 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                  (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)m, 0, 64);
  return bytes;
}

static uint64_t al256(uint64_t b) { return (b + 255) & ~255ull; }
static uint64_t row_ld(uint64_t n) { return (n + 15) & ~15ull; }
static uint64_t chain_tickets(const DesPlan &plan) { return 4ull * plan.rounds(); }
static uint64_t status_wpr(uint64_t n) { return (((n + 31) / 32) + 15) & ~15ull; }

// chained and pipelined down passes: tickets, per-position published chunk
// counts, chain states (all zeroed before every pass)
uint64_t des_chain_bytes(const DesPlan &plan, uint64_t n) {
  const uint64_t chunks = (n + dev::kDownChunk - 1) / dev::kDownChunk;
  return al256(chain_tickets(plan) * 4) + al256(plan.pos.size() * 4) +
         (uint64_t)plan.pos.size() * chunks * sizeof(dev::ChainState);
}

// Workspace parts, in order (256-B aligned): W and BK rows sized for u64,
// A, E, chunk sums, chain states, overflow flag, staged stats + table, sort path.
uint64_t des_workspace_bytes(const DesPlan &plan, uint64_t n, uint64_t stats_words, uint64_t table_rows) {
  const uint64_t nblk = (n + dev::kDesChunk - 1) / dev::kDesChunk;
  const uint64_t ld = row_ld(n);
  const uint64_t m = (uint64_t)plan.max_sort_pos * n;
  const uint64_t sort = m ? 2 * al256(m * 8) + 2 * al256(m * 4) + al256(sort_temp_bytes(m)) : 0;
  return 2 * al256((uint64_t)plan.pos.size() * ld * 8) + al256((uint64_t)plan.steps.size() * ld * 8) + al256(n * 8) +
         al256(n * 4) + al256((nblk + 1) * 8) + al256(des_chain_bytes(plan, n)) + 256 +
         al256((stats_words + table_rows * ISIM_DES_ROW_WORDS) * 8) +
         al256((uint64_t)plan.pos.size() * status_wpr(n) * 4) + sort;
}

void des_carve(DesLaunch &L, void *workspace) {
  const DesPlan &plan = *L.plan;
  const uint64_t n = L.n_traces, ld = row_ld(n);
  char *ws = (char *)workspace;
  auto take = [&](uint64_t bytes) {
    char *p = ws;
    ws += al256(bytes);
    return p;
  };
  L.W = take((uint64_t)plan.pos.size() * ld * 8);
  L.WF = take((uint64_t)plan.pos.size() * ld * 8);
  L.BK = take((uint64_t)plan.steps.size() * ld * 8);
  L.A = (uint64_t *)take(n * 8);
  L.E = (uint32_t *)take(n * 4);
  L.blk = (uint64_t *)take(((n + dev::kDesChunk - 1) / dev::kDesChunk + 1) * 8);
  L.chain = take(des_chain_bytes(plan, n));
  L.ovf = (uint32_t *)take(4);
  L.stage = (uint64_t *)take((L.stats_words + (uint64_t)L.table_rows * ISIM_DES_ROW_WORDS) * 8);
  L.stbits = (uint32_t *)take((uint64_t)plan.pos.size() * status_wpr(n) * 4);
  L.sort_ws = ws;
}

// The rounds of one batch with row type T: step begins,
// queues (fast: in place; sort path: radix sort first), finishes.
template <typename T>
static int des_rounds(const DesLaunch &L, dev::DesK k, uint32_t *tickets, hipStream_t stream) {
  using namespace dev;
  const DesPlan &pl = *L.plan;
  const uint64_t m_max = (uint64_t)pl.max_sort_pos * L.n_traces;
  char *sw = (char *)L.sort_ws;
  uint64_t *keys_a = (uint64_t *)sw, *keys_b = (uint64_t *)(sw + al256(m_max * 8));
  uint32_t *vals_a = (uint32_t *)(sw + 2 * al256(m_max * 8));
  uint32_t *vals_b = (uint32_t *)(sw + 2 * al256(m_max * 8) + al256(m_max * 4));
  void *sort_tmp = sw + 2 * al256(m_max * 8) + 2 * al256(m_max * 4);
  const size_t sort_tmp_bytes = sort_temp_bytes(m_max);
  k.sort_pos = L.d_sort_pos;
  // (position or row) x trace-range blocks: enough to fill the chip, >= 256 traces each
  // and at most ISIM_DES_MAX_SPLITS per position: every block flushes its
  // histogram and sums into the position's one table row by memory-side
  // atomics, which serialise per address (a one-position level in 4,096
  // blocks: ~90 us of atomics for 25 MB of rows)
  auto splits_for = [&](uint32_t width) {
    uint64_t sp = (ISIM_DES_SPLIT_TARGET + width - 1) / width;
    const uint64_t cap = (L.n_traces + 255) / 256;
    sp = sp < cap ? sp : cap;
    sp = sp < ISIM_DES_MAX_SPLITS ? sp : ISIM_DES_MAX_SPLITS;
    return (uint32_t)(sp ? sp : 1);
  };
  // the plan's variant order (des_plan.cpp): [single fused | single | replicated fused | replicated]
  static void (*const down[4])(DesK) = {des_down<T, false, true>, des_down<T, false, false>,
                                       des_down<T, true, true>, des_down<T, true, false>};
  static void (*const chain[2])(DesK) = {des_down_chain<T, true>, des_down_chain<T, false>};
  size_t seg = 0;
  uint32_t piped_to = 0;  // rounds below this one had their queues in a pipelined launch
  for (uint32_t r = 0; r < pl.rounds(); ++r) {
    if (ISIM_DES_PIPE && seg < pl.pipe.size() && pl.pipe[seg].r0 == r) {
      // the single-replica queues of rounds [r0, r1] in one launch (no step
      // begins, zero-hold, sort-path or replicated queues in them; finishes
      // only in r1)
      const DesPlan::PipeSeg &sg = pl.pipe[seg++];
      DesK kp = k;
      kp.level_pos = L.d_pipe;
      kp.pipe_dep = L.d_pipe + pl.pipe_pos.size();
      kp.level_begin = sg.off;
      kp.chain_ticket = tickets + 4 * r + 2;
      bool n32 = false;
      if constexpr (sizeof(T) == 4) {
        n32 = pl.pipe_n32;
        if (n32) hipLaunchKernelGGL((des_down_pipe<T, true>), dim3(sg.cnt), dim3(kDownThreads), 0, stream, kp);
      }
      if (!n32) hipLaunchKernelGGL((des_down_pipe<T, false>), dim3(sg.cnt), dim3(kDownThreads), 0, stream, kp);
      piped_to = sg.r1 + 1;
    }
    if (r < piped_to) goto finishes;
    {
    // 1. step begins (calls after calls)
    const uint32_t na = pl.arr_off[r + 1] - pl.arr_off[r];
    if (na) {
      k.level_begin = pl.arr_off[r];
      k.splits = splits_for(na);
      hipLaunchKernelGGL(des_arrive<T>, dim3(k.splits, na), dim3(kDesUpThreads), 0, stream, k);
    }
    // 2. queues.  Zero-hold services: start = arrival.
    const uint32_t nz = pl.zero_off[r + 1] - pl.zero_off[r];
    if (nz) {
      k.level_pos = L.d_zero_pos;
      k.level_begin = pl.zero_off[r];
      k.splits = splits_for(nz);
      hipLaunchKernelGGL(des_zero<T>, dim3(k.splits, nz), dim3(kDesUpThreads), 0, stream, k);
    }
    //    Single-replica groups narrower than the chip take the
    //    chained scan (many workgroups per position); wide groups and
    //    replicated services one workgroup per position.
    k.level_pos = L.d_fast_pos;
    if (ISIM_DES_MIX) {
      // single-replica positions (fused leaves or not): one launch
      const uint32_t b = pl.fast_split[5 * r], e = pl.fast_split[5 * r + 2];
      if (e > b) {
        k.level_begin = b;
        if (e - b < ISIM_DES_CHAIN_BELOW) {
          k.chain_ticket = tickets + 4 * r;
          hipLaunchKernelGGL(des_down_chain_mix<T>, dim3((e - b) * k.n_chunks), dim3(kDesThreads), 0, stream, k);
        } else {
          hipLaunchKernelGGL(des_down_mix<T>, dim3(e - b), dim3(kDownThreads), 0, stream, k);
        }
      }
    }
    for (uint32_t j = ISIM_DES_MIX ? 2 : 0; j < 4; ++j) {
      const uint32_t b = pl.fast_split[5 * r + j], e = pl.fast_split[5 * r + j + 1];
      if (e == b) continue;
      k.level_begin = b;
      if (j < 2 && e - b < ISIM_DES_CHAIN_BELOW) {
        k.chain_ticket = tickets + 4 * r + j;
        hipLaunchKernelGGL(chain[j], dim3((e - b) * k.n_chunks), dim3(kDesThreads), 0, stream, k);
      } else {
        hipLaunchKernelGGL(down[j], dim3(e - b), dim3(kDownThreads), 0, stream, k);
      }
    }
    for (uint32_t si = pl.sorted_off[r]; si < pl.sorted_off[r + 1]; ++si) {
      k.svc = pl.sorted[si];
      const uint64_t m = (uint64_t)k.svc.pos_cnt * L.n_traces;
      k.keys = keys_a;
      k.vals = vals_a;
      uint64_t g = (m + kDesUpThreads - 1) / kDesUpThreads;
      g = g < 4096 ? g : 4096;
      hipLaunchKernelGGL(des_sort_keys<T>, dim3((uint32_t)g), dim3(kDesUpThreads), 0, stream, k);
      size_t tb = sort_tmp_bytes;
      if (rocprim::radix_sort_pairs(sort_tmp, tb, keys_a, keys_b, vals_a, vals_b, (size_t)m, 0, 64, stream) !=
          hipSuccess)
        return 1;
      k.skeys = keys_b;
      k.svals = vals_b;
      hipLaunchKernelGGL(des_down_sorted<T>, dim3(1), dim3(kDesThreads), 0, stream, k);
    }
    }
  finishes:
    // 3. finishes, deepest group first
    k.level_pos = L.d_fin_pos;
    for (uint32_t gi = pl.fin_round_off[r]; gi < pl.fin_round_off[r + 1]; ++gi) {
      const uint32_t width = pl.fin_off[gi + 1] - pl.fin_off[gi];
      k.level_begin = pl.fin_off[gi];
      k.splits = splits_for(width);
      bool n32 = false;
      if constexpr (sizeof(T) == 4) {
        n32 = pl.up_n32;
        if (n32) hipLaunchKernelGGL((des_up<T, true>), dim3(k.splits, width), dim3(kDesUpThreads), 0, stream, k);
      }
      if (!n32) hipLaunchKernelGGL((des_up<T, false>), dim3(k.splits, width), dim3(kDesUpThreads), 0, stream, k);
    }
  }
  return 0;
}

// Host launcher: the whole DES of one batch on `stream` (no allocation; no
// host synchronisation unless the schedule is cyclic: its fixed-point passes
// read one flag per pass).
constexpr uint32_t kMaxPasses = 256;

static std::atomic<uint32_t> g_spin_limit{kDesSpinLimit};
uint32_t des_spin_limit() { return g_spin_limit.load(std::memory_order_relaxed); }
void des_set_spin_limit(uint32_t polls) { g_spin_limit.store(polls, std::memory_order_relaxed); }

int des_launch(const DesLaunch &L, void *stream_) {
  using namespace dev;
  hipStream_t stream = (hipStream_t)stream_;
  const bool narrow = !L.wide;
  const uint64_t table_words = (uint64_t)L.table_rows * ISIM_DES_ROW_WORDS;
  DesK k{};
  k.pos = (const DesPos *)L.d_pos;
  k.ext = (const DesPosExt *)L.d_ext;
  k.steps = (const DesStep *)L.d_steps;
  k.child = L.d_child;
  k.arr_ops = L.d_arr_ops;
  k.W = L.W;
  k.WF = L.WF;
  k.BK = L.BK;
  k.A = L.A;
  k.E = L.E;
  k.blk = L.blk;
  k.ovf = L.ovf;
  k.spin_limit = des_spin_limit();
  k.stbits = L.stbits;
  k.st_wpr = (uint32_t)status_wpr(L.n_traces);
  // statistics go to the staging copy, merged by des_commit unless the batch
  // is dropped (a 32-bit row overflowed, or no fixed point)
  k.stats = L.stage;
  k.table = L.stage + L.stats_words;
  k.records = L.d_records;
  k.N = L.n_traces;
  k.ld = row_ld(L.n_traces);
  k.trace_begin = L.trace_begin;
  k.mean_ns = L.mean_ns;
  k.k0 = (uint32_t)L.seed;
  k.k1 = (uint32_t)(L.seed >> 32);
  k.n_pos = L.n_pos;
  k.n_slots = L.n_slots;
  k.modeb = L.modeb;
  k.n_blk = (uint32_t)((L.n_traces + kDesChunk - 1) / kDesChunk);
  k.n_chunks = (uint32_t)((L.n_traces + kDownChunk - 1) / kDownChunk);
  const uint64_t tk_bytes = al256(chain_tickets(*L.plan) * 4);
  uint32_t *tickets = (uint32_t *)L.chain;
  k.prog = (uint32_t *)((char *)L.chain + tk_bytes);
  k.chain = (ChainState *)((char *)L.chain + tk_bytes + al256((uint64_t)L.n_pos * 4));
  const uint64_t chain_bytes = des_chain_bytes(*L.plan, L.n_traces);
  if (hipMemsetAsync(L.E, 0, L.n_traces * sizeof(uint32_t), stream) != hipSuccess) return 1;
  if (hipMemsetAsync(L.ovf, 0, 8, stream) != hipSuccess) return 1;  // overflow flag + changed flag
  if (hipMemsetAsync(L.stage, 0, (L.stats_words + table_words) * 8, stream) != hipSuccess) return 1;
  hipLaunchKernelGGL(des_arrivals, dim3(k.n_blk), dim3(kDesThreads), 0, stream, k);
  hipLaunchKernelGGL(des_scan_blocks, dim3(1), dim3(kDesThreads), 0, stream, k);
  hipLaunchKernelGGL(des_add_blocks, dim3(k.n_blk), dim3(kDesThreads), 0, stream, k);
  {
    const uint64_t threads = (uint64_t)((L.n_pos + 3) / 4) * k.st_wpr;
    hipLaunchKernelGGL(des_status, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, stream, k);
  }
  auto pass = [&](const DesK &kk) -> int {
    if (hipMemsetAsync(L.chain, 0, chain_bytes, stream) != hipSuccess) return 1;
    return narrow ? des_rounds<uint32_t>(L, kk, tickets, stream) : des_rounds<uint64_t>(L, kk, tickets, stream);
  };
  if (L.plan->cyclic) {
    // fixed point: back-edge rows start at 0 (a lower bound of every
    // relative time); quiet passes until no stored value changes, then the
    // pass that records the statistics
    const uint64_t rb = narrow ? 4 : 8;
    if (hipMemsetAsync(L.W, 0, (uint64_t)L.n_pos * k.ld * rb, stream) != hipSuccess ||
        hipMemsetAsync(L.WF, 0, (uint64_t)L.n_pos * k.ld * rb, stream) != hipSuccess ||
        hipMemsetAsync(L.BK, 0, (uint64_t)L.plan->steps.size() * k.ld * rb, stream) != hipSuccess)
      return 1;
    DesK kq = k;
    kq.quiet = 1;
    kq.changed = L.ovf + 1;
    uint32_t p = 0;
    for (; p < kMaxPasses; ++p) {
      if (hipMemsetAsync(kq.changed, 0, 4, stream) != hipSuccess) return 1;
      if (pass(kq)) return 1;
      uint32_t changed = 1;
      if (hipMemcpyAsync(&changed, kq.changed, 4, hipMemcpyDeviceToHost, stream) != hipSuccess ||
          hipStreamSynchronize(stream) != hipSuccess)
        return 1;
      if (!changed) break;
    }
    if (p == kMaxPasses) {
      static const uint32_t no_fixed_point = 2;
      if (hipMemcpyAsync(L.ovf, &no_fixed_point, 4, hipMemcpyHostToDevice, stream) != hipSuccess ||
          hipStreamSynchronize(stream) != hipSuccess)
        return 1;
    }
  }
  if (pass(k)) return 1;
  uint64_t fin_blocks = (L.n_traces + kDesUpThreads - 1) / kDesUpThreads;
  fin_blocks = fin_blocks < ISIM_DES_FIN_BLOCKS ? fin_blocks : ISIM_DES_FIN_BLOCKS;
  if (narrow) hipLaunchKernelGGL(des_finalize<uint32_t>, dim3((uint32_t)fin_blocks), dim3(kDesUpThreads), 0, stream, k);
  else hipLaunchKernelGGL(des_finalize<uint64_t>, dim3((uint32_t)fin_blocks), dim3(kDesUpThreads), 0, stream, k);
  if (L.n_slots > 0) {  // executed calls: every trace makes mult[slot] calls through each site
    uint32_t n_slots = L.n_slots;
    uint64_t n = L.n_traces;
    const uint32_t *mult = L.d_mult;
    uint64_t *st = k.stats;
    uint32_t *stage = nullptr;  // the DES counts its 500s itself (no staged walk flush)
    void *args[] = {&mult, &n_slots, &n, &st, &stage};
    if (hipLaunchKernel(stream_calls_kernel(), dim3((n_slots + 255) / 256), dim3(256), args, 0, stream) !=
        hipSuccess)
      return 1;
  }
  uint64_t g = (L.stats_words + table_words + 255) / 256;
  g = g < 1024 ? g : 1024;
  hipLaunchKernelGGL(des_commit, dim3((uint32_t)(g ? g : 1)), dim3(256), 0, stream, L.stage, L.d_stats, L.d_table,
                     L.stats_words, table_words, (const uint32_t *)L.ovf);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // namespace isim
