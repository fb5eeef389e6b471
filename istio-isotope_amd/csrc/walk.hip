// isim_walk — the hot path on gfx950 (CDNA4): one wavefront simulates 64
// independent request traces (one per lane) by interpreting the flattened
// service scripts of program.h in lock-step.  Semantics: "isim semantics v1"
// (DESIGN.md §2), i.e. isotope's Handler.ServeHTTP / execute recursion
// (isotope/service/pkg/srv/handler.go:37-79, executable.go:43-179) in virtual
// integer-nanosecond time.
//
// Execution model:
//  * The program counter, the current instruction (one s_load_dwordx8) and the
//    call depth are wave-uniform (SGPRs).  Per-lane booleans — "this lane's
//    trace executes the current invocation", "a step failed", "error in the
//    current concurrent step", "this invocation's own error draw" — are 64-bit
//    lane masks held in SGPRs and combined with scalar ALU ops.
//  * STATIC walks (no probabilistic calls, no mode-B abort that could skip a
//    step) execute the identical invocation sequence in every lane, so
//    virtual time and hop ids are wave-uniform: they live in SGPRs, and the
//    only per-lane work is the Philox error draw, the status masks and the
//    per-trace error count.  Other walks keep time (u32 or u64, chosen from
//    the program's static latency bound) and hop ids per lane.
//  * Call frames: uniform parts (return pc, masks, uniform time) are stored
//    in VGPR lanes (lane d holds frame d: v_writelane / v_readlane); per-lane
//    time and hop of dynamic walks go to an LDS stack [frame][lane].
//  * Error draws: word (h&3) of Philox4x32-10((t, h>>2, 0), seed), so one
//    block serves four consecutive invocations of a lane.
//  * Per-call-site counters (executed calls, callee 500s) are wave-reduced to
//    one ds_add per instruction into a workgroup LDS table and flushed to HBM
//    with global atomics once per workgroup; latency histograms are reduced
//    per batch with a wave "match" loop.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernel_abi.h"

namespace isim {
namespace dev {

constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;

__device__ __forceinline__ void philox10(uint32_t &c0, uint32_t &c1, uint32_t &c2, uint32_t &c3,
                                         uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c0 = n0;
    c1 = (uint32_t)p1;
    c2 = n2;
    c3 = (uint32_t)p0;
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
// v_writelane_b32: no clang builtin on this toolchain, so bind the LLVM
// intrinsic directly (value and lane index are wave-uniform).
__device__ int llvm_writelane(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t wrl(uint32_t v, uint32_t l, uint32_t old) {
  return (uint32_t)llvm_writelane((int)v, (int)l, (int)old);
}
__device__ __forceinline__ uint32_t uni(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// A 64-bit wave-uniform value kept in two VGPR-lane stacks.
struct U64Stack {
  uint32_t lo = 0, hi = 0;
  __device__ __forceinline__ void put(uint32_t d, uint64_t v) {
    lo = wrl((uint32_t)v, d, lo);
    hi = wrl((uint32_t)(v >> 32), d, hi);
  }
  __device__ __forceinline__ uint64_t get(uint32_t d) const {
    return (uint64_t)rdl(lo, d) | ((uint64_t)rdl(hi, d) << 32);
  }
};

// LDS counter add of a wave-uniform amount by one lane.
__device__ __forceinline__ void lds_add(uint32_t *p, uint32_t v) {
  if (lane_id() == 0) atomicAdd(p, v);
}

__device__ __forceinline__ void count(const KParams &kp, uint32_t *cnt, uint32_t idx, uint32_t v) {
  if (v == 0) return;
  if (cnt) {
    lds_add(cnt + idx, v);
  } else if (lane_id() == 0) {
    atomicAdd((unsigned long long *)(kp.stats + ISIM_ST_SITES + idx), (unsigned long long)v);
  }
}

__device__ __forceinline__ uint64_t u64of(uint32_t lo, uint32_t hi) {
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

__device__ __forceinline__ uint32_t prom_bucket(uint64_t t) {
  const uint64_t ms = 1000000ull;
  // service_request_duration_seconds buckets, srv/prometheus/handler.go:26-31
  const uint32_t e[32] = {7, 8, 9, 10, 11, 12, 14, 16, 18, 20, 25, 30, 35, 40, 45, 50,
                          60, 70, 80, 90, 100, 120, 140, 160, 180, 200, 250, 300, 350, 400, 450, 500};
  uint32_t b = 32;
#pragma unroll
  for (int i = 31; i >= 0; --i)
    if (t <= (uint64_t)e[i] * ms) b = (uint32_t)i;
  return b;
}

// Wave-aggregated LDS histogram add: one ds_add per distinct key.
__device__ __forceinline__ void hist_add(uint32_t *h, uint32_t key, uint64_t lanes) {
  while (lanes) {
    uint32_t leader = (uint32_t)__builtin_ctzll(lanes);
    uint32_t k = rdl(key, leader);
    uint64_t m = ballot(key == k) & lanes;
    if (lane_id() == leader) atomicAdd(h + k, popc(m));
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
    uint64_t w = __shfl_xor(v, o, 64);
    v = w > v ? w : v;
  }
  return v;
}

// Workgroup-shared accumulators (LDS).
struct WgAcc {
  unsigned long long sum_latency, sum_hops, sum_err, n500, ntr, notmin, max;
};

template <bool STATIC, bool MODEB, typename TT>
__device__ __forceinline__ void walk_batch(const KParams &kp, uint64_t base, uint32_t *cnt,
                                           uint32_t *hist, WgAcc *acc_lds, TT *lstk,
                                           uint32_t *hstk) {
  const uint32_t lane = lane_id();
  const uint64_t idx = base + lane;
  const bool valid = idx < kp.n_traces;
  const uint64_t t = kp.trace_begin + idx;
  const uint32_t t_lo = (uint32_t)t, t_hi = (uint32_t)(t >> 32);
  const uint64_t all = ballot(valid);
  const uint32_t k0 = kp.seed_lo, k1 = kp.seed_hi;
  const Ins *__restrict__ prog = kp.prog;

  // ---- wave-uniform state
  uint32_t pc = 0, depth = 0;
  uint64_t live = all, failed = 0, cerr = 0, own = 0, root_st = 0;
  // STATIC: uniform time and hop counter
  uint64_t uacc = 0, ucmax = 0;
  uint32_t uhop = 0, ublk = 0xFFFFFFFFu;
  // ---- per-lane state
  TT acc = 0, cmax = 0;           // dynamic walks
  uint32_t myhop = 0, hopn = 0;   // dynamic walks
  uint32_t cblk = 0xFFFFFFFFu;    // dynamic walks: cached Philox block
  uint32_t x0 = 0, x1 = 0, x2 = 0, x3 = 0;
  uint32_t errh = 0;
  // ---- frame stacks in VGPR lanes
  uint32_t f_ret = 0;
  U64Stack f_live, f_failed, f_cerr, f_own, f_acc, f_cmax;

  // error draw for the lanes in `e` invoking a callee with flags/thr
  auto draw_err = [&](uint32_t flags, uint32_t thr, uint64_t e) -> uint64_t {
    if (flags & F_ERR_ALWAYS) return e;
    if (!(flags & F_ERR_DRAW)) return 0;
    bool hit;
    if constexpr (STATIC) {
      const uint32_t blk = uhop >> 2;
      if (blk != ublk) {  // uniform branch
        x0 = t_lo; x1 = t_hi; x2 = blk; x3 = 0;
        philox10(x0, x1, x2, x3, k0, k1);
        ublk = blk;
      }
      const uint32_t w = uhop & 3;
      uint32_t word;
      if (w == 0) word = x0;
      else if (w == 1) word = x1;
      else if (w == 2) word = x2;
      else word = x3;
      hit = word < thr;
    } else {
      const uint32_t blk = hopn >> 2;
      const uint64_t need = ballot(blk != cblk) & e;
      if (need) {
        if (lane_in(need)) {
          uint32_t a = t_lo, b = t_hi, c = blk, d = 0;
          philox10(a, b, c, d, k0, k1);
          x0 = a; x1 = b; x2 = c; x3 = d;
          cblk = blk;
        }
      }
      const uint32_t w = hopn & 3;
      const uint32_t lo = (w & 1) ? x1 : x0;
      const uint32_t hi = (w & 1) ? x3 : x2;
      hit = ((w & 2) ? hi : lo) < thr;
    }
    return ballot(hit) & e;
  };

  // probability skip draw (dynamic walks only): lanes of `a` that skip
  auto draw_skip = [&](uint32_t k, uint32_t q, uint64_t a) -> uint64_t {
    bool skip = false;
    if (lane_in(a)) {
      uint32_t c0 = t_lo, c1 = t_hi, c2 = myhop, c3 = 1u + (k >> 2);
      philox10(c0, c1, c2, c3, k0, k1);
      const uint32_t sel = k & 3;  // uniform
      const uint32_t word = sel == 0 ? c0 : sel == 1 ? c1 : sel == 2 ? c2 : c3;
      skip = (word % 100u) < 100u - q;
    }
    return ballot(skip) & a;
  };

  // fold a finished invocation (duration H + T per lane, status st) into
  // the caller frame for lanes `e`
  auto fold = [&](uint32_t flags, uint64_t H, TT T, uint64_t uT, uint64_t e, uint64_t st) {
    if (flags & F_ROOT) {
      root_st = st;
      if constexpr (STATIC) uacc = H + uT;
      else if (lane_in(e)) acc = (TT)H + T;
    } else if (flags & F_CONC) {
      if constexpr (STATIC) {
        const uint64_t v = H + uT;
        ucmax = v > ucmax ? v : ucmax;
      } else if (lane_in(e)) {
        const TT v = (TT)H + T;
        cmax = v > cmax ? v : cmax;
      }
      if constexpr (MODEB) cerr |= st;
    } else {
      if constexpr (STATIC) uacc += H + uT;
      else if (lane_in(e)) acc += (TT)H + T;
      if constexpr (MODEB) failed |= st;
    }
  };

  while (true) {
    const Ins in = prog[pc];
    const uint32_t op = in.opf & 0xFFu;
    const uint32_t flags = (in.opf >> 8) & 0xFFu;
    if (op == OP_HALT) break;
    switch (op) {
      case OP_SLEEP: {
        const uint64_t d = u64of(in.a_lo, in.a_hi);
        if constexpr (STATIC) uacc += d;
        else if (lane_in(live & ~failed)) acc += (TT)d;
        ++pc;
        break;
      }
      case OP_CBEGIN: {
        if constexpr (STATIC) ucmax = 0;
        else if (lane_in(live & ~failed)) cmax = 0;
        cerr = 0;
        ++pc;
        break;
      }
      case OP_CSLEEP: {
        const uint64_t d = u64of(in.a_lo, in.a_hi);
        if constexpr (STATIC) ucmax = d > ucmax ? d : ucmax;
        else if (lane_in(live & ~failed)) cmax = (TT)d > cmax ? (TT)d : cmax;
        ++pc;
        break;
      }
      case OP_CEND: {
        if constexpr (STATIC) uacc += ucmax;
        else if (lane_in(live & ~failed)) acc += cmax;
        if constexpr (MODEB) failed |= cerr & live;
        ++pc;
        break;
      }
      case OP_LEAF:
      case OP_CALL: {
        uint64_t e = live & ~failed;
        if constexpr (!STATIC) {
          if (flags & F_PROB) e &= ~draw_skip(in.k, in.opf >> 16, e);
          if (e == 0) {  // no lane makes this call
            ++pc;
            break;
          }
        }
        const uint64_t st_own = draw_err(flags, in.thr, e);
        if constexpr (STATIC) ++uhop;
        const uint32_t myh = hopn;
        if constexpr (!STATIC) {
          if (lane_in(e)) ++hopn;
        }
        if (!(flags & F_ROOT)) count(kp, cnt, in.slot, popc(e));
        const uint64_t H = u64of(in.a_lo, in.a_hi);
        if (op == OP_LEAF) {
          if (!(flags & F_ROOT)) count(kp, cnt, (uint32_t)kp.n_slots + in.slot, popc(st_own));
          if (lane_in(st_own)) ++errh;
          const uint64_t TL = u64of(in.b_lo, in.b_hi);
          fold(flags, H, (TT)TL, TL, e, st_own);
          ++pc;
        } else {
          // push the caller frame
          f_ret = wrl(pc + 1, depth, f_ret);
          f_own.put(depth, own);
          if constexpr (MODEB) f_cerr.put(depth, cerr);
          if constexpr (STATIC) {
            f_acc.put(depth, uacc);
            f_cmax.put(depth, ucmax);
            uacc = 0;
            ucmax = 0;
          } else {
            f_live.put(depth, live);
            f_failed.put(depth, failed);
            lstk[2 * depth * 64 + lane] = acc;
            lstk[(2 * depth + 1) * 64 + lane] = cmax;
            hstk[depth * 64 + lane] = myhop;
            acc = 0;
            cmax = 0;
            myhop = myh;
            live = e;
          }
          failed = 0;
          cerr = 0;
          own = st_own;
          ++depth;
          pc = in.b_lo;
        }
        break;
      }
      case OP_RET: {
        const uint64_t e = live;
        const uint64_t st = (failed | own) & e;
        const TT T = acc;
        const uint64_t uT = uacc;
        --depth;
        const uint32_t ret = rdl(f_ret, depth);
        own = f_own.get(depth);
        if constexpr (MODEB) cerr = f_cerr.get(depth);
        else cerr = 0;
        if constexpr (STATIC) {
          uacc = f_acc.get(depth);
          ucmax = f_cmax.get(depth);
          failed = 0;
        } else {
          live = f_live.get(depth);
          failed = f_failed.get(depth);
          acc = lstk[2 * depth * 64 + lane];
          cmax = lstk[(2 * depth + 1) * 64 + lane];
          myhop = hstk[depth * 64 + lane];
        }
        const Ins cin = prog[ret - 1];
        const uint32_t cflags = (cin.opf >> 8) & 0xFFu;
        if (!(cflags & F_ROOT)) count(kp, cnt, (uint32_t)kp.n_slots + cin.slot, popc(st));
        if (lane_in(st)) ++errh;
        fold(cflags, u64of(cin.a_lo, cin.a_hi), T, uT, e, st);
        pc = ret;
        break;
      }
      default:
        __builtin_trap();
    }
  }

  // ---- per-trace outputs
  uint64_t lat;
  uint32_t hops;
  if constexpr (STATIC) {
    lat = uacc;
    hops = uhop;
  } else {
    lat = (uint64_t)acc;
    hops = hopn;
  }
  const bool is500 = lane_in(root_st);
  if (kp.records != nullptr && valid) {
    uint4 r;
    r.x = (uint32_t)lat;
    r.y = (uint32_t)(lat >> 32);
    r.z = hops;
    r.w = (is500 ? 0x80000000u : 0u) | errh;
    *reinterpret_cast<uint4 *>(kp.records + idx) = r;
  }
  hist_add(hist, (is500 ? ISIM_N_PROM : 0u) + prom_bucket(lat), all);
  const uint32_t l2 = lat == 0 ? 0u : 64u - (uint32_t)__builtin_clzll(lat);
  hist_add(hist + 2 * ISIM_N_PROM, (is500 ? ISIM_N_LOG2 : 0u) + l2, all);
  const uint64_t s_lat = wave_sum64(valid ? lat : 0);
  const uint64_t s_hops = wave_sum64(valid ? (uint64_t)hops : 0);
  const uint64_t s_err = wave_sum64(valid ? (uint64_t)errh : 0);
  const uint64_t mx = wave_max64(valid ? lat : 0);
  const uint64_t nmn = wave_max64(valid ? ~lat : 0);
  if (lane == 0) {
    atomicAdd(&acc_lds->sum_latency, (unsigned long long)s_lat);
    atomicAdd(&acc_lds->sum_hops, (unsigned long long)s_hops);
    atomicAdd(&acc_lds->sum_err, (unsigned long long)s_err);
    atomicAdd(&acc_lds->n500, (unsigned long long)popc(root_st & all));
    atomicAdd(&acc_lds->ntr, (unsigned long long)popc(all));
    atomicMax(&acc_lds->max, (unsigned long long)mx);
    atomicMax(&acc_lds->notmin, (unsigned long long)nmn);
  }
}

template <bool STATIC, bool MODEB, typename TT>
__global__ void __launch_bounds__(kWgThreads) isim_walk(KParams kp) {
  extern __shared__ __align__(16) unsigned char lds[];
  WgAcc *acc = reinterpret_cast<WgAcc *>(lds);
  uint32_t *hist = reinterpret_cast<uint32_t *>(lds + kLdsAccBytes);
  uint32_t *cnt = kp.lds_counters ? hist + kHistWords : nullptr;
  unsigned char *stk = lds + kLdsAccBytes + kHistWords * 4 + (kp.lds_counters ? 8u * kp.n_slots : 0u);
  stk = (unsigned char *)(((uintptr_t)stk + 15) & ~(uintptr_t)15);
  const uint32_t wave = threadIdx.x >> 6;
  const uint32_t waves = blockDim.x >> 6;
  TT *lstk = nullptr;
  uint32_t *hstk = nullptr;
  if constexpr (!STATIC) {
    const uint32_t per_wave = kp.max_frames * 64u * (2u * sizeof(TT) + 4u);
    lstk = reinterpret_cast<TT *>(stk + wave * per_wave);
    hstk = reinterpret_cast<uint32_t *>(stk + wave * per_wave + kp.max_frames * 64u * 2u * sizeof(TT));
  }
  // zero the workgroup accumulators
  const uint32_t zero_words = (kLdsAccBytes / 4) + kHistWords + (kp.lds_counters ? 2u * kp.n_slots : 0u);
  uint32_t *z = reinterpret_cast<uint32_t *>(lds);
  for (uint32_t i = threadIdx.x; i < zero_words; i += blockDim.x) z[i] = 0;
  __syncthreads();

  const uint64_t n_batches = (kp.n_traces + 63) / 64;
  const uint64_t stride = (uint64_t)gridDim.x * waves;
  for (uint64_t b = (uint64_t)blockIdx.x * waves + wave; b < n_batches; b += stride)
    walk_batch<STATIC, MODEB, TT>(kp, b * 64, cnt, hist, acc, lstk, hstk);

  __syncthreads();
  // ---- flush workgroup accumulators to HBM
  unsigned long long *st = reinterpret_cast<unsigned long long *>(kp.stats);
  for (uint32_t i = threadIdx.x; i < kHistWords; i += blockDim.x)
    if (hist[i]) atomicAdd(st + ISIM_ST_PROM + i, (unsigned long long)hist[i]);
  if (cnt) {
    for (uint32_t i = threadIdx.x; i < 2u * kp.n_slots; i += blockDim.x)
      if (cnt[i]) atomicAdd(st + ISIM_ST_SITES + i, (unsigned long long)cnt[i]);
  }
  if (threadIdx.x == 0 && acc->ntr) {
    atomicAdd(st + ISIM_ST_N_TRACES, acc->ntr);
    atomicAdd(st + ISIM_ST_SUM_LATENCY, acc->sum_latency);
    atomicAdd(st + ISIM_ST_SUM_HOPS, acc->sum_hops);
    atomicAdd(st + ISIM_ST_SUM_ERR_HOPS, acc->sum_err);
    atomicAdd(st + ISIM_ST_N_500, acc->n500);
    atomicMax(st + ISIM_ST_NOT_MIN_LATENCY, acc->notmin);
    atomicMax(st + ISIM_ST_MAX_LATENCY, acc->max);
  }
}

}  // namespace dev

// Kernel table: [static][modeB][time64]
void *walk_kernel(bool is_static, bool modeb, bool time64) {
  using namespace dev;
  if (is_static) {
    return modeb ? (void *)&isim_walk<true, true, uint64_t> : (void *)&isim_walk<true, false, uint64_t>;
  }
  if (time64)
    return modeb ? (void *)&isim_walk<false, true, uint64_t> : (void *)&isim_walk<false, false, uint64_t>;
  return modeb ? (void *)&isim_walk<false, true, uint32_t> : (void *)&isim_walk<false, false, uint32_t>;
}

}  // namespace isim
