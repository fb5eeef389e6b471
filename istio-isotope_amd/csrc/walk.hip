// isim_walk — the hot path on gfx950 (CDNA4): one wavefront simulates 64
// independent request traces (one per lane) by interpreting the flattened
// service scripts of program.h in lock-step.  Semantics: "isim semantics v1"
// (DESIGN.md §2), i.e. isotope's Handler.ServeHTTP / execute recursion
// (isotope/service/pkg/srv/handler.go:37-79, executable.go:43-179) in virtual
// integer-nanosecond time.
//
// Execution model:
//  * The program counter, the current instruction and the call depth are
//    wave-uniform (SGPRs).  The next instruction is known before the current
//    one executes (pc+1, a CALL's target, or the return pc of a RET), so the
//    loop issues one s_load_dwordx16 of [npc-1, npc] first and consumes it on
//    the next iteration; for a RET the first half is the CALL record.
//  * Per-lane booleans — "this lane's trace executes the current invocation",
//    "a step failed", "error in the current concurrent step", "this
//    invocation's own error draw" — are 64-bit lane masks in SGPRs.
//  * STATIC walks (no probabilistic calls, no mode-B abort that could skip a
//    step) execute the identical invocation sequence in every lane, so virtual
//    time and hop ids are wave-uniform (SGPRs); the per-lane work is the
//    Philox error draws, the status masks and the per-trace error count.
//    Other walks keep time (u32 or u64 by the program's latency bound) and
//    hop ids per lane.
//  * Call frames: wave-uniform parts live in VGPR lanes (lane d holds frame
//    d: v_writelane / v_readlane); per-lane time and hop of dynamic walks go
//    to an LDS stack [frame][lane].
//  * Error draws: word (h&3) of Philox4x32-10((t_lo, t_hi, h>>2, 0), seed):
//    one block serves four consecutive invocations of a lane.
//  * Per-call-site counters (executed calls, callee 500s) are one ds_add per
//    instruction per wave into a workgroup LDS table, flushed to HBM with
//    global atomics once per workgroup; latency histograms are reduced per
//    64-trace batch with a wave "match" loop.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "kernel_abi.h"
#include "walk_dev.h"

#ifndef ISIM_STREAM_TPL
#define ISIM_STREAM_TPL 2
#endif
#ifndef ISIM_STREAM_WAVES
#define ISIM_STREAM_WAVES 8  // waves per SIMD the draw-stream kernel is compiled for
#endif

namespace isim {
namespace dev {

constexpr int kStreamTPL = ISIM_STREAM_TPL;  // traces per lane in the draw-stream kernel

// ======================================================================
// STATIC walk: uniform time (UT = u32 when the latency bound fits) and hops.
// ======================================================================
template <bool MODEB, typename UT>
__device__ __forceinline__ void walk_static(const Ctx &c, uint64_t trace_begin, uint64_t n_traces,
                                            uint64_t base) {
  const uint32_t lane = lane_id();
  const uint64_t idx = base + lane;
  const bool valid = idx < n_traces;
  const uint64_t t = trace_begin + idx;
  const uint32_t t_lo = (uint32_t)t, t_hi = (uint32_t)(t >> 32);
  const uint32_t t_hi_u = rfl(t_hi);
  const bool hi_uniform = ballot(t_hi != t_hi_u) == 0;  // the batch does not straddle 2^32
  const uint64_t all = ballot(valid);
  const Ins *__restrict__ prog = c.prog;

  UT acc = 0, cmax = 0;
  uint64_t own = 0, failed = 0, cerr = 0, root_st = 0;
  uint32_t hop = 0, have = 0xFFFFFFFFu, depth = 0, pc = 0;
  uint32_t x0 = 0, x1 = 0, x2 = 0, x3 = 0, errh = 0;
  LaneStack<uint32_t> f_ret;
  LaneStack<uint64_t> f_own, f_cerr;
  LaneStack<UT> f_acc, f_cmax;

  auto fold = [&](uint32_t flags, UT v, uint64_t st) {
    if (flags & F_ROOT) {
      root_st = st;
      acc = v;
    } else if (flags & F_CONC) {
      cmax = v > cmax ? v : cmax;
      if constexpr (MODEB) cerr |= st;
    } else {
      acc += v;
      if constexpr (MODEB) failed |= st;
    }
  };

  Ins cur = prog[0];
  while (true) {
    const uint32_t op = cur.opf & 0xFFu;
    if (op == OP_HALT) break;
    const uint32_t flags = (cur.opf >> 8) & 0xFFu;
    uint32_t npc = pc + 1;
    if (op == OP_CALL) npc = cur.b_lo;
    if (op == OP_RET) npc = f_ret.get(depth - 1);
    const Ins2 pre = *reinterpret_cast<const Ins2 *>(prog + (npc - 1));  // [npc-1, npc]
    switch (op) {
      case OP_SLEEP:
        acc += (UT)u64of(cur.a_lo, cur.a_hi);
        break;
      case OP_CBEGIN:
        cmax = 0;
        cerr = 0;
        break;
      case OP_CSLEEP: {
        const UT d = (UT)u64of(cur.a_lo, cur.a_hi);
        cmax = d > cmax ? d : cmax;
        break;
      }
      case OP_CEND:
        acc += cmax;
        if constexpr (MODEB) failed |= cerr;
        break;
      case OP_LEAF:
      case OP_CALL: {
        uint64_t st = 0;
        if (flags & F_ERR_ALWAYS) {
          st = all;
        } else if (flags & F_ERR_DRAW) {
          const uint32_t blk = hop >> 2;
          if (blk != have) {
            have = blk;
            uint32_t a = t_lo, b = t_hi, cc = blk, d = 0;
            if (hi_uniform) {
              // rounds 1-2 with the uniform counter words folded into SGPR math
              // keep the key schedule out of SGPRs between refills (recomputed
              // with 2 SALU adds per round instead of 20 hoisted registers)
              uint32_t k0a = c.k0, k1a = c.k1;
              asm volatile("" : "+s"(k0a), "+s"(k1a));
              const uint64_t q1 = (uint64_t)M1 * blk;                    // scalar
              const uint64_t p0 = (uint64_t)M0 * t_lo;                   // per lane
              const uint32_t u0 = (uint32_t)(q1 >> 32) ^ t_hi_u ^ k0a;   // uniform
              const uint32_t u1 = (uint32_t)q1;                          // uniform
              const uint32_t v2 = (uint32_t)(p0 >> 32) ^ k1a;            // per lane
              const uint32_t v3 = (uint32_t)p0;                          // per lane
              const uint32_t k0b = k0a + W0, k1b = k1a + W1;
              const uint64_t q0 = (uint64_t)M0 * u0;                     // scalar
              const uint64_t p1 = (uint64_t)M1 * v2;                     // per lane
              a = (uint32_t)(p1 >> 32) ^ u1 ^ k0b;
              b = (uint32_t)p1;
              cc = (uint32_t)(q0 >> 32) ^ v3 ^ k1b;
              d = (uint32_t)q0;
              uint32_t k0 = k0b + W0, k1 = k1b + W1;
#pragma unroll
              for (int r = 2; r < 10; ++r) {
                round1(a, b, cc, d, k0, k1);
                k0 += W0;
                k1 += W1;
              }
            } else {
              philox10(a, b, cc, d, c.k0, c.k1);
            }
            x0 = a;
            x1 = b;
            x2 = cc;
            x3 = d;
          }
          const uint32_t w = hop & 3u;
          const uint32_t lo = (w & 1u) ? x1 : x0;
          const uint32_t hi = (w & 1u) ? x3 : x2;
          st = ballot(((w & 2u) ? hi : lo) < cur.thr) & all;
        }
        ++hop;
        if (!(flags & F_ROOT)) count(c.gstats, c.cnt, cur.slot, popc(all));
        const UT H = (UT)u64of(cur.a_lo, cur.a_hi);
        if (op == OP_LEAF) {
          if (!(flags & F_ROOT)) count(c.gstats, c.cnt, c.n_slots + cur.slot, popc(st));
          if (lane_in(st)) ++errh;
          fold(flags, H + (UT)u64of(cur.b_lo, cur.b_hi), st);
        } else {
          f_ret.put(depth, pc + 1);
          f_own.put(depth, own);
          f_acc.put(depth, acc);
          f_cmax.put(depth, cmax);
          if constexpr (MODEB) f_cerr.put(depth, cerr);
          ++depth;
          acc = 0;
          cmax = 0;
          cerr = 0;
          failed = 0;
          own = st;
        }
        break;
      }
      case OP_RET: {
        const uint64_t st = (failed | own) & all;
        const UT T = acc;
        --depth;
        own = f_own.get(depth);
        acc = f_acc.get(depth);
        cmax = f_cmax.get(depth);
        if constexpr (MODEB) cerr = f_cerr.get(depth);
        failed = 0;  // static walks never call after a failed step
        const Ins &cin = pre.a;
        const uint32_t cflags = (cin.opf >> 8) & 0xFFu;
        if (!(cflags & F_ROOT)) count(c.gstats, c.cnt, c.n_slots + cin.slot, popc(st));
        if (lane_in(st)) ++errh;
        fold(cflags, (UT)u64of(cin.a_lo, cin.a_hi) + T, st);
        break;
      }
      default:
        __builtin_trap();
    }
    cur = pre.b;
    pc = npc;
  }
  finish_batch(c, idx, valid, all, (uint64_t)acc, hop, root_st, errh);
}

// ======================================================================
// DYNAMIC walk: per-lane time (TT) and hop ids, LDS frame stack.
// ======================================================================
// Per-service invocation durations (RecordResponseSent, srv/prometheus/
// handler.go:101-106): row = [code][33] bucket counts + [code] sums (ns).
// A leaf callee's duration is its fixed latency (bucket precomputed in the
// table word); a RET has per-lane durations.
__device__ __forceinline__ void leaf_duration(const Ctx &c, uint32_t w, uint64_t T, uint64_t e, uint64_t st) {
  if (lane_id() != 0) return;
  unsigned long long *row = (unsigned long long *)(c.svc_tab + (uint64_t)(w & kDurRowMask) * ISIM_SVC_DUR_WORDS);
  const uint32_t b = w >> 24;
  const uint32_t n5 = popc(st), n2 = popc(e) - n5;
  if (n2) {
    atomicAdd(row + b, (unsigned long long)n2);
    atomicAdd(row + 2 * ISIM_N_PROM, (unsigned long long)(T * n2));
  }
  if (n5) {
    atomicAdd(row + ISIM_N_PROM + b, (unsigned long long)n5);
    atomicAdd(row + 2 * ISIM_N_PROM + 1, (unsigned long long)(T * n5));
  }
}

__device__ __forceinline__ void ret_duration(const Ctx &c, uint32_t row_i, uint64_t T, uint64_t e, uint64_t st) {
  uint64_t *row = c.svc_tab + (uint64_t)row_i * ISIM_SVC_DUR_WORDS;
  const bool is5 = lane_in(st);
  hist_add_global(row, (is5 ? ISIM_N_PROM : 0u) + prom_bucket(T), e);
  const uint64_t s2 = wave_sum64(lane_in(e & ~st) ? T : 0);
  const uint64_t s5 = st ? wave_sum64(is5 ? T : 0) : 0;
  if (lane_id() == 0) {
    if (s2) atomicAdd((unsigned long long *)(row + 2 * ISIM_N_PROM), (unsigned long long)s2);
    if (s5) atomicAdd((unsigned long long *)(row + 2 * ISIM_N_PROM + 1), (unsigned long long)s5);
  }
}

template <bool MODEB, typename TT>
__device__ __forceinline__ void walk_dynamic(const Ctx &c, uint64_t trace_begin, uint64_t n_traces,
                                             uint64_t base, TT *__restrict__ lstk, uint32_t *__restrict__ hstk) {
  const uint32_t lane = lane_id();
  const uint64_t idx = base + lane;
  const bool valid = idx < n_traces;
  const uint64_t t = trace_begin + idx;
  const uint32_t t_lo = (uint32_t)t, t_hi = (uint32_t)(t >> 32);
  const uint64_t all = ballot(valid);
  const Ins *__restrict__ prog = c.prog;

  uint64_t live = all, failed = 0, cerr = 0, own = 0, root_st = 0;
  uint32_t depth = 0, pc = 0;
  TT acc = 0, cmax = 0;
  uint32_t myhop = 0, hopn = 0, cblk = 0xFFFFFFFFu;
  uint32_t x0 = 0, x1 = 0, x2 = 0, x3 = 0, errh = 0;
  LaneStack<uint32_t> f_ret;
  LaneStack<uint64_t> f_live, f_failed, f_cerr, f_own;

  auto fold = [&](uint32_t flags, uint64_t H, TT T, uint64_t e, uint64_t st) {
    if (flags & F_ROOT) {
      root_st = st;
      if (lane_in(e)) acc = (TT)H + T;
    } else if (flags & F_CONC) {
      if (lane_in(e)) {
        const TT v = (TT)H + T;
        cmax = v > cmax ? v : cmax;
      }
      if constexpr (MODEB) cerr |= st;
    } else {
      if (lane_in(e)) acc += (TT)H + T;
      if constexpr (MODEB) failed |= st;
    }
  };

  Ins cur = prog[0];
  while (true) {
    const uint32_t op = cur.opf & 0xFFu;
    if (op == OP_HALT) break;
    const uint32_t flags = (cur.opf >> 8) & 0xFFu;
    uint32_t npc = pc + 1;
    if (op == OP_CALL) npc = cur.b_lo;
    if (op == OP_RET) npc = f_ret.get(depth - 1);
    Ins2 pre = *reinterpret_cast<const Ins2 *>(prog + (npc - 1));
    const uint64_t act = live & ~failed;
    switch (op) {
      case OP_SLEEP:
        if (lane_in(act)) acc += (TT)u64of(cur.a_lo, cur.a_hi);
        break;
      case OP_CBEGIN:
        if (lane_in(act)) cmax = 0;
        cerr = 0;
        break;
      case OP_CSLEEP:
        if (lane_in(act)) {
          const TT d = (TT)u64of(cur.a_lo, cur.a_hi);
          cmax = d > cmax ? d : cmax;
        }
        break;
      case OP_CEND:
        if (lane_in(act)) acc += cmax;
        if constexpr (MODEB) failed |= cerr & live;
        break;
      case OP_LEAF:
      case OP_CALL: {
        uint64_t e = act;
        if (flags & F_PROB) {  // shouldSkipRequest: Intn(100) < 100 - p
          bool skip = false;
          if (lane_in(e)) {
            uint32_t c0 = t_lo, c1 = t_hi, c2 = myhop, c3 = 1u + (cur.k >> 2);
            philox10(c0, c1, c2, c3, c.k0, c.k1);
            const uint32_t sel = cur.k & 3u;
            const uint32_t word = sel == 0 ? c0 : sel == 1 ? c1 : sel == 2 ? c2 : c3;
            skip = (word % 100u) < 100u - (cur.opf >> 16);
          }
          e &= ~ballot(skip);
        }
        if (e == 0) {  // no lane makes this call: fall through to pc+1
          if (op == OP_CALL) {
            npc = pc + 1;
            pre = *reinterpret_cast<const Ins2 *>(prog + (npc - 1));
          }
          break;
        }
        uint64_t st = 0;
        if (flags & F_ERR_ALWAYS) {
          st = e;
        } else if (flags & F_ERR_DRAW) {
          const uint32_t blk = hopn >> 2;
          const uint64_t need = ballot(blk != cblk) & e;
          if (need && lane_in(need)) {
            uint32_t a = t_lo, b = t_hi, cc = blk, d = 0;
            philox10(a, b, cc, d, c.k0, c.k1);
            x0 = a;
            x1 = b;
            x2 = cc;
            x3 = d;
            cblk = blk;
          }
          const uint32_t w = hopn & 3u;
          const uint32_t lo = (w & 1u) ? x1 : x0;
          const uint32_t hi = (w & 1u) ? x3 : x2;
          st = ballot(((w & 2u) ? hi : lo) < cur.thr) & e;
        }
        const uint32_t myh = hopn;
        if (lane_in(e)) ++hopn;
        if (!(flags & F_ROOT)) count(c.gstats, c.cnt, cur.slot, popc(e));
        const uint64_t H = u64of(cur.a_lo, cur.a_hi);
        if (op == OP_LEAF) {
          if (!(flags & F_ROOT)) count(c.gstats, c.cnt, c.n_slots + cur.slot, popc(st));
          if (lane_in(st)) ++errh;
          if (c.svc_tab) leaf_duration(c, (flags & F_ROOT) ? c.root_dur : c.dur[cur.slot],
                                       u64of(cur.b_lo, cur.b_hi), e, st);
          fold(flags, H, (TT)u64of(cur.b_lo, cur.b_hi), e, st);
        } else {
          f_ret.put(depth, pc + 1);
          f_own.put(depth, own);
          f_live.put(depth, live);
          f_failed.put(depth, failed);
          if constexpr (MODEB) f_cerr.put(depth, cerr);
          lstk[(2 * depth) * 64 + lane] = acc;
          lstk[(2 * depth + 1) * 64 + lane] = cmax;
          hstk[depth * 64 + lane] = myhop;
          ++depth;
          acc = 0;
          cmax = 0;
          myhop = myh;
          live = e;
          failed = 0;
          cerr = 0;
          own = st;
        }
        break;
      }
      case OP_RET: {
        const uint64_t e = live;
        const uint64_t st = (failed | own) & e;
        const TT T = acc;
        --depth;
        own = f_own.get(depth);
        live = f_live.get(depth);
        failed = f_failed.get(depth);
        if constexpr (MODEB) cerr = f_cerr.get(depth);
        else cerr = 0;
        acc = lstk[(2 * depth) * 64 + lane];
        cmax = lstk[(2 * depth + 1) * 64 + lane];
        myhop = hstk[depth * 64 + lane];
        const Ins &cin = pre.a;
        const uint32_t cflags = (cin.opf >> 8) & 0xFFu;
        if (!(cflags & F_ROOT)) count(c.gstats, c.cnt, c.n_slots + cin.slot, popc(st));
        if (lane_in(st)) ++errh;
        if (c.svc_tab) ret_duration(c, ((cflags & F_ROOT) ? c.root_dur : c.dur[cin.slot]) & kDurRowMask,
                                    (uint64_t)T, e, st);
        fold(cflags, u64of(cin.a_lo, cin.a_hi), T, e, st);
        break;
      }
      default:
        __builtin_trap();
    }
    cur = pre.b;
    pc = npc;
  }
  finish_batch(c, idx, valid, all, (uint64_t)acc, hopn, root_st, errh);
}


// ======================================================================
// DRAW STREAM walk (static walks): every trace executes the same invocation
// sequence, so the program compiler lays the invocations out in hop order
// (one 8-byte Node each) and folds the trace-invariant latency (t_static),
// hop count and per-site call multiplicities (the executed-call counters are
// mult[slot] x n_traces, added by isim_stream_calls).  Per lane and
// invocation only the stochastic part remains: the Philox error draw, the
// 500 status (mode B: OR-ed up the call tree at each subtree close), the
// per-trace error count and the per-site error counters.  Four records share
// one Philox block and one s_load_dwordx8; two group buffers ping-pong so the
// next group's load is in flight while the current one is processed.
// ======================================================================
struct Node4 {
  Node n[4];
};
// The stream is read-only for the whole launch: reading it through the
// constant address space lets the compiler issue s_load_dwordx8 (a uniform
// global-space load after the loop's stores would become a VMEM load +
// v_readfirstlane with an immediate vmcnt wait).
typedef const __attribute__((address_space(4))) Node4 CNode4;
__device__ __forceinline__ Node4 load_group(CNode4 *p) {
  Node4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r.n[j].thr = p->n[j].thr;
    r.n[j].meta = p->n[j].meta;
  }
  return r;
}

// m = 2 m + (this lane in mask): one v_addc_co_u32 with the lane mask as carry-in
__device__ __forceinline__ void shift_in(uint32_t &m, uint64_t mask) {
  uint64_t co;
  asm("v_addc_co_u32 %0, %1, %0, %0, %2" : "+v"(m), "=s"(co) : "s"(mask));
}
// v += (this lane in mask)
__device__ __forceinline__ void add_lane(uint32_t &v, uint64_t mask) {
  uint64_t co;
  asm("v_addc_co_u32 %0, %1, 0, %0, %2" : "+v"(v), "=s"(co) : "s"(mask));
}

template <bool LDSC>
__device__ __forceinline__ void count_t(uint64_t *__restrict__ gstats, uint32_t *cnt, uint32_t idx, uint32_t v,
                                        bool lane0) {
  if (lane0) {
    if constexpr (LDSC) atomicAdd(cnt + idx, v);
    else atomicAdd((unsigned long long *)(gstats + ISIM_ST_SITES + idx), (unsigned long long)v);
  }
}

// Philox4x32-10 of counter (t_lo, t_hi, g, 0); rounds 1-2 fold the
// wave-uniform words (t_hi when the batch does not straddle 2^32, g, 0) into
// scalar math.
__device__ __forceinline__ void philox_group(uint32_t t_lo, uint32_t t_hi, uint32_t t_hi_u, bool hi_uniform,
                                             uint32_t g, uint32_t k0a, uint32_t k1a, uint32_t (&x)[4]) {
  uint32_t a = t_lo, b = t_hi, cc = g, d = 0;
  if (hi_uniform) {
    const uint64_t q1 = (uint64_t)M1 * g;                      // scalar
    const uint64_t p0 = (uint64_t)M0 * t_lo;                   // per lane
    const uint32_t u0 = (uint32_t)(q1 >> 32) ^ t_hi_u ^ k0a;   // uniform
    const uint32_t u1 = (uint32_t)q1;                          // uniform
    const uint32_t v2 = (uint32_t)(p0 >> 32) ^ k1a;            // per lane
    const uint32_t v3 = (uint32_t)p0;                          // per lane
    const uint32_t k0b = k0a + W0, k1b = k1a + W1;
    const uint64_t q0 = (uint64_t)M0 * u0;                     // scalar
    const uint64_t p1 = (uint64_t)M1 * v2;                     // per lane
    a = (uint32_t)(p1 >> 32) ^ (u1 ^ k0b);
    b = (uint32_t)p1;
    cc = v3 ^ ((uint32_t)(q0 >> 32) ^ k1b);
    d = (uint32_t)q0;
    uint32_t k0 = k0b + W0, k1 = k1b + W1;
#pragma unroll
    for (int r = 2; r < 10; ++r) {
      round1(a, b, cc, d, k0, k1);
      k0 += W0;
      k1 += W1;
    }
  } else {
    philox10(a, b, cc, d, k0a, k1a);
  }
  x[0] = a;
  x[1] = b;
  x[2] = cc;
  x[3] = d;
}

// TPL Philox blocks (one per trace of the lane) of counter (t_lo[u], t_hi, g, 0)
// in lockstep: the round keys and the scalar rounds 1-2 (all counter words
// but t_lo are wave-uniform) are shared by the TPL chains.
template <int TPL>
__device__ __forceinline__ void philox_lockstep(const uint32_t (&t_lo)[TPL], uint32_t t_hi_u, uint32_t g,
                                                uint32_t k0a, uint32_t k1a, uint32_t (&x)[TPL][4]) {
  const uint64_t q1 = (uint64_t)M1 * g;                      // scalar
  const uint32_t u0 = (uint32_t)(q1 >> 32) ^ t_hi_u ^ k0a;   // uniform
  const uint32_t u1 = (uint32_t)q1;                          // uniform
  const uint32_t k0b = k0a + W0, k1b = k1a + W1;
  const uint64_t q0 = (uint64_t)M0 * u0;                     // scalar (round 2)
  // a VOP3 reads one SGPR: pre-xor the uniform words (opaque, so the
  // compiler does not re-fold them into a two-SGPR v_bitop3 + v_mov)
  uint32_t uk0 = u1 ^ k0b, uk1 = (uint32_t)(q0 >> 32) ^ k1b;
  asm volatile("" : "+s"(uk0), "+s"(uk1));
  uint32_t a[TPL], b[TPL], cc[TPL], d[TPL];
#pragma unroll
  for (int u = 0; u < TPL; ++u) {
    const uint64_t p0 = (uint64_t)M0 * t_lo[u];              // per lane
    const uint32_t v2 = (uint32_t)(p0 >> 32) ^ k1a;
    const uint64_t p1 = (uint64_t)M1 * v2;
    a[u] = (uint32_t)(p1 >> 32) ^ uk0;
    b[u] = (uint32_t)p1;
    cc[u] = (uint32_t)p0 ^ uk1;
    d[u] = (uint32_t)q0;
  }
  uint32_t k0 = k0b + W0, k1 = k1b + W1;
#pragma unroll
  for (int r = 2; r < 10; ++r) {
    // recompute the round keys per group (2 s_add) instead of letting the
    // compiler hoist all 16 into SGPRs, which spill to VGPR lanes and come
    // back as v_readlane (VALU) in the hot loop
    asm volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
    for (int u = 0; u < TPL; ++u) round1(a[u], b[u], cc[u], d[u], k0, k1);
    k0 += W0;
    k1 += W1;
  }
#pragma unroll
  for (int u = 0; u < TPL; ++u) {
    x[u][0] = a[u];
    x[u][1] = b[u];
    x[u][2] = cc[u];
    x[u][3] = d[u];
  }
}



// TPL traces per lane: the wave walks 64*TPL traces through one pass over the
// stream, so the per-record scalar work (fetch, decode, counter adds) is
// shared and each lane runs TPL independent Philox chains (ILP).
// BS: mode B keeps the open invocations' statuses in a per-lane bit stack
// (bit p = running status of the frame at stack position p; VALU), for
// call depths <= 32 (kernel kind 5); otherwise (kind 4) as wave masks on a
// VGPR-lane stack.
template <bool MODEB, bool LDSC, int TPL, bool FULL, bool BS>
__device__ __forceinline__ void walk_stream(const Ctx &c, CNode4 *__restrict__ stream, uint32_t n_groups,
                                            uint32_t n_nodes, uint64_t t_static, uint64_t trace_begin,
                                            uint64_t n_traces, uint64_t base) {
  const uint32_t lane = lane_id();
  const bool lane0 = lane == 0;
  uint64_t idx[TPL], all[TPL];
  uint32_t t_lo[TPL], t_hi[TPL], t_hi_u[TPL];
  bool valid[TPL];
  bool hi_uniform = true;
#pragma unroll
  for (int u = 0; u < TPL; ++u) {
    idx[u] = base + 64u * u + lane;
    valid[u] = idx[u] < n_traces;
    const uint64_t t = trace_begin + idx[u];
    t_lo[u] = (uint32_t)t;
    t_hi[u] = (uint32_t)(t >> 32);
    t_hi_u[u] = rfl(t_hi[u]);
    hi_uniform = hi_uniform && ballot(t_hi[u] != t_hi_u[u]) == 0 && t_hi_u[u] == t_hi_u[0];  // no 2^32 straddle
    all[u] = ballot(valid[u]);
  }

  uint32_t errh[TPL];
  uint64_t root_st[TPL];
  // mode B: stack of open invocations; the top's running status in SGPRs
  uint64_t top[TPL];
  uint32_t top_slot = 0, depth = 0;
  LaneStack<uint64_t> s_mask[TPL];
  LaneStack<uint32_t> s_slot;
  // mode B, bit-stack form (BS): per lane and trace, bit p of stk_lo = the
  // running 500 status of the open frame at stack position p (p < 32)
  uint32_t stk_lo[TPL];
#pragma unroll
  for (int u = 0; u < TPL; ++u) {
    errh[u] = 0;
    root_st[u] = 0;
    top[u] = 0;
    stk_lo[u] = 0;
  }
  // set / test / clear bit p (wave-uniform, < 32) in the lanes of mask m: VALU only
  auto bs_set = [&](int u, uint32_t p, uint64_t m) {
    const uint32_t b = 1u << (p & 31u);
    stk_lo[u] |= lane_in(m) ? b : 0u;
  };
  auto bs_test = [&](int u, uint32_t p) -> uint64_t {
    const uint32_t b = 1u << (p & 31u);
    return ballot((stk_lo[u] & b) != 0u);
  };
  auto bs_clear = [&](int u, uint32_t p) {
    stk_lo[u] &= ~(1u << (p & 31u));
  };
  auto node = [&](uint32_t thr, uint32_t meta, const uint32_t (&xw)[TPL]) {
    const uint32_t slot = meta & 0xFFFFFFu;
    uint64_t own[TPL];
#pragma unroll
    for (int u = 0; u < TPL; ++u) own[u] = (meta & 0x80000000u) ? all[u] : (ballot(xw[u] < thr) & all[u]);
    if constexpr (!MODEB) {
      // mode A: an invocation's status is its own error draw; padding
      // records (thr 0, never always) draw nothing.  The root (record 0)
      // is peeled off before the loop.
      uint64_t any = 0;
      uint32_t n = 0;
#pragma unroll
      for (int u = 0; u < TPL; ++u) {
        add_lane(errh[u], own[u]);
        any |= own[u];
        n += popc(own[u]);
      }
      if (any) count_t<LDSC>(c.gstats, c.cnt, c.n_slots + slot, n, lane0);
    } else if constexpr (BS) {
      if (slot == kSlotPad) return;
      uint32_t k = (meta >> 24) & 0x7Fu;
      const uint32_t d = depth;  // this invocation's stack position
      if (k > 0) {
        // a leaf opens and closes here: its status is its own draw; it
        // fails the caller (the open frame at d-1) in mode B
        uint64_t any = 0;
        uint32_t n = 0;
#pragma unroll
        for (int u = 0; u < TPL; ++u) {
          add_lane(errh[u], own[u]);
          any |= own[u];
          n += popc(own[u]);
        }
        if (d == 0) {
#pragma unroll
          for (int u = 0; u < TPL; ++u) root_st[u] = own[u];
        } else if (any) {
          count_t<LDSC>(c.gstats, c.cnt, c.n_slots + slot, n, lane0);
#pragma unroll
          for (int u = 0; u < TPL; ++u) bs_set(u, d - 1, own[u]);
        }
        --k;
      } else {
        uint64_t any = 0;
#pragma unroll
        for (int u = 0; u < TPL; ++u) any |= own[u];
        if (any) {
#pragma unroll
          for (int u = 0; u < TPL; ++u) bs_set(u, d, own[u]);
        }
        s_slot.put(d, slot);
        depth = d + 1;
      }
      for (; k > 0; --k) {  // the frame at position depth-1 closes
        const uint32_t p = depth - 1;
        uint64_t st[TPL], any = 0;
#pragma unroll
        for (int u = 0; u < TPL; ++u) {
          st[u] = bs_test(u, p);
          any |= st[u];
        }
        if (p == 0) {
#pragma unroll
          for (int u = 0; u < TPL; ++u) {
            root_st[u] = st[u];
            add_lane(errh[u], st[u]);
          }
        } else if (any) {
          uint32_t n = 0;
#pragma unroll
          for (int u = 0; u < TPL; ++u) {
            add_lane(errh[u], st[u]);
            n += popc(st[u]);
            bs_set(u, p - 1, st[u]);  // mode B: a 500 fails the caller
            bs_clear(u, p);
          }
          count_t<LDSC>(c.gstats, c.cnt, c.n_slots + s_slot.get(p), n, lane0);
        }
        depth = p;
      }
    } else {
      if (slot == kSlotPad) return;
      uint32_t k = (meta >> 24) & 0x7Fu;
      if (k > 0 && depth > 0) {
        // a leaf (opens and closes here): no push; its status is its own
        // draw, OR-ed into the caller's running status
        uint64_t any = 0;
        uint32_t n = 0;
#pragma unroll
        for (int u = 0; u < TPL; ++u) {
          add_lane(errh[u], own[u]);
          any |= own[u];
          n += popc(own[u]);
          top[u] |= own[u];
        }
        if (any) count_t<LDSC>(c.gstats, c.cnt, c.n_slots + slot, n, lane0);
        --k;
      } else {
        if (depth > 0) {
#pragma unroll
          for (int u = 0; u < TPL; ++u) s_mask[u].put(depth - 1, top[u]);
          s_slot.put(depth - 1, top_slot);
        }
#pragma unroll
        for (int u = 0; u < TPL; ++u) top[u] = own[u];
        top_slot = slot;
        ++depth;
      }
      for (; k > 0; --k) {  // subtree closes
        uint64_t any = 0;
        uint32_t n = 0;
        uint64_t st[TPL];
#pragma unroll
        for (int u = 0; u < TPL; ++u) {
          st[u] = top[u];
          add_lane(errh[u], st[u]);
          any |= st[u];
          n += popc(st[u]);
        }
        if (any && top_slot != kSlotRoot) count_t<LDSC>(c.gstats, c.cnt, c.n_slots + top_slot, n, lane0);
        --depth;
        if (depth > 0) {
#pragma unroll
          for (int u = 0; u < TPL; ++u) top[u] = s_mask[u].get(depth - 1) | st[u];  // mode B: 500 fails the caller
          top_slot = s_slot.get(depth - 1);
        } else {
#pragma unroll
          for (int u = 0; u < TPL; ++u) root_st[u] = st[u];
        }
      }
    }
  };
  auto draws = [&](const Node4 &q, uint32_t g, uint32_t (&x)[TPL][4]) {
    if ((q.n[0].thr | q.n[1].thr | q.n[2].thr | q.n[3].thr) != 0) {
      if (hi_uniform) {
        philox_lockstep<TPL>(t_lo, t_hi_u[0], g, c.k0, c.k1, x);
      } else {
#pragma unroll
        for (int u = 0; u < TPL; ++u) philox_group(t_lo[u], t_hi[u], t_hi_u[u], hi_uniform, g, c.k0, c.k1, x[u]);
      }
    }
  };
  auto group = [&](const Node4 &q, uint32_t g) {
    uint32_t x[TPL][4];
#pragma unroll
    for (int u = 0; u < TPL; ++u) x[u][0] = x[u][1] = x[u][2] = x[u][3] = 0;
    draws(q, g, x);
    if constexpr (!MODEB) {
      // mode A, no errorRate-1 record in the group: per record one compare
      // per trace; counts only on the (rarer) records where some lane errs
      if (((q.n[0].meta | q.n[1].meta | q.n[2].meta | q.n[3].meta) & 0x80000000u) == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint64_t own[TPL], any = 0;
#pragma unroll
          for (int u = 0; u < TPL; ++u) {
            own[u] = ballot(x[u][j] < q.n[j].thr);
            if constexpr (!FULL) own[u] &= all[u];
            any |= own[u];
          }
          if (any) {
            uint32_t n = 0;
#pragma unroll
            for (int u = 0; u < TPL; ++u) {
              add_lane(errh[u], own[u]);
              n += popc(own[u]);
            }
            count_t<LDSC>(c.gstats, c.cnt, c.n_slots + (q.n[j].meta & 0xFFFFFFu), n, lane0);
          }
        }
        return;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t xw[TPL];
#pragma unroll
      for (int u = 0; u < TPL; ++u) xw[u] = x[u][j];
      node(q.n[j].thr, q.n[j].meta, xw);
    }
  };

  const Node4 bufA = load_group(stream);
  const Node4 bufB = load_group(stream + 1);  // zero tail padding when n_groups == 1
  {  // group 0: record 0 is the entry invocation (the client request)
    uint32_t x[TPL][4];
#pragma unroll
    for (int u = 0; u < TPL; ++u) x[u][0] = x[u][1] = x[u][2] = x[u][3] = 0;
    draws(bufA, 0, x);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t xw[TPL];
#pragma unroll
      for (int u = 0; u < TPL; ++u) xw[u] = x[u][j];
      if (j == 0 && !MODEB) {
#pragma unroll
        for (int u = 0; u < TPL; ++u) {
          const uint64_t own =
              (bufA.n[0].meta & 0x80000000u) ? all[u] : (ballot(xw[u] < bufA.n[0].thr) & all[u]);
          add_lane(errh[u], own);
          root_st[u] = own;
        }
      } else {
        node(bufA.n[j].thr, bufA.n[j].meta, xw);
      }
    }
  }
  // Group g+1 is loaded (unconditionally: the device buffer carries two zero
  // groups of tail padding) before group g is processed, and handed over by
  // a loop-carried copy after it, so the s_waitcnt for the load lands after
  // a whole group of Philox work.
  Node4 cur = bufB;
  for (uint32_t g = 1; g < n_groups; ++g) {
    const Node4 nxt = load_group(stream + g + 1);
    group(cur, g);
    cur = nxt;
  }
#pragma unroll
  for (int u = 0; u < TPL; ++u) finish_batch(c, idx[u], valid[u], all[u], t_static, n_nodes, root_st[u], errh[u]);
}

typedef const __attribute__((address_space(4))) StreamClose CClose;
typedef const __attribute__((address_space(4))) uint32_t CU32;
struct CloseBlk {
  StreamClose c[8];
};
__device__ __forceinline__ CloseBlk load_closes(CClose *p) {  // one s_load_dwordx16
  CloseBlk r;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    r.c[k].pre1 = p[k].pre1;
    r.c[k].rmask = p[k].rmask;
  }
  return r;
}

// Mode B on the draw stream without a stack (kernel kind 6).  An invocation
// responds 500 iff some invocation of its subtree drew an error (a 500 fails
// the caller's step, and the caller's step failure is its 500), and a
// subtree is the contiguous stream range [p, j] (DFS preorder).  So a lane
// only keeps, per trace, the error bits of the current chunk of 32 records
// (shifted in, one v_addc per record) and the position + 1 of its last
// erring record before the chunk; after each chunk the closes that end in it
// are tested against both (StreamClose, kernel_abi.h) and counted (a lane
// per close, one ds_add per 64 closes).  Leaves respond with their own draw
// (a lane per record, one ds_add per chunk); the entry's status is "any
// error at all".  No call-depth limit, no per-record branching
// on the stack.
template <bool LDSC, int TPL, bool FULL>
__device__ __forceinline__ void walk_stream_cl(const Ctx &c, CNode4 *__restrict__ stream, uint32_t n_groups,
                                               uint32_t n_nodes, uint64_t t_static, uint64_t trace_begin,
                                               uint64_t n_traces, uint64_t base, CClose *__restrict__ closes,
                                               const uint32_t *__restrict__ close_slot, CU32 *__restrict__ close_end,
                                               const uint32_t *__restrict__ stream_w) {
  const uint32_t lane = lane_id();
  uint64_t idx[TPL], all[TPL];
  uint32_t t_lo[TPL], t_hi[TPL], t_hi_u[TPL];
  bool valid[TPL];
  bool hi_uniform = true;
#pragma unroll
  for (int u = 0; u < TPL; ++u) {
    idx[u] = base + 64u * u + lane;
    valid[u] = idx[u] < n_traces;
    const uint64_t t = trace_begin + idx[u];
    t_lo[u] = (uint32_t)t;
    t_hi[u] = (uint32_t)(t >> 32);
    t_hi_u[u] = rfl(t_hi[u]);
    hi_uniform = hi_uniform && ballot(t_hi[u] != t_hi_u[u]) == 0 && t_hi_u[u] == t_hi_u[0];
    all[u] = ballot(valid[u]);
  }
  uint32_t errh[TPL], le[TPL];
#pragma unroll
  for (int u = 0; u < TPL; ++u) errh[u] = le[u] = 0;

  Node4 cur = load_group(stream);
  uint32_t cp = 0;
  const uint32_t n_chunks = (n_groups + kChunkGroups - 1) / kChunkGroups;
  for (uint32_t ch = 0; ch < n_chunks; ++ch) {
    const uint32_t g0 = ch * kChunkGroups;
    const uint32_t g1 = g0 + kChunkGroups < n_groups ? g0 + kChunkGroups : n_groups;
    // the chunk's first 64 close slots (one per lane), loaded before its Philox work
    uint32_t slotv = close_slot[cp + lane];  // zero tail padding
    const uint32_t nrec = 4u * (g1 - g0);
    const uint32_t rmeta = lane < nrec ? stream_w[2u * (ch * kChunkRecords + lane) + 1u] : kSlotPad;
    uint32_t lcnt = 0;
    uint32_t mb[TPL];
#pragma unroll
    for (int u = 0; u < TPL; ++u) mb[u] = 0;
    // one group: its Philox blocks, then per record the error bits shifted
    // into mb and the record's count in lane r of lcnt
    auto grp = [&](const Node4 &q, uint32_t g) {
      uint32_t x[TPL][4];
#pragma unroll
      for (int u = 0; u < TPL; ++u) x[u][0] = x[u][1] = x[u][2] = x[u][3] = 0;
      if ((q.n[0].thr | q.n[1].thr | q.n[2].thr | q.n[3].thr) != 0) {
        if (hi_uniform) {
          philox_lockstep<TPL>(t_lo, t_hi_u[0], g, c.k0, c.k1, x);
        } else {
#pragma unroll
          for (int u = 0; u < TPL; ++u) philox_group(t_lo[u], t_hi[u], t_hi_u[u], hi_uniform, g, c.k0, c.k1, x[u]);
        }
      }
      auto records = [&](bool always) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t thr = q.n[j].thr, meta = q.n[j].meta;
          uint32_t n = 0;
#pragma unroll
          for (int u = 0; u < TPL; ++u) {
            uint64_t own = ballot(x[u][j] < thr);
            if (always && (meta & 0x80000000u)) own = ~0ull;
            shift_in(mb[u], own);
            if constexpr (!FULL) own &= all[u];
            n += popc(own);
          }
          lcnt = wrl(n, 4u * (g - g0) + j, lcnt);  // lane r: record r's count
        }
      };
      // errorRate-1 records (always 500) are rare: a branch per record only
      // in the groups that hold one
      if (((q.n[0].meta | q.n[1].meta | q.n[2].meta | q.n[3].meta) & 0x80000000u) == 0) records(false);
      else records(true);
    };
    // two groups per trip, each group's records loaded one group ahead into
    // the other buffer (no register copy between them: with `cur = nxt` the
    // compiler waited for each prefetch right after issuing it, so every
    // group paid the scalar load's latency)
    uint32_t g = g0;
    for (; g + 1 < g1; g += 2) {
      // the load of b issues after cur has arrived (an empty asm reads cur):
      // scalar loads return out of order, so a wait for cur placed after
      // b's issue would wait for b too
      CNode4 *pb = stream + g + 1;
      asm volatile("" : "+s"(pb) : "s"(cur.n[0].thr));
      const Node4 b = load_group(pb);
      grp(cur, g);
      CNode4 *pc = stream + g + 2;  // zero tail padding
      asm volatile("" : "+s"(pc) : "s"(b.n[0].thr));
      cur = load_group(pc);
      grp(b, g + 1);
    }
    if (g < g1) {
      const Node4 b = load_group(stream + g + 1);
      grp(cur, g);
      cur = b;
    }
    // leaves respond with their own draw: their error counts (lane r =
    // record r) go to the site table in one ds_add, their 500s to errh
    {
      const uint32_t rslot = rmeta & 0xFFFFFFu;
      const bool leaf = (rmeta & 0x7F000000u) != 0 && rslot < kSlotPad;
      const uint32_t lm = __builtin_bitreverse32((uint32_t)ballot(leaf)) >> (32u - nrec);  // mb's bit order
#pragma unroll
      for (int u = 0; u < TPL; ++u) errh[u] += (uint32_t)__builtin_popcount(mb[u] & lm);
      if (leaf && lcnt) {
        if constexpr (LDSC) atomicAdd(c.cnt + c.n_slots + rslot, lcnt);
        else atomicAdd((unsigned long long *)(c.gstats + ISIM_ST_SITES + c.n_slots + rslot), (unsigned long long)lcnt);
      }
    }
    const uint32_t ce = close_end[ch];
    CloseBlk blk = load_closes(closes + cp);  // the chunk's first 8 closes
    // calling invocations whose subtree ends in this chunk, in segments of
    // up to 64: close i of a segment keeps its count in lane i of cntv, and
    // the segment's counts go to the site table in one ds_add
    while (cp < ce) {
      const uint32_t nseg = ce - cp < 64u ? ce - cp : 64u;
      uint32_t cntv = 0;
      for (uint32_t i = 0; i < nseg; i += 8) {
        const CloseBlk nb = load_closes(closes + cp + i + 8);  // zero tail padding
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (i + k >= nseg) break;
          const uint32_t pre1 = blk.c[k].pre1, rmask = blk.c[k].rmask;
          uint32_t n = 0;
#pragma unroll
          for (int u = 0; u < TPL; ++u) {
            uint64_t st = ballot((mb[u] & rmask) != 0u) | ballot(le[u] >= pre1);
            if constexpr (!FULL) st &= all[u];
            add_lane(errh[u], st);
            n += popc(st);
          }
          cntv = wrl(n, i + k, cntv);
        }
        blk = nb;
      }
      if (lane < nseg) {
        if constexpr (LDSC) atomicAdd(c.cnt + c.n_slots + slotv, cntv);
        else if (cntv) atomicAdd((unsigned long long *)(c.gstats + ISIM_ST_SITES + c.n_slots + slotv),
                                 (unsigned long long)cntv);
      }
      cp += nseg;
      if (cp < ce) slotv = close_slot[cp + lane];  // a chunk with more than 64 closes
    }
    const uint32_t top = ch * kChunkRecords + 4u * (g1 - g0);
#pragma unroll
    for (int u = 0; u < TPL; ++u) le[u] = mb[u] ? top - (uint32_t)__builtin_ctz(mb[u]) : le[u];
  }
#pragma unroll
  for (int u = 0; u < TPL; ++u) {
    const uint64_t root_st = ballot(le[u] != 0u) & all[u];
    add_lane(errh[u], root_st);
    finish_batch(c, idx[u], valid[u], all[u], t_static, n_nodes, root_st, errh[u]);
  }
}

// Mode B on the draw stream by sparse ancestor marking (kernel kind 8, the
// default; kernel_abi.h kMarkPadKey).  The walk is mode A's — one Philox block
// per group of 4 records, one compare per record and trace — plus, per record
// and trace, one v_min of the record's key into the lane's running minimum
// since its trace's last error.  Only where some lane errs (the branch mode A
// takes for its counters anyway) the erring lanes mark: +1 at the record (one
// ds_add for the wave), -1 at the LCA that minimum names (a ds_sub per
// erring lane), and the trace's new 500s depth(e) - depth(LCA) into its error
// count.  The entry responds 500 iff its trace erred at all.  Costs against
// the close list (kind 6): no per-chunk close tests (4,389 per trace on
// config 3), no error-bit shifts, no call-depth limit.
template <int TPL, bool FULL>
__device__ __forceinline__ void walk_stream_mark(const Ctx &c, CNode4 *__restrict__ stream, uint32_t n_groups,
                                                 uint32_t n_nodes, uint64_t t_static, uint64_t trace_begin,
                                                 uint64_t n_traces, uint64_t base) {
  const uint32_t lane = lane_id();
  const bool lane0 = lane == 0;
  uint64_t idx[TPL], all[TPL];
  uint32_t t_lo[TPL], t_hi[TPL], t_hi_u[TPL];
  bool valid[TPL];
  bool hi_uniform = true;
#pragma unroll
  for (int u = 0; u < TPL; ++u) {
    idx[u] = base + 64u * u + lane;
    valid[u] = idx[u] < n_traces;
    const uint64_t t = trace_begin + idx[u];
    t_lo[u] = (uint32_t)t;
    t_hi[u] = (uint32_t)(t >> 32);
    t_hi_u[u] = rfl(t_hi[u]);
    hi_uniform = hi_uniform && ballot(t_hi[u] != t_hi_u[u]) == 0 && t_hi_u[u] == t_hi_u[0];
    all[u] = ballot(valid[u]);
  }
  uint32_t errh[TPL], mk[TPL];
#pragma unroll
  for (int u = 0; u < TPL; ++u) {
    errh[u] = 0;
    mk[u] = 0xFFFFFFFFu;
  }
  uint32_t *marks = c.cnt;
  auto group = [&](const Node4 &q, uint32_t g) {
    uint32_t x[TPL][4];
#pragma unroll
    for (int u = 0; u < TPL; ++u) x[u][0] = x[u][1] = x[u][2] = x[u][3] = 0;
    if ((q.n[0].thr | q.n[1].thr | q.n[2].thr | q.n[3].thr) != 0) {
      if (hi_uniform) {
        philox_lockstep<TPL>(t_lo, t_hi_u[0], g, c.k0, c.k1, x);
      } else {
#pragma unroll
        for (int u = 0; u < TPL; ++u) philox_group(t_lo[u], t_hi[u], t_hi_u[u], hi_uniform, g, c.k0, c.k1, x[u]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t kw = q.n[j].meta;
      const uint32_t key = kw & kMarkKeyMask;
      const uint64_t always = (kw & 0x80000000u) ? ~0ull : 0ull;  // errorRate 1: no draw, always 500
      uint64_t own[TPL], any = 0;
#pragma unroll
      for (int u = 0; u < TPL; ++u) {
        own[u] = ballot(x[u][j] < q.n[j].thr) | always;
        if constexpr (!FULL) own[u] &= all[u];
        mk[u] = mk[u] < key ? mk[u] : key;
        any |= own[u];
      }
      if (any) {
        uint32_t n = 0;
#pragma unroll
        for (int u = 0; u < TPL; ++u) n += popc(own[u]);
        if (lane0) atomicAdd(marks + 4u * g + (uint32_t)j, n);
        const uint32_t d1 = (key >> 24) + 1u;
#pragma unroll
        for (int u = 0; u < TPL; ++u) {
          if (lane_in(own[u])) {
            atomicSub(marks + (mk[u] & kMarkPosMask), 1u);
            errh[u] += d1 - (mk[u] >> 24);
            mk[u] = 0xFFFFFFFFu;
          }
        }
      }
    }
  };
  // group g+1 is loaded (the device buffer carries two zero groups of tail
  // padding) before group g is processed (walk_stream)
  Node4 cur = load_group(stream);
  for (uint32_t g = 0; g < n_groups; ++g) {
    const Node4 nxt = load_group(stream + g + 1);
    group(cur, g);
    cur = nxt;
  }
#pragma unroll
  for (int u = 0; u < TPL; ++u) {
    const uint64_t root_st = ballot(errh[u] != 0u) & all[u];
    finish_batch(c, idx[u], valid[u], all[u], t_static, n_nodes, root_st, errh[u]);
  }
}

// Kind 8's per-launch fold (one workgroup): the launch's position marks
// (u32, wrapping: the -1s at an LCA reached often go "negative") become
// subtree sums S(v) = P[end(v)] - P[v - 1] over their prefix sums P — the
// launch's count of 500 responses of the invocation at record v, below 2^32
// (launch_walk's split) — added to the per-site 500 counters; the row is
// zeroed for the next launch that takes this work slot.
__global__ void __launch_bounds__(1024) isim_mark_fold(uint32_t *__restrict__ stage, uint32_t n, uint32_t words,
                                                       const uint32_t *__restrict__ end,
                                                       const uint32_t *__restrict__ slot,
                                                       uint64_t *__restrict__ gstats, uint32_t n_slots) {
  extern __shared__ __align__(16) unsigned char lds[];
  uint32_t *P = reinterpret_cast<uint32_t *>(lds);
  __shared__ uint32_t wtot[16];
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  for (uint32_t i = tid; i < words; i += nt) {
    P[i] = i < n ? stage[i] : 0u;
    stage[i] = 0u;
  }
  __syncthreads();
  // each thread a contiguous segment: local sums, a block scan of the
  // segment totals, then the segment rewritten as inclusive prefix sums
  const uint32_t seg = (n + nt - 1) / nt;
  const uint32_t b = tid * seg, e = b + seg < n ? b + seg : n;
  uint32_t tot = 0;
  for (uint32_t i = b; i < e; ++i) tot += P[i];
  const uint32_t lane = tid & 63u, wave = tid >> 6;
  uint32_t inc = tot;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d, 64);
    if (lane >= d) inc += o;
  }
  if (lane == 63) wtot[wave] = inc;
  __syncthreads();
  uint32_t pre = inc - tot;
  for (uint32_t w = 0; w < wave; ++w) pre += wtot[w];
  for (uint32_t i = b; i < e; ++i) {
    pre += P[i];
    P[i] = pre;
  }
  __syncthreads();
  unsigned long long *st = reinterpret_cast<unsigned long long *>(gstats + ISIM_ST_SITES + n_slots);
  for (uint32_t v = 1 + tid; v < n; v += nt) {
    const uint32_t s = P[end[v]] - P[v - 1];
    if (s) atomicAdd(st + slot[v], (unsigned long long)s);
  }
}

// Executed-call counters of a static walk: every trace makes mult[slot] calls
// through each reachable call site, so a launch over n_traces adds
// mult[slot] * n_traces (exact; added once per launch).
// draw-free static walks: n copies of one trace's record, n x its statistics
__global__ void __launch_bounds__(256) isim_fill_const(isim_trace_rec *__restrict__ rec, uint64_t n,
                                                       isim_trace_rec r, const uint64_t *__restrict__ s1,
                                                       uint64_t *__restrict__ gstats, uint32_t words) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x, stride = (uint64_t)gridDim.x * 256;
  if (rec) {
    // streaming stores, 4 in flight per lane
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = {(uint32_t)r.latency_ns, (uint32_t)(r.latency_ns >> 32), r.hops, r.status_err};
    u32x4 *out = reinterpret_cast<u32x4 *>(rec);
    uint64_t i = tid;
    for (; i + 3 * stride < n; i += 4 * stride) {
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) __builtin_nontemporal_store(v, out + i + u * stride);
    }
    for (; i < n; i += stride) __builtin_nontemporal_store(v, out + i);
  }
  unsigned long long *st = reinterpret_cast<unsigned long long *>(gstats);
  for (uint64_t w = tid; w < words; w += stride) {
    const uint64_t x = s1[w];
    if (!x) continue;
    if (w == ISIM_ST_NOT_MIN_LATENCY || w == ISIM_ST_MAX_LATENCY) atomicMax(st + w, (unsigned long long)x);
    else atomicAdd(st + w, (unsigned long long)(x * n));
  }
}

__global__ void isim_stream_calls(const uint32_t *__restrict__ mult, uint32_t n_slots, uint64_t n_traces,
                                  uint64_t *__restrict__ gstats, uint32_t *__restrict__ stage) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_slots) return;
  gstats[ISIM_ST_SITES + i] += (uint64_t)mult[i] * n_traces;
  if (stage) {  // the launch's staged 500 counts (u32) into the stats; the row is zero again after
    const uint32_t v = stage[i];
    if (v) {
      gstats[ISIM_ST_SITES + n_slots + i] += v;
      stage[i] = 0;
    }
  }
}

// KIND: 0 static/u32 time, 1 static/u64, 2 dynamic/u32, 3 dynamic/u64, 4 draw stream,
// 5 draw stream with the mode-B bit stack (call depth <= 32), 6 draw stream
// with the mode-B close list
// LDSC: per-site counters in the workgroup LDS table (else global atomics)
template <int KIND, bool MODEB, bool LDSC>
__global__ void __launch_bounds__(kWgThreads, KIND >= 4 ? ISIM_STREAM_WAVES : 1)
    isim_walk(const Ins *__restrict__ prog, isim_trace_rec *__restrict__ records, uint64_t *__restrict__ gstats,
              const uint32_t *__restrict__ dur, KParams kp) {
  using TT = typename std::conditional<KIND == 0 || KIND == 2, uint32_t, uint64_t>::type;
  constexpr bool STATIC = KIND < 2 || KIND >= 4;
  extern __shared__ __align__(16) unsigned char lds[];
  Ctx c;
  c.prog = prog;
  c.records = records;
  c.gstats = gstats;
  c.dur = dur;
  c.svc_tab = kp.svc_dur ? gstats + ISIM_ST_SVC_DUR(kp.n_slots) : nullptr;
  c.root_dur = kp.root_dur;
  c.acc = reinterpret_cast<WgAcc *>(lds);
  c.hist = reinterpret_cast<uint32_t *>(lds + kLdsAccBytes);
  c.cnt = LDSC ? c.hist + kHistWords : nullptr;
  c.n_slots = kp.n_slots;
  c.k0 = kp.seed_lo;
  c.k1 = kp.seed_hi;
  unsigned char *stk = lds + kLdsAccBytes + kHistWords * 4 + (LDSC ? 8u * kp.n_slots : 0u);
  stk = (unsigned char *)(((uintptr_t)stk + 15) & ~(uintptr_t)15);
  const uint32_t wave = threadIdx.x >> 6;
  const uint32_t waves = blockDim.x >> 6;
  TT *lstk = nullptr;
  uint32_t *hstk = nullptr;
  if constexpr (!STATIC) {
    const uint32_t per_wave = kp.max_frames * 64u * (2u * (uint32_t)sizeof(TT) + 4u);
    lstk = reinterpret_cast<TT *>(stk + wave * per_wave);
    hstk = reinterpret_cast<uint32_t *>(stk + wave * per_wave + kp.max_frames * 64u * 2u * (uint32_t)sizeof(TT));
  }
  const uint32_t zero_words = (kLdsAccBytes / 4) + kHistWords + (LDSC ? (KIND == 8 ? kp.mark_words : 2u * kp.n_slots) : 0u);
  uint32_t *z = reinterpret_cast<uint32_t *>(lds);
  for (uint32_t i = threadIdx.x; i < zero_words; i += blockDim.x) z[i] = 0;
  __syncthreads();

  constexpr uint64_t kBatch = KIND >= 4 ? 64ull * kStreamTPL : 64ull;
  const uint64_t n_batches = (kp.n_traces + kBatch - 1) / kBatch;
  const uint64_t stride = (uint64_t)gridDim.x * waves;
  // Batches: the first wave-stride statically, the rest claimed from the
  // launch's queues, so waves the SIMD arbiter favours take more batches and
  // the grid drains within about one batch of the last claim.  Queue q (the
  // workgroup's XCD; every queue in use has workgroups) deals batches
  // stride + nq c + q.
  const uint32_t nq = gridDim.x < kWorkQueues ? gridDim.x : kWorkQueues;
  const uint32_t q = blockIdx.x % nq;
  unsigned long long *queue = kp.work + q * kWorkLine;
  auto claim = [&]() -> uint64_t {
    unsigned long long v = 0;
    if (lane_id() == 0) v = atomicAdd(queue, 1ull);
    const uint64_t c = (uint64_t)rfl((uint32_t)(v >> 32)) << 32 | rfl((uint32_t)v);
    return stride + c * nq + q;
  };
  for (uint64_t b = (uint64_t)blockIdx.x * waves + wave; b < n_batches; b = claim()) {
    if constexpr (KIND >= 4) {
      const uint64_t base = b * 64 * kStreamTPL;
      CNode4 *st = (CNode4 *)(const __attribute__((address_space(1))) Ins *)prog;
      const uint32_t ng = kp.n_nodes ? (kp.n_nodes + 3) / 4 : 0;
      if constexpr (KIND == 8) {
        if (base + 64 * kStreamTPL <= kp.n_traces)
          walk_stream_mark<kStreamTPL, true>(c, st, ng, kp.n_nodes, kp.t_static, kp.trace_begin, kp.n_traces, base);
        else
          walk_stream_mark<kStreamTPL, false>(c, st, ng, kp.n_nodes, kp.t_static, kp.trace_begin, kp.n_traces, base);
      } else if constexpr (KIND == 6) {
        CClose *cl = (CClose *)(const __attribute__((address_space(1))) StreamClose *)kp.closes;
        CU32 *ce = (CU32 *)(const __attribute__((address_space(1))) uint32_t *)kp.close_end;
        if (base + 64 * kStreamTPL <= kp.n_traces)
          walk_stream_cl<LDSC, kStreamTPL, true>(c, st, ng, kp.n_nodes, kp.t_static, kp.trace_begin, kp.n_traces,
                                                 base, cl, kp.close_slot, ce, (const uint32_t *)prog);
        else
          walk_stream_cl<LDSC, kStreamTPL, false>(c, st, ng, kp.n_nodes, kp.t_static, kp.trace_begin, kp.n_traces,
                                                  base, cl, kp.close_slot, ce, (const uint32_t *)prog);
      } else if (base + 64 * kStreamTPL <= kp.n_traces)  // every lane of every trace slot valid
        walk_stream<MODEB, LDSC, kStreamTPL, true, KIND == 5>(c, st, ng, kp.n_nodes, kp.t_static, kp.trace_begin,
                                                   kp.n_traces, base);
      else
        walk_stream<MODEB, LDSC, kStreamTPL, false, KIND == 5>(c, st, ng, kp.n_nodes, kp.t_static, kp.trace_begin,
                                                    kp.n_traces, base);
    }
    else if constexpr (STATIC) walk_static<MODEB, TT>(c, kp.trace_begin, kp.n_traces, b * 64);
    else walk_dynamic<MODEB, TT>(c, kp.trace_begin, kp.n_traces, b * 64, lstk, hstk);
  }

  // every wave has stopped claiming once all have counted out: the last one re-arms the queue
  if (lane_id() == 0 && atomicAdd(kp.work + kWorkQueues * kWorkLine, 1ull) == stride - 1) {
    for (uint32_t i = 0; i <= kWorkQueues; ++i) atomicExch(kp.work + i * kWorkLine, 0ull);
  }
  __syncthreads();
  // ---- flush workgroup accumulators to HBM
  unsigned long long *st = reinterpret_cast<unsigned long long *>(gstats);
  for (uint32_t i = threadIdx.x; i < kHistWords; i += blockDim.x)
    if (c.hist[i]) atomicAdd(st + ISIM_ST_PROM + i, (unsigned long long)c.hist[i]);
  if constexpr (KIND == 8) {  // the position marks, folded into the site counters by isim_mark_fold
    for (uint32_t i = threadIdx.x; i < kp.mark_words; i += blockDim.x)
      if (c.cnt[i]) atomicAdd(kp.stage + i, c.cnt[i]);
  } else if constexpr (LDSC) {
    if (kp.stage) {  // draw stream: only the 500 counts are counted here (calls: isim_stream_calls)
      for (uint32_t i = threadIdx.x; i < kp.n_slots; i += blockDim.x)
        if (c.cnt[kp.n_slots + i]) atomicAdd(kp.stage + i, c.cnt[kp.n_slots + i]);
    } else {
      for (uint32_t i = threadIdx.x; i < 2u * kp.n_slots; i += blockDim.x)
        if (c.cnt[i]) atomicAdd(st + ISIM_ST_SITES + i, (unsigned long long)c.cnt[i]);
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

template <int K>
static void *pick(bool modeb, bool ldsc) {
  using namespace dev;
  if (ldsc) return modeb ? (void *)&isim_walk<K, true, true> : (void *)&isim_walk<K, false, true>;
  return modeb ? (void *)&isim_walk<K, true, false> : (void *)&isim_walk<K, false, false>;
}

void *walk_kernel(int kind, bool modeb, bool lds_counters) {
  switch (kind) {
    case 0: return pick<0>(modeb, lds_counters);
    case 1: return pick<1>(modeb, lds_counters);
    case 2: return pick<2>(modeb, lds_counters);
    case 3: return pick<3>(modeb, lds_counters);
    case 4: return pick<4>(modeb, lds_counters);
    case 5:  // the bit stack only exists in mode B
      if (!modeb) return pick<4>(false, lds_counters);
      return lds_counters ? (void *)&dev::isim_walk<5, true, true> : (void *)&dev::isim_walk<5, true, false>;
    case 8:  // sparse ancestor marking: mode B, position marks in LDS only
      if (!modeb) return pick<4>(false, lds_counters);
      return lds_counters ? (void *)&dev::isim_walk<8, true, true> : nullptr;
    default:  // 6: the close list only exists in mode B
      if (!modeb) return pick<4>(false, lds_counters);
      return lds_counters ? (void *)&dev::isim_walk<6, true, true> : (void *)&dev::isim_walk<6, true, false>;
  }
}

void *mark_fold_kernel() { return (void *)&dev::isim_mark_fold; }

void *stream_calls_kernel() { return (void *)&dev::isim_stream_calls; }
void *fill_const_kernel() { return (void *)&dev::isim_fill_const; }
uint32_t stream_traces_per_wave() { return 64u * (uint32_t)dev::kStreamTPL; }

}  // namespace isim
