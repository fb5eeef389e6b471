// The lane tree walk: one request trace per lane over the unrolled tree of
// potential invocations (kernel_abi.h TreeNode/TreeExt, program.cpp
// build_tree).  Shared, line for line, by the HIP kernel (tree.hip, kernel
// kind 7) and the CPU check of the encoding (tests/cpp/tree_walk_check.cpp).
//
// Semantics: isim semantics v1 — isotope's Handler.ServeHTTP /
// execute recursion (isotope/service/pkg/srv/handler.go:37-79,
// executable.go:43-179) for one trace, in virtual integer-nanosecond time:
//   * positions are visited in preorder; a call whose probability draw skips
//     it (shouldSkipRequest, executable.go:84-90) jumps over its subtree, so
//     the executed invocations get consecutive hop ids in preorder;
//   * the current (innermost open) invocation is the frame f_*; the calling
//     invocations below it live in a register stack of FRAMES entries indexed
//     per lane (unrolled selects, no scratch);
//   * a call step begins at its first call (TF_STEP): the previous step, if
//     concurrent, ends (acc += cmax; mode B: a callee 500 fails the step);
//     in mode B a failed script runs no further step; the non-call time since
//     the previous call step is added;
//   * an invocation closes when the walk passes its subtree: the time after
//     its last call step is added (unless it failed), its status is its own
//     error draw (or its failure in mode B), and H + T folds into the caller
//     (sum for a sequential call, max inside a concurrent step);
//   * a call's skip draw comes from its caller's block of four residues,
//     drawn when the caller opens (Lane::step).
#pragma once
#include <stdint.h>

#include "kernel_abi.h"

#if defined(__HIPCC__)
#define ISIM_TW __host__ __device__ __forceinline__
#define TW_PRAGMA_UNROLL _Pragma("unroll")
#else
#define ISIM_TW inline
#define TW_PRAGMA_UNROLL
#endif

namespace isim {
namespace tw {

// frame flags
constexpr uint32_t FL_INCONC = 1;      // the current step of this invocation is concurrent
constexpr uint32_t FL_FAILED = 2;      // mode B: a step failed (no further step runs)
constexpr uint32_t FL_CERR = 4;        // mode B: a callee of the current concurrent step responded 500
constexpr uint32_t FL_OWN = 8;         // the invocation's own error draw erred
constexpr uint32_t FL_CONC_CHILD = 16; // the invocation was called from a concurrent step

ISIM_TW uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

// Philox4x32-10 (Random123), key (k0, k1).
ISIM_TW void philox10(uint32_t &c0, uint32_t &c1, uint32_t &c2, uint32_t &c3, uint32_t k0, uint32_t k1) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(TW_NO_ASM)
  asm volatile("" : "+s"(k0), "+s"(k1));  // keep the key schedule in two SGPRs
#endif
#if !defined(TW_NO_UNROLL)
TW_PRAGMA_UNROLL  // unrolled: config 4 7.28 -> 7.18 ms (the loop's SALU counter and branch per round)
#endif
#ifndef TW_ROUNDS
#define TW_ROUNDS 10  // timing experiments only: Philox4x32-10 is the semantics
#endif
  for (int r = 0; r < TW_ROUNDS; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1, k0);
    const uint32_t n2 = xor3((uint32_t)(p0 >> 32), c3, k1);
    c0 = n0;
    c1 = (uint32_t)p1;
    c2 = n2;
    c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// A TreeNode as ONE 8-byte load, fields unpacked by shifts (layout:
// kernel_abi.h).  The kernel reads nodes from LDS or global memory through
// an accessor with `NodeW load(uint32_t p) const` (tree.hip); the CPU check
// through CpuNodes.
struct NodeW {
  uint32_t w0, w1;  // size | k << 16, prob | flags << 8 | slot << 16
  static constexpr bool kDag = false;
  ISIM_TW uint32_t child() const { return 0; }
  ISIM_TW uint32_t size() const { return w0 & 0xFFFFu; }
  ISIM_TW uint32_t k() const { return w0 >> 16; }
  ISIM_TW uint32_t prob() const { return w1 & 0xFFu; }
  ISIM_TW uint32_t flags() const { return (w1 >> 8) & 0xFFu; }
  ISIM_TW uint32_t slot() const { return w1 >> 16; }
  ISIM_TW uint32_t site() const { return slot(); }  // what the sink counts the call under
};
static_assert(sizeof(TreeNode) == sizeof(NodeW), "TreeNode is two words");
struct CpuNodes {
  const TreeNode *p;
  ISIM_TW NodeW load(uint32_t i) const {
    NodeW n;
    __builtin_memcpy(&n, p + i, sizeof n);
    return n;
  }
};
// A wide tree's TreeNodeW (kernel_abi.h): the same accessors on 32-bit fields
constexpr uint32_t kSiteLds = 0x80000000u;
struct NodeW4 {
  uint32_t sz, kk, pf, sl;  // size, k, prob | flags << 8 | LDS counter << 16, slot
  static constexpr bool kDag = false;
  ISIM_TW uint32_t child() const { return 0; }
  ISIM_TW uint32_t size() const { return sz; }
  ISIM_TW uint32_t k() const { return kk; }
  ISIM_TW uint32_t prob() const { return pf & 0xFFu; }
  ISIM_TW uint32_t flags() const { return (pf >> 8) & 0xFFu; }
  ISIM_TW uint32_t slot() const { return sl; }
  // a hot site's LDS counter | kSiteLds, else the slot (global atomics)
  ISIM_TW uint32_t site() const { return (pf >> 16) != 0xFFFFu ? kSiteLds | (pf >> 16) : sl; }
};
static_assert(sizeof(TreeNodeW) == sizeof(NodeW4), "TreeNodeW is four words");
struct CpuNodesW {
  const TreeNodeW *p;
  ISIM_TW NodeW4 load(uint32_t i) const {
    NodeW4 n;
    __builtin_memcpy(&n, p + i, sizeof n);
    return n;
  }
};
// The site graph (round 6, Program::tree_dag): when the unrolled tree of a
// DAG would exceed kTreeMaxWidePositions (shared callees multiply the
// potential invocations), the walk runs over ONE node per reachable call site
// instead — each service's sites contiguous in script order, node 0 the entry
// — with the same 16-byte TreeNodeW: size = the callee's first site node,
// k = call index | the callee's site count << 16.  A skipped call then
// advances by one node (not over a subtree), an open enters the callee's
// site range, and a close resumes the caller after the closing invocation's
// own site: the same preorder, hop ids and draws as the unrolled tree.
struct NodeD4 {
  uint32_t ch, kk, pf, sl;  // callee's first site node, k | callee's sites << 16, prob | flags | LDS counter, slot
  static constexpr bool kDag = true;
  ISIM_TW uint32_t child() const { return ch; }
  ISIM_TW uint32_t size() const { return kk >> 16; }  // the callee's sites (the children of the opened node)
  ISIM_TW uint32_t k() const { return kk & 0xFFFFu; }
  ISIM_TW uint32_t prob() const { return pf & 0xFFu; }
  ISIM_TW uint32_t flags() const { return (pf >> 8) & 0xFFu; }
  ISIM_TW uint32_t slot() const { return sl; }
  ISIM_TW uint32_t site() const { return (pf >> 16) != 0xFFFFu ? kSiteLds | (pf >> 16) : sl; }
};
static_assert(sizeof(TreeNodeW) == sizeof(NodeD4), "a site-graph node is a TreeNodeW");
struct CpuNodesD {
  const TreeNodeW *p;
  ISIM_TW NodeD4 load(uint32_t i) const {
    NodeD4 n;
    __builtin_memcpy(&n, p + i, sizeof n);
    return n;
  }
};
// the positions a skipped call passes: its subtree, or (site graph) its own node
template <class N>
ISIM_TW uint32_t skip_span(const N &n) {
  return N::kDag ? 1u : n.size();
}
template <class N>
struct dag_of {
  static constexpr bool value = N::kDag;
};
template <class N>
struct dag_of<const N> : dag_of<N> {};

ISIM_TW TreeExt load_ext(const TreeExt *ext, uint32_t p) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint4 v = reinterpret_cast<const uint4 *>(ext)[p];
  return TreeExt{v.x, v.y, v.z, v.w};
#else
  return ext[p];
#endif
}

ISIM_TW uint32_t word4(uint32_t w, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const uint32_t lo = (w & 1u) ? b : a;
  const uint32_t hi = (w & 1u) ? d : c;
  return (w & 2u) ? hi : lo;
}

constexpr uint32_t KB_SHIFT = 5;  // f_fl bits 5-15: the call block whose skip residues f_res holds
constexpr uint32_t KB_NONE = 0x7FFu;
#ifndef TW_SCAN
#define TW_SCAN 3
#endif
constexpr int kScan = TW_SCAN;    // skipped calls a step may pass after its action (tree.hip: uniform trips)
// the scan budget of a walk: kScan, or its node accessor's kScan (tree.hip:
// nodes read from HBM pass 2 — each scan is a dependent global load: c3p
// 22.7 -> 22.2 ms, c3s 21.7 -> 21.2, c4w 18.0 -> 18.0; nodes in LDS pass 3:
// config 4 runs 5.05 ms with 3, 5.68 with 2)
template <class N, class = void>
struct scan_of {
  static constexpr int value = kScan;
};
template <class N>
struct scan_of<N, decltype((void)N::kScan)> {
  static constexpr int value = N::kScan;
};

// The four skip draws of a Philox block reduced to what shouldSkipRequest
// compares (word % 100, 7 bits each): skip call k iff residue(k & 3) < 100 - p.
ISIM_TW uint32_t pack_res(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return (a % 100u) | (b % 100u) << 7 | (c % 100u) << 14 | (d % 100u) << 21;
}

// Sink: call(slot) per executed call; resp_leaf(slot, status) per response
// of a leaf callee (its duration is static); resp(slot, row word, T,
// status) per response of a calling callee (the entry's is the trace result);
// optionally exec(position, hop, caller hop, own error) per executed
// invocation, entry included (caller hop kNoCaller), and then dur(hop, T,
// status) per response of a callee (its duration without contention and its
// status: the own error, or in mode B a failed step) — the DES item engine's
// pre-walk (des_items.hip) records the executed invocations with them.
constexpr uint32_t kNoCaller = 0xFFFFFFFFu;
template <class S, class = void>
struct has_exec {
  static constexpr bool value = false;
};
template <class S>
struct has_exec<S, decltype((void)&S::exec)> {
  static constexpr bool value = true;
};
// or (a sink with kCloseRec) ONE rec_close(position, hop, caller hop,
// duration, status) per executed invocation when it closes — a leaf at its
// visit, the entry with duration 0 — so a record is written once, whole
template <class S, class = void>
struct close_rec {
  static constexpr bool value = false;
};
template <class S>
struct close_rec<S, decltype((void)S::kCloseRec)> {
  static constexpr bool value = S::kCloseRec;
};
//
// One step() is a MACRO step: process position p (a call: skip it, run a leaf
// callee, or open a calling callee), then pass up to kScan further calls whose
// skip draw says skip, then close the current invocation if the walk has
// passed its subtree.  A wave runs its 64 lanes' steps in lock step, so
// fewer, fuller steps per trace are what count (config 4: 25.9 -> 11.1
// wave iterations per 64 traces) — but so does what a step costs: until
// round 6 a step also closed FIRST when the previous one left the walk past
// its subtree (a chain of subtrees ending together), and that second close
// site, which some lane of a wave needs in ~96 % of its steps, cost more than
// the steps it saved (c4 5.57 -> 5.05 ms per 2^26 traces with 8.3 -> 9.2
// wave steps per 64 traces; c3p 25.2 -> 22.7 ms with 289 -> 305: DESIGN.md
// §5 round 6, tools/wave_sim.py).  The skip residues of an invocation are
// drawn once, when it opens, and kept in its frame (f_res), so returning from
// a callee never recomputes the caller's block and the scans need no draw.
// CONC: the walk has concurrent steps (without them no frame keeps a step max).
// SPILL: the FRAMES register frames are a ring over the top of the stack; the
// calling invocations below it are kept in memory at sp[(level *
// kTreeSpillWords + word) * sp_stride] (the kernel: global memory, one column
// per lane; the CPU check: a vector).
// DRAW: some callee draws its error against a threshold (without, no error
// block is cached: 5 registers fewer).
// TT: the time type — uint32_t when the walk's latency bound is below 2^32
// ns, else uint64_t (round 5: a sequential 10k-service tree's bound is ~30 s;
// every position's own H, tc and step facts still fit 32 bits, program.cpp)
// W: a wide tree (kernel_abi.h TreeNodeW): positions and hop ids take 32 bits,
// so a frame keeps its position and end, and its hop and flags, in separate
// words (two more registers per frame; the nodes come as NodeW4)
template <int FRAMES, bool MODEB, bool CONC = true, bool SPILL = false, bool DRAW = true, typename TT = uint32_t,
          bool W = false>
struct Lane {
  // u32 words of a spilled frame: pos|end, hop|flags, residues, time, step max (+ end, hop when wide)
  static constexpr uint32_t kSW0 = sizeof(TT) == 8 ? kTreeSpillWords64 : kTreeSpillWords;
  static constexpr uint32_t kSW = kSW0 + (W ? kTreeSpillWide : 0u);
  static constexpr uint32_t kWF = W && FRAMES > 0 ? FRAMES : 1;
  uint32_t t_lo = 0, t_hi = 0;
  uint32_t p = 0, d = 0, end = 0;
  uint32_t he = 0;  // executed invocations (hop ids handed out) | invocations that responded 500 << 16
  uint32_t he_err = 0;  // W: the 500s (he counts the hops alone)
  bool done = true;
  TT lat = 0;
  bool root500 = false;
  // current invocation: f_hf = hop | fl << 16 (fl: FL_* | call block of f_res << KB_SHIFT), packed
  // as its frame is (one register fewer; HF() shifts a flag into place); W: f_hf = fl, hop in f_hop
  uint32_t f_pos = 0, f_hf = 0, f_res = 0, f_hop = 0;
  TT f_acc = 0, f_cmax = 0;
  static constexpr uint32_t kHFS = W ? 0u : 16u;
  static constexpr uint32_t HF(uint32_t fl) { return fl << kHFS; }
  ISIM_TW uint32_t hops() const { return W ? he : he & 0xFFFFu; }
  ISIM_TW uint32_t errs() const { return W ? he_err : he >> 16; }
  ISIM_TW void add_err(bool e) {
    if (W) he_err += e ? 1u : 0u;
    else he += e ? 0x10000u : 0u;
  }
  ISIM_TW uint32_t cur_hop() const { return W ? f_hop : f_hf & 0xFFFFu; }
  ISIM_TW uint32_t f_kb() const { return (f_hf >> (kHFS + KB_SHIFT)) & KB_NONE; }
  ISIM_TW void set_kb(uint32_t kb) { f_hf = (f_hf & ~HF(KB_NONE << KB_SHIFT)) | HF(kb << KB_SHIFT); }
  // calling invocations below it: pos | end << 16, hop | fl << 16, residues, time (W: + end, hop)
  uint32_t s_pe[FRAMES > 0 ? FRAMES : 1], s_hf[FRAMES > 0 ? FRAMES : 1], s_res[FRAMES > 0 ? FRAMES : 1];
  uint32_t s_end[kWF], s_hop[kWF];
  TT s_acc[FRAMES > 0 ? FRAMES : 1], s_cmax[CONC && FRAMES > 0 ? FRAMES : 1];
  uint32_t *sp = nullptr;  // SPILL: this lane's column of the spill area
  uint32_t sp_stride = 1;
  // cached error block: words of Philox (t, ek_blk, 0, 0)
  uint32_t ek_blk = 0xFFFFFFFFu, e0 = 0, e1 = 0, e2 = 0, e3 = 0;

  // k0, k1: the Philox key (wave-uniform: passed in, never stored per lane)
  ISIM_TW bool own_error(uint32_t hop, uint32_t flags, uint32_t thr, uint32_t k0, uint32_t k1) {
    if (flags & TF_ERR_ALWAYS) return true;
    if (!DRAW || !(flags & TF_ERR_DRAW)) return false;
    const uint32_t b = hop >> 2;
    if (b != ek_blk) {
      uint32_t a = t_lo, bb = t_hi, c = b, dd = 0;
      philox10(a, bb, c, dd, k0, k1);
      e0 = a;
      e1 = bb;
      e2 = c;
      e3 = dd;
      ek_blk = b;
    }
    return word4(hop & 3u, e0, e1, e2, e3) < thr;
  }

  // skip residues of call block kb of the invocation with hop id `hop`
  ISIM_TW uint32_t residues(uint32_t hop, uint32_t kb, uint32_t k0, uint32_t k1) const {
    uint32_t a = t_lo, b = t_hi, c = hop, dd = 1u + kb;
    philox10(a, b, c, dd, k0, k1);
    return pack_res(a, b, c, dd);
  }

  // Starts a trace: the entry invocation (position 0, hop 0) opens in the
  // first step, through the same code as every other open (one Philox site
  // for skip residues per step, shared by the lanes that open and the lanes
  // that start).
  ISIM_TW void start(uint64_t trace) {
    t_lo = (uint32_t)trace;
    t_hi = (uint32_t)(trace >> 32);
    done = false;
    he = 0;
    he_err = 0;
    d = 0;
    lo = 0;
    hs = 0;
    ek_blk = 0xFFFFFFFFu;  // the error block belongs to the previous trace of the lane
    p = 0;
    end = 1;
    f_hf = 0;
  }

  ISIM_TW void fold(TT c, bool st, bool conc) {
    if (CONC && conc) {
      f_cmax = c > f_cmax ? c : f_cmax;
      if (MODEB && st) f_hf |= HF(FL_CERR);
    } else {
      f_acc += c;
      if (MODEB && st) f_hf |= HF(FL_FAILED);
    }
  }

  // SPILL (round 6): the register frames are a ring holding the TOP of the
  // stack — frames [lo, d) in slots (hs - (d - lo)) .. hs - 1 mod FRAMES —
  // and only frames below lo live in memory, at level = frame index.  A push
  // onto a full ring evicts its oldest frame (frame lo, in the slot the new
  // frame takes); a pop from an empty ring reads its frame from memory.  A walk
  // that moves up and down within FRAMES levels (the deep subtrees, where most
  // calling invocations are) touches no memory; the old layout (frames below
  // FRAMES in registers, every deeper push and pop in memory) paid a frame's
  // write and read for each of them.
  uint32_t lo = 0, hs = 0;
  ISIM_TW void ring_put(uint32_t slot, uint32_t pe, uint32_t hf, uint32_t res, TT acc, TT cmax, uint32_t en,
                        uint32_t hp) {
TW_PRAGMA_UNROLL
    for (int i = 0; i < FRAMES; ++i) {
      const bool m = slot == (uint32_t)i;
      s_pe[i] = m ? pe : s_pe[i];
      s_hf[i] = m ? hf : s_hf[i];
      s_res[i] = m ? res : s_res[i];
      s_acc[i] = m ? acc : s_acc[i];
      if (CONC) s_cmax[i] = m ? cmax : s_cmax[i];
      if (W) {
        s_end[i] = m ? en : s_end[i];
        s_hop[i] = m ? hp : s_hop[i];
      }
    }
  }
  ISIM_TW void ring_get(uint32_t slot, uint32_t &pe, uint32_t &hf, uint32_t &r, TT &a, TT &c, uint32_t &en,
                        uint32_t &hp) const {
TW_PRAGMA_UNROLL
    for (int i = 0; i < FRAMES; ++i) {
      const bool m = slot == (uint32_t)i;
      pe = m ? s_pe[i] : pe;
      hf = m ? s_hf[i] : hf;
      r = m ? s_res[i] : r;
      a = m ? s_acc[i] : a;
      if (CONC) c = m ? s_cmax[i] : c;
      if (W) {
        en = m ? s_end[i] : en;
        hp = m ? s_hop[i] : hp;
      }
    }
  }
  ISIM_TW void mem_put(uint32_t level, uint32_t pe, uint32_t hf, uint32_t res, TT acc, TT cmax, uint32_t en,
                       uint32_t hp) {
    uint32_t *q = sp + level * kSW * sp_stride;
    q[0] = pe;
    q[sp_stride] = hf;
    q[2 * sp_stride] = res;
    q[3 * sp_stride] = (uint32_t)acc;
    q[4 * sp_stride] = (uint32_t)cmax;
    if constexpr (sizeof(TT) == 8) {
      q[5 * sp_stride] = (uint32_t)((uint64_t)acc >> 32);
      q[6 * sp_stride] = (uint32_t)((uint64_t)cmax >> 32);
    }
    if constexpr (W) {
      q[kSW0 * sp_stride] = en;
      q[(kSW0 + 1) * sp_stride] = hp;
    }
  }
  ISIM_TW void mem_get(uint32_t level, uint32_t &pe, uint32_t &hf, uint32_t &r, TT &a, TT &c, uint32_t &en,
                       uint32_t &hp) const {
    const uint32_t *q = sp + level * kSW * sp_stride;
    pe = q[0];
    hf = q[sp_stride];
    r = q[2 * sp_stride];
    a = q[3 * sp_stride];
    c = q[4 * sp_stride];
    if constexpr (sizeof(TT) == 8) {
      a |= (TT)((uint64_t)q[5 * sp_stride] << 32);
      c |= (TT)((uint64_t)q[6 * sp_stride] << 32);
    }
    if constexpr (W) {
      en = q[kSW0 * sp_stride];
      hp = q[(kSW0 + 1) * sp_stride];
    }
  }

  ISIM_TW void push() {
    const uint32_t pe = W ? f_pos : f_pos | (end << 16), hf = f_hf;
    if constexpr (SPILL) {
      if (d - lo == (uint32_t)FRAMES) {  // a full ring: its oldest frame (in slot hs) to memory
        uint32_t ope = 0, ohf = 0, ores = 0, oen = 0, ohp = 0;
        TT oacc = 0, ocm = 0;
        ring_get(hs, ope, ohf, ores, oacc, ocm, oen, ohp);
        mem_put(lo, ope, ohf, ores, oacc, ocm, oen, ohp);
        ++lo;
      }
      ring_put(hs, pe, hf, f_res, f_acc, f_cmax, end, f_hop);
      hs = hs + 1u == (uint32_t)FRAMES ? 0u : hs + 1u;
    } else {
      ring_put(d, pe, hf, f_res, f_acc, f_cmax, end, f_hop);
    }
    ++d;
  }

  ISIM_TW void pop() {
    --d;
    uint32_t pe = 0, hf = 0, r = 0, en = 0, hp = 0;
    TT a = 0, c = 0;
    if constexpr (SPILL) {
      if (d >= lo) {
        hs = hs == 0u ? (uint32_t)FRAMES - 1u : hs - 1u;
        ring_get(hs, pe, hf, r, a, c, en, hp);
      } else {  // an empty ring: the frame from memory
        mem_get(d, pe, hf, r, a, c, en, hp);
        lo = d;
      }
    } else {
      ring_get(d, pe, hf, r, a, c, en, hp);
    }
    if constexpr (W) {
      f_pos = pe;
      end = en;
      f_hop = hp;
    } else {
      f_pos = pe & 0xFFFFu;
      end = pe >> 16;
    }
    f_hf = hf;
    f_res = r;
    f_acc = a;
    f_cmax = c;
  }

  // The step begin of call position p (TF_STEP: the previous concurrent step
  // ends, the non-call time since the previous call step is added — mode B
  // only, TF_XPRE: mode A folds it into the caller's tc —, a concurrent step
  // starts) on copies of the frame's time and flags; returns false when the
  // script has failed (mode B: it runs no further step).
  template <class N>
  ISIM_TW bool step_begin(const N &n, const TreeStep *stp, TT &acc, uint32_t &fl, TT &cm) const {
    if (!(n.flags() & TF_STEP)) return true;
    if (CONC && (fl & HF(FL_INCONC))) {
      acc += cm;
      if (MODEB && (fl & HF(FL_CERR))) fl |= HF(FL_FAILED);
      fl &= ~HF(FL_INCONC | FL_CERR);
    }
    if (MODEB && (fl & HF(FL_FAILED))) return false;
    if (n.flags() & (TF_XPRE | TF_XCMAX)) {
      const TreeStep x = stp[p];
      if (MODEB) acc += x.pre;  // TF_XPRE is never set in mode A (pre is 0 here then)
      cm = x.cmax0;
    } else {
      cm = 0;
    }
    if (CONC && (n.flags() & TF_CONC)) fl |= HF(FL_INCONC);
    return true;
  }

  // the skip draw of call n (its block's residues are in f_res)
  template <class N>
  ISIM_TW bool skipped(const N &n) const {
    return ((f_res >> (7u * (n.k() & 3u))) & 0x7Fu) < 100u - n.prob();
  }

  // close f_pos: its response folds into its caller (false: the entry responded)
  template <class Nodes, class Sink>
  ISIM_TW bool close(const Nodes &nodes, const TreeExt *ext, Sink &sink) {
    TT T = f_acc;
    uint32_t fl = f_hf;
    if (CONC && (fl & HF(FL_INCONC))) {
      T += f_cmax;
      if (MODEB && (fl & HF(FL_CERR))) fl |= HF(FL_FAILED);
    }
    const TreeExt x = load_ext(ext, f_pos);
    const bool failed = MODEB && (fl & HF(FL_FAILED));
    if (!failed) T += x.tc;
    const bool st = failed || (fl & HF(FL_OWN));
    add_err(st);
    if (f_pos == 0) {
      done = true;
      lat = T;
      root500 = st;
      if constexpr (close_rec<Sink>::value) sink.rec_close(0u, cur_hop(), kNoCaller, (TT)0, st);
      return false;
    }
    sink.resp(nodes.load(f_pos).site(), x.row, T, st);
    if constexpr (has_exec<Sink>::value) sink.dur(cur_hop(), T, st);
    const TT c = (TT)x.H + T;
    const bool cc = (fl & HF(FL_CONC_CHILD)) != 0;
    const uint32_t cpos = f_pos, chop = cur_hop();
    if constexpr (dag_of<decltype(nodes.load(0))>::value) p = cpos + 1u;  // the caller's next site
    pop();
    if constexpr (close_rec<Sink>::value) sink.rec_close(cpos, chop, cur_hop(), T, st);
    fold(c, st, cc);
    return true;
  }

  // process call position p (p < end)
  template <class Nodes, class Sink>
  ISIM_TW void process(const Nodes &nodes, const TreeExt *ext, const TreeStep *stp, Sink &sink, uint32_t k0,
                       uint32_t k1) {
    const auto n = nodes.load(p);
    if (!step_begin(n, stp, f_acc, f_hf, f_cmax)) {  // mode B: the script stops, close at the subtree's end
      p = end;
      return;
    }
    if (n.prob()) {  // shouldSkipRequest: word (k & 3) of Philox((t, caller hop, 1 + k/4, 0)) % 100 < 100 - p
      const uint32_t kb = (uint32_t)n.k() >> 2;
      if (f_kb() != kb) {  // a call block past the first four calls
        f_res = residues(cur_hop(), kb, k0, k1);
        set_kb(kb);
      }
      if (skipped(n)) {
        p += skip_span(n);
        return;
      }
    }
    const uint32_t hop = hops();
    he += 1u;
    const uint32_t fl = n.flags();
    const bool entry = p == 0;  // the trace's first step: the entry (no call site, no caller)
    if (!entry) sink.call(n.site());
    if (fl & TF_LEAF) {
      const TreeExt x = load_ext(ext, p);
      const bool own = own_error(hop, fl, x.thr, k0, k1);
      add_err(own);
      if constexpr (has_exec<Sink>::value) sink.exec(p, hop, entry ? kNoCaller : cur_hop(), own);
      if constexpr (close_rec<Sink>::value)
        sink.rec_close(p, hop, entry ? kNoCaller : cur_hop(), entry ? (TT)0 : (TT)x.tc, own);
      if (entry) {
        done = true;
        lat = x.tc;
        root500 = own;
        return;
      }
      sink.resp_leaf(n.site(), own);
      if constexpr (has_exec<Sink>::value) sink.dur(hop, x.tc, own);
      fold((TT)x.H + x.tc, own, (fl & TF_CONC) != 0);
      p += 1;
      return;
    }
    const bool own =
        (DRAW && (fl & TF_ERR_DRAW)) ? own_error(hop, fl, load_ext(ext, p).thr, k0, k1) : (fl & TF_ERR_ALWAYS) != 0;
    if constexpr (has_exec<Sink>::value) sink.exec(p, hop, entry ? kNoCaller : cur_hop(), own);
    if (!entry) push();
    f_pos = p;
    f_acc = 0;
    f_cmax = 0;
    const bool pk = (fl & TF_PROBK0) != 0;
    f_res = pk ? residues(hop, 0, k0, k1) : 0u;
    f_hf = (W ? 0u : hop) | HF((own ? FL_OWN : 0u) | ((fl & TF_CONC) ? FL_CONC_CHILD : 0u) | ((pk ? 0u : KB_NONE) << KB_SHIFT));
    if (W) f_hop = hop;
    if constexpr (dag_of<decltype(n)>::value) {  // the callee's site range
      p = n.child();
      end = p + n.size();
    } else {
      end = p + n.size();
      p += 1;
    }
  }

  // pass call position p if its skip draw (already in f_res) says skip
  template <class Nodes>
  ISIM_TW bool scan(const Nodes &nodes, const TreeStep *stp) {
    const auto n = nodes.load(p);
    if (!n.prob() || f_kb() != ((uint32_t)n.k() >> 2) || !skipped(n)) return false;
    TT acc = f_acc, cm = f_cmax;
    uint32_t fl = f_hf;
    if (!step_begin(n, stp, acc, fl, cm)) return false;
    f_acc = acc;
    f_hf = fl;
    f_cmax = cm;
    p += skip_span(n);
    return true;
  }

  // One macro step (see above).
  template <class Nodes, class Sink>
  ISIM_TW void step(const Nodes &nodes, const TreeExt *ext, const TreeStep *stp, Sink &sink, uint32_t k0,
                    uint32_t k1) {
#ifdef ISIM_TREE_DEBUG
    if (sink.bad(p, f_pos, d, SPILL ? (int)kTreeMaxFrames : FRAMES)) {
      done = true;
      return;
    }
#endif
    if (p < end) process(nodes, ext, stp, sink, k0, k1);  // (else the walk closes at the end of the step)
    bool go = !done;
TW_PRAGMA_UNROLL
    for (int i = 0; i < scan_of<Nodes>::value; ++i) {
      go = go && p < end && scan(nodes, stp);
    }
    // and close the invocation if the walk has passed its subtree (the step's
    // one close site; round 4 added it here, after the scans: config 4 12.5 ->
    // 10.4 wave iterations per 64 traces, 7.18 -> 7.03 ms per 2^26 traces)
    if (!done && p >= end) close(nodes, ext, sink);
  }
};

}  // namespace tw
}  // namespace isim
