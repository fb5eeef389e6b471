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
//     (sum for a sequential call, max inside a concurrent step).
#pragma once
#include <stdint.h>

#include "kernel_abi.h"

#if defined(__HIPCC__)
#define ISIM_TW __host__ __device__ __forceinline__
#else
#define ISIM_TW inline
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
#if defined(TW_UNROLL)
#pragma unroll
#endif
  for (int r = 0; r < 10; ++r) {
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

ISIM_TW uint32_t word4(uint32_t w, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const uint32_t lo = (w & 1u) ? b : a;
  const uint32_t hi = (w & 1u) ? d : c;
  return (w & 2u) ? hi : lo;
}

// Sink: call(slot) per executed call; resp(slot, row word, T, status) per
// response of a called invocation (the entry's is the trace result).
template <int FRAMES, bool MODEB>
struct Lane {
  uint32_t t_lo = 0, t_hi = 0;
  uint32_t p = 0, d = 0, end = 0, hopn = 0, errh = 0;
  bool done = true;
  uint32_t lat = 0;
  bool root500 = false;
  // current invocation
  uint32_t f_pos = 0, f_acc = 0, f_cmax = 0, f_hop = 0, f_fl = 0;
  // calling invocations below it
  uint32_t s_pos[FRAMES > 0 ? FRAMES : 1], s_acc[FRAMES > 0 ? FRAMES : 1], s_cmax[FRAMES > 0 ? FRAMES : 1],
      s_hop[FRAMES > 0 ? FRAMES : 1];
  // cached Philox blocks: skip draws (key: caller hop, block) and error draws (key: hop >> 2)
  uint32_t sk_hop = 0xFFFFFFFFu, sk_blk = 0, sk0 = 0, sk1 = 0, sk2 = 0, sk3 = 0;
  uint32_t ek_blk = 0xFFFFFFFFu, e0 = 0, e1 = 0, e2 = 0, e3 = 0;

  // k0, k1: the Philox key (wave-uniform: passed in, never stored per lane)
  ISIM_TW bool own_error(uint32_t hop, uint8_t flags, uint32_t thr, uint32_t k0, uint32_t k1) {
    if (flags & TF_ERR_ALWAYS) return true;
    if (!(flags & TF_ERR_DRAW)) return false;
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

  // Enters the entry invocation (hop 0).  A leaf entry responds at once.
  ISIM_TW void start(uint64_t trace, uint32_t key0, uint32_t key1, const TreeNode *nodes, const TreeExt *ext) {
    t_lo = (uint32_t)trace;
    t_hi = (uint32_t)(trace >> 32);
    done = false;
    hopn = 1;
    errh = 0;
    d = 0;
    sk_hop = 0xFFFFFFFFu;  // the Philox caches belong to the previous trace of the lane
    ek_blk = 0xFFFFFFFFu;
    const TreeNode n = nodes[0];
    const bool own = own_error(0, n.flags, n.thr, key0, key1);
    if (n.flags & TF_LEAF) {
      done = true;
      lat = ext[0].tc;
      root500 = own;
      errh = own ? 1u : 0u;
      return;
    }
    f_pos = 0;
    f_acc = 0;
    f_cmax = 0;
    f_hop = 0;
    f_fl = own ? FL_OWN : 0u;
    end = n.size;
    p = 1;
  }

  ISIM_TW void fold(uint32_t c, bool st, bool conc) {
    if (conc) {
      f_cmax = c > f_cmax ? c : f_cmax;
      if (MODEB && st) f_fl |= FL_CERR;
    } else {
      f_acc += c;
      if (MODEB && st) f_fl |= FL_FAILED;
    }
  }

  ISIM_TW void push() {
#pragma unroll
    for (int i = 0; i < FRAMES; ++i) {
      const bool m = d == (uint32_t)i;
      s_pos[i] = m ? (f_pos | (f_fl << 16)) : s_pos[i];
      s_acc[i] = m ? f_acc : s_acc[i];
      s_cmax[i] = m ? f_cmax : s_cmax[i];
      s_hop[i] = m ? f_hop : s_hop[i];
    }
    ++d;
  }

  ISIM_TW void pop() {
    --d;
    uint32_t a = 0, b = 0, c = 0, h = 0;
#pragma unroll
    for (int i = 0; i < FRAMES; ++i) {
      const bool m = d == (uint32_t)i;
      a = m ? s_pos[i] : a;
      b = m ? s_acc[i] : b;
      c = m ? s_cmax[i] : c;
      h = m ? s_hop[i] : h;
    }
    f_pos = a & 0xFFFFu;
    f_fl = a >> 16;
    f_acc = b;
    f_cmax = c;
    f_hop = h;
  }

  // One action: close the current invocation, or process position p.
  template <class Sink>
  ISIM_TW void step(const TreeNode *nodes, const TreeExt *ext, Sink &sink, uint32_t k0, uint32_t k1) {
#ifdef ISIM_TREE_DEBUG
    if (sink.bad(p, f_pos, d, FRAMES)) {
      done = true;
      return;
    }
#endif
    if (p >= end) {  // ---- close f_pos
      uint32_t T = f_acc, fl = f_fl;
      if (fl & FL_INCONC) {
        T += f_cmax;
        if (MODEB && (fl & FL_CERR)) fl |= FL_FAILED;
      }
      const TreeExt x = ext[f_pos];
      const bool failed = MODEB && (fl & FL_FAILED);
      if (!failed) T += x.tc;
      const bool st = failed || (fl & FL_OWN);
      errh += st ? 1u : 0u;
      if (f_pos == 0) {
        done = true;
        lat = T;
        root500 = st;
        return;
      }
      sink.resp(nodes[f_pos].slot, x.row, T, st);
      const uint32_t c = x.H + T;
      const bool cc = (fl & FL_CONC_CHILD) != 0;
      pop();
      end = f_pos + nodes[f_pos].size;
      fold(c, st, cc);
      return;
    }
    // ---- process the call at position p (a call command of f_pos's script)
    const TreeNode n = nodes[p];
    if (n.flags & TF_STEP) {
      if (f_fl & FL_INCONC) {
        f_acc += f_cmax;
        if (MODEB && (f_fl & FL_CERR)) f_fl |= FL_FAILED;
        f_fl &= ~(FL_INCONC | FL_CERR);
      }
      if (MODEB && (f_fl & FL_FAILED)) {  // the script stops: close at the subtree's end
        p = end;
        return;
      }
      f_acc += n.pre;
      if (n.flags & TF_CONC) {
        f_fl |= FL_INCONC;
        f_cmax = ext[p].cmax0;
      }
    }
    if (n.prob) {  // shouldSkipRequest: word (k & 3) of Philox((t, caller hop, 1 + k/4, 0)) % 100 < 100 - p
      const uint32_t blk = 1u + (n.k >> 2);
      if (sk_hop != f_hop || sk_blk != blk) {
        uint32_t a = t_lo, b = t_hi, c = f_hop, dd = blk;
        philox10(a, b, c, dd, k0, k1);
        sk0 = a;
        sk1 = b;
        sk2 = c;
        sk3 = dd;
        sk_hop = f_hop;
        sk_blk = blk;
      }
      if (word4(n.k & 3u, sk0, sk1, sk2, sk3) % 100u < 100u - n.prob) {
        p += n.size;
        return;
      }
    }
    const uint32_t hop = hopn++;
    const bool own = own_error(hop, n.flags, n.thr, k0, k1);
    sink.call(n.slot);
    if (n.flags & TF_LEAF) {
      const TreeExt x = ext[p];
      errh += own ? 1u : 0u;
      sink.resp(n.slot, x.row, x.tc, own);
      fold(x.H + x.tc, own, (n.flags & TF_CONC) != 0);
      p += 1;
      return;
    }
    push();
    f_pos = p;
    f_acc = 0;
    f_cmax = 0;
    f_hop = hop;
    f_fl = (own ? FL_OWN : 0u) | ((n.flags & TF_CONC) ? FL_CONC_CHILD : 0u);
    end = p + n.size;
    p += 1;
  }
};

}  // namespace tw
}  // namespace isim
