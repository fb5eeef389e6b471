// Shared between the host program compiler and the HIP walk kernel: the
// device instruction format and the kernel argument block.
#pragma once
#include <stdint.h>

#include "../../include/isim.h"

namespace isim {

enum Op : uint32_t {
  OP_HALT = 0,
  OP_SLEEP = 1,   // acc += d
  OP_CBEGIN = 2,  // cmax = 0, cerr = 0
  OP_CSLEEP = 3,  // cmax = max(cmax, d)
  OP_CEND = 4,    // acc += cmax; mode B: failed |= cerr
  OP_CALL = 5,    // invoke a service with a script that makes calls
  OP_LEAF = 6,    // invoke a service whose script makes no calls
  OP_RET = 7,     // end of a service body (respond)
};

enum Flag : uint32_t {
  F_CONC = 1,        // the call is a sub-command of a concurrent step
  F_PROB = 2,        // probability 1..99: draw to skip
  F_ERR_ALWAYS = 4,  // callee errorRate == 1
  F_ERR_DRAW = 8,    // 0 < callee errorRate < 1: draw against thr
  F_ROOT = 16,       // the client request into the entry (no call site)
};

// 32-byte instruction, read by the kernel with one scalar load.
struct Ins {
  uint32_t opf;   // op | flags << 8 | probability << 16
  uint32_t k;     // CALL/LEAF: index of the call command in the caller's script
  uint32_t thr;   // CALL/LEAF: callee error threshold (F_ERR_DRAW)
  uint32_t slot;  // CALL/LEAF: stats slot of the call site
  uint32_t a_lo, a_hi;  // CALL/LEAF: hop cost H; SLEEP/CSLEEP: duration
  uint32_t b_lo, b_hi;  // CALL: target pc (b_lo); LEAF: callee latency
};
static_assert(sizeof(Ins) == 32, "Ins must be 32 bytes");

// STATIC walks also compile to a draw stream: one record per invocation in
// hop (DFS preorder) order.  meta = slot (bits 0-23) | closes (24-30) | always (31).
struct Node {
  uint32_t thr;   // error threshold over the u32 draw (0: never)
  uint32_t meta;
};
static_assert(sizeof(Node) == 8, "Node must be 8 bytes");
constexpr uint32_t kSlotRoot = 0xFFFFFFu;  // the entry invocation (no call site)
constexpr uint32_t kSlotPad = 0xFFFFFEu;   // padding to a multiple of 4 records
constexpr uint32_t kMaxStreamNodes = 1u << 24;

// Mode B on the draw stream (kernel kind 6): the closes of calling
// invocations (subtrees with children, the entry excepted), in close order.
// The stream is walked in chunks of kChunkRecords records; per chunk a lane
// keeps the error bits of its records (record r of a chunk of n records at
// bit n-1-r) and, from earlier chunks, the position + 1 of its last erring
// record.  The invocation at stream position p whose subtree ends at record j
// responds 500 iff an invocation in [p, j] erred:
//   (bits & rmask) != 0  ||  last_err1 >= pre1
// rmask = the chunk bits of records [max(p, chunk start), j]; pre1 = p + 1
// when p lies before the chunk, else 0xFFFFFFFF (the test is never true).
struct StreamClose {
  uint32_t pre1;
  uint32_t rmask;
};
static_assert(sizeof(StreamClose) == 8, "StreamClose must be 8 bytes");
constexpr uint32_t kClosePad = 16;  // zero StreamClose records after the list (block prefetch)

// Mode B on the draw stream by sparse ancestor marking (kernel kind 8, the
// default): an invocation responds 500 iff an invocation of its subtree drew
// an error, i.e. the 500s of a trace are the union of the root paths of its
// erring invocations.  With e_1 < e_2 < ... the erring records (preorder),
// that union is counted per position by +1 at every e_i and -1 at
// LCA(e_{i-1}, e_i): the subtree sum of those marks at v is 1 iff v responded
// 500 (summed over traces: v's 500 count; linear, so all traces share one
// per-position table).  For preorder records u < w, LCA(u, w) is the parent of
// the shallowest record in (u, w], so a lane only keeps, per trace, the
// minimum of the records' keys since its last error; at an error that minimum
// names the LCA and its depth, and the trace's new 500s are
// depth(e_i) - depth(LCA).  Stream record (same 8-byte shape as Node):
// thr, and key = always (31) | depth (24-30) | parent record (0-23); the
// entry's parent is the sentinel record n (a counter nobody reads); padding
// records have key kMarkPadKey (above every real key).  A per-launch fold
// (isim_mark_fold) turns the position marks into subtree sums and adds them
// to the per-site 500 counters.
constexpr uint32_t kMarkPadKey = 0x7FFFFFFFu;
constexpr uint32_t kMarkKeyMask = 0x7FFFFFFFu;  // key without the always bit
constexpr uint32_t kMarkPosMask = 0xFFFFFFu;
constexpr uint32_t kChunkGroups = 8;                  // Philox groups (4 records) per chunk
constexpr uint32_t kChunkRecords = 4 * kChunkGroups;  // 32: one bit per record per lane

// Per-service duration table word: row (bits 0-23) | bucket of a leaf callee (24-31).
constexpr uint32_t kDurRowMask = 0xFFFFFFu;

// DYNAMIC walks on the lane tree walk (kernel kind 7, tree_walk.h): the
// invocation tree unrolled over every POTENTIAL invocation (each reachable
// call command, probabilistic or not) in preorder; a trace walks it on its
// own lane, skipping the subtree of a call its draw skips.  Position 0 is the
// entry.  What every visit of a position needs (TreeNode, 8 B) lives in LDS
// when it fits, else is read from global memory (L2-resident); what an
// executed position needs (TreeExt, 16 B) and the rare step facts (TreeStep)
// are read from global memory.
enum TreeFlag : uint8_t {
  TF_STEP = 1,        // first call of its step in the caller's script (the step begins here)
  TF_CONC = 2,        // the step is concurrent
  TF_LEAF = 4,        // the callee makes no calls
  TF_ERR_ALWAYS = 8,  // callee errorRate 1
  TF_ERR_DRAW = 16,   // 0 < callee errorRate < 1: draw against TreeExt.thr
  TF_PROBK0 = 32,     // the callee's script has a probabilistic call among its first 4 calls (its skip
                      // residues, Philox block (t, hop, 1, 0), are drawn when it opens)
  TF_XPRE = 64,       // TF_STEP: the step begin adds TreeStep.pre (mode B; mode A folds every step's pre
                      // into the caller's TreeExt.tc: without aborts every step runs)
  TF_XCMAX = 128,     // TF_STEP|TF_CONC: the concurrent step starts at TreeStep.cmax0 (its longest sleep)
};
// Program.tree_flags / KParams.tree_flags: what the walk contains
constexpr uint32_t kTreeAnyProb = 1;  // some position is a probabilistic call
constexpr uint32_t kTreeAnyDraw = 2;  // some position draws its error against a threshold
constexpr uint32_t kTreeAnyConc = 4;  // some call step is concurrent
constexpr uint32_t kTreeMaxCalls = 4 * 2047;  // calls per script: the skip-block index fits 11 flag bits
struct TreeNode {
  uint16_t size;   // positions in the subtree (itself included): a skipped call jumps over them
  uint16_t k;      // index of the call command in the caller's script (skip-draw block and word)
  uint8_t prob;    // 1..99: draw to skip; 0: always called
  uint8_t flags;   // TF_*
  uint16_t slot;   // stats slot of the call site
};
static_assert(sizeof(TreeNode) == 8, "TreeNode must be 8 bytes");
// WIDE trees (round 5): more than 65,535 potential invocations, call sites
// or rows, or per-slot counters that do not fit in LDS — 32-bit sizes and
// slots (16 B per position, read from global memory), every statistic by
// global atomics (tree.hip WideSink), the row index whole in TreeExt.row
struct TreeNodeW {
  uint32_t size;   // positions in the subtree (itself included)
  uint32_t k;      // index of the call command in the caller's script
  uint8_t prob;    // 1..99: draw to skip; 0: always called
  uint8_t flags;   // TF_*
  uint16_t lidx;   // the call site's LDS counter (0xFFFF: global atomics; program.cpp: the hottest sites)
  uint32_t slot;   // stats slot of the call site
};
static_assert(sizeof(TreeNodeW) == 16, "TreeNodeW must be 16 bytes");
struct TreeExt {
  uint32_t H;      // hop cost of the call
  uint32_t tc;     // leaf callee: its latency; else the time after its last call step (mode A: + the
                   // pre of every call step of its script)
  uint32_t row;    // non-leaf callee: index (bits 0-15) | placement (bits 16-31): the LDS word offset of
                   // the row's bucket table, kTreeStaticRow, kTreeGlobalDyn or kTreeGlobalStatic
  uint32_t thr;    // callee error threshold (TF_ERR_DRAW)
};
static_assert(sizeof(TreeExt) == 16, "TreeExt must be 16 bytes");
struct TreeStep {
  uint32_t pre;    // TF_XPRE: time the caller spends between its previous call step and this step
  uint32_t cmax0;  // TF_XCMAX: the longest sleep sub-command of the concurrent step
};
static_assert(sizeof(TreeStep) == 8, "TreeStep must be 8 bytes");
// Placement of a non-leaf callee's duration row (TreeExt.row bits 16-31).  In
// LDS (a sum index in bits 0-15): its code-200 duration sum, and when its
// bucket varies (prom_bucket(tmin) < prom_bucket(tmax)) a bucket table of the
// workgroup: a header word (b_lo | width << 8), then the counts.  Wide rows:
// a u64 sum, [code 200|500][width] u32 counts.  Compact rows (TreeLayout
// compact, when the wide ones do not all fit): a u32 sum (a wrap carries 2^32
// to the row in HBM), the code-200 counts as u16 pairs (ceil(width / 2)
// words; a field reaching 2^15 moves 2^15 to HBM), code-500 buckets and sums
// (errorRate-rare) by global atomics.  Flushed once per workgroup.  In global memory (the duration-table
// row in bits 0-15; rows the LDS budget does not hold, coldest first): sums,
// and buckets when they vary, by global atomics per response.  A static
// bucket follows from the slot counters at the flush.
constexpr uint32_t kTreeStaticRow = 0xFFFFu;     // LDS sum, static bucket
constexpr uint32_t kTreeGlobalDyn = 0xFFFEu;     // global sum and bucket
constexpr uint32_t kTreeGlobalStatic = 0xFFFDu;  // global sum, static bucket
constexpr uint32_t kTreeDynBucket = 0xFFu;       // slot_tbkt: the callee's bucket varies per invocation
constexpr uint32_t kTreeLeafSlot = 1u << 23;     // slot_tbkt: the callee is a leaf (sums from the counters)
constexpr uint32_t kTreeRowMask = 0xFFFFu;       // slot_tbkt / sum_row: the row (tree programs: < 2^16 rows)
struct TreeDynRow {
  uint32_t row, off, b_lo, width;  // off: word offset of the header in the LDS tables
};
constexpr uint32_t kTreeMaxPositions = 0xFFFFu;  // u16 sizes and slots
constexpr uint32_t kTreeRegFrames = 16;          // deepest register stack; deeper walks spill (kTreeMaxFrames)
constexpr uint32_t kTreeMaxFrames = 64;          // open calling invocations below the current one
constexpr uint32_t kTreeSpillWords = 5;          // u32 words of a spilled frame
constexpr uint32_t kTreeSpillWords64 = 7;        // ... with u64 time (acc and step max take two words each)
constexpr uint32_t kTreeSpillWide = 2;           // ... + position end and hop id of a wide tree's frame
// a wide tree's kernels keep fewer frames in registers (7 or 9 words each):
// 6 with u32 time, 4 with u64, the rest always in the spill area — at 8 the
// 1024-thread kernels ran out of their 128 VGPRs into scratch (32-144 B per lane)
inline uint32_t tree_wide_reg_frames(bool t64) { return t64 ? 4u : 6u; }
// register frames of the kind-7 kernel for a tree: the spill area holds the rest
inline uint32_t tree_reg_frames(uint32_t frames, bool t64, bool wide) {
  if (wide) return tree_wide_reg_frames(t64);
  return frames > kTreeRegFrames ? 8u : frames;
}
constexpr uint32_t kSpillAreas = 4;              // spill areas per (handler, device): launches in flight
// LDS of the kind-7 kernel, per workgroup: the budget for two 1024-thread
// workgroups per CU, and the whole CU.
constexpr uint32_t kTreeLutBytes = 512;  // the duration-bucket table by ceil(t / 1 ms), after the histograms
constexpr uint32_t kTreeLdsHalf = 80u * 1024u;
constexpr uint32_t kTreeLdsFull = 160u * 1024u;
// Layout chosen by the host (program.cpp place_tree): LDS byte offsets.
struct TreeLayout {
  uint32_t off_cnt;     // [2][n_slots] u32: executed calls, callee 500s
  uint32_t off_sums;    // [n_sum] code-200 duration sums of the LDS rows: u64, or u32 when compact (carries to HBM)
  uint32_t off_dyn;     // dyn_words u32: the bucket tables
  uint32_t off_nodes;   // [n_pos] TreeNode (nodes_lds)
  uint32_t bytes;       // total
  uint32_t nodes_lds;   // 1: the nodes in LDS; 0: read from global memory
  uint32_t wg_per_cu;   // 2: the layout fits kTreeLdsHalf
  uint32_t n_sum;       // LDS sum rows
  uint32_t compact;     // 1: compact rows (u32 sums, code-200 u16 bucket pairs, 500s in HBM): chosen when the
                        // wide rows (u64 sums, [code][width] u32 buckets) do not all fit
  uint32_t cnt16;       // 1: one u32 per slot, calls | 500s << 16, each kept below 2^15 (a field reaching
                        // 2^15 moves 2^15 to the stats at once); 0: [2][n_slots] u32
};

// Scalar kernel arguments (the program, records and stats pointers are
// separate __restrict__ kernel arguments so program fetches become s_load).
struct KParams {
  uint64_t trace_begin;
  uint64_t n_traces;
  uint32_t seed_lo, seed_hi;
  uint32_t n_slots;
  uint32_t max_frames;
  uint32_t lds_counters;    // 1: per-site counters in the LDS table
  uint32_t n_nodes;         // stream kernel: invocations per trace
  uint64_t t_static;        // stream kernel: the (trace-invariant) latency
  uint32_t svc_dur;         // dynamic walks: 1 = record per-service durations
  uint32_t root_dur;        // the entry's duration-table word (row | leaf bucket << 24)
  unsigned long long *work; // batch queues (kWorkWords): zero at launch, zeroed again by the last wave
  uint32_t *stage;          // draw stream: u32 per-site 500 counts of this launch (null: u64 atomics into stats)
  const StreamClose *closes;     // kind 6: close list (+kClosePad zero records of tail padding)
  const uint32_t *close_slot;    // kind 6: per close, the call-site slot of the closing invocation
  const uint32_t *close_end;     // kind 6: per chunk, closes up to and including it
  uint32_t mark_words;           // kind 8: position marks (records + the sentinel) in the LDS table
  const TreeExt *tree_ext;       // kind 7: per position (the nodes are the `prog` argument)
  const TreeStep *tree_step;     // kind 7: per position (read under TF_XPRE / TF_XCMAX)
  const TreeDynRow *tree_dyn;    // kind 7: rows with an LDS bucket table
  const uint32_t *sum_row;       // kind 7: per LDS sum index, its duration-table row
  const uint32_t *slot_tc;       // kind 7: per slot, the leaf callee's latency
  uint32_t *spill;               // kind 7: frames below the register stack ([level][word][lane])
  uint32_t spill_lanes;          // kind 7: lanes of the spill area (grid x workgroup size)
  uint32_t n_pos;                // kind 7: positions of the unrolled tree
  uint32_t n_rows;               // kind 7: duration-table rows
  uint32_t n_dyn;                // kind 7: entries of tree_dyn
  uint32_t dyn_words;            // kind 7: LDS words of the bucket tables
  uint32_t tree_flags;           // kind 7: kTreeAny*
  TreeLayout lay;                // kind 7: LDS layout
  const uint32_t *lds_slot;      // kind 7, wide tree: per LDS counter its slot (lay.off_cnt .. off_sums)
  uint32_t n_lds_slots;          // kind 7, wide tree: LDS counters
};

// Batch queues of one launch: one counter per XCD (workgroups are dealt to
// the 8 XCDs round-robin), each on its own 128-B line, then the count of
// waves done.  kWorkSlots sets of them per device, one per launch in flight.
constexpr uint32_t kWorkQueues = 8;
constexpr uint32_t kWorkLine = 16;                    // u64 words per 128-B line
constexpr uint32_t kWorkWords = (kWorkQueues + 1) * kWorkLine;
constexpr uint32_t kWorkSlots = 256;
// Draw-stream launches flush their per-site 500 counts as u32 atomics into a
// staging row of the launch's work slot (launch_walk's split keeps a launch's
// count at a site below 2^32); isim_stream_calls adds the row to the u64
// stats and zeroes it.  Graphs with more slots keep the u64 atomics.
constexpr uint32_t kStageMaxSlots = 1u << 16;

constexpr uint32_t kWgThreads = 1024;                 // max workgroup size (launch bound)
constexpr uint32_t kLdsAccBytes = 64;                 // WgAcc
constexpr uint32_t kHistWords = 2 * ISIM_N_PROM + 2 * ISIM_N_LOG2;

// walk.hip: kernel pointer for a walk variant.
// kind: 0/1 static interpreter u32/u64 time, 2/3 dynamic u32/u64, 4 draw stream,
// 5 draw stream + mode-B bit stack, 6 draw stream + mode-B close list,
// 7 lane tree walk (dynamic walks, tree.hip; `frames` = register stack depth).
void *walk_kernel(int kind, bool modeb, bool lds_counters);
// kind 7 variant (tree.hip, compiled once per mode and concurrency):
// register-stack depth (4, 6, 8, 12, 16; `spill`: 8 registers + the rest in
// global memory), nodes in LDS or global, the error-block cache.
void *tree_kernel_m0c0(uint32_t frames, bool spill, bool nodes_lds, bool draw, bool occ2, bool t64, bool wide,
                       bool dag);
void *tree_kernel_m0c1(uint32_t frames, bool spill, bool nodes_lds, bool draw, bool occ2, bool t64, bool wide,
                       bool dag);
void *tree_kernel_m1c0(uint32_t frames, bool spill, bool nodes_lds, bool draw, bool occ2, bool t64, bool wide,
                       bool dag);
void *tree_kernel_m1c1(uint32_t frames, bool spill, bool nodes_lds, bool draw, bool occ2, bool t64, bool wide,
                       bool dag);
// occ2: the LDS layout fits two workgroups per CU (kernels built for 80 VGPRs);
// t64: u64 time (Program::tree_t64); wide: a wide tree (Program::tree_wide);
// dag: the site graph (Program::tree_dag, wide)
inline void *tree_kernel(bool modeb, uint32_t frames, bool spill, bool nodes_lds, bool conc, bool draw, bool occ2,
                         bool t64, bool wide = false, bool dag = false) {
  if (modeb)
    return conc ? tree_kernel_m1c1(frames, spill, nodes_lds, draw, occ2, t64, wide, dag)
                : tree_kernel_m1c0(frames, spill, nodes_lds, draw, occ2, t64, wide, dag);
  return conc ? tree_kernel_m0c1(frames, spill, nodes_lds, draw, occ2, t64, wide, dag)
              : tree_kernel_m0c0(frames, spill, nodes_lds, draw, occ2, t64, wide, dag);
}
void *stream_calls_kernel();
void *mark_fold_kernel();  // kind 8: the per-launch fold of the position marks (walk.hip isim_mark_fold)
void *fill_const_kernel();  // (records, n, record, one-trace stats, stats, stats words)
uint32_t stream_traces_per_wave();

}  // namespace isim
