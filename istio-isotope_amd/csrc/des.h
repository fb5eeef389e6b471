// Per-replica worker-pool discrete-event simulation (BASELINE config 5,
// DESIGN.md §10 "isim DES semantics v1").
//
// Host side: the DES plan — the unrolled invocation tree of a static walk
// (one POSITION per invocation, in hop order = the draw stream's order), the
// per-position timing constants, and the positions grouped by depth (LEVELS).
// Device side (des.hip): a level-synchronous exact algorithm over all traces
// of a batch at once — top-down, one FIFO max-plus scan per position over the
// traces (the replica queue); bottom-up, finish times, statuses, durations.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/isim.h"
#include "graph.h"
#include "program.h"

namespace isim {

constexpr uint32_t kDesNoParent = 0xFFFFFFFFu;
constexpr uint32_t kDesMaxReplicas = 64;  // per-replica carries of a leaf position live in LDS
constexpr uint32_t kDesMaxRounds = 65536; // schedule length limit (each round is a few launches per batch)
constexpr uint32_t kDesFlagAlways = 1u;   // errorRate 1
constexpr uint32_t kDesFlagLeaf = 2u;     // no call step
constexpr uint32_t kDesFlagFused = 4u;    // fast-path leaf: finished by its queue pass (no up pass)
// non-fused position whose invocation durations its caller's up block records
// (round 3, des.hip des_up: the caller holds S(caller) + off, the arrival, so
// this position's block reads no arrival row); its index among the caller's
// such children in bits kDesDurShift.. of the flags
constexpr uint32_t kDesFlagParentDur = 8u;
constexpr uint32_t kDesDurShift = 8;
constexpr uint32_t kDesDurKids = 8;       // per caller
// rows are relative to the arrival of the trace's group of kDesGroupTraces
// (one DPP row of the 32-bit-key queue pass: 16 lanes x kDesN32Per traces);
// the 32-bit keys need (t - t_group) x hold < 2^31
constexpr uint32_t kDesN32Per = 4;
constexpr uint64_t kDesGroupTraces = 16ull * kDesN32Per;
constexpr uint64_t kDesN32HoldMax = (1ull << 31) / kDesGroupTraces;
constexpr uint32_t kDesUpChildLds = 1024; // callers with more children record none (their ids are not staged in LDS)
// non-fused position whose finish needs no start row: one call step, no step
// begins, and every callee's hop cost at least the step's longest sleep, so
// F(c) >= a(c) = S + pre + H(c) >= S + floor for each callee c and
// F = max_c F(c) + post (des_up reads S only for callee durations)
constexpr uint32_t kDesFlagNoStart = 16u;

// One invocation position of the unrolled tree (64 bytes, device layout).
struct DesPos {
  uint32_t parent;     // caller's position (kDesNoParent: the entry)
  uint32_t row;        // duration-table row of the service (Program::svc_row)
  uint32_t slot;       // stats slot of the call site (kSlotRoot: the entry)
  uint32_t reps;       // replicas of the service (numReplicas, >= 1)
  uint64_t off;        // arrival = start(parent) + off: the caller's pre-call sleeps + H
  uint64_t hold;       // worker hold time: the service's sleep total
  uint64_t floor;      // leaf: script time; else pre-call sleeps + longest sleep of the call step
  uint64_t post;       // sleeps after the call step
  uint32_t child_off, child_cnt;  // children in DesPlan::child
  uint32_t thr;        // error threshold over the u32 draw
  uint32_t flags;      // kDesFlag*
};
static_assert(sizeof(DesPos) == 64, "DesPos must be 64 bytes");

// A service whose queue needs the sort path: several
// positions per trace, or arrivals not in trace order (a caller upstream
// has replicas, or the call is not in the caller's first call step).
struct DesSortSvc {
  uint32_t row;       // duration-table row
  uint32_t reps;      // replicas
  uint32_t pos_off;   // its positions in DesPlan::sort_pos (hop order)
  uint32_t pos_cnt;
  uint64_t hold;      // worker hold time
};

// Per position, for scripts with several call steps (16 bytes, device layout).
struct DesPosExt {
  uint32_t bk_in;      // BK row whose value + off is the arrival (kDesNone: start(parent) + off)
  uint32_t bk_last;    // BK row of the position's own last call step (kDesNone: one call step or none)
  uint32_t last_child; // index in its children list where the last call step's children start
  uint32_t pad;
};

// The begin time of call step k of a position, BK[id][t]:
// step 1: start + add; step k > 1: max(BK[prev] + smax, max F(step k-1 callees)) + add.
struct DesStep {
  uint32_t pos;        // the calling position
  uint32_t prev;       // BK row of step k-1 (kDesNone for step 1)
  uint64_t add;        // step 1: sleeps before it; k > 1: sleeps between steps k-1 and k
  uint64_t smax;       // longest sleep of step k-1's concurrent sub-commands
  uint32_t child_off;  // step k-1's callees: positions child[child_off .. +child_cnt)
  uint32_t child_cnt;
};
static_assert(sizeof(DesStep) == 32, "DesStep must be 32 bytes");
constexpr uint32_t kDesNone = 0xFFFFFFFFu;
// step_round flag: a step begin whose callee-finish edges the cyclic schedule
// cut (des_plan.cpp): it reads the previous pass's callee maxima (des_items.hip)
constexpr uint32_t kDesStepCut = 0x80000000u;

// Per position, for the item engine of dynamic walks (des_items.hip; 16 bytes, device layout).
struct DesItemPos {
  uint32_t qround;     // round of its queue (the service's, or its own for a zero-hold service)
  uint32_t fgroup;     // finish group (DesPlan::fin_off index)
  uint16_t kstep;      // its call step in the caller's script
  uint16_t nsteps;     // call steps of its own script
  uint32_t bk_first;   // nsteps >= 2: the DesStep id of its first call step (kDesNone otherwise)
};
static_assert(sizeof(DesItemPos) == 16, "DesItemPos must be 16 bytes");

struct DesPlan {
  // item engine (des_items.hip): a dynamic walk (probabilistic calls, or mode-B aborts)
  // over the tree of potential invocations; only executed invocations
  // (ITEMS) are simulated
  bool items = false;
  bool modeb = false;                // error mode B: the item engine's walks draw errors, failed steps end scripts
  std::vector<DesItemPos> item_pos;  // [n_pos]
  std::vector<uint32_t> step_round;  // [steps]: the round of each BK op | kDesStepCut
  uint32_t item_acc = 1;             // per item: callee finish maxima, one per call step (>= 1)
  uint32_t item_bk = 0;              // per item: BK slots (the most call steps of a multi-step script; 0: none)
  // per round: every position queued in it needs no sort — its service has
  // no other position and one replica and its arrivals come in trace order
  // (the static engine's fast-path condition), or no hold (start = arrival):
  // the round scans its items in their (position, trace) order directly
  std::vector<uint8_t> round_nosort;
  std::vector<DesPos> pos;           // hop order (position 0 = the entry)
  std::vector<DesPosExt> ext;        // [n_pos]
  std::vector<uint32_t> child;       // children lists (positions, call-step order)
  std::vector<DesStep> steps;        // BK rows
  std::vector<uint32_t> slot_mult;   // per slot: calls through it per trace
  uint32_t n_levels = 0, max_width = 0;  // invocation-tree depth, widest depth
  bool general = false;              // some script has several call steps
  bool cyclic = false;               // the schedule runs as passes to a fixed point (back edges cut)
  // the schedule: rounds of (step begins, queues, finishes)
  std::vector<uint32_t> arr_ops, arr_off;        // BK rows computed in round r
  std::vector<uint32_t> fast_pos, fast_off;      // single-position trace-ordered services
  // [rounds][5]: a round's fast positions by kernel variant (des_down<MULTI, FUSED>):
  // [v][0..1) fused single replica, [1..2) single, [2..3) fused replicated, [3..4) replicated
  std::vector<uint32_t> fast_split;
  std::vector<uint32_t> zero_pos, zero_off;      // positions of zero-hold services: start = arrival
  std::vector<DesSortSvc> sorted;                // sort-path services
  std::vector<uint32_t> sorted_off;
  std::vector<uint32_t> sort_pos;                // positions of the sort-path services
  std::vector<uint32_t> fin_pos, fin_off;        // finish groups (one depth each), deepest first
  std::vector<uint32_t> fin_round_off;           // [rounds + 1] into the finish groups
  uint32_t max_sort_pos = 0;         // most positions of one sort-path service
  uint32_t max_rep_bits = 0;         // sort keys: bits of the largest replica index of a sort-path service
  uint64_t max_hold = 0;             // longest worker hold time of any position (queue scan keys)
  // pipelined queue segments (des.hip des_down_pipe): runs of >= 2 rounds whose
  // queues are all single-replica fast positions and whose finishes all come in
  // the run's last round; every position of a run in ONE launch, a position's
  // chunks waiting on its caller's published chunk count
  struct PipeSeg {
    uint32_t r0, r1;    // rounds [r0, r1]
    uint32_t off, cnt;  // positions pipe_pos[off, off + cnt)
  };
  std::vector<PipeSeg> pipe;
  std::vector<uint32_t> pipe_pos;    // round order, within a round non-fused first
  std::vector<uint32_t> pipe_dep;    // per pipe_pos: the position whose start row it waits on (kDesNone: none)
  // every pipelined position's holds and offsets fit the 32-bit queue keys
  // (des.hip down1_chunk_n32: hold < kDesN32HoldMax, off and a leaf's floor < 2^30)
  bool pipe_n32 = false;
  // no step begins and every finish constant (off, floor, post) below 2^30:
  // des_up's finish quads in 32-bit arithmetic (des.hip up_quad32)
  bool up_n32 = false;
  uint32_t rounds() const { return (uint32_t)arr_off.size() - 1; }
};

// Device buffers and sizes of one DES batch (des.hip: des_launch).
struct DesLaunch {
  const DesPlan *plan;               // host copy (the schedule)
  const void *d_pos, *d_ext, *d_steps;  // DesPos[n_pos], DesPosExt[n_pos], DesStep[]
  const uint32_t *d_child, *d_fast_pos, *d_sort_pos, *d_fin_pos, *d_arr_ops, *d_zero_pos;
  const uint32_t *d_pipe;            // pipe_pos then pipe_dep
  const uint32_t *d_mult;            // per slot: calls per trace (executed-call counters)
  // workspace parts (des_carve)
  void *W, *WF, *BK;                 // rows [n_pos][ld] (starts, finishes), [steps][ld] of u32 or u64
  uint64_t *A, *blk;                 // [N] arrival times, chunk sums
  uint32_t *E;                       // [N] per-trace 500 count
  void *chain;                       // chained-scan states of the down pass (des_chain_bytes)
  uint32_t *ovf;                     // narrow rows: overflow flag
  uint64_t *stage;                   // narrow rows: staged stats (stats_words) + table
  uint32_t *stbits;                  // own error status bits [n_pos][words of 32 traces]
  void *sort_ws;                     // sort path (keys, values, radix-sort temp)
  // caller buffers
  uint64_t *d_stats, *d_table;
  isim_trace_rec *d_records;         // may be null
  uint64_t n_traces, trace_begin, mean_ns, seed;
  uint64_t stats_words;
  uint32_t table_rows;
  uint32_t n_pos, n_slots, modeb;
  bool wide;                         // u64 rows (ISIM_DES_FLAG_WIDE); else u32 rows + overflow retry
};

// Workspace bytes for a batch of n traces (every part 256-B aligned; rows
// sized for u64 so one workspace serves both row widths).
uint64_t des_workspace_bytes(const DesPlan &plan, uint64_t n, uint64_t stats_words, uint64_t table_rows);
// Points L's workspace parts into `workspace` (L.plan, n_traces, stats_words, table_rows set).
void des_carve(DesLaunch &L, void *workspace);
int des_launch(const DesLaunch &L, void *stream);
// Polls a decoupled look-back (des.hip chain pass, pipelined pass; des_items.hip
// k_qscan) makes for a predecessor before it gives up and FAILS the batch (a
// device fault flag: the batch is not accumulated and the call reports it).
// Default 2^26 (never expected: tickets order the tiles); 0 makes every
// look-back fail at once (isim_debug_set_spin_limit, tests only).
constexpr uint32_t kDesSpinLimit = 1u << 26;
uint32_t des_spin_limit();
void des_set_spin_limit(uint32_t polls);
// Bit of ISIM_ST_DES_RETRY's high word: batches dropped for a device fault
constexpr uint64_t kDesFaultUnit = 1ull << 32;
// Chained-scan workspace of the down pass: a ticket counter per launch, then
// one 32-byte state per (position, chunk of 4096 traces); zeroed per batch.
uint64_t des_chain_bytes(const DesPlan &plan, uint64_t n);

// Rows one trace reads and writes in a batch's queue and finish passes (one
// pass of a cyclic schedule): what des.hip's kernels move per trace, 4 or 8
// bytes each (the algorithmic bytes of the roofline).
void des_row_traffic(const DesPlan &plan, uint32_t &reads, uint32_t &writes);

// Returns ISIM_OK or ISIM_EINVAL with the reason in `err` when the graph is
// outside the DES class.
int build_des_plan(const ServiceGraph &g, const Program &p, bool modeb, DesPlan &out, std::string &err);

// The item engine (des_items.hip): one batch of a dynamic walk's DES.  Device
// per-trace workspace bytes; the per-item arrays are allocated on `stream`
// from `pool` (the handler's private hipMemPool_t on this device) once the
// batch's executed invocations are counted.
struct DesItemsReport {
  uint32_t passes;  // passes over the rounds (cyclic schedules: the quiet ones and the recording one)
  uint32_t syncs;   // host synchronisations of the stream
  uint64_t items;   // executed invocations
};
struct DesItemsLaunch {
  const DesPlan *plan;
  const void *d_pos, *d_item_pos, *d_steps;  // DesPos[n_pos], DesItemPos[n_pos], DesStep[]
  const uint32_t *d_step_round;              // [steps]
  const void *d_nodes, *d_ext, *d_tstep;     // the lane tree walk's TreeNode/TreeExt/TreeStep
  uint32_t tree_frames, tree_flags, n_nodes;
  uint32_t tree_t64;  // the walk keeps u64 time (Program::tree_t64)
  uint32_t tree_wide;  // a wide tree: 16-byte nodes (Program::tree_wide)
  void *workspace;
  uint64_t *d_stats, *d_table;
  isim_trace_rec *d_records;
  uint64_t n_traces, trace_begin, mean_ns, seed;
  uint32_t n_slots;
  uint32_t flags;  // isim_params.flags (ISIM_FLAG_DES_*: the independent-check paths)
  void *pool;  // hipMemPool_t
  DesItemsReport *report;  // filled when the batch ends (null: none)
};
uint64_t des_items_workspace_bytes(uint64_t n);
int des_items_launch(const DesItemsLaunch &L, void *stream, std::string &err);

// -ln(w / 2^24), w = (u >> 8) + 1, in Q24 fixed point:
// log1p(i/256) table, 16-bit linear interpolation.  Shared by host and device.
constexpr int32_t kLnQ24[257] = {
#include "des_ln_table.inc"
};
constexpr int64_t kLn2Q24 = 11629080;  // round(ln 2 * 2^24)

inline uint64_t des_exp_q24_host(uint32_t u) {
  const uint32_t w = (u >> 8) + 1u;
  const int e = 31 - __builtin_clz(w);
  const uint32_t f = (w << (24 - e)) & 0xFFFFFFu;
  const uint32_t idx = f >> 16, rem = f & 0xFFFFu;
  const int64_t lnm = kLnQ24[idx] + ((((int64_t)kLnQ24[idx + 1] - kLnQ24[idx]) * (int64_t)rem) >> 16);
  return (uint64_t)(24 * kLn2Q24 - ((int64_t)e * kLn2Q24 + lnm));
}

}  // namespace isim
