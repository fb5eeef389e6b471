// Flattening of a loaded ServiceGraph into the device program the walk
// kernel interprets.
//
// One code block per reachable non-leaf service (its script, in order),
// ending in RET; a call is CALL (jump into the callee's block, return to the
// next instruction) or LEAF (callee without calls: its whole invocation —
// error draw, counters, fixed latency — in one instruction).  pc 0 invokes
// the entry (the client request), pc 1 halts.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/isim.h"
#include "graph.h"
#include "kernel_abi.h"

namespace isim {



struct Program {
  std::vector<Ins> code;
  int32_t entry = -1;
  int32_t n_services = 0, n_sites = 0, n_slots = 0;
  int32_t max_depth = 0;   // deepest call chain from the entry (entry = 1)
  int32_t max_frames = 0;  // CALL frames the kernel stack needs (client frame included)
  bool static_walk = false;
  int32_t time_bits = 64;
  uint64_t max_latency = 0, hops_upper = 0;
  std::vector<int32_t> slot_site, slot_callee;  // per slot
  std::vector<int32_t> site_slot;               // per site (-1: unreachable)
  std::vector<int32_t> site_callee;             // per site
  std::vector<uint64_t> site_hop;               // per site: hop cost H (ns)
  // draw stream (static walks whose unrolled invocation tree is <= kMaxStreamNodes)
  std::vector<Node> stream;                     // padded to a multiple of 4
  uint32_t stream_nodes = 0;                    // invocations per trace (unpadded)
  std::vector<uint32_t> stream_mult;            // per slot: calls through it per trace
  std::vector<StreamClose> stream_closes;       // mode B (kind 6): closes of calling invocations
  std::vector<uint32_t> stream_close_slot;      // per close: call-site slot
  std::vector<uint32_t> stream_close_end;       // per chunk of kChunkRecords records
  std::vector<Node> stream_mark;                // mode B (kind 8): thr | key (kernel_abi.h), padded like stream
  std::vector<uint32_t> stream_end;             // kind 8: per record, the last record of its subtree
  // per-service invocation durations (RecordResponseSent, prometheus/handler.go:101-106)
  std::vector<uint64_t> svc_time;   // per service: T_max; the exact duration when static_walk
  std::vector<int32_t> svc_row;     // per service: row in the duration table (-1: unreachable)
  std::vector<int32_t> row_svc;     // per row: service (rows = reachable services, preorder)
  std::vector<uint32_t> slot_dur;   // per slot: callee row | leaf-callee bucket << 24
  uint32_t root_dur = 0;            // the entry: row 0 | bucket << 24 when the entry is a leaf
  // lane tree walk (kernel kind 7, dynamic walks): the unrolled tree of potential
  // invocations when it fits (tree_nodes empty otherwise; tree_why says why)
  // (tree_nodes_w: every tree in the wide format — the host-side view the DES
  // plan reads; tree_nodes: the 8-byte device nodes, empty for a wide tree)
  std::vector<TreeNode> tree_nodes;
  std::vector<TreeNodeW> tree_nodes_w;
  bool tree_wide = false;           // a wide tree (kernel_abi.h TreeNodeW): 32-bit fields, global statistics
  bool tree_dag = false;            // the site graph (tree_walk.h NodeD4): one node per call site, always wide
  std::vector<uint16_t> tree_slot_lds;  // wide: per slot its LDS counter (0xFFFF: global atomics)
  std::vector<uint32_t> tree_lds_slot;  // wide: per LDS counter its slot
  std::vector<TreeExt> tree_ext;
  std::vector<TreeStep> tree_step;
  std::vector<uint32_t> slot_tbkt;  // per slot: callee row | kTreeLeafSlot | static duration bucket << 24
                                    // (kTreeDynBucket: it varies)
  std::vector<uint32_t> slot_tc;    // per slot: the leaf callee's latency (0 for a calling callee)
  std::vector<TreeDynRow> tree_dyn; // LDS rows whose duration bucket varies: their LDS bucket tables
  uint32_t tree_dyn_words = 0;
  std::vector<uint32_t> sum_row;    // per LDS sum index: its row
  std::vector<uint32_t> tree_row_place, tree_row_index, tree_row_blo;  // per row (place_tree)
  TreeLayout tree_layout{};
  uint32_t tree_frames = 0;         // frames the walk needs (open calling invocations - 1)
  bool tree_t64 = false;            // the latency bound reaches 2^32 ns: the walk keeps u64 time
  uint32_t tree_mult = 0;           // most positions through one slot or into one bucket-table row (LDS u32
                                    // counter overflow guard)
  uint32_t tree_flags = 0;          // kTreeAnyProb | kTreeAnyDraw | kTreeAnyConc
  std::string tree_why;
  bool has_tree() const { return !tree_nodes_w.empty(); }
  uint32_t tree_positions() const { return (uint32_t)tree_nodes_w.size(); }
};

// Bucket of an invocation duration on the service_request_duration_seconds
// edges (prometheus/handler.go:26-31, `le`): 0..31, 32 = +Inf.
uint32_t prom_bucket_ns(uint64_t t);

// Returns an isim_status; on error `err` holds the message.
int compile_program(const ServiceGraph &g, int32_t entry, const isim_params &p, Program &out,
                    std::string &err);

// First service with the name, -1 if absent (extractService, srv/graph.go:97-109).
int32_t service_index(const ServiceGraph &g, const std::string &name);

}  // namespace isim
