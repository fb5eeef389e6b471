/*
 * isim.h — C ABI of the MI355X-native isotope trace simulator ("isim").
 *
 * This is the drop-in boundary for ONE hot path of adalrsjr1/istio-isotope:
 * executing isotope service-graph scripts (isotope/service/pkg/srv) for many
 * independent request traces, over graphs loaded with isotope's own
 * service-graph schema (isotope/convert/pkg/graph).  Plain C types only: a Go
 * host binds it through cgo, Python through ctypes.
 *
 * Reference interfaces replaced (file:line relative to the reference repo):
 *   isim_graph_unmarshal_json  <- (*graph.ServiceGraph).UnmarshalJSON
 *                                 isotope/convert/pkg/graph/unmarshal.go:30-48
 *                                 (reached through sigs.k8s.io/yaml.Unmarshal,
 *                                 isotope/service/pkg/srv/graph.go:82-94; the
 *                                 host does the YAML->JSON step)
 *   isim_handler_create        <- srv.HandlerFromServiceGraphYAML(path, name)
 *                                 isotope/service/pkg/srv/graph.go:34-60
 *                                 (extractService :97-109, extractServiceTypes :113-120)
 *   isim_serve / isim_serve_device
 *                              <- Handler.ServeHTTP  isotope/service/pkg/srv/handler.go:37-79
 *                                 + execute / executeRequestCommand /
 *                                 executeConcurrentCommand executable.go:43-179,
 *                                 run for n_traces independent client requests
 *                                 in virtual integer-nanosecond time
 *   stats words                <- prometheus.Record* isotope/service/pkg/srv/prometheus/handler.go:87-106
 *   isim_multi_* / isim_stats_allreduce_device / isim_stats_merge
 *                              <- the per-pod Prometheus scrape of those counters
 *                                 (prometheus/handler.go:37-69, one registry per
 *                                 pod): here one RCCL all-reduce over the ranks
 *                                 that each walked a shard of the traces
 *
 * Semantics: "isim semantics v1" (SURVEY.md Appendix A).
 * Errors: every function returns an isim_status; isim_last_error() gives a
 * thread-local message (the Go error text for graph-load errors).
 * Thread-safety: distinct handles may be used concurrently; a handle may be
 * served from several threads onto different devices.
 */
#ifndef ISIM_H
#define ISIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ISIM_ABI_VERSION 10

#if defined(__GNUC__)
#define ISIM_API __attribute__((visibility("default")))
#else
#define ISIM_API
#endif

typedef enum {
  ISIM_OK = 0,
  ISIM_EINVAL = 1,   /* bad argument, or no isEntrypoint service */
  ISIM_ENOMEM = 2,
  ISIM_EHIP = 3,     /* HIP runtime error */
  ISIM_EPARSE = 4,   /* graph load error: the Go error text is in isim_last_error() */
  ISIM_ECYCLE = 5,   /* call cycle reachable from the entry (would recurse forever) */
  ISIM_EDEPTH = 6,   /* call depth above isim_params.max_depth (<= 64) */
  ISIM_ERANGE = 7,   /* hop cost / latency bound overflows int64 */
  ISIM_ENOTFOUND = 8,/* service name not in graph */
  ISIM_ENODEV = 9,   /* no usable gfx950 device */
  ISIM_ECOMM = 10    /* RCCL error, or RCCL cannot be loaded (isim_multi_*) */
} isim_status;

/* Error propagation mode. */
#define ISIM_MODE_A 0u /* reference: a callee's 500 is swallowed (executable.go:131-143) */
#define ISIM_MODE_B 1u /* EXT: a callee's 500 fails the calling step and aborts the script */

typedef struct isim_graph isim_graph;
typedef struct isim_handler isim_handler;

/* Simulation parameters (the hop-cost model replaces the HTTP transport of
 * isotope/service/pkg/srv/request.go:30-64):
 *   H(call) = hop_base_ns + floor((size*req_ps_per_byte + responseSize(callee)*resp_ps_per_byte)/1000) */
typedef struct {
  uint64_t seed;             /* Philox4x32-10 key = (seed_lo, seed_hi) */
  uint64_t hop_base_ns;
  uint64_t req_ps_per_byte;
  uint64_t resp_ps_per_byte;
  uint32_t error_mode;       /* ISIM_MODE_A / ISIM_MODE_B */
  uint32_t max_depth;        /* 0 = 64; at most 64 */
  uint32_t flags;            /* ISIM_FLAG_* */
  uint32_t reserved;         /* must be 0 */
} isim_params;

/* isim_params.flags */
#define ISIM_FLAG_NO_STREAM 1u  /* run static walks on the interpreter kernel instead of the draw stream */
#define ISIM_FLAG_NO_SVC_DUR 2u /* dynamic walks: do not record per-service invocation durations */
#define ISIM_FLAG_WALK_ALL 4u   /* draw-free static walks: walk every trace (default: walk one, fill the rest) */
#define ISIM_FLAG_BIT_STACK 8u  /* mode B on the draw stream: the bit-stack kernel (kind 5, call depth <= 32;
                                   kind 4 deeper) instead of the close-list kernel (kind 6) */
#define ISIM_FLAG_DYNAMIC 16u   /* treat every walk as dynamic: the general kernels with per-lane time and hop
                                   ids (kind 7, or 2/3) even when every trace executes the same invocations
                                   (parity tests of the general path on static graphs; no DES) */
#define ISIM_FLAG_WAVE_WALK 32u /* dynamic walks on the wave-walk interpreter (kinds 2/3: a wave walks the union
                                   of its 64 traces' call paths) instead of the lane tree walk (kind 7) */
#define ISIM_FLAG_CLOSE_LIST 64u /* mode B on the draw stream: the close-list kernel (kind 6) instead of sparse
                                    ancestor marking (kind 8, the default when its per-invocation mark table
                                    fits the LDS) */
/* Independent-check paths (the same results by a different algorithm; tests
 * compare them with the defaults at sizes the CPU oracle does not reach): */
#define ISIM_FLAG_TREE_WIDE 128u      /* dynamic walks: the wide lane-tree format (16-byte nodes, 32-bit frames)
                                         for any tree, not only past the 8-byte nodes' 16-bit fields */
#define ISIM_FLAG_DES_SCAN_BY_KEY 256u /* DES item engine: every queue by rocPRIM's scan by key over max-plus maps
                                         instead of the one-pass look-back scan (k_qscan) */
#define ISIM_FLAG_DES_SORT_ALL 512u   /* DES item engine, cyclic schedules: sort every queue round of every pass
                                         (no reuse of the previous pass's sorted order) */
#define ISIM_FLAG_DES_TWO_SORTS 1024u /* DES item engine: every sorted queue round by two stable sorts (replica |
                                         arrival, then service) instead of one combined key */
#define ISIM_FLAG_TREE_DAG 2048u      /* dynamic walks: the lane walk over the site graph (one node per call site)
                                         for any graph, not only where the unrolled tree would pass 2^24 positions */

/* One 16-byte record per simulated request trace. */
typedef struct {
  uint64_t latency_ns;       /* T(entry): virtual duration of the entry's ServeHTTP */
  uint32_t hops;             /* executed invocations (entry included) */
  uint32_t status_err;       /* bit31: entry responded 500; bits0-30: invocations that responded 500 */
} isim_trace_rec;

/* Layout of the u64 stats buffer filled by isim_serve*.  Offsets in words. */
#define ISIM_ST_N_TRACES 0
#define ISIM_ST_SUM_LATENCY 1
#define ISIM_ST_SUM_HOPS 2
#define ISIM_ST_SUM_ERR_HOPS 3
#define ISIM_ST_N_500 4
#define ISIM_ST_NOT_MIN_LATENCY 5 /* ~min latency (so min and max both merge with MAX) */
#define ISIM_ST_MAX_LATENCY 6
#define ISIM_ST_DES_RETRY 7       /* DES batches NOT accumulated: low 32 bits, a latency reached 2^31 ns in
                                     32-bit rows (rerun them with ISIM_DES_FLAG_WIDE; isim_serve_des does), or
                                     a cyclic schedule found no fixed point within 256 passes; high 32 bits,
                                     batches FAILED by a device fault (a queue pass's decoupled look-back gave
                                     up waiting for an earlier tile: an error, never retried — isim_serve_des
                                     and the item engine return ISIM_EHIP; such a batch writes no record and
                                     counts no trace, and the item engine's per-site / DES-table words it may
                                     have added are undefined: discard the buffers) */
#define ISIM_ST_PROM 8            /* [2][33] latency histogram, Prometheus duration buckets
                                     (prometheus/handler.go:26-31), index [status500][bucket] */
#define ISIM_N_PROM 33
#define ISIM_ST_LOG2 (ISIM_ST_PROM + 2 * ISIM_N_PROM) /* [2][64] latency histogram by bit length */
#define ISIM_N_LOG2 64
#define ISIM_ST_SITES (ISIM_ST_LOG2 + 2 * ISIM_N_LOG2) /* [2][n_slots]: executed calls, then callee 500s,
                                                          per reachable call site slot */
/* Per-service duration table (service_request_duration_seconds and its _sum,
 * prometheus/handler.go:55-69,101-106), one row of ISIM_SVC_DUR_WORDS per
 * reachable service: [code 200|500][33] bucket counts, then the two duration
 * sums in ns.  Present in the stats buffer only when info.svc_dur_rows > 0
 * (dynamic walks); for static walks every invocation of a service lasts the
 * same T(s) and isim_stats_fold_durations derives the table from the
 * counters. */
#define ISIM_SVC_DUR_WORDS (2 * ISIM_N_PROM + 2)
#define ISIM_ST_SVC_DUR(n_slots) (ISIM_ST_SITES + 2 * (uint64_t)(n_slots))

/* Per-service row of the DES table filled by isim_serve_des* (config 5,
 * DESIGN.md §10): the service's invocation durations from request receipt to
 * response, queueing included, as ISIM_SVC_DUR_WORDS ([code][33] buckets on
 * the Prometheus duration edges, then the [code] sums in ns), followed by
 * the replica-queue figures.  Rows follow the duration-table row order
 * (reachable services in preorder; isim_des_fold maps them to services). */
#define ISIM_DES_COUNT ISIM_SVC_DUR_WORDS          /* invocations */
#define ISIM_DES_SUM_WAIT (ISIM_SVC_DUR_WORDS + 1) /* sum of queue waits, ns */
#define ISIM_DES_MAX_WAIT (ISIM_SVC_DUR_WORDS + 2) /* longest queue wait, ns */
#define ISIM_DES_SUM_HOLD (ISIM_SVC_DUR_WORDS + 3) /* worker busy time, ns */
#define ISIM_DES_ROW_WORDS (ISIM_SVC_DUR_WORDS + 4)

typedef struct {
  int32_t n_services;        /* services in the graph */
  int32_t n_sites;           /* call commands in the graph (document order) */
  int32_t n_slots;           /* call sites reachable from the entry (stats slots) */
  int32_t entry;             /* entry service index */
  int32_t max_depth;         /* deepest call chain from the entry (entry = 1) */
  int32_t static_walk;       /* 1: every invocation executes in every trace */
  int32_t time_bits;         /* 32 or 64: per-lane time width of the kernel */
  int32_t program_len;       /* instructions in the device program */
  uint64_t max_latency_ns;   /* static upper bound of any trace's latency */
  uint64_t hops_upper;       /* static upper bound of invocations per trace */
  uint64_t stats_words;      /* u64 words of the stats buffer */
  int32_t svc_dur_rows;      /* rows of the device duration table (0: derived on the host) */
  int32_t n_reachable;       /* services reachable from the entry */
  uint64_t draw_groups;      /* draw stream: groups of 4 invocations with an error draw (one Philox4x32-10
                                block per trace each); 0 for draw-free and dynamic walks */
} isim_handler_info;

/* Launch configuration chosen for a device (filled on first use of that device). */
typedef struct {
  int32_t wg_threads;        /* workgroup size (multiple of 64) */
  int32_t lds_bytes;         /* dynamic LDS per workgroup */
  int32_t lds_counters;      /* 1: per-site counters in LDS; 0: global atomics */
  int32_t blocks_per_cu;     /* resident workgroups per CU (occupancy query) */
  int32_t max_blocks;        /* resident workgroups on the device (grid cap) */
  int32_t kernel_kind;       /* 0/1 static interpreter u32/u64 time, 2/3 dynamic u32/u64, 4 draw stream,
                                5 draw stream with the mode-B bit stack (call depth <= 32),
                                6 draw stream with the mode-B close list (ISIM_FLAG_CLOSE_LIST, or a stream
                                too long for kind 8's LDS mark table),
                                7 lane tree walk (dynamic walks whose unrolled tree of potential
                                invocations has at most 2^24 positions; else 2/3),
                                8 draw stream with mode-B sparse ancestor marking (the default in mode B) */
  int32_t fill;              /* 1: a draw-free static walk: one trace walked, batches are a record fill
                                (isim_fill_const) + n x its statistics (off with ISIM_FLAG_WALK_ALL) */
  int32_t tree_wide;         /* kind 7 on a wide tree (more than 65,535 positions, call sites or rows, or
                                per-site counters past the LDS): 16-byte nodes, the hottest sites counted
                                in LDS, the rest by global atomics; 2: kind 7 on the site
                                graph (one node per call site: a DAG whose unrolled tree would pass 2^24
                                positions, or ISIM_FLAG_TREE_DAG), wide as 1; else 0 */
  uint64_t max_launch_traces; /* isim_serve_device splits a batch into launches of at most this many traces
                                 (per-workgroup u32 LDS counters must not wrap) */
} isim_launch_info;

ISIM_API const char *isim_last_error(void);
ISIM_API int isim_abi_version(void);

/* ---- graph (convert/pkg/graph) ---- */
ISIM_API int isim_graph_unmarshal_json(const char *json, size_t len, isim_graph **out);
ISIM_API void isim_graph_free(isim_graph *g);
ISIM_API int isim_graph_num_services(const isim_graph *g);
/* Exact implementation-neutral dump of the decoded graph.
 * Writes at most cap bytes (NUL-terminated when it fits); *len = bytes needed. */
ISIM_API int isim_graph_canonical_json(const isim_graph *g, char *buf, size_t cap, size_t *len);
/* json.Marshal(graph.ServiceGraph): svc/service.go:25-51 json tags + omitempty,
 * script.Script.MarshalJSON (script/script.go:24-31, command.go:30-53),
 * ByteSize/Percentage/ServiceType MarshalJSON (size/byte_size.go:31-34,
 * pct/percentage.go:32-35, svctype/service_type.go:45-48).  Same buffer
 * contract as isim_graph_canonical_json. */
ISIM_API int isim_graph_marshal_json(const isim_graph *g, char *buf, size_t cap, size_t *len);
/* graphviz.ServiceGraphToDotLanguage (convert/pkg/graphviz/graphviz.go:28-41):
 * the Graphviz DOT text of `isotope convert graphviz`. */
ISIM_API int isim_graph_to_dot(const isim_graph *g, char *buf, size_t cap, size_t *len);
/* extractService: first service with that name (graph.go:97-109); -1 if absent. */
/* ---- Kubernetes manifests (convert/pkg/kubernetes) ----
 * Replaces kubernetes.ServiceGraphToKubernetesManifests(serviceGraph,
 * serviceNodeSelector, serviceImage, serviceMaxIdleConnectionsPerHost,
 * clientNodeSelector, clientImage, environmentName)
 * (isotope/convert/pkg/kubernetes/kubernetes.go:56-63): Namespace, ConfigMap
 * (the graph as yaml.Marshal), per service a Deployment + Service (+ RBAC
 * rules under ISTIO), the Fortio client Deployment + Service, YAML documents
 * joined by "---\n" exactly as sigs.k8s.io/yaml v1.2.0 renders k8s.io/api
 * v0.18.0 objects.  Node selectors are n key/value pairs [k0, v0, k1, v1, ...]
 * (the CLI's "k=v" flag, cmd/kubernetes.go:96-108).  EXT: the reference stamps
 * time.Now() and names RBAC rules with uuid.New(); here every
 * creationTimestamp is creation_timestamp_s (UTC, RFC 3339) and the rule
 * names are v4 UUIDs from Philox4x32-10 keyed by rbac_seed. */
typedef struct {
  const char *service_image;                 /* "" / NULL: omitted, as Go's omitempty */
  const char *client_image;
  const char *environment_name;              /* "NONE" or "ISTIO" (strings.EqualFold); NULL = "NONE" */
  const char *const *service_node_selector;  /* 2 * n_service_node_selector strings */
  const char *const *client_node_selector;   /* 2 * n_client_node_selector strings */
  int32_t n_service_node_selector;
  int32_t n_client_node_selector;
  int32_t service_max_idle_connections_per_host;
  int32_t reserved;                          /* 0 */
  int64_t creation_timestamp_s;              /* unix seconds of every metadata.creationTimestamp */
  uint64_t rbac_seed;                        /* RBAC rule names (environment ISTIO, numRbacPolicies > 0) */
} isim_k8s_params;
/* Writes at most cap bytes (NUL-terminated when it fits); *len = bytes needed. */
ISIM_API int isim_graph_to_k8s_manifests(const isim_graph *g, const isim_k8s_params *p, char *buf, size_t cap,
                                         size_t *len);
/* yaml.Marshal(graph) (sigs.k8s.io/yaml: JSONToYAML of json.Marshal) — the ConfigMap payload. */
ISIM_API int isim_graph_marshal_yaml(const isim_graph *g, char *buf, size_t cap, size_t *len);
ISIM_API int isim_graph_service_index(const isim_graph *g, const char *name);

/* ---- units (convert/pkg/graph/size, pct, script/sleep_command.go) ---- */
ISIM_API int isim_size_from_string(const char *s, uint64_t *out);        /* size.FromString */
ISIM_API int isim_duration_parse(const char *s, int64_t *out_ns);        /* time.ParseDuration */
ISIM_API int isim_percentage_from_string(const char *s, double *out);    /* pct.FromString */

/* ---- handler (service/pkg/srv) ---- */
/* service_name NULL: the first service with isEntrypoint: true. */
ISIM_API int isim_handler_create(const isim_graph *g, const char *service_name, const isim_params *p,
                        isim_handler **out);
ISIM_API void isim_handler_free(isim_handler *h);
ISIM_API int isim_handler_info_get(const isim_handler *h, isim_handler_info *out);
/* Prepares `device` (uploads the program) and reports the launch configuration. */
ISIM_API int isim_handler_launch_info(isim_handler *h, int device, isim_launch_info *out);
/* Map of stats slots to the graph: slot -> call-site id (document order) and
 * callee service index.  Arrays of info.n_slots entries. */
ISIM_API int isim_handler_slots(const isim_handler *h, int32_t *slot_site, int32_t *slot_callee);

/* Serve n_traces requests (trace ids [trace_begin, trace_begin+n_traces)) on
 * the current HIP device, asynchronously on `hip_stream` (a hipStream_t, NULL =
 * default stream).  d_records: device array of n_traces records or NULL.
 * d_stats: device array of info.stats_words u64; ACCUMULATED into (zero it
 * first; ~min word starts at 0).  No host synchronisation, no allocation:
 * graph-capturable after the first call on a device.
 * Concurrency limit: the walk kernels claim batches from per-launch queue
 * sets (and draw-stream kernels stage their per-site 500 counts in per-launch
 * u32 rows, folded into d_stats by the launch's last kernel) that rotate
 * over 256 sets per (handler, device); at most 256 launches
 * of one handler may be in flight on one device at once (launches on ONE
 * stream are ordered and never collide; with more than 256 streams in
 * flight, order them with events or use one handler per stream).  A lane tree
 * walk deeper than its register frames (16 calling invocations on narrow
 * trees, fewer on wide ones) spills frames to one of up to 4 areas per
 * (handler, device), each allocated when a stream first needs it: each such
 * launch waits for the previous launch that used its area (an event recorded
 * after every spilling launch), so launches on different streams never share
 * frames.  A spilling walk cannot be graph-captured: on a capturing stream it
 * returns ISIM_EINVAL. */
ISIM_API int isim_serve_device(isim_handler *h, uint64_t trace_begin, uint64_t n_traces,
                      isim_trace_rec *d_records, uint64_t *d_stats, void *hip_stream);

/* Synchronous convenience: host buffers (either may be NULL), device `device`. */
ISIM_API int isim_serve(isim_handler *h, int device, uint64_t trace_begin, uint64_t n_traces,
               isim_trace_rec *h_records, uint64_t *h_stats);

/* Fold a stats buffer into per-service / per-call-site counters:
 * svc_calls[n_services] = incoming requests (RecordRequestReceived),
 * svc_errs[n_services]  = responses with code 500 (RecordResponseSent),
 * site_calls[n_sites]   = executed calls per call command (RecordRequestSent).
 * Any output may be NULL. */
ISIM_API int isim_stats_fold(const isim_handler *h, const uint64_t *stats, uint64_t *svc_calls,
                    uint64_t *svc_errs, uint64_t *site_calls);

/* Per-service invocation-duration histograms (RecordResponseSent's duration
 * observation, prometheus/handler.go:101-106, made at handler.go:56-58):
 * svc_dur[n_services][ISIM_SVC_DUR_WORDS] = per service [code][33] bucket
 * counts (non-cumulative; code 0 = 200, 1 = 500) then the [code] sums in ns.
 * ISIM_EINVAL when the handler was created with ISIM_FLAG_NO_SVC_DUR for a
 * dynamic walk. */
ISIM_API int isim_stats_fold_durations(const isim_handler *h, const uint64_t *stats, uint64_t *svc_dur);

/* ---- per-replica worker-pool DES (BASELINE config 5) ----
 * Open-loop Poisson arrivals of the client requests at the entry; every
 * replica of a service (svc.Service.NumReplicas, convert/pkg/graph/svc/
 * service.go:30-31) is a FIFO queue in front of ONE worker, held for the
 * invocation's sleep total; an invocation's script (Handler.ServeHTTP,
 * handler.go:37-79) starts when the worker takes it.  Statuses, hops and
 * call counters are those of the walk; latencies and the per-service
 * durations include queueing; in mode B a failed call step ends its script
 * there (the worker hold stays the sleep total).  Exact (bit-identical to the
 * sequential event-driven oracle) for the DES graph class of DESIGN.md
 * §10.1: static walks of at most 2^24 invocations and 65536 replicas per
 * service, and dynamic walks (probabilistic calls; in mode B, a step after
 * one that can fail) whose lane-tree-walk tree was built
 * (isim_des_info.items; isim_des_info_get returns ISIM_EINVAL with the
 * reason otherwise).  Times
 * are kept per trace relative to its arrival: in 32-bit rows by default;
 * a batch with a latency of 2^31 ns (2.1 s) or more is then not accumulated
 * (ISIM_ST_DES_RETRY counts it) and must be rerun with ISIM_DES_FLAG_WIDE
 * (64-bit rows).  A graph whose call-step
 * schedule is cyclic (a service with sleeps invoked both inside a caller's
 * call step and after it) runs as passes to a fixed point; its batches
 * synchronize hip_stream once per pass. */
#define ISIM_DES_FLAG_WIDE 1u    /* 64-bit rows: any latency */
typedef struct {
  uint64_t mean_interarrival_ns; /* 1 .. 2^34: mean gap of the exponential arrivals */
  uint32_t flags;                /* 0 or ISIM_DES_FLAG_WIDE */
  uint32_t reserved;             /* must be 0 */
} isim_des_params;

typedef struct {
  int32_t n_positions;           /* invocations per trace */
  int32_t n_levels;              /* depth of the invocation tree */
  int32_t max_width;             /* widest level */
  int32_t table_rows;            /* rows of the DES table (reachable services) */
  int32_t n_fused;               /* leaf positions finished in their queue pass (no up pass) */
  int32_t cyclic;                /* 1: the call-step schedule is cyclic (fixed-point passes) */
  int32_t row_reads;             /* rows one trace's batch reads (queue + finish passes, one pass), 4 or 8 B each */
  int32_t row_writes;            /* rows it writes (the algorithmic bytes of bench.py's roofline) */
  int32_t items;                 /* 1: a dynamic walk (probabilistic calls, mode-B aborts) on the item engine (DESIGN.md
                                    §10.9): positions are the tree's POTENTIAL invocations, a batch simulates the
                                    executed ones and synchronizes hip_stream at its item count and bucket sizes,
                                    once per sort round whose arrival range it reads back, and (a cyclic schedule)
                                    once per quiet pass — isim_des_last_batch reports the count */
} isim_des_info;

ISIM_API int isim_des_info_get(const isim_handler *h, isim_des_info *out);

/* The item engine's (isim_des_info.items) last batch served through this
 * handler, on any device, for reports: passes over the rounds (a cyclic
 * schedule's quiet passes and the recording pass; 1 otherwise), host
 * synchronisations of hip_stream (the item count, bucket sizes, each sort
 * round's arrival range, each quiet pass's change flag), executed
 * invocations.  Zero before the first item-engine batch. */
typedef struct {
  uint32_t passes;
  uint32_t syncs;
  uint64_t items;
} isim_des_batch_stats;
ISIM_API int isim_des_last_batch(const isim_handler *h, isim_des_batch_stats *out);
/* Device workspace a batch of n_traces needs (either row width: 8 B per invocation per trace + ~40 B per trace). */
ISIM_API int isim_des_workspace_bytes(const isim_handler *h, uint64_t n_traces, uint64_t *bytes);
/* One DES batch (trace ids [trace_begin, trace_begin+n_traces), arrivals from
 * time 0, all replicas idle) on the current device, asynchronously on
 * hip_stream.  d_records may be NULL; d_stats (info.stats_words) and
 * d_des_table (table_rows * ISIM_DES_ROW_WORDS) are ACCUMULATED into. */
ISIM_API int isim_serve_des_device(isim_handler *h, const isim_des_params *p, uint64_t trace_begin,
                          uint64_t n_traces, isim_trace_rec *d_records, uint64_t *d_stats,
                          uint64_t *d_des_table, void *d_workspace, uint64_t workspace_bytes,
                          void *hip_stream);
/* Synchronous convenience: host buffers (any may be NULL). */
ISIM_API int isim_serve_des(isim_handler *h, int device, const isim_des_params *p, uint64_t trace_begin,
                   uint64_t n_traces, isim_trace_rec *h_records, uint64_t *h_stats, uint64_t *h_des_table);
/* DES table rows -> svc_rows[n_services][ISIM_DES_ROW_WORDS] (zero for unreachable services). */
ISIM_API int isim_des_fold(const isim_handler *h, const uint64_t *des_table, uint64_t *svc_rows);
/* Test hook (no reference counterpart): the polls a DES queue pass's decoupled
 * look-back makes for an earlier tile before it fails the batch (device
 * fault flag; default 2^26, never reached in practice).  0 makes every
 * look-back fail at once, so tests can drive the error path.  Process-wide; read at each DES launch. */
ISIM_API void isim_debug_set_spin_limit(uint32_t polls);
ISIM_API uint32_t isim_debug_spin_limit(void);

/* ---- multi-device: trace shards + one RCCL all-reduce ----
 * north_star: traces shard evenly across the GPUs of a node; the histograms
 * and counters merge with one RCCL all-reduce over xGMI.  An isim_multi is an
 * RCCL communicator with one or more LOCAL devices: one process per GPU
 * (isim_multi_init_rank, the id exchanged out of band, e.g. by the Go host)
 * or one process driving several GPUs (isim_multi_init_all).  Global rank r
 * walks the shard [trace_begin + r*n_per_rank, +n_per_rank); Philox keys use
 * the global trace id, so any rank count gives identical per-trace results.
 * The merge is SUM over every stats word except [~min, max], which merge by
 * MAX; DES tables (isim_des_table_allreduce_device) SUM except
 * ISIM_DES_MAX_WAIT (MAX).  RCCL is loaded at run time (dlopen of
 * librccl.so.1) on the first isim_multi_* call; ISIM_ECOMM if it cannot be. */
typedef struct isim_multi isim_multi;
typedef struct {
  char internal[128];            /* an ncclUniqueId */
} isim_multi_id;
/* New communicator id (on ONE process; send its 128 bytes to every rank). */
ISIM_API int isim_multi_get_id(isim_multi_id *id);
/* Local checks a rank makes BEFORE the collective creation, so that the
 * ranks can agree on them out of band first: RCCL loads and `device` can be
 * selected.  No communication. */
ISIM_API int isim_multi_precheck(int device);
/* This process is rank `rank` of n_ranks, on HIP device `device` (ncclCommInitRank; collective over the ranks).
 * Created non-blocking (ncclCommInitRankConfig, blocking = 0) when RCCL has it, and polled: if the
 * peers do not all arrive within ISIM_MULTI_TIMEOUT_S seconds (environment, default 120) the
 * communicator is aborted and ISIM_ECOMM returned.  Collectives and isim_serve_multi's wait are polled
 * the same way (hipStreamQuery + ncclCommGetAsyncError), so a rank whose peer aborted or never came
 * returns ISIM_ECOMM instead of waiting forever. */
ISIM_API int isim_multi_init_rank(const isim_multi_id *id, int n_ranks, int rank, int device, isim_multi **out);
/* One process, n_devices local devices = ranks 0..n-1 in the order given (ncclCommInitAll). */
ISIM_API int isim_multi_init_all(const int *devices, int n_devices, isim_multi **out);
ISIM_API void isim_multi_free(isim_multi *m);
/* Aborts the communicator (ncclCommAbort on every local comm): a rank that
 * fails before a collective calls it so that its peers' pending or next
 * collectives fail with ISIM_ECOMM instead of waiting forever.  The handle
 * is then only good for isim_multi_free; collectives on it return ECOMM. */
ISIM_API int isim_multi_abort(isim_multi *m);
ISIM_API int isim_multi_info(const isim_multi *m, int *n_ranks, int *n_local, int *first_rank);
/* In-place all-reduce of the stats buffers of the local devices (d_stats[i]
 * on local device i, enqueued on hip_streams[i]; hip_streams may be NULL =
 * default streams).  Asynchronous; collective over all ranks. */
ISIM_API int isim_stats_allreduce_device(const isim_handler *h, isim_multi *m, uint64_t *const *d_stats,
                                void *const *hip_streams);
/* The same for DES tables (n_reachable * ISIM_DES_ROW_WORDS words each). */
ISIM_API int isim_des_table_allreduce_device(const isim_handler *h, isim_multi *m, uint64_t *const *d_tables,
                                    void *const *hip_streams);
/* Synchronous sharded batch: every local device walks its rank's shard; the
 * merged stats (identical on every rank) go to h_stats, the local shards'
 * records (n_local * n_per_rank, local device order) to h_records; either may
 * be NULL.  Collective over all ranks.  A local HIP failure before the
 * all-reduce aborts the communicator when it has remote ranks
 * (isim_multi_abort), so the peers return ECOMM rather than hang. */
ISIM_API int isim_serve_multi(isim_handler *h, isim_multi *m, uint64_t trace_begin, uint64_t n_per_rank,
                     isim_trace_rec *h_records, uint64_t *h_stats);
/* Host-side merges (the same rules): dst += src. */
ISIM_API int isim_stats_merge(const isim_handler *h, uint64_t *dst, const uint64_t *src);
ISIM_API int isim_des_table_merge(const isim_handler *h, uint64_t *dst, const uint64_t *src);

#ifdef __cplusplus
}
#endif
#endif /* ISIM_H */
