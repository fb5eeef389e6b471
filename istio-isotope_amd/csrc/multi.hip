// Multi-device serving and the RCCL merge of the statistics (include/isim.h
// "multi-device").
//
// north_star: "Traces shard evenly across the 8 GPUs of one node, and the
// histograms and counters merge with one RCCL all-reduce over xGMI."  The
// reference has no such step (every isotope pod is scraped by its own
// Prometheus, prometheus/handler.go:37-69); here a trace batch is split into
// per-rank shards with no data-path exchange, and the only collective is the
// merge of the u64 stats buffers: SUM over the counters and histograms, MAX
// over the two extrema words (stored as [~min, max] so both merge by MAX).
//
// RCCL is loaded at run time (dlopen) on the first isim_multi_* call, so
// libisim itself does not depend on it; a process that already holds RCCL
// (torch's bundled librccl.so) shares that copy.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/isim.h"

namespace isim {
int set_error(int code, const std::string &msg);  // api.hip
}

static_assert(sizeof(isim_multi_id) == sizeof(ncclUniqueId), "isim_multi_id must hold an ncclUniqueId");

namespace {

// isim_last_error() reads api.hip's thread-local message
int mfail(int code, const std::string &msg) { return isim::set_error(code, msg); }

struct Rccl {
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommInitAll) CommInitAll = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclCommAbort) CommAbort = nullptr;  // optional
  decltype(&ncclCommInitRankConfig) CommInitRankConfig = nullptr;  // optional: non-blocking init
  decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;    // optional: polled waits
  decltype(&ncclAllReduce) AllReduce = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  bool ok = false;
  std::string why;
};

const Rccl &rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void *lib = nullptr;
    for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((lib = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
    if (!lib) {
      r.why = std::string("cannot load RCCL (librccl.so.1): ") + dlerror();
      return;
    }
    auto sym = [&](auto &fn, const char *name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(lib, name));
      return fn != nullptr;
    };
    r.ok = sym(r.GetUniqueId, "ncclGetUniqueId") && sym(r.CommInitRank, "ncclCommInitRank") &&
           sym(r.CommInitAll, "ncclCommInitAll") && sym(r.CommDestroy, "ncclCommDestroy") &&
           sym(r.AllReduce, "ncclAllReduce") && sym(r.GroupStart, "ncclGroupStart") &&
           sym(r.GroupEnd, "ncclGroupEnd") && sym(r.GetErrorString, "ncclGetErrorString");
    if (!r.ok) r.why = "RCCL library lacks an nccl* entry point";
    (void)sym(r.CommAbort, "ncclCommAbort");
    (void)sym(r.CommInitRankConfig, "ncclCommInitRankConfig");
    (void)sym(r.CommGetAsyncError, "ncclCommGetAsyncError");
  });
  return r;
}

#define RCCLCHK(expr)                                                                        \
  do {                                                                                       \
    ncclResult_t e_ = (expr);                                                                \
    if (e_ != ncclSuccess) return mfail(ISIM_ECOMM, std::string(#expr) + ": " + R.GetErrorString(e_)); \
  } while (0)

#define HIPCHK(expr)                                                                         \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess) return mfail(ISIM_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// Inside ncclGroupStart..ncclGroupEnd: an error closes the group and restores
// the caller's device before returning (an open group would swallow the next
// collective of this thread).
#define GRPCHK(expr)                                                                         \
  do {                                                                                       \
    ncclResult_t e_ = (expr);                                                                \
    if (e_ != ncclSuccess) {                                                                 \
      (void)R.GroupEnd();                                                                    \
      (void)hipSetDevice(prev);                                                              \
      return mfail(ISIM_ECOMM, std::string(#expr) + ": " + R.GetErrorString(e_));            \
    }                                                                                        \
  } while (0)

// Gathers / scatters word `w` of each `row_words`-word row (the DES table's
// MAX word) so that it can be all-reduced with MAX apart from the SUM of the
// table.
__global__ void gather_words(const uint64_t *tab, uint64_t *out, uint32_t rows, uint32_t row_words, uint32_t w) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < rows) out[i] = tab[(uint64_t)i * row_words + w];
}
__global__ void scatter_words(uint64_t *tab, const uint64_t *in, uint32_t rows, uint32_t row_words, uint32_t w) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < rows) tab[(uint64_t)i * row_words + w] = in[i];
}

// How long a rank waits for its peers (communicator creation, a collective)
// before it aborts the communicator and returns ISIM_ECOMM: a peer that failed
// locally before entering a collective never arrives, and over xGMI nothing
// else tells the waiting rank.  ISIM_MULTI_TIMEOUT_S (seconds), default 120.
double multi_timeout_s() {
  const char *e = std::getenv("ISIM_MULTI_TIMEOUT_S");
  const double v = e ? std::atof(e) : 0.0;
  return v > 0 ? v : 120.0;
}

}  // namespace

struct isim_multi {
  int n_ranks = 0;                 // ranks of the communicator (all processes)
  int first_rank = 0;              // global rank of local device 0
  std::vector<int> devices;        // local devices, in rank order
  std::vector<ncclComm_t> comms;   // one per local device
  std::vector<uint64_t *> scratch; // per local device: MAX-word staging of a DES table (grown on demand)
  std::vector<uint64_t> scratch_words;
  bool aborted = false;            // isim_multi_abort: comms aborted, handle only freeable
  bool nonblocking = false;        // comms created with blocking = 0: calls may return ncclInProgress
  ~isim_multi() {
    const Rccl &R = rccl();
    for (size_t i = 0; i < comms.size(); ++i) {
      if (hipSetDevice(devices[i]) == hipSuccess && scratch[i]) (void)hipFree(scratch[i]);
      if (comms[i] && R.ok) (void)R.CommDestroy(comms[i]);
    }
  }
};

namespace {

int stats_words_of(const isim_handler *h, uint64_t &words, uint32_t &rows) {
  isim_handler_info info;
  const int rc = isim_handler_info_get(h, &info);
  if (rc != ISIM_OK) return rc;
  words = info.stats_words;
  rows = (uint32_t)info.n_reachable;
  return ISIM_OK;
}

// Waits until no local communicator of m is ncclInProgress (a non-blocking
// communicator's init, or the enqueue of a group), polling
// ncclCommGetAsyncError; on an asynchronous error or after the timeout the
// communicator is aborted and ISIM_ECOMM returned.
int settle(isim_multi *m, const char *what) {
  const Rccl &R = rccl();
  if (!m->nonblocking || !R.CommGetAsyncError) return ISIM_OK;
  const auto t0 = std::chrono::steady_clock::now();
  const double limit = multi_timeout_s();
  for (;;) {
    bool pending = false;
    for (ncclComm_t c : m->comms) {
      if (!c) continue;
      ncclResult_t a = ncclSuccess;
      const ncclResult_t q = R.CommGetAsyncError(c, &a);
      if (q != ncclSuccess || (a != ncclSuccess && a != ncclInProgress)) {
        const std::string why = R.GetErrorString(q != ncclSuccess ? q : a);
        (void)isim_multi_abort(m);
        return mfail(ISIM_ECOMM, std::string(what) + ": " + why);
      }
      pending = pending || a == ncclInProgress;
    }
    if (!pending) return ISIM_OK;
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
      (void)isim_multi_abort(m);
      return mfail(ISIM_ECOMM, std::string(what) + ": no answer from the peer ranks within ISIM_MULTI_TIMEOUT_S");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

// Waits for the local streams after a collective: hipStreamQuery polled
// beside ncclCommGetAsyncError, so that a peer that aborted (or never came)
// ends this rank's wait with ISIM_ECOMM after the timeout instead of a
// hipStreamSynchronize that never returns.  Returns the first failure.
int wait_streams(isim_multi *m, const std::vector<void *> &streams) {
  const Rccl &R = rccl();
  const auto t0 = std::chrono::steady_clock::now();
  const double limit = multi_timeout_s();
  std::vector<bool> done(streams.size(), false);
  for (;;) {
    bool all = true;
    for (size_t i = 0; i < streams.size(); ++i) {
      if (done[i]) continue;
      if (hipSetDevice(m->devices[i]) != hipSuccess) return mfail(ISIM_EHIP, "hipSetDevice failed");
      const hipError_t q = hipStreamQuery((hipStream_t)streams[i]);
      if (q == hipSuccess) {
        done[i] = true;
        continue;
      }
      if (q != hipErrorNotReady) return mfail(ISIM_EHIP, std::string("walk or all-reduce failed: ") + hipGetErrorString(q));
      all = false;
      if (R.CommGetAsyncError && m->comms[i]) {
        ncclResult_t a = ncclSuccess;
        if (R.CommGetAsyncError(m->comms[i], &a) == ncclSuccess && a != ncclSuccess && a != ncclInProgress) {
          (void)isim_multi_abort(m);
          return mfail(ISIM_ECOMM, std::string("all-reduce: ") + R.GetErrorString(a));
        }
      }
    }
    if (all) return ISIM_OK;
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
      (void)isim_multi_abort(m);
      return mfail(ISIM_ECOMM, "all-reduce: no answer from the peer ranks within ISIM_MULTI_TIMEOUT_S");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
}

}  // namespace

extern "C" {

int isim_multi_get_id(isim_multi_id *id) {
  if (!id) return mfail(ISIM_EINVAL, "null argument");
  const Rccl &R = rccl();
  if (!R.ok) return mfail(ISIM_ECOMM, R.why);
  ncclUniqueId u;
  RCCLCHK(R.GetUniqueId(&u));
  std::memcpy(id, &u, sizeof(u));
  return ISIM_OK;
}

int isim_multi_init_rank(const isim_multi_id *id, int n_ranks, int rank, int device, isim_multi **out) {
  if (!id || !out || n_ranks < 1 || rank < 0 || rank >= n_ranks || device < 0)
    return mfail(ISIM_EINVAL, "bad argument");
  const Rccl &R = rccl();
  if (!R.ok) return mfail(ISIM_ECOMM, R.why);
  int prev = 0;
  HIPCHK(hipGetDevice(&prev));
  HIPCHK(hipSetDevice(device));
  isim_multi *m = new (std::nothrow) isim_multi();
  if (!m) return mfail(ISIM_ENOMEM, "out of memory");
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  // non-blocking when RCCL offers it: the creation is polled with a timeout,
  // so a peer that failed before reaching its own init cannot hold this rank
  // inside ncclCommInitRank forever
  const bool nb = R.CommInitRankConfig && R.CommGetAsyncError;
  ncclResult_t e;
  if (nb) {
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    e = R.CommInitRankConfig(&c, n_ranks, u, rank, &cfg);
  } else {
    e = R.CommInitRank(&c, n_ranks, u, rank);
  }
  (void)hipSetDevice(prev);
  if (e != ncclSuccess && !(nb && e == ncclInProgress)) {
    if (c && R.CommAbort) (void)R.CommAbort(c);
    delete m;
    return mfail(ISIM_ECOMM, std::string("ncclCommInitRank: ") + R.GetErrorString(e));
  }
  m->n_ranks = n_ranks;
  m->first_rank = rank;
  m->devices = {device};
  m->comms = {c};
  m->scratch = {nullptr};
  m->scratch_words = {0};
  m->nonblocking = nb;
  if (const int rc = settle(m, "ncclCommInitRank")) {
    delete m;
    return rc;
  }
  *out = m;
  return ISIM_OK;
}

int isim_multi_init_all(const int *devices, int n_devices, isim_multi **out) {
  if (!devices || !out || n_devices < 1) return mfail(ISIM_EINVAL, "bad argument");
  const Rccl &R = rccl();
  if (!R.ok) return mfail(ISIM_ECOMM, R.why);
  isim_multi *m = new (std::nothrow) isim_multi();
  if (!m) return mfail(ISIM_ENOMEM, "out of memory");
  m->devices.assign(devices, devices + n_devices);
  m->comms.assign(n_devices, nullptr);
  m->scratch.assign(n_devices, nullptr);
  m->scratch_words.assign(n_devices, 0);
  int prev = 0;
  (void)hipGetDevice(&prev);
  const ncclResult_t e = R.CommInitAll(m->comms.data(), n_devices, devices);
  (void)hipSetDevice(prev);
  if (e != ncclSuccess) {
    m->comms.assign(n_devices, nullptr);
    delete m;
    return mfail(ISIM_ECOMM, std::string("ncclCommInitAll: ") + R.GetErrorString(e));
  }
  m->n_ranks = n_devices;
  m->first_rank = 0;
  *out = m;
  return ISIM_OK;
}

void isim_multi_free(isim_multi *m) { delete m; }

int isim_multi_precheck(int device) {
  if (device < 0) return mfail(ISIM_EINVAL, "bad argument");
  const Rccl &R = rccl();
  if (!R.ok) return mfail(ISIM_ECOMM, R.why);
  int count = 0, prev = 0;
  HIPCHK(hipGetDeviceCount(&count));
  // checked against the count first: a failed hipSetDevice would leave the
  // error as the thread's last HIP error, for the caller's next HIP check
  if (device >= count) return mfail(ISIM_EHIP, "no HIP device " + std::to_string(device));
  HIPCHK(hipGetDevice(&prev));
  const hipError_t e = hipSetDevice(device);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return mfail(ISIM_EHIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
  }
  return ISIM_OK;
}

int isim_multi_abort(isim_multi *m) {
  if (!m) return mfail(ISIM_EINVAL, "null argument");
  const Rccl &R = rccl();
  if (!m->aborted && R.ok) {
    for (size_t i = 0; i < m->comms.size(); ++i) {
      if (!m->comms[i]) continue;
      if (R.CommAbort) (void)R.CommAbort(m->comms[i]);
      else (void)R.CommDestroy(m->comms[i]);
      m->comms[i] = nullptr;
    }
  }
  m->aborted = true;
  return ISIM_OK;
}

int isim_multi_info(const isim_multi *m, int *n_ranks, int *n_local, int *first_rank) {
  if (!m) return mfail(ISIM_EINVAL, "null argument");
  if (n_ranks) *n_ranks = m->n_ranks;
  if (n_local) *n_local = (int)m->devices.size();
  if (first_rank) *first_rank = m->first_rank;
  return ISIM_OK;
}

int isim_stats_allreduce_device(const isim_handler *h, isim_multi *m, uint64_t *const *d_stats,
                                void *const *hip_streams) {
  if (!h || !m || !d_stats) return mfail(ISIM_EINVAL, "null argument");
  for (size_t i = 0; i < m->devices.size(); ++i)
    if (!d_stats[i]) return mfail(ISIM_EINVAL, "null device buffer");
  uint64_t words = 0;
  uint32_t rows = 0;
  if (const int rc = stats_words_of(h, words, rows)) return rc;
  const Rccl &R = rccl();
  if (m->aborted) return mfail(ISIM_ECOMM, "communicator aborted (isim_multi_abort)");
  int prev = 0;
  HIPCHK(hipGetDevice(&prev));
  RCCLCHK(R.GroupStart());
  for (size_t i = 0; i < m->devices.size(); ++i) {
    uint64_t *s = d_stats[i];
    hipStream_t st = hip_streams ? (hipStream_t)hip_streams[i] : nullptr;
    constexpr uint64_t lo = ISIM_ST_NOT_MIN_LATENCY, hi = ISIM_ST_MAX_LATENCY + 1;
    GRPCHK(R.AllReduce(s, s, lo, ncclUint64, ncclSum, m->comms[i], st));
    GRPCHK(R.AllReduce(s + lo, s + lo, hi - lo, ncclUint64, ncclMax, m->comms[i], st));
    GRPCHK(R.AllReduce(s + hi, s + hi, words - hi, ncclUint64, ncclSum, m->comms[i], st));
  }
  {
    const ncclResult_t e = R.GroupEnd();
    (void)hipSetDevice(prev);
    if (e != ncclSuccess && !(m->nonblocking && e == ncclInProgress))
      return mfail(ISIM_ECOMM, std::string("ncclGroupEnd: ") + R.GetErrorString(e));
  }
  return settle(m, "stats all-reduce");
}

int isim_des_table_allreduce_device(const isim_handler *h, isim_multi *m, uint64_t *const *d_tables,
                                    void *const *hip_streams) {
  if (!h || !m || !d_tables) return mfail(ISIM_EINVAL, "null argument");
  uint64_t words = 0;
  uint32_t rows = 0;
  if (const int rc = stats_words_of(h, words, rows)) return rc;
  if (rows == 0) return ISIM_OK;
  for (size_t i = 0; i < m->devices.size(); ++i)
    if (!d_tables[i]) return mfail(ISIM_EINVAL, "null device buffer");
  if (m->aborted) return mfail(ISIM_ECOMM, "communicator aborted (isim_multi_abort)");
  const Rccl &R = rccl();
  int prev = 0;
  HIPCHK(hipGetDevice(&prev));
  const uint32_t W = ISIM_DES_ROW_WORDS, blocks = (rows + 255) / 256;
  for (size_t i = 0; i < m->devices.size(); ++i) {
    HIPCHK(hipSetDevice(m->devices[i]));
    if (m->scratch_words[i] < rows) {
      if (m->scratch[i]) HIPCHK(hipFree(m->scratch[i]));
      m->scratch[i] = nullptr;
      m->scratch_words[i] = 0;
      HIPCHK(hipMalloc(&m->scratch[i], rows * sizeof(uint64_t)));
      m->scratch_words[i] = rows;
    }
    hipStream_t st = hip_streams ? (hipStream_t)hip_streams[i] : nullptr;
    hipLaunchKernelGGL(gather_words, dim3(blocks), dim3(256), 0, st, d_tables[i], m->scratch[i], rows, W,
                       (uint32_t)ISIM_DES_MAX_WAIT);
    HIPCHK(hipGetLastError());
  }
  RCCLCHK(R.GroupStart());
  for (size_t i = 0; i < m->devices.size(); ++i) {
    hipStream_t st = hip_streams ? (hipStream_t)hip_streams[i] : nullptr;
    GRPCHK(R.AllReduce(d_tables[i], d_tables[i], (size_t)rows * W, ncclUint64, ncclSum, m->comms[i], st));
    GRPCHK(R.AllReduce(m->scratch[i], m->scratch[i], rows, ncclUint64, ncclMax, m->comms[i], st));
  }
  {
    const ncclResult_t e = R.GroupEnd();
    if (e != ncclSuccess && !(m->nonblocking && e == ncclInProgress)) {
      (void)hipSetDevice(prev);
      return mfail(ISIM_ECOMM, std::string("ncclGroupEnd: ") + R.GetErrorString(e));
    }
  }
  if (const int rc = settle(m, "DES table all-reduce")) {
    (void)hipSetDevice(prev);
    return rc;
  }
  for (size_t i = 0; i < m->devices.size(); ++i) {
    HIPCHK(hipSetDevice(m->devices[i]));
    hipStream_t st = hip_streams ? (hipStream_t)hip_streams[i] : nullptr;
    hipLaunchKernelGGL(scatter_words, dim3(blocks), dim3(256), 0, st, d_tables[i], m->scratch[i], rows, W,
                       (uint32_t)ISIM_DES_MAX_WAIT);
    HIPCHK(hipGetLastError());
  }
  (void)hipSetDevice(prev);
  return ISIM_OK;
}

int isim_serve_multi(isim_handler *h, isim_multi *m, uint64_t trace_begin, uint64_t n_per_rank,
                     isim_trace_rec *h_records, uint64_t *h_stats) {
  if (!h || !m) return mfail(ISIM_EINVAL, "null argument");
  uint64_t words = 0;
  uint32_t rows = 0;
  if (const int rc = stats_words_of(h, words, rows)) return rc;
  const size_t L = m->devices.size();
  std::vector<uint64_t *> d_stats(L, nullptr);
  std::vector<isim_trace_rec *> d_rec(L, nullptr);
  std::vector<void *> streams(L, nullptr);
  int prev = 0;
  HIPCHK(hipGetDevice(&prev));
  int rc = ISIM_OK;
  for (size_t i = 0; i < L && rc == ISIM_OK; ++i) {
    hipStream_t s = nullptr;
    if (hipSetDevice(m->devices[i]) != hipSuccess || hipStreamCreate(&s) != hipSuccess) {
      rc = mfail(ISIM_EHIP, "hipStreamCreate failed");
      break;
    }
    streams[i] = s;
    if (hipMalloc(&d_stats[i], words * 8) != hipSuccess || hipMemsetAsync(d_stats[i], 0, words * 8, s) != hipSuccess ||
        (h_records && n_per_rank && hipMalloc(&d_rec[i], n_per_rank * sizeof(isim_trace_rec)) != hipSuccess)) {
      rc = mfail(ISIM_EHIP, "hipMalloc failed");
      break;
    }
    // shard of global rank first_rank + i (isim/dist.py shard_begin with step 0)
    const uint64_t begin = trace_begin + (uint64_t)(m->first_rank + (int)i) * n_per_rank;
    rc = isim_serve_device(h, begin, n_per_rank, d_rec[i], d_stats[i], s);
  }
  // a local failure before the collective: abort the communicator so the
  // peer ranks' all-reduce fails (ECOMM) instead of waiting for this rank
  if (rc != ISIM_OK && m->n_ranks > (int)L) (void)isim_multi_abort(m);
  if (rc == ISIM_OK) rc = isim_stats_allreduce_device(h, m, d_stats.data(), streams.data());
  // polled, not hipStreamSynchronize: a peer that aborted ends the wait (ECOMM)
  if (rc == ISIM_OK) rc = wait_streams(m, streams);
  for (size_t i = 0; i < L && rc == ISIM_OK; ++i) {
    if (hipSetDevice(m->devices[i]) != hipSuccess) {
      rc = mfail(ISIM_EHIP, "hipSetDevice failed");
      break;
    }
    if (i == 0 && h_stats && hipMemcpy(h_stats, d_stats[0], words * 8, hipMemcpyDeviceToHost) != hipSuccess)
      rc = mfail(ISIM_EHIP, "copy stats failed");
    if (rc == ISIM_OK && h_records && d_rec[i] &&
        hipMemcpy(h_records + i * n_per_rank, d_rec[i], n_per_rank * sizeof(isim_trace_rec),
                  hipMemcpyDeviceToHost) != hipSuccess)
      rc = mfail(ISIM_EHIP, "copy records failed");
  }
  for (size_t i = 0; i < L; ++i) {
    if (hipSetDevice(m->devices[i]) != hipSuccess) continue;
    if (streams[i]) (void)hipStreamSynchronize((hipStream_t)streams[i]);
    if (d_rec[i]) (void)hipFree(d_rec[i]);
    if (d_stats[i]) (void)hipFree(d_stats[i]);
    if (streams[i]) (void)hipStreamDestroy((hipStream_t)streams[i]);
  }
  (void)hipSetDevice(prev);
  return rc;
}

int isim_stats_merge(const isim_handler *h, uint64_t *dst, const uint64_t *src) {
  if (!h || !dst || !src) return mfail(ISIM_EINVAL, "null argument");
  uint64_t words = 0;
  uint32_t rows = 0;
  if (const int rc = stats_words_of(h, words, rows)) return rc;
  for (uint64_t w = 0; w < words; ++w)
    dst[w] = (w == ISIM_ST_NOT_MIN_LATENCY || w == ISIM_ST_MAX_LATENCY) ? std::max(dst[w], src[w]) : dst[w] + src[w];
  return ISIM_OK;
}

int isim_des_table_merge(const isim_handler *h, uint64_t *dst, const uint64_t *src) {
  if (!h || !dst || !src) return mfail(ISIM_EINVAL, "null argument");
  uint64_t words = 0;
  uint32_t rows = 0;
  if (const int rc = stats_words_of(h, words, rows)) return rc;
  for (uint64_t w = 0; w < (uint64_t)rows * ISIM_DES_ROW_WORDS; ++w)
    dst[w] = w % ISIM_DES_ROW_WORDS == ISIM_DES_MAX_WAIT ? std::max(dst[w], src[w]) : dst[w] + src[w];
  return ISIM_OK;
}

}  // extern "C"
