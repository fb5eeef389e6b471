/*
 * isim_oracle.c — CPU oracle of the isotope script executor in virtual time.
 * TEST INFRASTRUCTURE ONLY: used by tests/ as the parity checker and by
 * bench.py as the "port" cpu_baseline.  Never linked into the product.
 *
 * Plain-C restatement, one request trace at a time, of
 *   Handler.ServeHTTP            isotope/service/pkg/srv/handler.go:37-79
 *   execute                      isotope/service/pkg/srv/executable.go:43-76
 *   executeSleepCommand          executable.go:78-82   (virtual t += max(d,0))
 *   shouldSkipRequest            executable.go:84-90   (Philox draw, EXT)
 *   executeRequestCommand        executable.go:94-144  (H + T(callee); 500 swallowed in mode A)
 *   executeConcurrentCommand     executable.go:148-179 (max over children, OR of errors)
 *   prometheus.Record*           srv/prometheus/handler.go:87-106
 * under "isim semantics v1" (DESIGN.md §2).  It walks the *service graph*
 * recursively, exactly as the reference recursion over HTTP does; it shares no
 * code or data layout with the product's flattened program.
 *
 * Parallel over traces with OpenMP (each thread keeps private stats that are
 * summed at the end), so it doubles as the multi-core CPU baseline.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { K_SLEEP = 0, K_CALL = 1, K_CONC = 2 };

typedef struct {
    int32_t kind;      /* K_SLEEP / K_CALL / K_CONC */
    int32_t site;      /* K_CALL: call-site id */
    int32_t k;         /* K_CALL: index of this call command in the script */
    int32_t sub_off;   /* K_CONC: first sub-command in cmds[] */
    int32_t sub_len;   /* K_CONC: number of sub-commands */
    int32_t pad;
    int64_t sleep_ns;  /* K_SLEEP */
} ocmd;

typedef struct {
    int32_t n_services, n_sites;
    const uint64_t *thr;        /* [n_services] error threshold (2^32 = always) */
    const int32_t *step_off;    /* [n_services] */
    const int32_t *step_len;    /* [n_services] */
    const ocmd *cmds;           /* steps and concurrent sub-commands */
    const int32_t *site_callee; /* [n_sites] */
    const int32_t *site_prob;   /* [n_sites] 0..100 */
    const uint64_t *site_hop;   /* [n_sites] H = hop cost in ns (precomputed by the caller) */
} ograph;

typedef struct {
    uint64_t seed;
    int32_t error_mode;         /* 0 = A (reference), 1 = B (propagate) */
    int32_t entry;
} oparams;

/* Stats layout (u64 words):
 * [0] n_traces [1] sum_latency [2] sum_hops [3] sum_err_hops [4] n_500
 * [5] min_latency [6] max_latency
 * [8 .. 8+2*33)    latency prometheus buckets [status][33]
 * [74 .. 74+2*64)  latency log2 buckets [status][64]
 * [202 .. +n_services) svc_calls, then svc_errs [n_services], then site_calls [n_sites]
 * then svc_dur [n_services][68]: per service, invocation durations on the
 *   Prometheus duration buckets [code 200|500][33] + duration sums [2] in ns
 *   (RecordResponseSent, prometheus/handler.go:101-106, observed at
 *   handler.go:56-58 with the invocation's own duration)
 */
#define ST_HDR 8
#define N_PROM 33
#define N_LOG2 64
#define ST_PROM ST_HDR
#define ST_LOG2 (ST_PROM + 2 * N_PROM)
#define ST_SVC (ST_LOG2 + 2 * N_LOG2)
#define SVC_DUR_WORDS (2 * N_PROM + 2)

static const uint64_t PROM_EDGES_NS[32] = {
    7000000ull, 8000000ull, 9000000ull, 10000000ull, 11000000ull, 12000000ull, 14000000ull,
    16000000ull, 18000000ull, 20000000ull, 25000000ull, 30000000ull, 35000000ull, 40000000ull,
    45000000ull, 50000000ull, 60000000ull, 70000000ull, 80000000ull, 90000000ull, 100000000ull,
    120000000ull, 140000000ull, 160000000ull, 180000000ull, 200000000ull, 250000000ull,
    300000000ull, 350000000ull, 400000000ull, 450000000ull, 500000000ull};

static int prom_bucket(uint64_t T) {
    for (int j = 0; j < 32; ++j)
        if (T <= PROM_EDGES_NS[j]) return j;
    return 32;
}

static void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

void isim_oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    memcpy(out, ctr, 16);
    philox(out, key[0], key[1]);
}

typedef struct {
    const ograph *g;
    const oparams *p;
    uint64_t *st;
    uint64_t t;
    uint32_t next_hop, err_hops;
    uint32_t cblk, cvalid;       /* cache of the last error-draw block */
    uint32_t cw[4];
} tstate;

/* error draw of hop h: word (h&3) of philox((t_lo,t_hi,h>>2,0), seed) */
static uint32_t err_draw(tstate *s, uint32_t h) {
    if (!s->cvalid || s->cblk != (h >> 2)) {
        uint32_t c[4] = {(uint32_t)s->t, (uint32_t)(s->t >> 32), h >> 2, 0};
        philox(c, (uint32_t)s->p->seed, (uint32_t)(s->p->seed >> 32));
        memcpy(s->cw, c, 16);
        s->cblk = h >> 2;
        s->cvalid = 1;
    }
    return s->cw[h & 3];
}

/* shouldSkipRequest (executable.go:84-90) with Intn(100) := draw % 100 */
static int skip_call(tstate *s, uint32_t hop, int32_t k, int32_t q) {
    if (q == 0 || q >= 100) return 0;
    uint32_t c[4] = {(uint32_t)s->t, (uint32_t)(s->t >> 32), hop, 1u + ((uint32_t)k >> 2)};
    philox(c, (uint32_t)s->p->seed, (uint32_t)(s->p->seed >> 32));
    return (c[k & 3] % 100u) < (uint32_t)(100 - q);
}

static uint64_t invoke(tstate *s, int32_t svc, int *err_out);

static uint64_t call(tstate *s, const ocmd *c, uint32_t hop, int *executed, int *err) {
    const ograph *g = s->g;
    *executed = 0;
    *err = 0;
    if (skip_call(s, hop, c->k, g->site_prob[c->site])) return 0;
    int e = 0;
    uint64_t tc = invoke(s, g->site_callee[c->site], &e);
    s->st[ST_SVC + 2 * (uint64_t)g->n_services + (uint64_t)c->site] += 1;  /* RecordRequestSent */
    *executed = 1;
    *err = e;
    return g->site_hop[c->site] + tc;
}

static uint64_t invoke(tstate *s, int32_t svc, int *err_out) {
    const ograph *g = s->g;
    uint32_t hop = s->next_hop++;
    s->st[ST_SVC + svc] += 1;                     /* RecordRequestReceived */
    uint64_t thr = g->thr[svc];
    /* the respond-point draw is keyed by (t, hop); drawing it here, in hop
     * order, lets consecutive hops share a Philox block */
    int own = thr >= (1ull << 32) ? 1 : (thr > 0 ? (uint64_t)err_draw(s, hop) < thr : 0);
    uint64_t T = 0;
    int failed = 0;
    const ocmd *steps = g->cmds + g->step_off[svc];
    for (int32_t i = 0; i < g->step_len[svc] && !failed; ++i) {
        const ocmd *c = &steps[i];
        if (c->kind == K_SLEEP) {
            T += c->sleep_ns > 0 ? (uint64_t)c->sleep_ns : 0;
        } else if (c->kind == K_CALL) {
            int ex, e;
            T += call(s, c, hop, &ex, &e);
            if (s->p->error_mode == 1 && e) failed = 1;
        } else {
            uint64_t m = 0;
            int cerr = 0;
            for (int32_t j = 0; j < c->sub_len; ++j) {
                const ocmd *x = &g->cmds[c->sub_off + j];
                uint64_t dt;
                if (x->kind == K_SLEEP) {
                    dt = x->sleep_ns > 0 ? (uint64_t)x->sleep_ns : 0;
                } else {
                    int ex, e;
                    dt = call(s, x, hop, &ex, &e);
                    if (s->p->error_mode == 1 && e) cerr = 1;
                }
                if (dt > m) m = dt;
            }
            T += m;
            if (cerr) failed = 1;
        }
    }
    int err = failed ? 1 : own;
    if (err) {
        s->st[ST_SVC + g->n_services + svc] += 1;
        s->err_hops += 1;
    }
    uint64_t *dur = s->st + ST_SVC + 2 * (uint64_t)g->n_services + (uint64_t)g->n_sites +
                    (uint64_t)svc * SVC_DUR_WORDS;
    dur[err * N_PROM + prom_bucket(T)] += 1;
    dur[2 * N_PROM + err] += T;
    *err_out = err;
    return T;
}

uint64_t isim_oracle_stats_words(int32_t n_services, int32_t n_sites) {
    return ST_SVC + 2 * (uint64_t)n_services + (uint64_t)n_sites + (uint64_t)n_services * SVC_DUR_WORDS;
}

/* records: 16 B per trace {u64 latency, u32 hops, u32 (status500<<31)|err_hops}
 * (may be NULL); stats: isim_oracle_stats_words() u64, zeroed by the caller. */
int isim_oracle_run(const ograph *g, const oparams *p, uint64_t trace_begin, uint64_t n_traces,
                    uint64_t *records, uint64_t *stats, int n_threads) {
    uint64_t words = isim_oracle_stats_words(g->n_services, g->n_sites);
    stats[5] = ~0ull;
#ifdef _OPENMP
    if (n_threads <= 0) n_threads = omp_get_max_threads();
#else
    n_threads = 1;
#endif
    uint64_t *priv = (uint64_t *)calloc((size_t)n_threads * words, sizeof(uint64_t));
    if (!priv) return 2;
    for (int i = 0; i < n_threads; ++i) priv[(size_t)i * words + 5] = ~0ull;
#ifdef _OPENMP
#pragma omp parallel num_threads(n_threads)
#endif
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        uint64_t *st = priv + (size_t)tid * words;
        tstate s;
        memset(&s, 0, sizeof(s));
        s.g = g;
        s.p = p;
        s.st = st;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 256)
#endif
        for (int64_t i = 0; i < (int64_t)n_traces; ++i) {
            s.t = trace_begin + (uint64_t)i;
            s.next_hop = 0;
            s.err_hops = 0;
            s.cvalid = 0;
            int e = 0;
            uint64_t T = invoke(&s, p->entry, &e);
            if (records) {
                records[2 * i] = T;
                records[2 * i + 1] = (uint64_t)s.next_hop | ((uint64_t)(((uint32_t)e << 31) | s.err_hops) << 32);
            }
            st[0] += 1;
            st[1] += T;
            st[2] += s.next_hop;
            st[3] += s.err_hops;
            st[4] += (uint64_t)e;
            if (T < st[5]) st[5] = T;
            if (T > st[6]) st[6] = T;
            st[ST_PROM + e * N_PROM + prom_bucket(T)] += 1;
            int l = T == 0 ? 0 : 64 - __builtin_clzll(T);
            st[ST_LOG2 + e * N_LOG2 + l] += 1;
        }
    }
    for (int i = 0; i < n_threads; ++i) {
        const uint64_t *ps = priv + (size_t)i * words;
        for (uint64_t w = 0; w < words; ++w) {
            if (w == 5) { if (ps[w] < stats[w]) stats[w] = ps[w]; }
            else if (w == 6) { if (ps[w] > stats[w]) stats[w] = ps[w]; }
            else stats[w] += ps[w];
        }
    }
    free(priv);
    return 0;
}
