/*
 * des_oracle.c — CPU oracle of the per-replica worker-pool DES (BASELINE
 * config 5, DESIGN.md §10 "isim DES semantics v1").  TEST INFRASTRUCTURE
 * ONLY: the parity checker for the product's level-synchronous GPU DES and
 * the "port" cpu_baseline of bench.py --config c5.  Never linked into the
 * product.
 *
 * A plain sequential discrete-event simulation: one global binary heap of
 * invocation ARRIVE events ordered by (time, trace id, hop id); each replica
 * is a FIFO queue in front of one worker, held for the invocation's hold time
 * (its sleep total); an invocation's script starts when the worker takes it;
 * a call step sends its requests when it begins and ends when its last
 * callee finishes, then the script goes on (any number of call steps).  After the heap drains,
 * each trace's finish times, statuses and stats are computed by recursion
 * over the SERVICE GRAPH (as isim_oracle.c's invoke() does), so this shares
 * no code or layout with the product's position arrays and level scans.
 *
 * Probabilistic calls: before the simulation, a walk of each trace (as
 * isim_oracle.c's invoke(): shouldSkipRequest with Intn(100) := draw % 100,
 * hop ids counting EXECUTED invocations in preorder) fixes which calls
 * execute and every executed invocation's hop id; a skipped call sends no
 * request, holds nothing and takes no time.  In mode B (EXT) the walk also
 * draws the errors: a step with a callee that responded 500 fails the script
 * (handler.go:66-75 with the 500 propagated), whose later commands never run
 * — the walk records the command after which each invocation stops, and the
 * simulation responds to the caller there (the worker hold stays the
 * service's sleep total).
 *
 * Reference anchors (the simulated behaviour, not a Go transcription):
 *   Handler.ServeHTTP          isotope/service/pkg/srv/handler.go:37-79
 *   executeRequestCommand      executable.go:94-144  (request -> callee ServeHTTP)
 *   executeConcurrentCommand   executable.go:148-179 (wait for all)
 *   svc.Service.NumReplicas    convert/pkg/graph/svc/service.go:30-31 (replicas behind a service)
 *   prometheus.Record*         srv/prometheus/handler.go:87-106
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { K_SLEEP = 0, K_CALL = 1, K_CONC = 2 };

typedef struct {
    int32_t kind, site, k, sub_off, sub_len, pad;
    int64_t sleep_ns;
} ocmd;

typedef struct {
    int32_t n_services, n_sites;
    const uint64_t *thr;
    const int32_t *step_off;
    const int32_t *step_len;
    const ocmd *cmds;
    const int32_t *site_callee;
    const int32_t *site_prob;
    const uint64_t *site_hop;
} ograph;

typedef struct {
    uint64_t seed;
    int32_t error_mode;
    int32_t entry;
} oparams;

typedef struct {
    uint64_t mean_interarrival_ns;
    const int32_t *replicas;    /* [n_services] numReplicas (values < 1 count as 1) */
} odes;

#define N_PROM 33
#define N_LOG2 64
#define ST_PROM 8
#define ST_LOG2 (ST_PROM + 2 * N_PROM)
#define ST_SVC (ST_LOG2 + 2 * N_LOG2)
#define SVC_DUR_WORDS (2 * N_PROM + 2)
#define DES_ROW 72 /* [code][33] durations, [2] duration sums, count, sum wait, max wait, sum hold */

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

static uint32_t draw(uint64_t seed, uint64_t t, uint32_t w2, uint32_t w3, int word) {
    uint32_t c[4] = {(uint32_t)t, (uint32_t)(t >> 32), w2, w3};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    return c[word];
}

/* ---- exponential inter-arrival times in integer arithmetic */
static int64_t LN_Q24[257];
static int ln_ready = 0;
static void ln_init(void) {
    if (ln_ready) return;
    for (int i = 0; i <= 256; ++i) LN_Q24[i] = llround(log1p(i / 256.0) * 16777216.0);
    ln_ready = 1;
}
void isim_oracle_des_ln_table(int64_t *out) { ln_init(); memcpy(out, LN_Q24, sizeof LN_Q24); }

/* E = -ln(w / 2^24) in Q24 for w = (u >> 8) + 1 in [1, 2^24] */
uint64_t isim_oracle_des_exp_q24(uint32_t u) {
    ln_init();
    const uint32_t w = (u >> 8) + 1u;
    int e = 31 - __builtin_clz(w);              /* 0..24 */
    const uint32_t f = (w << (24 - e)) & 0xFFFFFFu;  /* 24-bit fraction of w / 2^e */
    const uint32_t idx = f >> 16, rem = f & 0xFFFFu;
    const int64_t lnm = LN_Q24[idx] + (((LN_Q24[idx + 1] - LN_Q24[idx]) * (int64_t)rem) >> 16);
    const int64_t LN2_Q24 = 11629080;           /* round(ln 2 * 2^24) */
    return (uint64_t)(24 * LN2_Q24 - (e * LN2_Q24 + lnm));
}

static uint64_t interarrival(const odes *d, uint64_t seed, uint64_t t) {
    const uint32_t u = draw(seed, t, 0u, 0x80000001u, 0);
    return (d->mean_interarrival_ns * isim_oracle_des_exp_q24(u)) >> 24;
}

/* ---- static structure of the graph ---- */
typedef struct {
    const ograph *g;
    const oparams *p;
    const odes *d;
    uint32_t *size;   /* [n_services] invocations in a call of the service (subtree size) */
    uint32_t *ncalls; /* [n_services] call commands of the script (concurrent sub-commands included) */
    uint64_t *hold;   /* [n_services] total sleep */
    int32_t *nrep;
} sctx;

static uint64_t sl(int64_t d) { return d > 0 ? (uint64_t)d : 0; }

static uint32_t subtree(sctx *c, int32_t s) {
    if (c->size[s]) return c->size[s];
    const ograph *g = c->g;
    uint64_t n = 1, hold = 0;
    uint32_t nc = 0;
    for (int32_t i = 0; i < g->step_len[s]; ++i) {
        const ocmd *x = &g->cmds[g->step_off[s] + i];
        if (x->kind == K_SLEEP) hold += sl(x->sleep_ns);
        else if (x->kind == K_CALL) {
            n += subtree(c, g->site_callee[x->site]);
            ++nc;
        } else
            for (int32_t j = 0; j < x->sub_len; ++j) {
                const ocmd *y = &g->cmds[x->sub_off + j];
                if (y->kind == K_SLEEP) hold += sl(y->sleep_ns);
                else {
                    n += subtree(c, g->site_callee[y->site]);
                    ++nc;
                }
            }
    }
    c->ncalls[s] = nc;
    c->size[s] = (uint32_t)n;
    c->hold[s] = hold;
    return (uint32_t)n;
}

/* ---- the executed invocations of one trace (skips; mode B: aborts) ---- */
#define NO_HOP 0xFFFFFFFFu
typedef struct {
    const sctx *c;
    uint64_t t;
    uint32_t next;       /* next hop id = executed invocations so far */
    uint32_t kid_next;
    uint32_t *kid_base;  /* [nodes] per hop: its entries in kid */
    uint32_t *kid;       /* per (hop, call command k): the callee's hop, NO_HOP when skipped or aborted */
    uint32_t *stop;      /* [nodes] per hop: script commands that run (mode B: up to the failed step) */
} pwalk;

/* shouldSkipRequest (executable.go:84-90) with Intn(100) := draw % 100 (isim_oracle.c skip_call) */
static int skip_call(uint64_t seed, uint64_t t, uint32_t hop, int32_t k, int32_t q) {
    if (q == 0 || q >= 100) return 0;
    return draw(seed, t, hop, 1u + ((uint32_t)k >> 2), k & 3) % 100u < (uint32_t)(100 - q);
}

/* own error draw of invocation `hop` of service s (the respond point) */
static int own_error(const sctx *c, uint64_t t, int32_t s, uint32_t hop) {
    const uint64_t thr = c->g->thr[s];
    if (thr >= (1ull << 32)) return 1;
    return thr > 0 && (uint64_t)draw(c->p->seed, t, hop >> 2, 0u, (int)(hop & 3)) < thr;
}

/* *err: the invocation's status 500 (mode B: a failed step or its own error) */
static uint32_t pre_walk(pwalk *w, int32_t s, int *err) {
    const ograph *g = w->c->g;
    const int modeb = w->c->p->error_mode == 1;
    const uint32_t hop = w->next++;
    const uint32_t base = w->kid_next;
    w->kid_base[hop] = base;
    w->kid_next += w->c->ncalls[s];
    int failed = 0;
    uint32_t stop = (uint32_t)g->step_len[s];
    for (int32_t i = 0; i < g->step_len[s]; ++i) {
        const ocmd *x = &g->cmds[g->step_off[s] + i];
        const int32_t nsub = x->kind == K_CONC ? x->sub_len : 1;
        int cerr = 0;
        for (int32_t j = 0; j < nsub; ++j) {
            const ocmd *y = x->kind == K_CONC ? &g->cmds[x->sub_off + j] : x;
            if (y->kind != K_CALL) continue;
            int e = 0;
            w->kid[base + (uint32_t)y->k] =
                failed || skip_call(w->c->p->seed, w->t, hop, y->k, g->site_prob[y->site])
                    ? NO_HOP
                    : pre_walk(w, g->site_callee[y->site], &e);
            cerr |= e;
        }
        if (modeb && cerr && !failed) {  /* the script responds after this step */
            failed = 1;
            stop = (uint32_t)i + 1u;
        }
    }
    w->stop[hop] = stop;
    *err = modeb && (failed || own_error(w->c, w->t, s, hop));  /* mode A: unused, not drawn */
    return hop;
}

/* ---- event heap ---- */
typedef struct {
    uint64_t time, t;
    uint32_t hop;
    int32_t svc;
} ev;

static int ev_less(const ev *a, const ev *b) {
    if (a->time != b->time) return a->time < b->time;
    if (a->t != b->t) return a->t < b->t;
    return a->hop < b->hop;
}

typedef struct {
    ev *v;
    size_t n, cap;
} heap;

static int hpush(heap *h, ev e) {
    if (h->n == h->cap) {
        size_t nc = h->cap ? 2 * h->cap : 1024;
        ev *nv = (ev *)realloc(h->v, nc * sizeof(ev));
        if (!nv) return 0;
        h->v = nv;
        h->cap = nc;
    }
    size_t i = h->n++;
    h->v[i] = e;
    while (i > 0) {
        size_t p = (i - 1) / 2;
        if (!ev_less(&h->v[i], &h->v[p])) break;
        ev tmp = h->v[i]; h->v[i] = h->v[p]; h->v[p] = tmp;
        i = p;
    }
    return 1;
}

static ev hpop(heap *h) {
    ev top = h->v[0];
    h->v[0] = h->v[--h->n];
    size_t i = 0;
    for (;;) {
        size_t l = 2 * i + 1, r = l + 1, m = i;
        if (l < h->n && ev_less(&h->v[l], &h->v[m])) m = l;
        if (r < h->n && ev_less(&h->v[r], &h->v[m])) m = r;
        if (m == i) break;
        ev tmp = h->v[i]; h->v[i] = h->v[m]; h->v[m] = tmp;
        i = m;
    }
    return top;
}

/* ---- per-trace recursion after the simulation ---- */
typedef struct {
    sctx *c;
    const uint64_t *S, *A;  /* [nodes] start and arrival of this trace's invocations */
    const uint32_t *kid_base, *kid;  /* the trace's executed calls (pwalk) */
    uint64_t t;
    uint64_t *st, *des;
    uint32_t err_hops;
} fstate;

/* returns the finish time of invocation (svc, hop); *err = its status 500 */
static uint64_t finish(fstate *f, int32_t s, uint32_t hop, int *err) {
    const sctx *c = f->c;
    const ograph *g = c->g;
    uint64_t *st = f->st;
    st[ST_SVC + s] += 1;  /* RecordRequestReceived */
    uint64_t T = f->S[hop];
    const uint32_t *kid = f->kid + f->kid_base[hop];
    int failed = 0;
    for (int32_t i = 0; i < g->step_len[s] && !failed; ++i) {
        const ocmd *x = &g->cmds[g->step_off[s] + i];
        if (x->kind == K_SLEEP) {
            T += sl(x->sleep_ns);
        } else if (x->kind == K_CALL) {
            int e = 0;
            const uint32_t h = kid[x->k];
            if (h == NO_HOP) continue;  /* skipped: no request, no time */
            T = finish(f, g->site_callee[x->site], h, &e);  /* response at the callee's finish */
            st[ST_SVC + 2 * (uint64_t)g->n_services + (uint64_t)x->site] += 1;
            if (f->c->p->error_mode == 1 && e) failed = 1;
        } else {
            uint64_t m = T;
            int cerr = 0;
            for (int32_t j = 0; j < x->sub_len; ++j) {
                const ocmd *y = &g->cmds[x->sub_off + j];
                uint64_t end;
                if (y->kind == K_SLEEP) {
                    end = T + sl(y->sleep_ns);
                } else {
                    int e = 0;
                    const uint32_t h = kid[y->k];
                    if (h == NO_HOP) continue;
                    end = finish(f, g->site_callee[y->site], h, &e);
                    st[ST_SVC + 2 * (uint64_t)g->n_services + (uint64_t)y->site] += 1;
                    if (f->c->p->error_mode == 1 && e) cerr = 1;
                }
                if (end > m) m = end;
            }
            T = m;
            if (cerr) failed = 1;
        }
    }
    const int e = failed ? 1 : own_error(c, f->t, s, hop);
    if (e) {
        st[ST_SVC + g->n_services + s] += 1;
        f->err_hops += 1;
    }
    const uint64_t dur = T - f->A[hop];  /* request receipt to response (handler.go:56-58) */
    uint64_t *row = f->des + (uint64_t)s * DES_ROW;
    row[e * N_PROM + prom_bucket(dur)] += 1;
    row[2 * N_PROM + e] += dur;
    row[68] += 1;
    const uint64_t w = f->S[hop] - f->A[hop];
    row[69] += w;
    if (w > row[70]) row[70] = w;
    row[71] += c->hold[s];
    *err = e;
    return T;
}

/* ---- per-invocation script progress during the simulation: a call step
 * sends its requests when it begins and ends when its last callee finishes
 * (the response arrives at the callee's finish); the script then goes on */
#define NO_PARENT 0xFFFFFFFFu
typedef struct {
    uint64_t T, runmax;
    uint32_t parent, next, step, pending;
    int32_t svc;
} istate;

typedef struct {
    const sctx *c;
    heap *h;
    istate *is;      /* [n_traces][nodes] */
    uint32_t nodes;
    uint64_t trace_begin;
    const uint32_t *kid_base, *kid;  /* [n_traces][nodes]: the executed calls (pwalk) */
    const uint32_t *stop;            /* [n_traces][nodes]: commands each invocation runs (pwalk) */
} sim;

static int advance(sim *m, uint64_t i, uint32_t hop);

static int notify(sim *m, uint64_t i, uint32_t hop, uint64_t fin) {
    istate *st = &m->is[i * m->nodes + hop];
    if (fin > st->runmax) st->runmax = fin;
    if (--st->pending) return 1;
    st->T = st->runmax;
    return advance(m, i, hop);
}

/* 0: skipped (no request); 1: sent; -1: out of memory */
static int push_call(sim *m, uint64_t i, istate *st, uint32_t hop, const ocmd *x) {
    const ograph *g = m->c->g;
    const int32_t cs = g->site_callee[x->site];
    const uint32_t ch = m->kid[i * m->nodes + m->kid_base[i * m->nodes + hop] + (uint32_t)x->k];
    if (ch == NO_HOP) return 0;
    istate *cst = &m->is[i * m->nodes + ch];
    cst->parent = hop;
    cst->svc = cs;
    ev ce = {st->T + g->site_hop[x->site], m->trace_begin + i, ch, cs};
    st->pending++;
    return hpush(m->h, ce) ? 1 : -1;
}

static int advance(sim *m, uint64_t i, uint32_t hop) {
    const ograph *g = m->c->g;
    istate *st = &m->is[i * m->nodes + hop];
    const int32_t s = st->svc;
    const uint32_t stop = m->stop[i * m->nodes + hop];
    while (st->step < stop) {
        const ocmd *x = &g->cmds[g->step_off[s] + st->step];
        st->step++;
        if (x->kind == K_SLEEP) {
            st->T += sl(x->sleep_ns);
        } else if (x->kind == K_CALL) {
            st->runmax = st->T;
            const int r = push_call(m, i, st, hop, x);
            if (r < 0) return 0;
            if (r > 0) return 1;  /* waits for the callee */
        } else {
            uint64_t smax = 0;
            for (int32_t j = 0; j < x->sub_len; ++j) {
                const ocmd *y = &g->cmds[x->sub_off + j];
                if (y->kind == K_SLEEP && sl(y->sleep_ns) > smax) smax = sl(y->sleep_ns);
            }
            st->runmax = st->T + smax;
            for (int32_t j = 0; j < x->sub_len; ++j) {
                const ocmd *y = &g->cmds[x->sub_off + j];
                if (y->kind == K_CALL && push_call(m, i, st, hop, y) < 0) return 0;
            }
            if (st->pending) return 1;  /* waits for all callees */
            st->T = st->runmax;
        }
    }
    /* the script has ended: respond to the caller */
    if (st->parent != NO_PARENT) return notify(m, i, st->parent, st->T);
    return 1;
}

uint64_t isim_oracle_des_stats_words(int32_t n_services, int32_t n_sites) {
    return ST_SVC + 2 * (uint64_t)n_services + (uint64_t)n_sites;
}

/* records: 16 B per trace {latency, hops | (status500<<31 | err_hops) << 32} or NULL;
 * stats: isim_oracle_des_stats_words() u64, zeroed (~min word handled here);
 * des: [n_services][72] u64, zeroed.  Returns 0, 2 on allocation failure. */
int isim_oracle_des_run(const ograph *g, const oparams *p, const odes *d, uint64_t trace_begin,
                        uint64_t n_traces, uint64_t *records, uint64_t *stats, uint64_t *des) {
    const int32_t n = g->n_services;
    sctx c;
    c.g = g;
    c.p = p;
    c.d = d;
    c.size = (uint32_t *)calloc((size_t)n, sizeof(uint32_t));
    c.ncalls = (uint32_t *)calloc((size_t)n, sizeof(uint32_t));
    c.hold = (uint64_t *)calloc((size_t)n, sizeof(uint64_t));
    if (!c.size || !c.ncalls || !c.hold) return 2;
    const uint32_t nodes = subtree(&c, p->entry);
    /* replica queues: busy-until per (service, replica) */
    uint64_t *qoff = (uint64_t *)calloc((size_t)n + 1, sizeof(uint64_t));
    for (int32_t s = 0; s < n; ++s) qoff[s + 1] = qoff[s] + (uint64_t)(d->replicas[s] > 1 ? d->replicas[s] : 1);
    uint64_t *busy = (uint64_t *)calloc((size_t)qoff[n], sizeof(uint64_t));
    uint64_t *S = (uint64_t *)malloc((size_t)n_traces * nodes * sizeof(uint64_t));
    uint64_t *A = (uint64_t *)malloc((size_t)n_traces * nodes * sizeof(uint64_t));
    uint64_t *arr = (uint64_t *)malloc((size_t)(n_traces ? n_traces : 1) * sizeof(uint64_t));
    heap h = {0, 0, 0};
    if (!qoff || !busy || !S || !A || !arr) return 2;
    /* open-loop arrivals at the entry: A_t = sum of inter-arrival times */
    uint64_t now = 0;
    for (uint64_t i = 0; i < n_traces; ++i) {
        now += interarrival(d, p->seed, trace_begin + i);
        arr[i] = now;
        ev e = {now, trace_begin + i, 0, p->entry};
        if (!hpush(&h, e)) return 2;
    }
    istate *is = (istate *)calloc((size_t)n_traces * nodes, sizeof(istate));
    /* each trace's executed calls and hop ids (every call command of an
     * executed invocation is a distinct potential position: <= nodes entries) */
    uint32_t *kid_base = (uint32_t *)malloc((size_t)(n_traces ? n_traces : 1) * nodes * sizeof(uint32_t));
    uint32_t *kid = (uint32_t *)malloc((size_t)(n_traces ? n_traces : 1) * nodes * sizeof(uint32_t));
    uint32_t *stop = (uint32_t *)malloc((size_t)(n_traces ? n_traces : 1) * nodes * sizeof(uint32_t));
    uint32_t *hops = (uint32_t *)malloc((size_t)(n_traces ? n_traces : 1) * sizeof(uint32_t));
    if (!is || !kid_base || !kid || !stop || !hops) return 2;
    for (uint64_t i = 0; i < n_traces; ++i) {
        is[i * nodes].parent = NO_PARENT;
        is[i * nodes].svc = p->entry;
        pwalk w = {&c, trace_begin + i, 0, 0, kid_base + i * nodes, kid + i * nodes, stop + i * nodes};
        int e = 0;
        (void)pre_walk(&w, p->entry, &e);
        hops[i] = w.next;
    }
    sim m = {&c, &h, is, nodes, trace_begin, kid_base, kid, stop};
    while (h.n) {
        const ev e = hpop(&h);
        const uint64_t i = e.t - trace_begin;
        const int32_t s = e.svc;
        const int32_t R = d->replicas[s] > 1 ? d->replicas[s] : 1;
        const uint32_t r = R > 1 ? draw(p->seed, e.t, e.hop, 0x80000002u, 0) % (uint32_t)R : 0u;
        uint64_t *b = &busy[qoff[s] + r];
        const uint64_t start = e.time > *b ? e.time : *b;  /* FIFO, one worker */
        *b = start + c.hold[s];
        S[i * nodes + e.hop] = start;
        A[i * nodes + e.hop] = e.time;
        /* the script runs from `start` */
        istate *st = &is[i * nodes + e.hop];
        st->T = start;
        st->step = 0;
        st->pending = 0;
        if (!advance(&m, i, e.hop)) return 2;
    }
    free(is);
    stats[5] = ~0ull;
    for (uint64_t i = 0; i < n_traces; ++i) {
        fstate f = {&c, S + i * nodes, A + i * nodes, kid_base + i * nodes, kid + i * nodes, trace_begin + i, stats, des, 0};
        int e = 0;
        const uint64_t F = finish(&f, p->entry, 0, &e);
        const uint64_t L = F - arr[i];
        if (records) {
            records[2 * i] = L;
            records[2 * i + 1] = (uint64_t)hops[i] | ((uint64_t)(((uint32_t)e << 31) | f.err_hops) << 32);
        }
        stats[0] += 1;
        stats[1] += L;
        stats[2] += hops[i];
        stats[3] += f.err_hops;
        stats[4] += (uint64_t)e;
        if (L < stats[5]) stats[5] = L;
        if (L > stats[6]) stats[6] = L;
        stats[ST_PROM + e * N_PROM + prom_bucket(L)] += 1;
        const int l = L == 0 ? 0 : 64 - __builtin_clzll(L);
        stats[ST_LOG2 + e * N_LOG2 + l] += 1;
    }
    free(h.v);
    free(hops);
    free(stop);
    free(kid);
    free(kid_base);
    free(arr);
    free(A);
    free(S);
    free(busy);
    free(qoff);
    free(c.hold);
    free(c.ncalls);
    free(c.size);
    return 0;
}
