/*
 * tb_ref.c -- independent C restatement of the reference's token-bucket acquire
 * script (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this
 * library (as the checker / the timed CPU baseline).  The product path is the HIP
 * engine behind include/tbe.h and never links this file.
 *
 * Follows /root/reference/DistributedRateLimiting.Redis/TokenBucket/
 * RedisTokenBucketRateLimiter.cs (alias TB in SURVEY.md):
 *   TB:202-203  new_t = sec + usec / 1e6        (tbr_new_t)
 *   TB:210-215  HGETALL or default {cap, new_t}  (absent: t_us == TBR_ABSENT)
 *   TB:218      delta_t = math.max(0, new_t - prev.t)
 *   TB:221      new_v = math.max(0, math.min(cap, prev.v + delta_t * fill_rate))
 *   TB:224-236  success = new_v >= p; on success v -= p, HSET v,t, EXPIRE ttl
 *   TB:238 + TB:64-81  reply {success, trunc(new_v)}
 * Parity status: see oracle/semantics.py header (no reference-produced vectors
 * exist; pinned by KATs, the Python restatement and the Lua-replay fixtures).
 *
 * Build: gcc -O2 -ffp-contract=off -fno-fast-math -fPIC -shared -pthread
 * (no FMA contraction: the script does a multiply then an add, two roundings).
 */
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define TBR_ABSENT INT64_MIN

/* Contraction is disabled by the build flags (-ffp-contract=off); tests/test_oracle.py
 * checks the object code for vfmadd instructions. */

typedef struct {
    uint64_t n_keys;
    double cap;
    double rate;
    int64_t ttl_ms;
    double *v;
    int64_t *t_us;
} tbr_table;

static inline double lua_max(double a, double b) { return (b > a) ? b : a; }
static inline double lua_min(double a, double b) { return (b < a) ? b : a; }

double tbr_new_t(int64_t ts_us) {
    int64_t sec = ts_us / 1000000;
    int64_t usec = ts_us % 1000000;
    return (double)sec + ((double)usec / 1000000.0);
}

double tbr_fill_rate(int32_t tokens_per_period, int64_t period_ticks) {
    double total_seconds = (double)period_ticks / 10000000.0;
    return (double)tokens_per_period / total_seconds;
}

int64_t tbr_ttl_seconds(int32_t capacity, double rate) {
    return (int64_t)ceil(lua_min(lua_max((double)capacity / rate, 1.0), 31536000.0));
}

tbr_table *tbr_create(uint64_t n_keys, int32_t token_limit, double fill_rate) {
    if (token_limit <= 0 || !(fill_rate > 0.0) || isinf(fill_rate)) return NULL;
    tbr_table *tb = (tbr_table *)calloc(1, sizeof(tbr_table));
    if (!tb) return NULL;
    tb->n_keys = n_keys;
    tb->cap = (double)token_limit;
    tb->rate = fill_rate;
    tb->ttl_ms = tbr_ttl_seconds(token_limit, fill_rate) * 1000;
    tb->v = (double *)malloc(n_keys * sizeof(double));
    tb->t_us = (int64_t *)malloc(n_keys * sizeof(int64_t));
    if (!tb->v || !tb->t_us) {
        free(tb->v); free(tb->t_us); free(tb);
        return NULL;
    }
    for (uint64_t k = 0; k < n_keys; ++k) { tb->v[k] = tb->cap; tb->t_us[k] = TBR_ABSENT; }
    return tb;
}

void tbr_destroy(tbr_table *tb) {
    if (!tb) return;
    free(tb->v); free(tb->t_us); free(tb);
}

/* One script evaluation.  Returns 1 on grant; *remaining = trunc(new_v). */
static inline int tbr_acquire_one(tbr_table *tb, uint64_t key, int32_t p, int64_t ts_us,
                                  int32_t *remaining) {
    double new_t = tbr_new_t(ts_us);
    int64_t pt_us = tb->t_us[key];
    double pv, pt;
    if (pt_us != TBR_ABSENT && (ts_us / 1000) > (pt_us / 1000) + tb->ttl_ms) {
        /* Passive expiry: HGETALL (TB:210) on a lapsed key deletes it, whatever the
         * script decides next. */
        tb->t_us[key] = pt_us = TBR_ABSENT;
        tb->v[key] = tb->cap;
    }
    if (pt_us == TBR_ABSENT) {
        pv = tb->cap; pt = new_t;                       /* TB:213-215 (absent) */
    } else {
        pv = tb->v[key]; pt = tbr_new_t(pt_us);         /* TB:211-212 */
    }
    double delta_t = lua_max(0.0, new_t - pt);                      /* TB:218 */
    double x = lua_max(0.0, lua_min(tb->cap, pv + (delta_t * tb->rate)));  /* TB:221 */
    int ok = x >= (double)p;                                        /* TB:224 */
    if (ok) {
        x = x - (double)p;                                          /* TB:227 */
        tb->v[key] = x;                                             /* TB:230 */
        tb->t_us[key] = ts_us;
    }
    *remaining = (int32_t)(int64_t)x;                               /* TB:238, TB:73 */
    return ok;
}

/* Validates like the engine (include/tbe.h): returns 0, or -1 on an invalid request
 * (nothing applied). */
int tbr_validate(const tbr_table *tb, const uint64_t *keys, const int32_t *permits,
                 const int64_t *ts_us, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i)
        if (keys[i] >= tb->n_keys || permits[i] < 0 || ts_us[i] < 0) return -1;
    return 0;
}

int tbr_acquire_batch(tbr_table *tb, const uint64_t *keys, const int32_t *permits,
                      const int64_t *ts_us, uint64_t n, uint8_t *granted, int32_t *remaining) {
    if (tbr_validate(tb, keys, permits, ts_us, n)) return -1;
    for (uint64_t i = 0; i < n; ++i)
        granted[i] = (uint8_t)tbr_acquire_one(tb, keys[i], permits[i], ts_us[i], &remaining[i]);
    return 0;
}

/* Key-sharded multi-threaded baseline: thread j owns keys with key % T == j and walks
 * the whole batch in arrival order, so per-key order is preserved. */
typedef struct {
    tbr_table *tb; const uint64_t *keys; const int32_t *permits; const int64_t *ts;
    uint64_t n; uint8_t *granted; int32_t *remaining; int tid, nthreads;
} tbr_job;

static void *tbr_worker(void *arg) {
    tbr_job *j = (tbr_job *)arg;
    for (uint64_t i = 0; i < j->n; ++i) {
        uint64_t k = j->keys[i];
        if ((int)(k % (uint64_t)j->nthreads) != j->tid) continue;
        j->granted[i] = (uint8_t)tbr_acquire_one(j->tb, k, j->permits[i], j->ts[i], &j->remaining[i]);
    }
    return NULL;
}

int tbr_acquire_batch_mt(tbr_table *tb, const uint64_t *keys, const int32_t *permits,
                         const int64_t *ts_us, uint64_t n, uint8_t *granted, int32_t *remaining,
                         int nthreads) {
    if (nthreads <= 1) return tbr_acquire_batch(tb, keys, permits, ts_us, n, granted, remaining);
    if (tbr_validate(tb, keys, permits, ts_us, n)) return -1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    tbr_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (tbr_job){tb, keys, permits, ts_us, n, granted, remaining, t, nthreads};
        pthread_create(&th[t], NULL, tbr_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}

/* (v, t) as stored in the Redis hash; returns 0 when absent (or expired at ts_us >= 0). */
int tbr_query(const tbr_table *tb, uint64_t key, int64_t ts_us, double *v, double *t) {
    if (key >= tb->n_keys) return 0;
    int64_t pt = tb->t_us[key];
    if (pt == TBR_ABSENT) return 0;
    if (ts_us >= 0 && (ts_us / 1000) > (pt / 1000) + tb->ttl_ms) return 0;
    *v = tb->v[key];
    *t = tbr_new_t(pt);
    return 1;
}

/* Raw state export for bulk parity checks: v bits and grant timestamps (TBR_ABSENT). */
void tbr_export(const tbr_table *tb, double *v, int64_t *t_us) {
    memcpy(v, tb->v, tb->n_keys * sizeof(double));
    memcpy(t_us, tb->t_us, tb->n_keys * sizeof(int64_t));
}

/* ------------------------------------------------------------------ trace generator
 * Identical to oracle/trace.py and csrc/tbe_gen.hip (splitmix64 finaliser over a
 * counter). */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void tbr_gen_uniform_keys(uint64_t seed, uint64_t n_keys, uint64_t g0, uint64_t n, uint64_t *out) {
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t r = mix64(seed + (g0 + i) * 0x9E3779B97F4A7C15ull);
        out[i] = ((r >> 32) * n_keys) >> 32;
    }
}

void tbr_gen_permits(uint64_t seed, uint64_t g0, uint64_t n, int32_t lo, int32_t hi, int32_t *out) {
    uint64_t span = (uint64_t)(hi - lo + 1);
    for (uint64_t i = 0; i < n; ++i) {
        if (lo == hi) { out[i] = lo; continue; }
        uint64_t r = mix64((seed ^ 0xA5A5A5A5A5A5A5A5ull) + (g0 + i) * 0x9E3779B97F4A7C15ull);
        out[i] = lo + (int32_t)(((r >> 32) * span) >> 32);
    }
}

void tbr_gen_timestamps(int64_t batch, uint64_t n, int64_t interval_us, int64_t t0_us, int64_t *out) {
    for (uint64_t i = 0; i < n; ++i)
        out[i] = t0_us + batch * interval_us + (int64_t)(((__int128)i * interval_us) / (__int128)n);
}

/* ------------------------------------------------------------------ token bucket with queue
 * C restatement of oracle/semantics.py QueueingTokenBucketTable (the build's spec for the
 * non-compiling TokenBucketWithQueue limiter, Q:67-165 + Q:237-271 + TB script + DQ order).
 * Per key: a ring of QueueLimit entries {request id, permits} (permits >= 1, so at most
 * QueueLimit entries), head, count and qsum (= _queueCount). */
enum { TBRQ_FAILED = 0, TBRQ_GRANTED = 1, TBRQ_QUEUED = 2, TBRQ_REJECTED = 3 };

typedef struct {
    tbr_table *tb;
    int32_t token_limit, queue_limit, order;   /* order: 0 OldestFirst, 1 NewestFirst */
    uint32_t ring_cap;
    int64_t *ring_id;
    int32_t *ring_p;
    uint32_t *head, *count;
    int64_t *qsum;
} tbrq_table;

tbrq_table *tbrq_create(uint64_t n_keys, int32_t token_limit, double fill_rate, int32_t queue_limit,
                        int32_t order) {
    if (queue_limit < 0 || (order != 0 && order != 1)) return NULL;
    tbrq_table *q = (tbrq_table *)calloc(1, sizeof(tbrq_table));
    if (!q) return NULL;
    q->tb = tbr_create(n_keys, token_limit, fill_rate);
    q->token_limit = token_limit;
    q->queue_limit = queue_limit;
    q->order = order;
    q->ring_cap = (uint32_t)(queue_limit > 0 ? queue_limit : 1);
    q->ring_id = (int64_t *)calloc(n_keys * q->ring_cap, sizeof(int64_t));
    q->ring_p = (int32_t *)calloc(n_keys * q->ring_cap, sizeof(int32_t));
    q->head = (uint32_t *)calloc(n_keys, sizeof(uint32_t));
    q->count = (uint32_t *)calloc(n_keys, sizeof(uint32_t));
    q->qsum = (int64_t *)calloc(n_keys, sizeof(int64_t));
    if (!q->tb || !q->ring_id || !q->ring_p || !q->head || !q->count || !q->qsum) {
        tbr_destroy(q->tb); free(q->ring_id); free(q->ring_p); free(q->head); free(q->count);
        free(q->qsum); free(q);
        return NULL;
    }
    return q;
}

void tbrq_destroy(tbrq_table *q) {
    if (!q) return;
    tbr_destroy(q->tb);
    free(q->ring_id); free(q->ring_p); free(q->head); free(q->count); free(q->qsum); free(q);
}

/* One WaitAsync (Q:67-134).  Evicted ids (NewestFirst) are appended to evicted[] with
 * the causing request's index; returns the status. */
static int tbrq_acquire_one(tbrq_table *q, uint64_t key, int32_t p, int64_t ts_us, int64_t id,
                            uint64_t cause, int32_t *remaining, int64_t *ev_id, uint64_t *ev_cause,
                            uint64_t *n_ev, uint64_t max_ev) {
    *remaining = -1;
    if (p > q->token_limit) return TBRQ_REJECTED;                           /* Q:70-73 */
    uint32_t cap = q->ring_cap;
    uint64_t base = key * cap;
    if (p == 0 || !(q->count[key] > 0 && q->order == 0)) {                  /* Q:153 */
        if (tbr_acquire_one(q->tb, key, p, ts_us, remaining)) return TBRQ_GRANTED;
    }
    if ((int64_t)q->queue_limit - q->qsum[key] < p) {                       /* Q:92 */
        if (q->order == 1 && p <= q->queue_limit) {                         /* Q:94-109 */
            while ((int64_t)q->queue_limit - q->qsum[key] < p) {
                uint32_t h = q->head[key];
                if (*n_ev < max_ev) { ev_id[*n_ev] = q->ring_id[base + h]; ev_cause[*n_ev] = cause; }
                (*n_ev)++;
                q->qsum[key] -= q->ring_p[base + h];
                q->head[key] = (h + 1) % cap;
                q->count[key]--;
            }
        } else {
            return TBRQ_FAILED;                                              /* Q:113 */
        }
    }
    uint32_t tail = (q->head[key] + q->count[key]) % cap;                   /* EnqueueTail */
    q->ring_id[base + tail] = id;
    q->ring_p[base + tail] = p;
    q->count[key]++;
    q->qsum[key] += p;
    return TBRQ_QUEUED;
}

int tbrq_acquire_batch(tbrq_table *q, const uint64_t *keys, const int32_t *permits,
                       const int64_t *ts_us, uint64_t n, int64_t id_base, uint8_t *status,
                       int32_t *remaining, int64_t *ev_id, uint64_t *ev_cause, uint64_t max_ev,
                       uint64_t *n_ev) {
    if (tbr_validate(q->tb, keys, permits, ts_us, n)) return -1;
    *n_ev = 0;
    for (uint64_t i = 0; i < n; ++i)
        status[i] = (uint8_t)tbrq_acquire_one(q, keys[i], permits[i], ts_us[i], id_base + (int64_t)i,
                                              i, &remaining[i], ev_id, ev_cause, n_ev, max_ev);
    return 0;
}

/* One replenish tick (Q:237-271) over every key, in key order. */
int tbrq_refresh(tbrq_table *q, int64_t ts_us, uint64_t *log_key, int64_t *log_id,
                 int32_t *log_remaining, uint64_t max_log, uint64_t *n_log) {
    if (ts_us < 0) return -1;
    *n_log = 0;
    uint32_t cap = q->ring_cap;
    for (uint64_t k = 0; k < q->tb->n_keys; ++k) {
        while (q->count[k] > 0) {
            uint32_t idx = (q->order == 0) ? q->head[k] : (q->head[k] + q->count[k] - 1) % cap;
            int32_t rem;
            if (!tbr_acquire_one(q->tb, k, q->ring_p[k * cap + idx], ts_us, &rem)) break;
            if (*n_log < max_log) {
                log_key[*n_log] = k; log_id[*n_log] = q->ring_id[k * cap + idx];
                log_remaining[*n_log] = rem;
            }
            (*n_log)++;
            q->qsum[k] -= q->ring_p[k * cap + idx];
            if (q->order == 0) q->head[k] = (q->head[k] + 1) % cap;
            q->count[k]--;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ key-sharded queue oracle
 * The same restatement at full benchmark sizes (config D: 1e8 keys, 2^26-request
 * batches): keys are independent, so thread t applies, in arrival order, exactly the
 * requests of the keys k % T == t (waits), or drains the keys of one contiguous range
 * (ticks).  Logs go to per-thread growable buffers and are merged in thread order: the
 * tick log stays in key order; eviction logs are compared after sorting by (cause, id),
 * as the engine reports them. */
typedef struct {
    int64_t *id;
    uint64_t *a;      /* cause index (evictions) or key (tick log) */
    int32_t *rem;     /* tick log only */
    uint64_t n, cap;
} tbrq_log;

static int tbrq_log_push(tbrq_log *l, uint64_t a, int64_t id, int32_t rem) {
    if (l->n == l->cap) {
        uint64_t c = l->cap ? l->cap * 2 : 4096;
        int64_t *ni = (int64_t *)realloc(l->id, c * sizeof(int64_t));
        if (!ni) return -1;
        l->id = ni;
        uint64_t *na = (uint64_t *)realloc(l->a, c * sizeof(uint64_t));
        if (!na) return -1;
        l->a = na;
        int32_t *nr = (int32_t *)realloc(l->rem, c * sizeof(int32_t));
        if (!nr) return -1;
        l->rem = nr;
        l->cap = c;
    }
    l->a[l->n] = a;
    l->id[l->n] = id;
    l->rem[l->n] = rem;
    l->n++;
    return 0;
}

static void tbrq_log_free(tbrq_log *l) {
    free(l->id); free(l->a); free(l->rem);
    memset(l, 0, sizeof *l);
}

/* Merged log of the last tbrq_*_mt call (owned by the library, see tbrq_mt_log). */
static tbrq_log g_mt_log;

typedef struct {
    tbrq_table *q; const uint64_t *keys; const int32_t *permits; const int64_t *ts;
    uint64_t n; int64_t id_base; uint8_t *status; int32_t *remaining;
    int64_t tick_us; uint64_t k0, k1;
    int tid, nthreads, err;
    tbrq_log log;
} tbrq_job;

static void *tbrq_wait_worker(void *arg) {
    tbrq_job *j = (tbrq_job *)arg;
    int64_t ev_id[64];
    uint64_t ev_cause[64];
    for (uint64_t i = 0; i < j->n; ++i) {
        uint64_t k = j->keys[i];
        if ((int)(k % (uint64_t)j->nthreads) != j->tid) continue;
        uint64_t m = 0;
        /* one request evicts at most QueueLimit entries; 64 at a time, the rest counted */
        j->status[i] = (uint8_t)tbrq_acquire_one(j->q, k, j->permits[i], j->ts[i], j->id_base + (int64_t)i,
                                                 i, &j->remaining[i], ev_id, ev_cause, &m, 64);
        if (m > 64) { j->err = 1; m = 64; }
        for (uint64_t e = 0; e < m; ++e)
            if (tbrq_log_push(&j->log, ev_cause[e], ev_id[e], 0)) j->err = 1;
    }
    return NULL;
}

static void *tbrq_tick_worker(void *arg) {
    tbrq_job *j = (tbrq_job *)arg;
    tbrq_table *q = j->q;
    uint32_t cap = q->ring_cap;
    for (uint64_t k = j->k0; k < j->k1; ++k) {
        while (q->count[k] > 0) {
            uint32_t idx = (q->order == 0) ? q->head[k] : (q->head[k] + q->count[k] - 1) % cap;
            int32_t rem;
            if (!tbr_acquire_one(q->tb, k, q->ring_p[k * cap + idx], j->tick_us, &rem)) break;
            if (tbrq_log_push(&j->log, k, q->ring_id[k * cap + idx], rem)) j->err = 1;
            q->qsum[k] -= q->ring_p[k * cap + idx];
            if (q->order == 0) q->head[k] = (q->head[k] + 1) % cap;
            q->count[k]--;
        }
    }
    return NULL;
}

static int tbrq_run_mt(tbrq_job *jobs, int nthreads, void *(*fn)(void *)) {
    pthread_t th[256];
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, fn, &jobs[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    tbrq_log_free(&g_mt_log);
    int err = 0;
    for (int t = 0; t < nthreads; ++t) {
        for (uint64_t e = 0; e < jobs[t].log.n; ++e)
            if (tbrq_log_push(&g_mt_log, jobs[t].log.a[e], jobs[t].log.id[e], jobs[t].log.rem[e])) err = 1;
        err |= jobs[t].err;
        tbrq_log_free(&jobs[t].log);
    }
    return err ? -2 : 0;
}

/* WaitAsync batch, key-sharded over nthreads; *n_ev = evictions (tbrq_mt_log). */
int tbrq_acquire_batch_mt(tbrq_table *q, const uint64_t *keys, const int32_t *permits,
                          const int64_t *ts_us, uint64_t n, int64_t id_base, uint8_t *status,
                          int32_t *remaining, int nthreads, uint64_t *n_ev) {
    if (tbr_validate(q->tb, keys, permits, ts_us, n)) return -1;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    tbrq_job jobs[256];
    memset(jobs, 0, sizeof jobs);
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].q = q; jobs[t].keys = keys; jobs[t].permits = permits; jobs[t].ts = ts_us;
        jobs[t].n = n; jobs[t].id_base = id_base; jobs[t].status = status; jobs[t].remaining = remaining;
        jobs[t].tid = t; jobs[t].nthreads = nthreads;
    }
    int rc = tbrq_run_mt(jobs, nthreads, tbrq_wait_worker);
    *n_ev = g_mt_log.n;
    return rc;
}

/* One replenish tick, keys split into nthreads contiguous ranges; log in key order. */
int tbrq_refresh_mt(tbrq_table *q, int64_t ts_us, int nthreads, uint64_t *n_log) {
    if (ts_us < 0) return -1;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    tbrq_job jobs[256];
    memset(jobs, 0, sizeof jobs);
    uint64_t nk = q->tb->n_keys;
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].q = q; jobs[t].tick_us = ts_us;
        jobs[t].k0 = nk * (uint64_t)t / (uint64_t)nthreads;
        jobs[t].k1 = nk * (uint64_t)(t + 1) / (uint64_t)nthreads;
    }
    int rc = tbrq_run_mt(jobs, nthreads, tbrq_tick_worker);
    *n_log = g_mt_log.n;
    return rc;
}

/* Copy out the merged log of the last *_mt call: (a, id, rem) = (cause, id, 0) for
 * evictions, (key, id, remaining) for a tick.  Returns the entries copied. */
uint64_t tbrq_mt_log(uint64_t *a, int64_t *id, int32_t *rem, uint64_t max) {
    uint64_t m = g_mt_log.n < max ? g_mt_log.n : max;
    if (m) {
        memcpy(a, g_mt_log.a, m * sizeof(uint64_t));
        memcpy(id, g_mt_log.id, m * sizeof(int64_t));
        memcpy(rem, g_mt_log.rem, m * sizeof(int32_t));
    }
    return m;
}

/* Queue contents of one key, oldest first: returns the entry count. */
uint32_t tbrq_queue_of(const tbrq_table *q, uint64_t key, int64_t *ids, int32_t *permits, uint32_t max) {
    uint32_t c = q->count[key], cap = q->ring_cap;
    for (uint32_t j = 0; j < c && j < max; ++j) {
        uint32_t idx = (q->head[key] + j) % cap;
        ids[j] = q->ring_id[key * cap + idx];
        permits[j] = q->ring_p[key * cap + idx];
    }
    return c;
}

tbr_table *tbrq_bucket_table(tbrq_table *q) { return q->tb; }

/* CancelQueueState.TrySetCanceled (Q:480-506), as oracle/semantics.py
 * QueueingTokenBucketTable.cancel: 1 iff `id` was queued on `key`; _queueCount drops by its
 * permits (Q:499) and the registration leaves the deque at once, the entries behind it
 * closing up in order. */
int tbrq_cancel(tbrq_table *q, uint64_t key, int64_t id) {
    uint32_t cap = q->ring_cap, c = q->count[key], h = q->head[key];
    uint64_t base = key * cap;
    for (uint32_t j = 0; j < c; ++j) {
        if (q->ring_id[base + (h + j) % cap] != id) continue;
        q->qsum[key] -= q->ring_p[base + (h + j) % cap];
        for (uint32_t m = j; m + 1 < c; ++m) {
            q->ring_id[base + (h + m) % cap] = q->ring_id[base + (h + m + 1) % cap];
            q->ring_p[base + (h + m) % cap] = q->ring_p[base + (h + m + 1) % cap];
        }
        q->count[key] = c - 1;
        return 1;
    }
    return 0;
}

/* ------------------------------------------------------------------ approximate limiter
 * C restatement of one client of ApproximateTokenBucket/RedisApproximateTokenBucketRateLimiter.cs
 * ("A"), for every key, plus that client's replica of the global tier (the Redis hash
 * the sync script keeps).  Independent of oracle/semantics.py ApproxClient /
 * ApproxGlobalTable, which it must agree with bit for bit (tests/test_approx_oracle.py):
 *   A:36-37    AvailableTokens = max(0, (int)ceil((TokenLimit - global) / est) - local)
 *   A:84-113   AcquireCore;  A:116-183 WaitAsyncCore;  A:185-214 TryLeaseUnsynchronized
 *   A:241-270  sync script: decay, EWMA period, HSET, EXPIRE 86400, reply {v', "%.14g" p'}
 *   A:430-443  swap local -> count, (int)r[0], double.Parse(r[1]), Math.Round (banker's)
 *   A:462-501  drain: head (OldestFirst) / tail (NewestFirst) while AvailableTokens >= Count
 * Zero-permit waits while throttled queue with Count 0, at most zero_slots per key
 * (DESIGN.md §2c).  All int arithmetic is C# unchecked int32. */
enum { TBA_FAILED = 0, TBA_GRANTED = 1, TBA_QUEUED = 2, TBA_REJECTED = 3 };
#define TBA_TTL_MS (86400LL * 1000)

typedef struct {
    uint64_t n_keys;
    int32_t token_limit, queue_limit, order, zero_slots;
    double decay_rate, period_s;
    uint32_t ring_cap;
    int32_t *cap, *local, *global_;   /* cap = (int)ceil((TokenLimit - global) / est), cached per sync */
    double *est;
    uint32_t *head, *count, *zc;
    int32_t *qsum;
    int64_t *ring_id;
    int32_t *ring_p;
    double *gv, *gp;                  /* global tier replica {v, p, t} */
    int64_t *gt;
} tba_table;

static inline int32_t tba_wrap(int64_t x) { return (int32_t)(uint32_t)(uint64_t)x; }

static inline int32_t tba_to_int(double x) {   /* C# (int)double on x64 */
    if (!(x > -2147483649.0 && x < 2147483648.0)) return INT32_MIN;
    return (int32_t)x;
}

static inline int32_t tba_avail(const tba_table *a, uint64_t k) {
    int32_t d = tba_wrap((int64_t)a->cap[k] - (int64_t)a->local[k]);
    return d > 0 ? d : 0;
}

static double tba_round_trip_14g(double x) {   /* Lua tostring -> C# double.Parse */
    char buf[64];
    snprintf(buf, sizeof buf, "%.14g", x);
    return strtod(buf, NULL);
}

void tba_destroy(tba_table *a);

tba_table *tba_create(uint64_t n_keys, int32_t token_limit, int32_t tokens_per_period, int64_t period_ticks,
                      int32_t queue_limit, int32_t order, int32_t zero_slots) {
    if (token_limit <= 0 || tokens_per_period <= 0 || period_ticks <= 0 || queue_limit < 0 ||
        (order != 0 && order != 1) || zero_slots < 0)
        return NULL;
    tba_table *a = (tba_table *)calloc(1, sizeof(tba_table));
    if (!a) return NULL;
    a->n_keys = n_keys;
    a->token_limit = token_limit;
    a->queue_limit = queue_limit;
    a->order = order;
    a->zero_slots = zero_slots;
    a->decay_rate = tbr_fill_rate(tokens_per_period, period_ticks);
    a->period_s = (double)period_ticks / 10000000.0;
    a->ring_cap = (uint32_t)((queue_limit > 0 ? queue_limit : 1) + zero_slots);
    a->cap = (int32_t *)malloc(n_keys * sizeof(int32_t));
    a->local = (int32_t *)calloc(n_keys, sizeof(int32_t));
    a->global_ = (int32_t *)calloc(n_keys, sizeof(int32_t));
    a->est = (double *)malloc(n_keys * sizeof(double));
    a->head = (uint32_t *)calloc(n_keys, sizeof(uint32_t));
    a->count = (uint32_t *)calloc(n_keys, sizeof(uint32_t));
    a->zc = (uint32_t *)calloc(n_keys, sizeof(uint32_t));
    a->qsum = (int32_t *)calloc(n_keys, sizeof(int32_t));
    a->ring_id = (int64_t *)calloc(n_keys * a->ring_cap, sizeof(int64_t));
    a->ring_p = (int32_t *)calloc(n_keys * a->ring_cap, sizeof(int32_t));
    a->gv = (double *)calloc(n_keys, sizeof(double));
    a->gp = (double *)calloc(n_keys, sizeof(double));
    a->gt = (int64_t *)malloc(n_keys * sizeof(int64_t));
    if (!a->cap || !a->local || !a->global_ || !a->est || !a->head || !a->count || !a->zc || !a->qsum ||
        !a->ring_id || !a->ring_p || !a->gv || !a->gp || !a->gt) {
        tba_destroy(a);
        return NULL;
    }
    for (uint64_t k = 0; k < n_keys; ++k) {
        a->cap[k] = token_limit;     /* global 0, est 1 */
        a->est[k] = 1.0;
        a->gt[k] = TBR_ABSENT;
    }
    return a;
}

void tba_destroy(tba_table *a) {
    if (!a) return;
    free(a->cap); free(a->local); free(a->global_); free(a->est); free(a->head); free(a->count);
    free(a->zc); free(a->qsum); free(a->ring_id); free(a->ring_p); free(a->gv); free(a->gp); free(a->gt);
    free(a);
}

/* AcquireCore (wait = 0) or WaitAsyncCore (wait = 1) of one request.  *avail_out =
 * AvailableTokens after it (-1 when rejected). */
static int tba_acquire_one(tba_table *a, uint64_t k, int32_t p, int wait, int64_t id, uint64_t cause,
                           int32_t *avail_out, tbrq_log *ev) {
    uint32_t rc = a->ring_cap;
    uint64_t base = k * rc;
    int32_t avail = tba_avail(a, k);
    int st;
    *avail_out = -1;
    if (p > a->token_limit) return TBA_REJECTED;                               /* A:87-90, A:119-122 */
    if (p == 0 && (avail > 0 || !wait)) {                                        /* A:93-102, A:127-130 */
        st = avail > 0 ? TBA_GRANTED : TBA_FAILED;
    } else if (p == 0) {                                                         /* queued with Count 0 */
        if ((int32_t)a->zc[k] < a->zero_slots) {
            uint32_t tail = (a->head[k] + a->count[k]) % rc;
            a->ring_id[base + tail] = id;
            a->ring_p[base + tail] = 0;
            a->count[k]++;
            a->zc[k]++;
            st = TBA_QUEUED;
        } else {
            st = TBA_FAILED;
        }
    } else if (avail >= p && avail != 0 && (a->qsum[k] == 0 || a->order == 1)) {  /* A:191-209 */
        a->local[k] = tba_wrap((int64_t)a->local[k] + p);
        st = TBA_GRANTED;
    } else if (!wait) {
        st = TBA_FAILED;                                                         /* A:111 */
    } else {
        st = TBA_QUEUED;
        if ((int64_t)a->queue_limit - a->qsum[k] < p) {                          /* A:141 */
            if (a->order == 1 && p <= a->queue_limit) {                          /* A:143-158 */
                while ((int64_t)a->queue_limit - a->qsum[k] < p) {
                    uint32_t h = a->head[k];
                    if (ev && tbrq_log_push(ev, cause, a->ring_id[base + h], 0)) return -1;
                    a->qsum[k] -= a->ring_p[base + h];
                    if (a->ring_p[base + h] == 0) a->zc[k]--;
                    a->head[k] = (h + 1) % rc;
                    a->count[k]--;
                }
            } else {
                st = TBA_FAILED;                                                 /* A:159-163 */
            }
        }
        if (st == TBA_QUEUED) {                                                  /* A:166-181 */
            uint32_t tail = (a->head[k] + a->count[k]) % rc;
            a->ring_id[base + tail] = id;
            a->ring_p[base + tail] = p;
            a->count[k]++;
            a->qsum[k] += p;
        }
    }
    *avail_out = tba_avail(a, k);
    return st;
}

typedef struct {
    tba_table *a; const uint64_t *keys; const int32_t *permits; uint64_t n; int wait; int64_t id_base;
    uint8_t *status; int32_t *avail;
    const int32_t *all_counts; uint32_t n_clients, my; int64_t ts, stagger; uint64_t k0, k1;
    int tid, nthreads, err;
    tbrq_log log;
} tba_job;

static void *tba_acquire_worker(void *arg) {
    tba_job *j = (tba_job *)arg;
    for (uint64_t i = 0; i < j->n; ++i) {
        uint64_t k = j->keys[i];
        if (j->nthreads > 1 && (int)(k % (uint64_t)j->nthreads) != j->tid) continue;
        int st = tba_acquire_one(j->a, k, j->permits[i], j->wait, j->id_base + (int64_t)i, i, &j->avail[i], &j->log);
        if (st < 0) { j->err = 1; return NULL; }
        j->status[i] = (uint8_t)st;
    }
    return NULL;
}

/* One refresh epoch (A:412-508) for keys [k0, k1): replay the n_clients sync calls
 * (client r at ts + r*stagger with count all_counts[r*n_keys + k]) on this replica, take
 * client `my`'s reply, then drain.  Log: (key, request id, AvailableTokens after). */
static void *tba_sync_worker(void *arg) {
    tba_job *j = (tba_job *)arg;
    tba_table *a = j->a;
    const int64_t ttl_ms = TBA_TTL_MS;
    for (uint64_t k = j->k0; k < j->k1; ++k) {
        double v = a->gv[k], pp = a->gp[k];
        int64_t t = a->gt[k];
        int32_t my_global = 0;
        double my_period = 0.0;
        for (uint32_t r = 0; r < j->n_clients; ++r) {
            int64_t ts = j->ts + (int64_t)r * j->stagger;
            double new_t = tbr_new_t(ts);                                          /* A:241-242 */
            int present = t != TBR_ABSENT && !((ts / 1000) > (t / 1000) + ttl_ms); /* EXPIRE A:268 */
            double pv = present ? v : 0.0, ppv = present ? pp : 0.0;               /* A:247-252 */
            double pt = present ? tbr_new_t(t) : new_t;
            double dt = lua_max(0.0, new_t - pt);                                  /* A:255 */
            double nv = lua_max(0.0, pv - (dt * a->decay_rate)) +
                        (double)j->all_counts[(uint64_t)r * a->n_keys + k];        /* A:258 */
            double np = (ppv * 0.8) + (dt * 0.2);                                  /* A:262 */
            v = nv; pp = np; t = ts;                                               /* A:265 */
            if (r == j->my) {
                my_global = (int32_t)(int64_t)nv;                                  /* A:270 -> A:441 */
                my_period = tba_round_trip_14g(np);                                /* A:270 -> A:442 */
            }
        }
        a->gv[k] = v; a->gp[k] = pp; a->gt[k] = t;
        double q = a->period_s / my_period;                                        /* A:443 */
        double rnd = rint(q);                                                      /* banker's */
        a->est[k] = (rnd != rnd) ? rnd : (rnd > 1.0 ? rnd : 1.0);
        a->global_[k] = my_global;
        a->cap[k] = tba_to_int(ceil((double)tba_wrap((int64_t)a->token_limit - my_global) / a->est[k]));
        uint32_t rc = a->ring_cap;
        while (a->count[k] > 0) {                                                  /* A:467-501 */
            uint32_t idx = a->order == 0 ? a->head[k] : (a->head[k] + a->count[k] - 1) % rc;
            int32_t c = a->ring_p[k * rc + idx];
            if (tba_avail(a, k) < c) break;                                        /* A:474 */
            a->qsum[k] -= c;
            a->local[k] = tba_wrap((int64_t)a->local[k] + c);
            if (c == 0) a->zc[k]--;
            if (a->order == 0) a->head[k] = (a->head[k] + 1) % rc;
            a->count[k]--;
            if (tbrq_log_push(&j->log, k, a->ring_id[k * rc + idx], tba_avail(a, k))) j->err = 1;
        }
    }
    return NULL;
}

static int tba_run(tba_job *jobs, int nthreads, void *(*fn)(void *)) {
    pthread_t th[256];
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, fn, &jobs[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    tbrq_log_free(&g_mt_log);
    int err = 0;
    for (int t = 0; t < nthreads; ++t) {
        for (uint64_t e = 0; e < jobs[t].log.n; ++e)
            if (tbrq_log_push(&g_mt_log, jobs[t].log.a[e], jobs[t].log.id[e], jobs[t].log.rem[e])) err = 1;
        err |= jobs[t].err;
        tbrq_log_free(&jobs[t].log);
    }
    return err ? -2 : 0;
}

static int tba_clamp_threads(int t) { return t < 1 ? 1 : (t > 256 ? 256 : t); }

/* A batch of AcquireCore (wait = 0) / WaitAsyncCore (wait = 1) requests, key-sharded over
 * nthreads; *n_ev = evictions (tbrq_mt_log: cause index, request id). */
int tba_acquire_batch(tba_table *a, const uint64_t *keys, const int32_t *permits, uint64_t n, int wait,
                      int64_t id_base, uint8_t *status, int32_t *avail, int nthreads, uint64_t *n_ev) {
    for (uint64_t i = 0; i < n; ++i)
        if (keys[i] >= a->n_keys || permits[i] < 0) return -1;
    nthreads = tba_clamp_threads(nthreads);
    tba_job jobs[256];
    memset(jobs, 0, sizeof jobs);
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].a = a; jobs[t].keys = keys; jobs[t].permits = permits; jobs[t].n = n; jobs[t].wait = wait;
        jobs[t].id_base = id_base; jobs[t].status = status; jobs[t].avail = avail;
        jobs[t].tid = t; jobs[t].nthreads = nthreads;
    }
    int rc = tba_run(jobs, nthreads, tba_acquire_worker);
    *n_ev = g_mt_log.n;
    return rc;
}

/* A:430-435 for every key: counts[k] = _localThrottleScore; _localThrottleScore = 0. */
void tba_collect(tba_table *a, int32_t *counts) {
    for (uint64_t k = 0; k < a->n_keys; ++k) {
        counts[k] = a->local[k];
        a->local[k] = 0;
    }
}

/* One refresh epoch of client `my` among n_clients (all_counts[r * n_keys + k]); *n_log =
 * drained registrations (tbrq_mt_log: key, request id, AvailableTokens after), key order. */
int tba_sync(tba_table *a, const int32_t *all_counts, uint32_t n_clients, uint32_t my, int64_t ts_us,
             int64_t stagger_us, int nthreads, uint64_t *n_log) {
    if (n_clients == 0 || my >= n_clients || ts_us < 0 || stagger_us < 0) return -1;
    nthreads = tba_clamp_threads(nthreads);
    tba_job jobs[256];
    memset(jobs, 0, sizeof jobs);
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].a = a; jobs[t].all_counts = all_counts; jobs[t].n_clients = n_clients; jobs[t].my = my;
        jobs[t].ts = ts_us; jobs[t].stagger = stagger_us;
        jobs[t].k0 = a->n_keys * (uint64_t)t / (uint64_t)nthreads;
        jobs[t].k1 = a->n_keys * (uint64_t)(t + 1) / (uint64_t)nthreads;
    }
    int rc = tba_run(jobs, nthreads, tba_sync_worker);
    *n_log = g_mt_log.n;
    return rc;
}

/* Bulk state for parity checks: local tier (local, global, est, AvailableTokens, queued
 * count) and the global replica (v, p, t_us; absent: t_us = INT64_MIN, v = p = 0). */
void tba_export(const tba_table *a, int32_t *local, int32_t *global_score, double *est, int32_t *avail,
                uint32_t *queued, double *v, double *p, int64_t *t_us) {
    for (uint64_t k = 0; k < a->n_keys; ++k) {
        if (local) local[k] = a->local[k];
        if (global_score) global_score[k] = a->global_[k];
        if (est) est[k] = a->est[k];
        if (avail) avail[k] = tba_avail(a, k);
        if (queued) queued[k] = a->count[k];
        if (v) v[k] = a->gt[k] == TBR_ABSENT ? 0.0 : a->gv[k];
        if (p) p[k] = a->gt[k] == TBR_ABSENT ? 0.0 : a->gp[k];
        if (t_us) t_us[k] = a->gt[k];
    }
}

/* Queue of one key, oldest first: returns the entry count. */
/* CancelQueueState.TrySetCanceled (A:545-556), as oracle/semantics.py ApproxClient.cancel:
 * 1 iff `id` was queued on `key`; _queueCount drops by its permits; removed at once. */
int tba_cancel(tba_table *a, uint64_t key, int64_t id) {
    uint32_t rc = a->ring_cap, c = a->count[key], h = a->head[key];
    uint64_t base = key * rc;
    for (uint32_t j = 0; j < c; ++j) {
        if (a->ring_id[base + (h + j) % rc] != id) continue;
        const int32_t p = a->ring_p[base + (h + j) % rc];
        a->qsum[key] -= p;
        if (p == 0) a->zc[key]--;
        for (uint32_t m = j; m + 1 < c; ++m) {
            a->ring_id[base + (h + m) % rc] = a->ring_id[base + (h + m + 1) % rc];
            a->ring_p[base + (h + m) % rc] = a->ring_p[base + (h + m + 1) % rc];
        }
        a->count[key] = c - 1;
        return 1;
    }
    return 0;
}

uint32_t tba_queue_of(const tba_table *a, uint64_t key, int64_t *ids, int32_t *permits, uint32_t max) {
    uint32_t c = a->count[key], rc = a->ring_cap;
    for (uint32_t j = 0; j < c && j < max; ++j) {
        uint32_t idx = (a->head[key] + j) % rc;
        ids[j] = a->ring_id[key * rc + idx];
        permits[j] = a->ring_p[key * rc + idx];
    }
    return c;
}
