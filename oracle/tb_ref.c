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
