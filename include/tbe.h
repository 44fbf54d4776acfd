/*
 * tbe.h -- C ABI of the MI355X batched token-bucket engine ("tbe").
 *
 * This is the drop-in boundary.  In the reference every decision is one
 * StackExchange.Redis script round-trip; the entry points below replace those
 * call sites with batched calls into an HBM-resident bucket table on one GPU.
 * References are to /root/reference/DistributedRateLimiting.Redis/ (aliases as in
 * TB = TokenBucket/RedisTokenBucketRateLimiter.cs, PTB =
 * TokenBucket/PartitionedRedisTokenBucketRateLimiter.cs, TBO = TokenBucket/
 * RedisTokenBucketRateLimiterOptions.cs).
 *
 * Conventions
 *  - Plain pointers and sizes only; no C++ or HIP types cross this boundary.
 *  - Every function returns a tbe_status; no exception ever crosses the ABI.
 *  - An engine is NOT re-entrant: one submitting thread per engine.  Batch order
 *    is arrival order: request i of a batch is decided after request i-1 of the
 *    same batch and after every request of earlier batches (the order Redis
 *    serialises script calls in, TB:63).
 *  - Keys are dense ids in [0, n_keys).  Mapping InstanceName + resourceID
 *    strings (PTB:42) to ids is the caller's job.
 *  - Timestamps are injected microseconds since the Unix epoch (>= 0); they play
 *    the role of Redis `TIME` inside the script (TB:202-203).
 */
#ifndef TBE_H_
#define TBE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TBE_ABI_VERSION 1

typedef enum tbe_status {
    TBE_OK = 0,
    TBE_EINVAL = 1,     /* bad argument / invalid request in a batch (nothing applied):
                           ArgumentException / ArgumentOutOfRangeException (TB:24-42) */
    TBE_ENOMEM = 2,     /* device or host allocation failed */
    TBE_EDEVICE = 3,    /* HIP runtime error; the engine should be destroyed */
    TBE_EDISPOSED = 4,  /* engine already disposed: ObjectDisposedException (TB:158-164) */
    TBE_ERANGE = 5      /* permits > TokenLimit where the limiter forbids it (A:87-90) */
} tbe_status;

typedef enum tbe_kind {
    TBE_KIND_TOKEN_BUCKET = 0,   /* TokenBucket/ (TB, PTB)                                */
    TBE_KIND_QUEUEING = 1,       /* TokenBucketWithQueue/           */
    TBE_KIND_APPROXIMATE = 2     /* ApproximateTokenBucket/        */
} tbe_kind;

/* Limiter options (TBO:9-85) plus engine sizing.  The Redis connection options
 * (Configuration, ConfigurationOptions, ConnectionMultiplexerFactory, TBO:48-60) and
 * the ProfilingSession (TBO:70) have no counterpart: the "connection" is the device. */
typedef struct tbe_config {
    uint32_t struct_size;                 /* sizeof(tbe_config); sizes down to
                                             offsetof(tbe_config, zero_wait_slots) (the first
                                             published layout) are accepted, and the fields
                                             past struct_size read as 0 */
    int32_t kind;                         /* tbe_kind */
    uint64_t n_keys;                      /* table capacity, 1 <= n_keys <= 2^32 */
    int32_t token_limit;                  /* TokenLimit (TBO:43), > 0 */
    int32_t tokens_per_period;            /* TokensPerPeriod (TBO:30), > 0 */
    int64_t replenishment_period_ticks;   /* ReplenishmentPeriod in .NET ticks (100 ns), > 0 */
    int32_t queue_limit;                  /* QueueLimit (queueing kind: 0..65535; ignored otherwise) */
    int32_t queue_order;                  /* 0 = OldestFirst, 1 = NewestFirst */
    int32_t device;                       /* HIP device ordinal; -1 = current device */
    uint32_t flags;                       /* TBE_FLAG_* */
    uint64_t max_batch;                   /* expected largest batch (workspace pre-sizing); 0 = grow on demand */
    int32_t zero_wait_slots;              /* approximate kind: queue entries per key for zero-permit
                                             waits (A:127-181; see tbe_approx_acquire_batch); 0 for
                                             the other kinds.  max(1, queue_limit) + zero_wait_slots
                                             <= 65535 */
    int32_t reserved;                     /* 0 */
} tbe_config;

#define TBE_FLAG_STAGE_TIMING 0x1u        /* record per-stage HIP events (tbe_stage_times) */
#define TBE_FLAG_NO_PACK 0x2u             /* token bucket: keep the wide pass records even where
                                             the packed 8-byte form applies (A/B checks) */
#define TBE_FLAG_NO_HOT 0x4u              /* token bucket: no hot-key runs (A/B checks); keys
                                             that take >= 2048 requests of a batch otherwise get
                                             a run of their own two batches later */
#define TBE_FLAG_NO_PIPELINE 0x8u         /* token bucket: run every stage of a batch on one
                                             stream (A/B checks); by default batch b+1's
                                             partition overlaps batch b's fold */
#define TBE_FLAG_NO_NARROW 0x10u          /* keep 4-byte replies through the fold and the
                                             un-partition passes (A/B checks) instead of the
                                             narrower forms: token bucket 1-byte replies
                                             (packed records, TokenLimit <= 127); queueing kind
                                             1-byte (TokenLimit <= 62) and 2-byte (<= 16382)
                                             replies; approximate kind 2-byte replies
                                             (TokenLimit <= 16382) */
#define TBE_FLAG_UNSCATTER_ALL 0x20u      /* token bucket (A/B checks): the last partition pass
                                             writes plain records and its permutation, and its
                                             own un-partition pass runs.  By default (>= 2
                                             passes, packed records) it writes fold records that
                                             carry each request's position in its input, and the
                                             fold puts every reply straight there */
#define TBE_FLAG_RERANK 0x80u             /* packed records (A/B checks): the final
                                             un-partition re-ranks pass 0's tiles from one-byte
                                             digits the first histogram wrote (k_unrank) instead
                                             of gathering through pass 0's stored permutation:
                                             0.4 GB less traffic per config-B batch, 0.06 ms
                                             slower */
#define TBE_FLAG_FOLD_TIMING 0x100u        /* record HIP events around the fold stage only
                                             (tbe_stage_times reports the fold alone): the
                                             dominant kernel's time at two events per batch
                                             instead of a pair per stage, each event record
                                             leaving the stream idle for microseconds */
#define TBE_FLAG_HIST_RECORDS 0x40u       /* packed records, 2 passes (A/B checks): the second
                                             pass's histogram reads the first pass's 8-byte
                                             records.  By default the first pass also writes each
                                             request's second digit as one byte beside its record,
                                             and that histogram reads those */

typedef struct tbe_engine tbe_engine;

/* Fill rate the engine computes from the options exactly like FillRatePerSecond
 * (TBO:82-85): (double)tokens_per_period / (ticks / 1e7).  Raw f64, as the script
 * literal `fill_rate` (TB:185) round-trips it. */
double tbe_fill_rate(int32_t tokens_per_period, int64_t replenishment_period_ticks);

/* Replaces the constructor + lazy connect (TB:22-46, TB:111-151).  Allocates the
 * table (16 B per key) on the device, every key absent. */
tbe_status tbe_create(const tbe_config *config, tbe_engine **out_engine);

/* Replaces Dispose / DisposeAsyncCore (TB:85-109).  NULL is ignored. */
void tbe_destroy(tbe_engine *engine);

/* Human-readable description of the last non-OK status on this engine (never NULL);
 * with engine == NULL, of the calling thread's last failed tbe_create. */
const char *tbe_last_error(const tbe_engine *engine);

/* Replaces n sequential IDatabase.ScriptEvaluateAsync(_acquireScript,
 * {BucketId, PermitCount}) calls (TB:63; PTB:42) and their reply parsing (TB:64-81).
 * Host buffers; synchronous.  granted[i] = 1 iff reply[0] == 1 (TB:76); remaining[i]
 * = reply[1] = trunc(new_v) after the decision (TB:73, TB:238).
 * Invalid batch (key >= n_keys, permits < 0, ts_us < 0): TBE_EINVAL, no state change,
 * outputs unspecified. */
tbe_status tbe_acquire_batch(tbe_engine *engine, const uint64_t *keys, const int32_t *permits,
                             const int64_t *ts_us, uint64_t n, uint8_t *granted,
                             int32_t *remaining);

/* Same decision on device-resident buffers.  Returns once enqueued; a batch found
 * invalid on the device is skipped (no state change) and reported by tbe_synchronize.
 * `stream` (a hipStream_t): the engine waits on it for the inputs and makes it wait for
 * the replies, so work enqueued on it afterwards may read the replies and overwrite the
 * inputs.  NULL: the inputs must be complete when the call is made and stay untouched
 * until the replies are; the replies are complete at tbe_synchronize (or for any later
 * call on this engine).  Batches are applied in call order either way; consecutive
 * batches of a token-bucket engine overlap on the device (TBE_FLAG_NO_PIPELINE). */
tbe_status tbe_acquire_batch_device(tbe_engine *engine, const uint64_t *d_keys,
                                    const int32_t *d_permits, const int64_t *d_ts_us,
                                    uint64_t n, uint8_t *d_granted, int32_t *d_remaining,
                                    void *stream);

/* Page-locked host memory for the host-buffer calls' arrays (the caller
 * owns its buffers, pinning recommended).  Copies from it run as direct DMA, without the
 * staging copy a pageable buffer needs; the C# host pins its batch arrays this way
 * instead of GCHandle-pinning managed arrays.  bytes == 0 gives NULL.  Free with
 * tbe_free_host (NULL is ignored). */
tbe_status tbe_alloc_host(uint64_t bytes, void **out);
void tbe_free_host(void *p);

/* Waits for every enqueued batch; TBE_EINVAL if any of them was invalid since the
 * last call (the sticky flag is then cleared). */
tbe_status tbe_synchronize(tbe_engine *engine);

/* Bucket state exactly as the Redis hash would hold it (HGETALL of the key, TB:210):
 * *present = 0 if absent or expired at ts_us (pass ts_us < 0 to skip the expiry test);
 * otherwise *v = field v and *t = field t (= new_t of the last grant, TB:203/230). */
tbe_status tbe_query(tbe_engine *engine, uint64_t key, int64_t ts_us, double *v, double *t,
                     int32_t *present);

/* Bulk state export for parity checks: v[k] and the last grant's injected timestamp
 * t_us[k] (INT64_MIN when never granted) for keys [first, first + count). */
tbe_status tbe_export_state(tbe_engine *engine, uint64_t first, uint64_t count, double *v,
                            int64_t *t_us);

/* Restore of an exported range (snapshot/restore of the bucket hashes, the state Redis
 * persists; the in-process queues of the queueing kind are not part of it, as they are
 * not in the reference): keys [first, first + count) take {v[k], t_us[k]}; t_us =
 * INT64_MIN makes the key absent.  Token-bucket and queueing kinds.  t_us must be
 * INT64_MIN or >= 0; ordered after every batch enqueued before the call. */
tbe_status tbe_import_state(tbe_engine *engine, uint64_t first, uint64_t count, const double *v,
                            const int64_t *t_us);

/* ---------------------------------------------------------------- TokenBucketWithQueue
 * Engines created with kind = TBE_KIND_QUEUEING.  The reference limiter
 * (TokenBucketWithQueue/RedisTokenBucketRateLimiter.cs, "Q") is commented out and does
 * not compile; its semantics are fixed in DESIGN.md §2b (a lease is one TB script call;
 * queue order follows System.Collections.Generic/Deque.cs).  Per-key queues hold at most
 * QueueLimit entries (permits >= 1 each). */
#define TBE_WAIT_FAILED 0    /* CreateFailedTokenLease (Q:113, Q:383-388) */
#define TBE_WAIT_GRANTED 1   /* SuccessfulLease (Q:85-88) */
#define TBE_WAIT_QUEUED 2    /* registration enqueued (Q:117-132); completes via tbe_refresh */
#define TBE_WAIT_REJECTED 3  /* permits > TokenLimit: ArgumentOutOfRangeException (Q:70-73) */

/* Replaces n WaitAsyncCore calls (Q:67-134).  Request i gets id id_base + i (0 <= id <
 * 2^47).  status[i] is a TBE_WAIT_* code; remaining[i] = trunc(new_v) of the script call
 * made for the request, or -1 when no call was made (OldestFirst with a non-empty queue,
 * or REJECTED).  Queued requests that a NewestFirst admission evicted (Q:94-109) are
 * retrievable with tbe_evicted until the next batch; *n_evicted gets their number. */
tbe_status tbe_wait_batch(tbe_engine *engine, const uint64_t *keys, const int32_t *permits,
                          const int64_t *ts_us, uint64_t n, int64_t id_base, uint8_t *status,
                          int32_t *remaining, uint64_t *n_evicted);

/* AttemptAcquire on a queueing limiter (TryLeaseUnsynchronized only, Q:136-165): like
 * tbe_wait_batch but a request that cannot lease is FAILED instead of queued (nothing is
 * ever enqueued or evicted).  OldestFirst with a non-empty queue fails without a script
 * call (remaining -1).  The reference's own AcquireCore is a stub (Q:62-65). */
tbe_status tbe_queue_attempt_batch(tbe_engine *engine, const uint64_t *keys, const int32_t *permits,
                                   const int64_t *ts_us, uint64_t n, uint8_t *status,
                                   int32_t *remaining);

/* Evictions of the last tbe_wait_batch, sorted by (causing request index, request id):
 * cause_index[j] is the batch index of the request whose admission evicted request_id[j]. */
tbe_status tbe_evicted(tbe_engine *engine, uint64_t *cause_index, int64_t *request_id,
                       uint64_t capacity, uint64_t *n_written);

/* One replenish tick at ts_us (the timer-driven drain, Q:237-271): for every key with a
 * non-empty queue, grant the head (OldestFirst) or tail (NewestFirst) while the script
 * grants.  *n_granted gets the number of queued requests completed; fetch them with
 * tbe_refresh_log. */
tbe_status tbe_refresh(tbe_engine *engine, int64_t ts_us, uint64_t *n_granted);

/* Grants of the last tbe_refresh in (key, drain order): key, request id and
 * trunc(new_v) after the grant. */
tbe_status tbe_refresh_log(tbe_engine *engine, uint64_t *keys, int64_t *request_id,
                           int32_t *remaining, uint64_t capacity, uint64_t *n_written);

/* Device-pointer tbe_wait_batch (wait = 1, Q:67-134) / tbe_queue_attempt_batch (wait = 0,
 * Q:136-165): every buffer is device memory on the engine's GPU, the call only enqueues
 * (stream semantics as tbe_acquire_batch_device) and the replies equal the host-buffer
 * call's.  NewestFirst evictions are fetched with tbe_evicted (which then synchronises).
 * Invalid requests skip the batch and surface at tbe_synchronize. */
tbe_status tbe_wait_batch_device(tbe_engine *engine, const uint64_t *d_keys, const int32_t *d_permits,
                                 const int64_t *d_ts_us, uint64_t n, int64_t id_base, int32_t wait,
                                 uint8_t *d_status, int32_t *d_remaining, void *stream);

/* Upper bound on the grants one tbe_refresh_device can log: min(entries possibly queued,
 * n_keys * min(max(1, QueueLimit), TokenLimit)) -- a queued entry holds >= 1 permit and
 * a tick grants at most TokenLimit tokens per key. */
tbe_status tbe_refresh_bound(tbe_engine *engine, uint64_t *bound);

/* Device-pointer tbe_refresh (Q:237-271): enqueues one replenish tick at ts_us.  Grants
 * land in the caller's device buffers as (key << 16 | drain position, request id,
 * trunc(new_v)), grouped arbitrarily across keys, and *d_count (device u32) receives
 * their number.  capacity must be >= tbe_refresh_bound (TBE_EINVAL otherwise), so no
 * grant is ever dropped. */
tbe_status tbe_refresh_device(tbe_engine *engine, int64_t ts_us, uint64_t *d_keyseq,
                              int64_t *d_request_id, int32_t *d_remaining, uint64_t capacity,
                              uint32_t *d_count, void *stream);

/* tbe_wait_batch_device followed by tbe_refresh_device(tick_ts_us), fused: the batch's
 * fold drains every key of its bucket at tick_ts_us right after the batch's requests,
 * on the rows and queue headers it already holds in LDS, so the tick costs no separate
 * pass over the table (Q:67-134 then Q:237-271; results, logs and engine state equal
 * the two calls').  capacity must cover tbe_refresh_bound as it stands AFTER the batch
 * (the batch's own enqueues count).  An invalid batch skips the tick too (the call is
 * one unit); it surfaces at tbe_synchronize like any device batch. */
tbe_status tbe_wait_batch_tick_device(tbe_engine *engine, const uint64_t *d_keys, const int32_t *d_permits,
                                      const int64_t *d_ts_us, uint64_t n, int64_t id_base, int32_t wait,
                                      uint8_t *d_status, int32_t *d_remaining, int64_t tick_ts_us,
                                      uint64_t *d_keyseq, int64_t *d_request_id, int32_t *d_log_remaining,
                                      uint64_t capacity, uint32_t *d_count, void *stream);

/* Queue of one key, oldest first (Deque enumeration order, DQ:116-125). */
tbe_status tbe_queue_of(tbe_engine *engine, uint64_t key, int64_t *request_id, int32_t *permits,
                        uint32_t capacity, uint32_t *count);

/* Cancellation of queued requests (the CancellationToken registration of a queued
 * WaitAsync: CancelQueueState.TrySetCanceled, Q:480-506 / A:531-557), queueing and
 * approximate kinds.  Cancels are applied in call order; cancelled[i] = 1 when
 * request_ids[i] was queued on keys[i] and is now removed: _queueCount (qsum) drops by its
 * permits and the entries behind it keep their order.  0 when it is not queued there
 * (already granted, evicted, failed or canceled: TrySetCanceled returns false).  Decision
 * (DESIGN.md §2b): the entry leaves the queue at once, so the drain neither grants it nor
 * waits on it; the reference leaves it in its deque until the drain dequeues it, which
 * consumes its tokens and, in A:489, adds them back twice.
 * Ordered after every batch enqueued before the call; synchronous.  *n_cancelled gets
 * the number of 1s.  key >= n_keys: TBE_EINVAL, nothing canceled. */
tbe_status tbe_queue_cancel(tbe_engine *engine, const uint64_t *keys, const int64_t *request_ids,
                            uint64_t n, uint8_t *cancelled, uint64_t *n_cancelled);

/* ---------------------------------------------------------------- ApproximateTokenBucket
 * Engines created with kind = TBE_KIND_APPROXIMATE hold ONE client's local tier for every
 * key (ApproximateTokenBucket/RedisApproximateTokenBucketRateLimiter.cs, "A") plus a
 * replica of the shared global tier (the sync script's Redis hash, A:241-270).  Status
 * codes are the TBE_WAIT_* values; available[i] is AvailableTokens (A:37) after the
 * decision (-1 for REJECTED). */

/* wait = 0: AcquireCore (A:84-113, never queues); wait = 1: WaitAsyncCore (A:116-183).
 * A zero-permit wait while AvailableTokens is 0 queues with Count 0 (A:127-181: TryLease
 * fails on `availableTokens != 0` and `QueueLimit - _queueCount < 0` never holds), holds
 * no queue permits, completes at the first drain that reaches it (A:474: AvailableTokens
 * >= 0) and is evicted from the head like any registration (A:145-156).  The reference
 * queues any number of them; a key holds at most tbe_config.zero_wait_slots, beyond which
 * the wait is FAILED. */
tbe_status tbe_approx_acquire_batch(tbe_engine *engine, const uint64_t *keys, const int32_t *permits,
                                    uint64_t n, int32_t wait, int64_t id_base, uint8_t *status,
                                    int32_t *available, uint64_t *n_evicted);

/* Device-pointer tbe_approx_acquire_batch (A:84-183): device buffers, enqueue only
 * (stream semantics as tbe_acquire_batch_device); evictions via tbe_evicted. */
tbe_status tbe_approx_acquire_batch_device(tbe_engine *engine, const uint64_t *d_keys,
                                           const int32_t *d_permits, uint64_t n, int32_t wait,
                                           int64_t id_base, uint8_t *d_status, int32_t *d_available,
                                           void *stream);

/* Refresh step 1 (A:430-435): d_counts[k] = _localThrottleScore of key k, then 0.
 * d_counts is device memory for n_keys int32 (the caller exchanges it between clients,
 * e.g. an RCCL all-gather over xGMI). */
tbe_status tbe_approx_collect(tbe_engine *engine, int32_t *d_counts, void *stream);

/* Refresh step 2 (A:439-508): replay the sync script for every key, once per client in
 * client order, client r at ts_us + r*stagger_us with LocalCount d_all_counts[r*n_keys+k]
 * (device memory, n_clients * n_keys int32), keep client `my_client`'s reply (global
 * score, period via "%.14g" -> est), then drain the queues; fetch the completed queued
 * requests with tbe_refresh_log.  n_clients = 1 with summed counts makes the node one
 * client (an all-reduce instead of an all-gather).
 * Completion contract: the kernel runs on the engine's stream, ordered after the engine's
 * own earlier batches but after NO other stream, so d_all_counts must be complete when
 * this is called (e.g. the producer stream synchronised).  A caller whose counts come from
 * work still in flight on another stream (an RCCL all-gather, torch.cat on a side stream)
 * uses tbe_approx_sync_stream.  Returns when the replay and the drain log are done. */
tbe_status tbe_approx_sync(tbe_engine *engine, const int32_t *d_all_counts, uint32_t n_clients,
                           uint32_t my_client, int64_t ts_us, int64_t stagger_us, uint64_t *n_granted);

/* tbe_approx_sync ordered after `stream` (a hipStream_t; NULL = tbe_approx_sync): the
 * engine records an event on it and its stream waits for that event before the replay
 * reads d_all_counts, so the counts may still be being produced on `stream` at the call
 * (A:439).  No host synchronisation of `stream` is needed. */
tbe_status tbe_approx_sync_stream(tbe_engine *engine, const int32_t *d_all_counts, uint32_t n_clients,
                                  uint32_t my_client, int64_t ts_us, int64_t stagger_us, void *stream,
                                  uint64_t *n_granted);

/* RefreshAsync of a limiter that is the only client of its global tier (A:412-508): the
 * same as tbe_approx_collect followed by tbe_approx_sync with n_clients = 1, as one kernel
 * pass over the local tier (each key's local count is swapped to 0 and used as the sync
 * call's LocalCount; no host round trip between the two).  Completed queued requests via
 * tbe_refresh_log. */
tbe_status tbe_approx_refresh(tbe_engine *engine, int64_t ts_us, uint64_t *n_granted);

/* Local-tier state of one key: _localThrottleScore, _globalThrottleScore,
 * _instanceCountEstimate, AvailableTokens (GetAvailablePermits, A:81), queued requests. */
tbe_status tbe_approx_query(tbe_engine *engine, uint64_t key, int32_t *local, int32_t *global_score,
                            double *est, int32_t *available, uint32_t *queued);

/* Snapshot/restore of the approximate kind's replica of the global tier: per key the
 * Redis hash {v, p, t} that the sync script writes with a one-day TTL (A:265-268);
 * t_us[k] is the injected TIME of the key's last sync, INT64_MIN when absent (then v = p
 * = 0, the script's default, A:250-252).  The local tier is in-process state in the
 * reference (A:36-40) and is not part of it.  Import: t_us must be INT64_MIN or >= 0;
 * both calls are ordered after every batch and sync enqueued before them.  Every rank of
 * a node imports the same snapshot so that the replicas stay identical. */
tbe_status tbe_approx_export_state(tbe_engine *engine, uint64_t first, uint64_t count, double *v,
                                   double *p, int64_t *t_us);
tbe_status tbe_approx_import_state(tbe_engine *engine, uint64_t first, uint64_t count, const double *v,
                                   const double *p, const int64_t *t_us);

/* How the engine lays a batch out (for reports and tests): *passes = 8-bit partition
 * passes over the bucket id, *r_bits = log2 of the keys per bucket (one workgroup
 * each), *packed: bit 0 set when the passes move packed 8-byte request records (token
 * bucket kind) rather than the wide {key, permits, ts} records, bit 1 set
 * when hot keys get runs of their own (TBE_FLAG_NO_HOT clears it), bit 2 set when
 * consecutive device batches overlap (TBE_FLAG_NO_PIPELINE clears it), bit 3 set when
 * replies travel as one byte (TBE_FLAG_NO_NARROW clears it), bit 4 set when the queueing
 * or approximate kind's replies travel as two bytes, bit 5 set when the last partition
 * pass writes fold records (TBE_FLAG_UNSCATTER_ALL clears it; used by batches whose
 * reply position and time offset fit), bit 6 set when the second
 * pass's histogram reads the one-byte digit stream (TBE_FLAG_HIST_RECORDS clears it),
 * bit 7 set when the final un-partition re-ranks pass 0's tiles (TBE_FLAG_RERANK sets
 * it), bit 8 set when pass 0 writes narrow 4-byte records (token bucket and queueing kinds
 * with fold records and the digit stream, and the approximate kind's AcquireCore batches; a
 * batch uses them when it uses fold records), bit 9 set when the queueing kind stores its
 * per-key queue headers in 32 bits (QueueLimit <= 1024). */
tbe_status tbe_layout(const tbe_engine *engine, uint32_t *passes, uint32_t *r_bits, uint32_t *packed);

/* The record layout a batch of n requests takes (diagnostics and tests):
 * out[0] partition passes, out[1] 1 if the last pass writes fold records, out[2] their
 * reply-position bits (ceil_log2 n), out[3] their time-offset bits, out[4] the pass-0
 * record's key bits, out[5] permit-code bits, out[6] pass-0 time-offset bits, out[7]
 * r_bits, and when n_out > 8, out[8] 1 if the batch is a sparse token-bucket batch
 * (fewer than R >> TBE_SPARSE_GATE_SHIFT = R/8 requests per bucket on average, R = 2^r_bits
 * keys per bucket: one wave per sparse bucket, the dense buckets listed for the wide
 * fold; hot-key runs only from 2^TBE_HOT_SPARSE_MIN_LOG2 = 2^20 requests, a smaller
 * sparse batch leaves the hot sets as they are).  n_out must be >= 8.  A request
 * whose time offset does not fit takes the escape form (its time is read from the
 * previous record / the caller's array). */
tbe_status tbe_batch_format(const tbe_engine *engine, uint64_t n, uint32_t *out, uint32_t n_out);

/* Per-stage device time (ms) accumulated since the last call, when
 * TBE_FLAG_STAGE_TIMING is set: out[0..n_out) = {hist, colscan, scatter, bounds,
 * fold, unscatter}.  Returns the number of stages written via *n_written. */
tbe_status tbe_stage_times(tbe_engine *engine, double *out, uint32_t n_out, uint32_t *n_written);

#ifdef __cplusplus
}
#endif

#endif /* TBE_H_ */
