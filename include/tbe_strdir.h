/*
 * tbe_strdir.h -- device-resident string-key directory, C ABI.
 *
 * The reference's bucket key is the exact string InstanceName + resourceID
 * (PartitionedRedisTokenBucketRateLimiter.cs:42, `BucketId = InstanceName + resourceID`);
 * Redis keys are compared byte for byte, so two resource ids never share a bucket.  This
 * directory maps such strings to the engine's dense key ids in HBM, batch at a time:
 *
 *   - a directory belongs to one limiter and holds its InstanceName as `prefix`; the
 *     strings passed per request are the resourceIDs (the key is prefix + resourceID);
 *   - strings are compared byte for byte (a 64-bit hash only chooses the slot: at 1e8
 *     keys two of them share a hash with probability ~2.7e-4), so the
 *     mapping is collision-free;
 *   - ids are assigned exactly like tbe_dir_* (tbe_cluster.h): strings new to the
 *     directory get consecutive counters in order of first occurrence (batches in call
 *     order, arrival order inside a batch) and id = a fixed bijection of [0, capacity)
 *     applied to the counter.  An id depends only on that order, never on hashes.
 *
 * Batch layout (Arrow-style string array): string i is bytes [offs[i], offs[i+1]) of
 * `bytes`; offs has n + 1 u64 entries, non-decreasing, offs[n] <= n_bytes; a string is
 * at most 65536 bytes; `bytes` is 8-byte aligned.  A request whose offsets break these
 * rules gets id UINT64_MAX and the directory's error state (tbe_sdir_size: TBE_EINVAL).
 *
 * Limits: `capacity` ids and `arena_bytes` bytes of key text (each key takes its length
 * rounded up to 8).  A batch that brings more new keys than either limit leaves the
 * directory in the TBE_ERANGE state: keys that got an id keep it, unique; the others get
 * UINT64_MAX (an engine batch containing them is rejected) and the directory must be
 * recreated.
 *
 * All device calls enqueue on `stream` (hipStream_t; NULL = the default stream).
 */
#ifndef TBE_STRDIR_H_
#define TBE_STRDIR_H_

#include <stdint.h>

#include "tbe.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tbe_string_directory tbe_string_directory;

/* prefix: InstanceName (prefix_len bytes, may be 0). */
tbe_status tbe_sdir_create(uint64_t capacity, uint64_t arena_bytes, const char *prefix, uint32_t prefix_len,
                           int32_t device, tbe_string_directory **out);
void tbe_sdir_destroy(tbe_string_directory *dir);

/* d_ids[i] = id of string i (assigning new ones).  n < 2^32. */
tbe_status tbe_sdir_assign_device(tbe_string_directory *dir, const uint8_t *d_bytes, uint64_t n_bytes,
                                  const uint64_t *d_offs, uint64_t n, uint64_t *d_ids, void *stream);
/* d_ids[i] = id of string i, UINT64_MAX for a string never assigned (nothing changes). */
tbe_status tbe_sdir_lookup_device(tbe_string_directory *dir, const uint8_t *d_bytes, uint64_t n_bytes,
                                  const uint64_t *d_offs, uint64_t n, uint64_t *d_ids, void *stream);
/* Host buffers (staged through the directory's device; synchronises before returning). */
tbe_status tbe_sdir_assign(tbe_string_directory *dir, const uint8_t *bytes, uint64_t n_bytes,
                           const uint64_t *offs, uint64_t n, uint64_t *ids);

/* Ids assigned so far (synchronises).  TBE_ERANGE after a capacity or arena overflow (or
 * a string whose hashes collided in all four probe rounds: never observed with 64-bit
 * hashes), TBE_EINVAL after a malformed batch. */
tbe_status tbe_sdir_size(tbe_string_directory *dir, uint64_t *n_ids);

/* Key text of an id (resourceID part, without the prefix): *len = its length; copies
 * min(len, cap) bytes to buf.  TBE_EINVAL for an id never assigned.  Synchronises. */
tbe_status tbe_sdir_key_of(tbe_string_directory *dir, uint64_t id, uint8_t *buf, uint64_t cap, uint64_t *len);

/* Assign path: 0 = automatic (default), 1 = full pass, 2 = warm path.  The warm path first
 * resolves every string of the batch that is already known (one lookup pass: hash,
 * probe, byte compare with the stored text) and runs the assign passes over the misses
 * only, listed in arrival order; automatic takes it while the last batch whose id count
 * has come back brought new keys for less than half of its requests.  Ids, errors and
 * the directory's state are the same on either path. */
tbe_status tbe_sdir_set_mode(tbe_string_directory *dir, int32_t mode);

/* Test hook: keep only the low `bits` (1..62) bits of every string hash, so that distinct
 * strings share hashes often and the byte comparison and re-probe rounds run.  Ids do not
 * change (they depend only on first occurrence).  Only before the first assign. */
tbe_status tbe_sdir_set_hash_bits(tbe_string_directory *dir, uint32_t bits);

#ifdef __cplusplus
}
#endif

#endif /* TBE_STRDIR_H_ */
