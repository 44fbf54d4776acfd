/*
 * tbe_cluster.h -- multi-GPU data path of the engine, C ABI.
 *
 * The reference distributes by letting every client process share ONE Redis key space
 * (README:1-9; the bucket key is InstanceName + resourceID, PTB:42).  Here each GPU
 * owns a hash partition of the keys and holds their buckets in its own HBM:
 *
 *   owner(key) = ((mix64(key) >> 32) * n_owners) >> 32
 *              = mix64(key) >> (64 - log2 n_owners)      for a power-of-two n_owners
 *
 * Requests that arrive at the wrong GPU are routed with one all-to-all (RCCL over xGMI,
 * driven by the host through torch.distributed): tbe_route_plan_device groups a batch by
 * owner, stably (arrival order kept inside each owner's group), tbe_route_pack_device
 * lays the groups out as the all-to-all's send buffer, and after the owners decide,
 * tbe_route_gather_device puts the replies back in arrival order.  On the owner, a
 * device-resident key directory (tbe_dir_*) turns the owned global keys into dense local
 * bucket ids, collision-free (it compares whole keys).  Everything stays in HBM; only the
 * n_owners group sizes cross to the host (the all-to-all's split sizes).
 *
 * All calls enqueue on `stream` (hipStream_t, NULL = the default stream) and return
 * TBE_OK, or TBE_EINVAL for bad arguments (nothing enqueued).
 */
#ifndef TBE_CLUSTER_H_
#define TBE_CLUSTER_H_

#include <stdint.h>

#include "tbe.h"

#ifdef __cplusplus
extern "C" {
#endif

/* owner(key) as above, on the host (the device kernels use the same function). */
uint32_t tbe_key_owner(uint64_t key, uint32_t n_owners);

/* Stable partition of a batch by owner, 1 <= n_owners <= 256, n < 2^32:
 * d_counts[o] (u64) = requests of owner o; d_pos[i] = position of request i in the
 * owner-grouped order (owner-major, arrival order inside an owner).  Uses a workspace
 * of tbe_route_workspace_bytes(n, n_owners) bytes at d_work. */
uint64_t tbe_route_workspace_bytes(uint64_t n, uint32_t n_owners);
tbe_status tbe_route_plan_device(const uint64_t *d_keys, uint64_t n, uint32_t n_owners, void *d_work,
                                 uint32_t *d_pos, uint64_t *d_counts, void *stream);

/* ---------------------------------------------------------------- owner maps
 * Table-driven ownership (DESIGN.md §7 "owner maps"): owner(key) = map[vnode(key)], with
 * vnode(key) = mix64(key) >> 52, one of TBE_OWNER_MAP_SIZE virtual nodes, and `map` a u8
 * array of TBE_OWNER_MAP_SIZE owners (4-byte aligned), the same on every GPU.  The map
 * v -> (v * n_owners) >> 12 is the hash partition above for a power-of-two n_owners; a
 * balanced map gives the virtual nodes of hot keys' owners fewer others, so a Zipf
 * stream's owner loads even out (SURVEY.md §7 hard part iii).  A key still has exactly
 * one owner; the map must not change while any owner holds state. */
#define TBE_OWNER_MAP_BITS 12
#define TBE_OWNER_MAP_SIZE 4096
uint32_t tbe_key_vnode(uint64_t key);
/* tbe_route_plan_device with owner = d_owner_map[vnode(key)] (d_owner_map NULL: the hash
 * partition, exactly tbe_route_plan_device); every map entry must be < n_owners. */
tbe_status tbe_route_plan_map_device(const uint64_t *d_keys, uint64_t n, uint32_t n_owners,
                                     const uint8_t *d_owner_map, void *d_work, uint32_t *d_pos,
                                     uint64_t *d_counts, void *stream);
/* d_counts[v] (u64, TBE_OWNER_MAP_SIZE of them, zeroed first) = requests of the batch on
 * virtual node v: the load histogram a balanced map is built from. */
tbe_status tbe_vnode_count_device(const uint64_t *d_keys, uint64_t n, uint64_t *d_counts, void *stream);

/* Send buffer of the routing all-to-all: out[pos[i]] = {key, ts_us, permits} as three
 * int64 per request (d_out holds 3n). */
tbe_status tbe_route_pack_device(const uint32_t *d_pos, uint64_t n, const uint64_t *d_keys,
                                 const int32_t *d_permits, const int64_t *d_ts_us, int64_t *d_out,
                                 void *stream);

/* Replies back to arrival order: out[i*cols + c] = in[pos[i]*cols + c], 1 <= cols <= 8. */
tbe_status tbe_route_gather_device(const uint32_t *d_pos, uint64_t n, const int64_t *d_in, uint32_t cols,
                                   int64_t *d_out, void *stream);

/* ---------------------------------------------------------------- key directory
 * Global key (any u64 but UINT64_MAX) -> dense local id in [0, capacity), assigned when a
 * key is first seen: keys new to the directory get consecutive counters in order of
 * first occurrence (batches in call order, arrival order inside a batch), and the id is
 * a fixed bijection of [0, capacity) applied to the counter (so hot keys, which are seen
 * first, do not crowd the first buckets).  Collision-free: the table stores whole keys.
 * Capacity: once a batch brings more new keys than `capacity` ids remain, tbe_dir_size
 * reports TBE_ERANGE from then on and the directory must be recreated.  In such a batch
 * every key that gets an id keeps a unique one in [0, capacity), but which of the new
 * keys get one is unspecified (the hash table, 2x capacity, may fill up first); the
 * others get UINT64_MAX, and an engine batch containing them is rejected as invalid. */
typedef struct tbe_directory tbe_directory;

tbe_status tbe_dir_create(uint64_t capacity, int32_t device, tbe_directory **out);
void tbe_dir_destroy(tbe_directory *dir);
/* d_ids[i] = id of d_keys[i] (assigning new ones).  n < 2^32. */
tbe_status tbe_dir_assign_device(tbe_directory *dir, const uint64_t *d_keys, uint64_t n, uint64_t *d_ids,
                                 void *stream);
/* d_ids[i] = id of d_keys[i], UINT64_MAX for a key never assigned (nothing changes). */
tbe_status tbe_dir_lookup_device(tbe_directory *dir, const uint64_t *d_keys, uint64_t n, uint64_t *d_ids,
                                 void *stream);
/* Ids assigned so far (synchronises the directory's device). */
tbe_status tbe_dir_size(tbe_directory *dir, uint64_t *n_ids);
/* The same without synchronising: enqueues on `stream` a copy of {ids assigned, error
 * bits} (two u64; error bits != 0 once a batch exceeded the capacity, the condition
 * tbe_dir_size reports as TBE_ERANGE) into out2, pinned host or device memory.  Lets a
 * caller notice an overflow a batch later without a device synchronisation per batch;
 * the batch that overflowed is caught by the engine anyway (its UINT64_MAX ids make the
 * engine batch invalid). */
tbe_status tbe_dir_state_async(tbe_directory *dir, uint64_t *out2, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* TBE_CLUSTER_H_ */
