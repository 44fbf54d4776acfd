// tbe_cluster.hip -- multi-GPU data path (include/tbe_cluster.h): stable
// routing partition of request batches by owner GPU and the per-GPU key directory.
//
// Routing: the reference serialises every client's script calls in one Redis (README:1-9),
// so any order in which a key's requests reach it is a valid serial order.  A batch that
// arrives at one GPU is grouped by owner with a stable partition (arrival order kept per
// owner); the all-to-all concatenates the groups by source rank, so each owner applies a
// key's requests in (source rank, arrival) order.
//
// Directory: InstanceName + resourceID is an exact string in Redis (PTB:42), never a
// hash; the directory keeps whole keys, so two keys never share a bucket.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <new>

#include "../../include/tbe_cluster.h"
#include "tbe_device.hpp"
#include "tbe_hash.hpp"

using namespace tbe;

namespace {

constexpr int kRtBlock = 512;
constexpr int kRtItems = 8;
constexpr int kRtTile = kRtBlock * kRtItems;   // 4096 requests per routing tile
constexpr uint32_t kMaxOwners = 256;

// Owner of a key: the hash partition, or the owner map's entry for its virtual node
// (`m` = the workgroup's LDS copy of the map, filled by load_owner_map).
__device__ __forceinline__ uint32_t route_owner(uint64_t key, uint32_t G, const uint8_t *m) {
    return m ? (uint32_t)m[key_vnode(key)] : key_owner(key, G);
}
// Entries >= G are clamped to G - 1 on the way into LDS, so a malformed map (the header
// requires every entry < n_owners; cluster.py validates before calling) misroutes requests
// but can never index the per-owner arrays out of bounds.
__device__ __forceinline__ const uint8_t *load_owner_map(const uint8_t *__restrict__ omap, uint8_t *lds,
                                                         uint32_t G) {
    if (!omap) return nullptr;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(omap);
    uint32_t *dst = reinterpret_cast<uint32_t *>(lds);
    const uint32_t top = G - 1u;
    for (uint32_t j = threadIdx.x; j < kOwnerMapSize / 4; j += blockDim.x) {
        const uint32_t w = src[j];
        uint32_t o = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) o |= min((w >> (8 * b)) & 0xFFu, top) << (8 * b);
        dst[j] = o;
    }
    __syncthreads();
    return lds;
}

// Per-tile request count of every owner.
__global__ __launch_bounds__(kRtBlock) void k_route_count(const uint64_t *__restrict__ keys, uint64_t n,
                                                          uint32_t G, const uint8_t *__restrict__ omap,
                                                          uint32_t *__restrict__ tile_counts) {
    __shared__ uint32_t c[kMaxOwners];
    __shared__ __attribute__((aligned(16))) uint8_t mlds[kOwnerMapSize];
    const int tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * kRtTile;
    for (uint32_t j = tid; j < G; j += kRtBlock) c[j] = 0;
    const uint8_t *m = load_owner_map(omap, mlds, G);   // (its barrier also publishes c[])
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kRtItems; ++it) {
        const uint64_t i = base + (uint64_t)it * kRtBlock + tid;
        if (i < n) atomicAdd(&c[route_owner(keys[i], G, m)], 1u);
    }
    __syncthreads();
    for (uint32_t j = tid; j < G; j += kRtBlock) tile_counts[(uint64_t)blockIdx.x * G + j] = c[j];
}

// One workgroup: per owner, the exclusive scan of its tile counts (in place) and its
// total; then owner bases (exclusive scan over owners).
constexpr int kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void k_route_scan(uint32_t *__restrict__ tile_counts, uint32_t ntiles,
                                                             uint32_t G, uint64_t *__restrict__ owner_counts,
                                                             uint32_t *__restrict__ owner_base) {
    __shared__ uint32_t wsum[kScanThreads / 64];
    __shared__ uint32_t totals[kMaxOwners];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (ntiles + kScanThreads - 1) / kScanThreads;
    for (uint32_t o = 0; o < G; ++o) {
        uint32_t sum = 0;
        for (uint32_t k = 0; k < per; ++k) {
            const uint32_t tile = t * per + k;
            if (tile < ntiles) sum += tile_counts[(uint64_t)tile * G + o];
        }
        uint32_t tot;
        uint32_t run = block_excl_scan<kScanThreads>(sum, wsum, &tot);
        for (uint32_t k = 0; k < per; ++k) {
            const uint32_t tile = t * per + k;
            if (tile < ntiles) {
                const uint32_t c = tile_counts[(uint64_t)tile * G + o];
                tile_counts[(uint64_t)tile * G + o] = run;
                run += c;
            }
        }
        if (t == 0) totals[o] = tot;
    }
    __syncthreads();
    if (t == 0) {
        uint32_t acc = 0;
        for (uint32_t o = 0; o < G; ++o) {
            owner_base[o] = acc;
            owner_counts[o] = totals[o];
            acc += totals[o];
        }
    }
}

// Position of every request in the owner-grouped order: owner base + the tile's offset
// in that owner's group + the request's stable rank among the tile's requests of that
// owner (wave ballot-match ranking, as the partition passes use).
__global__ __launch_bounds__(kRtBlock) void k_route_pos(const uint64_t *__restrict__ keys, uint64_t n, uint32_t G,
                                                        const uint8_t *__restrict__ omap,
                                                        const uint32_t *__restrict__ tile_off,
                                                        const uint32_t *__restrict__ owner_base,
                                                        uint32_t *__restrict__ pos) {
    __shared__ RankLds<kRtBlock> L;
    __shared__ uint16_t cnt[kRtItems * (kRtBlock / 64) * kDigits];
    __shared__ __attribute__((aligned(16))) uint8_t mlds[kOwnerMapSize];
    const int tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * kRtTile;
    const int nvalid = (int)min<uint64_t>(kRtTile, n - base);
    const uint8_t *m = load_owner_map(omap, mlds, G);
    uint32_t own[kRtItems], lpos[kRtItems];
#pragma unroll
    for (int it = 0; it < kRtItems; ++it) {
        const int e = it * kRtBlock + tid;
        own[it] = e < nvalid ? route_owner(keys[base + e], G, m) : 0u;
    }
    rank_tile<kRtBlock, kRtItems>(own, 0, nvalid, L, cnt, lpos);
#pragma unroll
    for (int it = 0; it < kRtItems; ++it) {
        const int e = it * kRtBlock + tid;
        if (e < nvalid) {
            const uint32_t o = own[it];
            pos[base + e] = owner_base[o] + tile_off[(uint64_t)blockIdx.x * G + o] + lpos[it] - L.lstart[o];
        }
    }
}

// Requests per virtual node (owner-map balancing): an LDS histogram per workgroup over a
// grid-stride range, added to the 4096 global counters once.
__global__ __launch_bounds__(kRtBlock) void k_vnode_count(const uint64_t *__restrict__ keys, uint64_t n,
                                                          unsigned long long *__restrict__ counts) {
    __shared__ uint32_t h[kOwnerMapSize];
    for (uint32_t j = threadIdx.x; j < kOwnerMapSize; j += kRtBlock) h[j] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * kRtBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kRtBlock + threadIdx.x; i < n; i += stride)
        atomicAdd(&h[key_vnode(keys[i])], 1u);
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < kOwnerMapSize; j += kRtBlock)
        if (h[j]) atomicAdd(&counts[j], (unsigned long long)h[j]);
}

__global__ void k_route_pack(const uint32_t *__restrict__ pos, uint64_t n, const uint64_t *__restrict__ keys,
                             const int32_t *__restrict__ permits, const int64_t *__restrict__ ts,
                             int64_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t q = (uint64_t)pos[i] * 3;
        out[q] = (int64_t)keys[i];
        out[q + 1] = ts[i];
        out[q + 2] = permits[i];
    }
}

__global__ void k_route_gather(const uint32_t *__restrict__ pos, uint64_t n, const int64_t *__restrict__ in,
                               uint32_t cols, int64_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t q = (uint64_t)pos[i] * cols;
        for (uint32_t c = 0; c < cols; ++c) out[i * cols + c] = in[q + c];
    }
}

// ---------------------------------------------------------------- directory
constexpr uint64_t kEmptyKey = ~0ull;
constexpr uint32_t kNoId = 0xFFFFFFFFu;
constexpr int kDirBlock = 256;
constexpr int kDirTile = 1024;   // requests per flag block (4 per thread)

// Find or claim the slot of every key (linear probing on the whole key); a slot claimed
// in this batch records the arrival index of its first request (atomicMin).
__global__ __launch_bounds__(kDirBlock) void k_dir_claim(const uint64_t *__restrict__ keys, uint64_t n,
                                                         uint64_t *__restrict__ skey,
                                                         const uint32_t *__restrict__ sid,
                                                         uint32_t *__restrict__ sfirst, uint64_t smask,
                                                         uint32_t *__restrict__ slot_of,
                                                         unsigned long long *__restrict__ err) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t key = keys[i];
        uint32_t found = kNoId;
        if (key != kEmptyKey) {
            uint64_t h = mix64(key) & smask;
            for (uint64_t probe = 0; probe <= smask; ++probe) {
                const uint64_t cur = skey[h];
                if (cur == key) {
                    found = (uint32_t)h;
                    break;
                }
                if (cur == kEmptyKey) {
                    const unsigned long long prev =
                        atomicCAS(reinterpret_cast<unsigned long long *>(&skey[h]), kEmptyKey, key);
                    if (prev == kEmptyKey || prev == key) {
                        found = (uint32_t)h;
                        break;
                    }
                }
                h = (h + 1) & smask;
            }
        }
        slot_of[i] = found;
        if (found == kNoId) {
            atomicOr(err, 1ull);            // UINT64_MAX key, or a full table
        } else if (sid[found] == kNoId) {
            atomicMin(&sfirst[found], (uint32_t)i);
        }
    }
}

__device__ __forceinline__ bool dir_is_new(const uint32_t *slot_of, const uint32_t *sid, const uint32_t *sfirst,
                                           uint64_t i) {
    const uint32_t sl = slot_of[i];
    return sl != kNoId && sid[sl] == kNoId && sfirst[sl] == (uint32_t)i;
}

// New keys per block of kDirTile requests.
__global__ __launch_bounds__(kDirBlock) void k_dir_count(const uint32_t *__restrict__ slot_of, uint64_t n,
                                                         const uint32_t *__restrict__ sid,
                                                         const uint32_t *__restrict__ sfirst,
                                                         uint32_t *__restrict__ bsum) {
    __shared__ uint32_t wsum[kDirBlock / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kDirTile;
    uint32_t c = 0;
    for (int k = 0; k < kDirTile / kDirBlock; ++k) {
        const uint64_t i = base + (uint64_t)threadIdx.x * (kDirTile / kDirBlock) + k;
        if (i < n && dir_is_new(slot_of, sid, sfirst, i)) ++c;
    }
    uint32_t tot;
    (void)block_excl_scan<kDirBlock>(c, wsum, &tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// Exclusive scan of the block counts (in place); base = ids assigned before this batch;
// the running total advances, clamped at capacity (overflow: sticky error).
__global__ __launch_bounds__(kScanThreads) void k_dir_scan(uint32_t *__restrict__ bsum, uint32_t nblk,
                                                           unsigned long long *__restrict__ state,
                                                           uint64_t capacity) {
    __shared__ uint32_t wsum[kScanThreads / 64];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nblk + kScanThreads - 1) / kScanThreads;
    uint32_t sum = 0;
    for (uint32_t k = 0; k < per; ++k) {
        const uint32_t j = t * per + k;
        if (j < nblk) sum += bsum[j];
    }
    uint32_t tot;
    uint32_t run = block_excl_scan<kScanThreads>(sum, wsum, &tot);
    for (uint32_t k = 0; k < per; ++k) {
        const uint32_t j = t * per + k;
        if (j < nblk) {
            const uint32_t c = bsum[j];
            bsum[j] = run;
            run += c;
        }
    }
    if (t == 0) {
        const unsigned long long before = state[0];   // ids assigned so far
        state[2] = before;                            // this batch's base
        unsigned long long after = before + tot;
        if (after > capacity) {
            after = capacity;
            state[1] |= 2ull;                         // capacity exceeded
        }
        state[0] = after;
    }
}

// Assign ids to the new keys: counter = base + rank among the batch's new keys (block
// prefix + rank in block), id = bijection of the counter; beyond capacity, none.
__global__ __launch_bounds__(kDirBlock) void k_dir_assign(const uint32_t *__restrict__ slot_of, uint64_t n,
                                                          uint32_t *__restrict__ sid,
                                                          const uint32_t *__restrict__ sfirst,
                                                          const uint32_t *__restrict__ bsum,
                                                          const unsigned long long *__restrict__ state,
                                                          uint64_t capacity, uint64_t imask, uint32_t ish) {
    __shared__ uint32_t wsum[kDirBlock / 64];
    constexpr int PER = kDirTile / kDirBlock;
    const uint64_t base = (uint64_t)blockIdx.x * kDirTile;
    bool nw[PER];
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const uint64_t i = base + (uint64_t)threadIdx.x * PER + k;
        nw[k] = i < n && dir_is_new(slot_of, sid, sfirst, i);
        c += nw[k];
    }
    uint32_t tot;
    uint32_t r = block_excl_scan<kDirBlock>(c, wsum, &tot);   // every thread has read sid before it returns
    const uint64_t b0 = (uint64_t)state[2] + bsum[blockIdx.x];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        if (!nw[k]) continue;
        const uint64_t i = base + (uint64_t)threadIdx.x * PER + k;
        const uint64_t counter = b0 + r++;
        if (counter < capacity) sid[slot_of[i]] = (uint32_t)scramble_walk(counter, capacity, imask, ish);
    }
}

__global__ void k_dir_gather(const uint32_t *__restrict__ slot_of, uint64_t n, const uint32_t *__restrict__ sid,
                             uint64_t *__restrict__ ids) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t sl = slot_of[i];
        const uint32_t id = sl == kNoId ? kNoId : sid[sl];
        ids[i] = id == kNoId ? ~0ull : (uint64_t)id;
    }
}

// Read-only lookup: id, or UINT64_MAX for a key the directory has never assigned.
__global__ __launch_bounds__(kDirBlock) void k_dir_lookup(const uint64_t *__restrict__ keys, uint64_t n,
                                                          const uint64_t *__restrict__ skey,
                                                          const uint32_t *__restrict__ sid, uint64_t smask,
                                                          uint64_t *__restrict__ ids) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t key = keys[i];
        uint64_t id = ~0ull;
        if (key != kEmptyKey) {
            uint64_t h = mix64(key) & smask;
            for (uint64_t probe = 0; probe <= smask; ++probe) {
                const uint64_t cur = skey[h];
                if (cur == key) {
                    if (sid[h] != kNoId) id = sid[h];
                    break;
                }
                if (cur == kEmptyKey) break;
                h = (h + 1) & smask;
            }
        }
        ids[i] = id;
    }
}

__global__ void k_dir_init(uint64_t *__restrict__ skey, uint32_t *__restrict__ sid, uint32_t *__restrict__ sfirst,
                           uint64_t nslots) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nslots; j += stride) {
        skey[j] = kEmptyKey;
        sid[j] = kNoId;
        sfirst[j] = kNoId;
    }
}

unsigned grid_for(uint64_t n, unsigned block, unsigned cap = 8192) {
    const uint64_t g = (n + block - 1) / block;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, cap));
}

}  // namespace

struct tbe_directory {
    uint64_t capacity = 0;
    uint64_t nslots = 0;
    int device = 0;
    uint64_t imask = 0;
    uint32_t ish = 0;
    uint64_t *skey = nullptr;
    uint32_t *sid = nullptr;
    uint32_t *sfirst = nullptr;
    unsigned long long *state = nullptr;   // [0] ids assigned, [1] error bits, [2] batch base
    uint32_t *slot_of = nullptr;           // per-request slot of the current batch
    uint32_t *bsum = nullptr;
    uint64_t tmp_cap = 0;
};

extern "C" {

uint32_t tbe_key_owner(uint64_t key, uint32_t n_owners) { return n_owners ? key_owner(key, n_owners) : 0u; }

uint64_t tbe_route_workspace_bytes(uint64_t n, uint32_t n_owners) {
    const uint64_t ntiles = (n + kRtTile - 1) / kRtTile;
    return (ntiles * (uint64_t)n_owners + kMaxOwners) * sizeof(uint32_t);
}

tbe_status tbe_route_plan_device(const uint64_t *d_keys, uint64_t n, uint32_t n_owners, void *d_work,
                                 uint32_t *d_pos, uint64_t *d_counts, void *stream) {
    return tbe_route_plan_map_device(d_keys, n, n_owners, nullptr, d_work, d_pos, d_counts, stream);
}

uint32_t tbe_key_vnode(uint64_t key) { return key_vnode(key); }

tbe_status tbe_route_plan_map_device(const uint64_t *d_keys, uint64_t n, uint32_t n_owners,
                                     const uint8_t *d_owner_map, void *d_work, uint32_t *d_pos,
                                     uint64_t *d_counts, void *stream) {
    if (n_owners == 0 || n_owners > kMaxOwners || n >= (1ull << 32) || !d_counts) return TBE_EINVAL;
    if (d_owner_map && (reinterpret_cast<uintptr_t>(d_owner_map) & 3u)) return TBE_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    if (n == 0) return hipMemsetAsync(d_counts, 0, n_owners * sizeof(uint64_t), st) == hipSuccess ? TBE_OK : TBE_EDEVICE;
    if (!d_keys || !d_work || !d_pos) return TBE_EINVAL;
    const uint32_t ntiles = (uint32_t)((n + kRtTile - 1) / kRtTile);
    uint32_t *tile = static_cast<uint32_t *>(d_work);
    uint32_t *obase = tile + (uint64_t)ntiles * n_owners;
    k_route_count<<<ntiles, kRtBlock, 0, st>>>(d_keys, n, n_owners, d_owner_map, tile);
    k_route_scan<<<1, kScanThreads, 0, st>>>(tile, ntiles, n_owners, d_counts, obase);
    k_route_pos<<<ntiles, kRtBlock, 0, st>>>(d_keys, n, n_owners, d_owner_map, tile, obase, d_pos);
    return hipGetLastError() == hipSuccess ? TBE_OK : TBE_EDEVICE;
}

tbe_status tbe_vnode_count_device(const uint64_t *d_keys, uint64_t n, uint64_t *d_counts, void *stream) {
    if (!d_counts || (n && !d_keys)) return TBE_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(d_counts, 0, kOwnerMapSize * sizeof(uint64_t), st) != hipSuccess) return TBE_EDEVICE;
    if (n == 0) return TBE_OK;
    k_vnode_count<<<grid_for(n, kRtBlock, 1024), kRtBlock, 0, st>>>(
        d_keys, n, reinterpret_cast<unsigned long long *>(d_counts));
    return hipGetLastError() == hipSuccess ? TBE_OK : TBE_EDEVICE;
}

tbe_status tbe_route_pack_device(const uint32_t *d_pos, uint64_t n, const uint64_t *d_keys, const int32_t *d_permits,
                                 const int64_t *d_ts_us, int64_t *d_out, void *stream) {
    if (n == 0) return TBE_OK;
    if (!d_pos || !d_keys || !d_permits || !d_ts_us || !d_out) return TBE_EINVAL;
    k_route_pack<<<grid_for(n, 256), 256, 0, (hipStream_t)stream>>>(d_pos, n, d_keys, d_permits, d_ts_us, d_out);
    return hipGetLastError() == hipSuccess ? TBE_OK : TBE_EDEVICE;
}

tbe_status tbe_route_gather_device(const uint32_t *d_pos, uint64_t n, const int64_t *d_in, uint32_t cols,
                                   int64_t *d_out, void *stream) {
    if (n == 0) return TBE_OK;
    if (!d_pos || !d_in || !d_out || cols == 0 || cols > 8) return TBE_EINVAL;
    k_route_gather<<<grid_for(n, 256), 256, 0, (hipStream_t)stream>>>(d_pos, n, d_in, cols, d_out);
    return hipGetLastError() == hipSuccess ? TBE_OK : TBE_EDEVICE;
}

tbe_status tbe_dir_create(uint64_t capacity, int32_t device, tbe_directory **out) {
    if (!out) return TBE_EINVAL;
    *out = nullptr;
    if (capacity == 0 || capacity > 0xFFFFFFFEull) return TBE_EINVAL;
    tbe_directory *d = new (std::nothrow) tbe_directory();
    if (!d) return TBE_ENOMEM;
    if (device >= 0) {
        if (hipSetDevice(device) != hipSuccess) { delete d; return TBE_EDEVICE; }
        d->device = device;
    } else if (hipGetDevice(&d->device) != hipSuccess) {
        delete d;
        return TBE_EDEVICE;
    }
    d->capacity = capacity;
    uint64_t ns = 1;
    while (ns < 2 * capacity) ns <<= 1;   // load <= 1/2
    d->nslots = ns;
    scramble_params(capacity, d->imask, d->ish);
    bool ok = hipMalloc(&d->skey, ns * sizeof(uint64_t)) == hipSuccess &&
              hipMalloc(&d->sid, ns * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&d->sfirst, ns * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&d->state, 4 * sizeof(unsigned long long)) == hipSuccess;
    if (!ok) {
        tbe_dir_destroy(d);
        return TBE_ENOMEM;
    }
    k_dir_init<<<grid_for(ns, 256), 256>>>(d->skey, d->sid, d->sfirst, ns);
    if (hipMemset(d->state, 0, 4 * sizeof(unsigned long long)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        tbe_dir_destroy(d);
        return TBE_EDEVICE;
    }
    *out = d;
    return TBE_OK;
}

void tbe_dir_destroy(tbe_directory *d) {
    if (!d) return;
    (void)hipSetDevice(d->device);
    (void)hipDeviceSynchronize();
    for (void *p : {(void *)d->skey, (void *)d->sid, (void *)d->sfirst, (void *)d->state, (void *)d->slot_of,
                    (void *)d->bsum})
        if (p) (void)hipFree(p);
    delete d;
}

tbe_status tbe_dir_assign_device(tbe_directory *d, const uint64_t *d_keys, uint64_t n, uint64_t *d_ids, void *stream) {
    if (!d) return TBE_EINVAL;
    if (n == 0) return TBE_OK;
    if (!d_keys || !d_ids || n >= (1ull << 32)) return TBE_EINVAL;
    if (hipSetDevice(d->device) != hipSuccess) return TBE_EDEVICE;
    hipStream_t st = (hipStream_t)stream;
    if (n > d->tmp_cap) {
        // the previous batch may still be using the old buffers
        if (hipDeviceSynchronize() != hipSuccess) return TBE_EDEVICE;
        if (d->slot_of) (void)hipFree(d->slot_of);
        if (d->bsum) (void)hipFree(d->bsum);
        d->slot_of = nullptr;
        d->bsum = nullptr;
        d->tmp_cap = 0;
        const uint64_t cap = std::max<uint64_t>(n, 1u << 16);
        if (hipMalloc(&d->slot_of, cap * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc(&d->bsum, ((cap + kDirTile - 1) / kDirTile) * sizeof(uint32_t)) != hipSuccess)
            return TBE_ENOMEM;
        d->tmp_cap = cap;
    }
    const uint32_t nblk = (uint32_t)((n + kDirTile - 1) / kDirTile);
    k_dir_claim<<<grid_for(n, kDirBlock), kDirBlock, 0, st>>>(d_keys, n, d->skey, d->sid, d->sfirst, d->nslots - 1,
                                                             d->slot_of, d->state + 1);
    k_dir_count<<<nblk, kDirBlock, 0, st>>>(d->slot_of, n, d->sid, d->sfirst, d->bsum);
    k_dir_scan<<<1, kScanThreads, 0, st>>>(d->bsum, nblk, d->state, d->capacity);
    k_dir_assign<<<nblk, kDirBlock, 0, st>>>(d->slot_of, n, d->sid, d->sfirst, d->bsum, d->state, d->capacity,
                                             d->imask, d->ish);
    k_dir_gather<<<grid_for(n, 256), 256, 0, st>>>(d->slot_of, n, d->sid, d_ids);
    return hipGetLastError() == hipSuccess ? TBE_OK : TBE_EDEVICE;
}

tbe_status tbe_dir_lookup_device(tbe_directory *d, const uint64_t *d_keys, uint64_t n, uint64_t *d_ids, void *stream) {
    if (!d) return TBE_EINVAL;
    if (n == 0) return TBE_OK;
    if (!d_keys || !d_ids) return TBE_EINVAL;
    if (hipSetDevice(d->device) != hipSuccess) return TBE_EDEVICE;
    k_dir_lookup<<<grid_for(n, kDirBlock), kDirBlock, 0, (hipStream_t)stream>>>(d_keys, n, d->skey, d->sid,
                                                                               d->nslots - 1, d_ids);
    return hipGetLastError() == hipSuccess ? TBE_OK : TBE_EDEVICE;
}

tbe_status tbe_dir_state_async(tbe_directory *d, uint64_t *out2, void *stream) {
    if (!d || !out2) return TBE_EINVAL;
    if (hipSetDevice(d->device) != hipSuccess) return TBE_EDEVICE;
    return hipMemcpyAsync(out2, d->state, 2 * sizeof(uint64_t), hipMemcpyDefault, (hipStream_t)stream) == hipSuccess
               ? TBE_OK
               : TBE_EDEVICE;
}

tbe_status tbe_dir_size(tbe_directory *d, uint64_t *n_ids) {
    if (!d || !n_ids) return TBE_EINVAL;
    if (hipSetDevice(d->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return TBE_EDEVICE;
    unsigned long long st[2] = {0, 0};
    if (hipMemcpy(st, d->state, sizeof st, hipMemcpyDeviceToHost) != hipSuccess) return TBE_EDEVICE;
    *n_ids = st[0];
    return st[1] ? TBE_ERANGE : TBE_OK;
}

}  // extern "C"
