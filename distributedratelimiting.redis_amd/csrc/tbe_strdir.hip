// tbe_strdir.hip -- device string-key directory (include/tbe_strdir.h, SURVEY.md §8(f)
// row 2): InstanceName + resourceID (PartitionedRedisTokenBucketRateLimiter.cs:42) ->
// dense key id, exact byte comparison, ids by first occurrence.
//
// Layout in HBM (nslots = pow2 >= 2 * capacity, load <= 1/2):
//   stag[s]   u64  the slot's tag (below), ~0 = empty
//   sid[s]    u32  the key's id once assigned (kNoId before)
//   sfirst[s] u32  arrival index of the key's first request in the batch that claimed it
//   sloc[s]   u64  bit 63 | (arena offset << 17) | length of the key's text, once assigned
//   iloc[id]  u64  the same per id (tbe_sdir_key_of)
//   arena     key text (resourceID bytes), each key at an 8-byte aligned offset
//
// A string's tag in probe round k (0..3) is (k << 62) | (H_k(string) & hmask), H_k a
// 64-bit hash seeded from the prefix and k.  Tags are unique in the table: a batch's
// requests with equal tags land on one slot (CAS), and its representative -- the stored
// text of an assigned key, else the batch's first request that landed there -- is
// compared byte for byte with every request.  Requests whose text differs (different
// strings, equal tags) move to the next round's tag; round k's tags only ever meet
// round k's claims, so a slot's first request is settled within the round that claims
// it.  Lookups follow the same rounds: the first slot tagged like the string whose text
// matches is its key; an empty slot before any tagged one means "never assigned".
#include <hip/hip_runtime.h>

#include <algorithm>
#include <new>
#include <vector>

#include "../../include/tbe_strdir.h"
#include "tbe_device.hpp"
#include "tbe_hash.hpp"

using namespace tbe;

namespace {

constexpr uint64_t kEmptyTag = ~0ull;
constexpr uint32_t kNoId = 0xFFFFFFFFu;
constexpr uint32_t kMaxLen = 1u << 16;
constexpr int kRounds = 4;
constexpr int kSdBlock = 256;
constexpr int kSdTile = 1024;            // requests per count/assign block (4 per thread)
constexpr int kSdScan = 1024;
constexpr unsigned kListGrid = 1024;     // workgroups of a probe round over the collided list
constexpr uint64_t kLocValid = 1ull << 63;
constexpr double kWarmShare = 0.5;       // warm path while the last batch's new keys stay below this share

__device__ __host__ __forceinline__ uint32_t loc_len(uint64_t loc) { return (uint32_t)(loc & (2 * kMaxLen - 1)); }
__device__ __host__ __forceinline__ uint64_t loc_off(uint64_t loc) { return (loc >> 17) & ((1ull << 46) - 1); }

// error bits (state[1])
constexpr unsigned long long kErrBatch = 1, kErrRange = 2, kErrRounds = 4, kErrArena = 8, kErrFull = 16;

struct SdParams {
    uint64_t seed[kRounds];
    uint64_t hmask;
};

// 8 bytes of a string starting at its byte 8k (bytes past its end read as 0).  `safe` =
// the largest multiple of 8 such that [0, safe) is readable; words past it are read
// byte by byte up to the string's end.
__device__ __forceinline__ uint64_t sd_word(const uint8_t *__restrict__ base, uint64_t safe, uint64_t off,
                                            uint32_t len, uint32_t k) {
    const uint64_t p = off + 8ull * k;
    const uint32_t rem = len - 8u * k;
    const uint64_t a = p & ~7ull;
    const uint32_t sh = (uint32_t)(p & 7) * 8u;
    uint64_t w;
    if (a + 16 <= safe) {
        const uint64_t lo = *reinterpret_cast<const uint64_t *>(base + a);
        if (sh) {
            const uint64_t hi = *reinterpret_cast<const uint64_t *>(base + a + 8);
            w = (lo >> sh) | (hi << (64 - sh));
        } else {
            w = lo;
        }
    } else {
        w = 0;
        const uint32_t m = rem < 8 ? rem : 8;
        for (uint32_t b = 0; b < m; ++b) w |= (uint64_t)base[p + b] << (8 * b);
    }
    if (rem < 8) w &= (1ull << (8 * rem)) - 1;
    return w;
}

__device__ __forceinline__ uint64_t sd_hash(const uint8_t *__restrict__ base, uint64_t safe, uint64_t off,
                                            uint32_t len, uint64_t seed) {
    uint64_t h = mix64(seed ^ ((uint64_t)len * 0x9E3779B97F4A7C15ull));
    for (uint32_t k = 0; 8u * k < len; ++k) h = mix64(h ^ sd_word(base, safe, off, len, k));
    return h;
}

__device__ __forceinline__ uint64_t sd_tag(uint32_t round, uint64_t h, uint64_t hmask) {
    const uint64_t t = ((uint64_t)round << 62) | (h & hmask);
    return t == kEmptyTag ? t - 1 : t;
}

__device__ __forceinline__ bool sd_equal(const uint8_t *__restrict__ a, uint64_t asafe, uint64_t aoff,
                                         const uint8_t *__restrict__ b, uint64_t bsafe, uint64_t boff,
                                         uint32_t len) {
    for (uint32_t k = 0; 8u * k < len; ++k)
        if (sd_word(a, asafe, aoff, len, k) != sd_word(b, bsafe, boff, len, k)) return false;
    return true;
}

// Offsets of string i, validated (false: malformed).
__device__ __forceinline__ bool sd_span(const uint64_t *__restrict__ offs, uint64_t i, uint64_t n_bytes,
                                        uint64_t &off, uint32_t &len) {
    const uint64_t a = offs[i], b = offs[i + 1];
    if (b < a || b > n_bytes || b - a > kMaxLen) return false;
    off = a;
    len = (uint32_t)(b - a);
    return true;
}

struct SdBatch {
    const uint8_t *bytes;
    const uint64_t *offs;
    uint64_t n_bytes;
    uint64_t safe;         // n_bytes rounded down to 8
};
struct SdArena {
    const uint8_t *bytes;
    uint64_t safe;
};

// Probe round `round`: find or claim the slot tagged like each request's string (over
// all requests in round 0, over the collided list after).  A slot claimed in this batch
// records the arrival index of its first request (atomicMin).
__global__ __launch_bounds__(kSdBlock) void k_sd_claim(SdBatch B, uint64_t n, const uint32_t *__restrict__ list,
                                                       const uint32_t *__restrict__ list_n, uint32_t round,
                                                       SdParams P, uint64_t *__restrict__ stag,
                                                       const uint32_t *__restrict__ sid,
                                                       uint32_t *__restrict__ sfirst, uint64_t smask,
                                                       uint32_t *__restrict__ slot_of,
                                                       unsigned long long *__restrict__ err) {
    const uint64_t count = list ? *list_n : n;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < count; t += stride) {
        const uint64_t i = list ? list[t] : t;
        uint64_t off;
        uint32_t len;
        if (!sd_span(B.offs, i, B.n_bytes, off, len)) {
            slot_of[i] = kNoId;
            atomicOr(err, kErrBatch);
            continue;
        }
        const uint64_t tag = sd_tag(round, sd_hash(B.bytes, B.safe, off, len, P.seed[round]), P.hmask);
        uint32_t found = kNoId;
        uint64_t h = mix64(tag) & smask;
        for (uint64_t probe = 0; probe <= smask; ++probe) {
            const uint64_t cur = stag[h];
            if (cur == tag) {
                found = (uint32_t)h;
                break;
            }
            if (cur == kEmptyTag) {
                const unsigned long long prev =
                    atomicCAS(reinterpret_cast<unsigned long long *>(&stag[h]), kEmptyTag, tag);
                if (prev == kEmptyTag || prev == tag) {
                    found = (uint32_t)h;
                    break;
                }
            }
            h = (h + 1) & smask;
        }
        slot_of[i] = found;
        if (found == kNoId) atomicOr(err, kErrFull);
        else if (sid[found] == kNoId) atomicMin(&sfirst[found], (uint32_t)i);
    }
}

// Compare every request of the round with its slot's representative; a mismatch clears
// the request's slot and lists it for the next round (wave-aggregated appends).
__global__ __launch_bounds__(kSdBlock) void k_sd_verify(SdBatch B, uint64_t n, const uint32_t *__restrict__ list,
                                                        const uint32_t *__restrict__ list_n, SdArena A,
                                                        const uint32_t *__restrict__ sid,
                                                        const uint32_t *__restrict__ sfirst,
                                                        const uint64_t *__restrict__ sloc,
                                                        uint32_t *__restrict__ slot_of,
                                                        uint32_t *__restrict__ next, uint32_t *__restrict__ next_n,
                                                        unsigned long long *__restrict__ err) {
    const uint64_t count = list ? *list_n : n;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x; t0 < count; t0 += stride) {
        const uint64_t t = t0 + threadIdx.x;
        bool moved = false;
        uint64_t i = 0;
        if (t < count) {
            i = list ? list[t] : t;
            const uint32_t s = slot_of[i];
            if (s != kNoId) {
                const uint64_t off = B.offs[i];
                const uint32_t len = (uint32_t)(B.offs[i + 1] - off);
                const uint32_t id = sid[s];
                bool eq;
                if (id != kNoId) {
                    const uint64_t loc = sloc[s];
                    eq = loc_len(loc) == len && sd_equal(A.bytes, A.safe, loc_off(loc), B.bytes, B.safe, off, len);
                } else {
                    const uint32_t j = sfirst[s];
                    if (j == (uint32_t)i) {
                        eq = true;
                    } else {
                        const uint64_t jo = B.offs[j];
                        eq = (uint32_t)(B.offs[j + 1] - jo) == len && sd_equal(B.bytes, B.safe, jo, B.bytes, B.safe, off, len);
                    }
                }
                if (!eq) {
                    slot_of[i] = kNoId;
                    moved = true;
                }
            }
        }
        const uint64_t m = __ballot(moved);
        if (m) {
            if (!next) {
                if (moved) atomicOr(err, kErrRounds);
                continue;
            }
            const int leader = __ffsll((long long)m) - 1;
            uint32_t base = 0;
            if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(next_n, (uint32_t)__popcll(m));
            base = __shfl(base, leader, 64);
            if (moved) next[base + __popcll(m & lanemask_lt())] = (uint32_t)i;
        }
    }
}

__device__ __forceinline__ bool sd_is_new(const uint32_t *slot_of, const uint32_t *sid, const uint32_t *sfirst,
                                          uint64_t i) {
    const uint32_t sl = slot_of[i];
    return sl != kNoId && sid[sl] == kNoId && sfirst[sl] == (uint32_t)i;
}

__device__ __forceinline__ uint32_t sd_room(const uint64_t *offs, uint64_t i) {
    return (uint32_t)((offs[i + 1] - offs[i] + 7) & ~7ull);
}

// Request at position t of a pass over the batch: t itself, or list[t] when the pass
// runs over an ordered list of requests (the warm path's misses, in arrival order).
__device__ __forceinline__ bool sd_at(const uint32_t *__restrict__ list, uint64_t count, uint64_t t, uint64_t &i) {
    if (t >= count) return false;
    i = list ? list[t] : t;
    return true;
}

// New keys and their arena bytes per block of kSdTile requests (of the batch, or of the
// ordered list: list / list_n).
__global__ __launch_bounds__(kSdBlock) void k_sd_count(const uint64_t *__restrict__ offs, uint64_t n,
                                                       const uint32_t *__restrict__ slot_of,
                                                       const uint32_t *__restrict__ sid,
                                                       const uint32_t *__restrict__ sfirst,
                                                       uint32_t *__restrict__ bsum, uint32_t *__restrict__ bbytes,
                                                       const uint32_t *__restrict__ list = nullptr,
                                                       const uint32_t *__restrict__ list_n = nullptr) {
    __shared__ uint32_t wsum[kSdBlock / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kSdTile;
    const uint64_t count = list ? *list_n : n;
    uint32_t c = 0, nb = 0;
    for (int k = 0; k < kSdTile / kSdBlock; ++k) {
        uint64_t i;
        if (sd_at(list, count, base + (uint64_t)threadIdx.x * (kSdTile / kSdBlock) + k, i) &&
            sd_is_new(slot_of, sid, sfirst, i)) {
            ++c;
            nb += sd_room(offs, i);
        }
    }
    uint32_t tc, tb;
    (void)block_excl_scan<kSdBlock>(c, wsum, &tc);
    __syncthreads();
    (void)block_excl_scan<kSdBlock>(nb, wsum, &tb);
    if (threadIdx.x == 0) {
        bsum[blockIdx.x] = tc;
        bbytes[blockIdx.x] = tb;
    }
}

// Exclusive scans of the block counts and bytes (bytes into u64 bbase); state[0] ids
// assigned, [1] error bits, [2] this batch's id base, [3] arena bytes used, [4] this
// batch's arena base.
__global__ __launch_bounds__(kSdScan) void k_sd_scan(uint32_t *__restrict__ bsum, const uint32_t *__restrict__ bbytes,
                                                     uint64_t *__restrict__ bbase, uint32_t nblk,
                                                     unsigned long long *__restrict__ state, uint64_t capacity,
                                                     uint64_t arena_bytes) {
    __shared__ uint32_t wsum[kSdScan / 64];
    __shared__ unsigned long long part[kSdScan];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nblk + kSdScan - 1) / kSdScan;
    uint32_t sum = 0;
    unsigned long long bs = 0;
    for (uint32_t k = 0; k < per; ++k) {
        const uint32_t j = t * per + k;
        if (j < nblk) {
            sum += bsum[j];
            bs += bbytes[j];
        }
    }
    uint32_t tot;
    uint32_t run = block_excl_scan<kSdScan>(sum, wsum, &tot);
    // bytes: u64 scan through LDS (one thread per 1024 partials; nblk is small)
    part[t] = bs;
    __syncthreads();
    if (t == 0) {
        unsigned long long acc = 0;
        for (uint32_t k = 0; k < kSdScan; ++k) {
            const unsigned long long v = part[k];
            part[k] = acc;
            acc += v;
        }
    }
    __syncthreads();
    unsigned long long brun = part[t];
    for (uint32_t k = 0; k < per; ++k) {
        const uint32_t j = t * per + k;
        if (j < nblk) {
            const uint32_t c = bsum[j];
            bsum[j] = run;
            run += c;
            bbase[j] = brun;
            brun += bbytes[j];
        }
    }
    if (t == kSdScan - 1) {
        const unsigned long long before = state[0];
        state[2] = before;
        unsigned long long after = before + tot;
        if (after > capacity) {
            after = capacity;
            state[1] |= kErrRange;
        }
        state[0] = after;
        const unsigned long long abefore = state[3];
        state[4] = abefore;
        unsigned long long aafter = abefore + brun;
        if (aafter > arena_bytes) {
            aafter = arena_bytes;
            state[1] |= kErrArena | kErrRange;
        }
        state[3] = aafter;
    }
}

// Assign ids (counter = base + rank among the batch's new keys, id = its bijection) and
// store the new keys' text; beyond capacity or arena, none.
__global__ __launch_bounds__(kSdBlock) void k_sd_assign(SdBatch B, uint64_t n, const uint32_t *__restrict__ slot_of,
                                                        uint32_t *__restrict__ sid, const uint32_t *__restrict__ sfirst,
                                                        uint64_t *__restrict__ sloc, uint64_t *__restrict__ iloc,
                                                        uint8_t *__restrict__ arena, const uint32_t *__restrict__ bsum,
                                                        const uint64_t *__restrict__ bbase,
                                                        const unsigned long long *__restrict__ state,
                                                        uint64_t capacity, uint64_t arena_bytes, uint64_t imask,
                                                        uint32_t ish, const uint32_t *__restrict__ list = nullptr,
                                                        const uint32_t *__restrict__ list_n = nullptr) {
    __shared__ uint32_t wsum[kSdBlock / 64];
    constexpr int PER = kSdTile / kSdBlock;
    const uint64_t base = (uint64_t)blockIdx.x * kSdTile;
    const uint64_t count = list ? *list_n : n;
    bool nw[PER];
    uint64_t iv[PER];
    uint32_t c = 0, nb = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        nw[k] = sd_at(list, count, base + (uint64_t)threadIdx.x * PER + k, iv[k]) &&
                sd_is_new(slot_of, sid, sfirst, iv[k]);
        c += nw[k];
        nb += nw[k] ? sd_room(B.offs, iv[k]) : 0u;
    }
    uint32_t tc, tb;
    uint32_t r = block_excl_scan<kSdBlock>(c, wsum, &tc);   // every thread has read sid before it returns
    __syncthreads();
    uint32_t rb = block_excl_scan<kSdBlock>(nb, wsum, &tb);
    const uint64_t c0 = (uint64_t)state[2] + bsum[blockIdx.x];
    const uint64_t a0 = (uint64_t)state[4] + bbase[blockIdx.x];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        if (!nw[k]) continue;
        const uint64_t i = iv[k];
        const uint64_t counter = c0 + r++;
        const uint64_t off = B.offs[i];
        const uint32_t len = (uint32_t)(B.offs[i + 1] - off);
        const uint64_t aoff = a0 + rb;
        rb += (len + 7) & ~7u;
        if (counter >= capacity || aoff + ((len + 7) & ~7u) > arena_bytes) continue;
        for (uint32_t w = 0; 8u * w < len; ++w)
            *reinterpret_cast<uint64_t *>(arena + aoff + 8ull * w) = sd_word(B.bytes, B.safe, off, len, w);
        const uint32_t id = (uint32_t)scramble_walk(counter, capacity, imask, ish);
        const uint64_t loc = kLocValid | (aoff << 17) | len;
        sloc[slot_of[i]] = loc;
        iloc[id] = loc;
        sid[slot_of[i]] = id;
    }
}

__global__ void k_sd_gather(const uint32_t *__restrict__ slot_of, uint64_t n, const uint32_t *__restrict__ sid,
                            uint64_t *__restrict__ ids, const uint32_t *__restrict__ list = nullptr,
                            const uint32_t *__restrict__ list_n = nullptr) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t count = list ? *list_n : n;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < count; t += stride) {
        const uint64_t i = list ? list[t] : t;
        const uint32_t sl = slot_of[i];
        const uint32_t id = sl == kNoId ? kNoId : sid[sl];
        ids[i] = id == kNoId ? ~0ull : (uint64_t)id;
    }
}

__global__ __launch_bounds__(kSdBlock) void k_sd_lookup(SdBatch B, uint64_t n, SdParams P,
                                                        const uint64_t *__restrict__ stag,
                                                        const uint32_t *__restrict__ sid,
                                                        const uint64_t *__restrict__ sloc, uint64_t smask, SdArena A,
                                                        uint64_t *__restrict__ ids) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t id = ~0ull;
        uint64_t off;
        uint32_t len;
        if (sd_span(B.offs, i, B.n_bytes, off, len)) {
            bool done = false;
            for (uint32_t round = 0; round < (uint32_t)kRounds && !done; ++round) {
                const uint64_t tag = sd_tag(round, sd_hash(B.bytes, B.safe, off, len, P.seed[round]), P.hmask);
                uint64_t h = mix64(tag) & smask;
                for (uint64_t probe = 0; probe <= smask; ++probe) {
                    const uint64_t cur = stag[h];
                    if (cur == kEmptyTag) {
                        done = true;   // no slot carries this tag: never assigned
                        break;
                    }
                    if (cur == tag) {
                        const uint32_t s_id = sid[h];
                        const uint64_t loc = sloc[h];
                        if (s_id != kNoId && loc_len(loc) == len &&
                            sd_equal(A.bytes, A.safe, loc_off(loc), B.bytes, B.safe, off, len)) {
                            id = s_id;
                            done = true;
                        }
                        break;         // tags are unique: try the next round's
                    }
                    h = (h + 1) & smask;
                }
            }
        }
        ids[i] = id;
    }
}

// ---------------------------------------------------------------- warm path
// Most strings of a steady-state batch are already known.  k_sd_resolve answers them the
// way a lookup does (every probe round, byte compare with the stored text) and leaves
// UINT64_MAX for the misses; a stable compaction lists the misses in arrival order, and
// the assign machinery (claim / verify rounds, count, scan, assign, gather) runs over that
// list only.  Ids are unchanged: the known strings keep theirs, and the new ones get
// counters in arrival order, exactly as a full pass assigns them.
__device__ __forceinline__ uint64_t sd_find(const SdBatch &B, uint64_t i, const SdParams &P,
                                            const uint64_t *__restrict__ stag, const uint32_t *__restrict__ sid,
                                            const uint64_t *__restrict__ sloc, uint64_t smask, const SdArena &A) {
    uint64_t off;
    uint32_t len;
    if (!sd_span(B.offs, i, B.n_bytes, off, len)) return ~0ull;   // the claim round flags it
    for (uint32_t round = 0; round < (uint32_t)kRounds; ++round) {
        const uint64_t tag = sd_tag(round, sd_hash(B.bytes, B.safe, off, len, P.seed[round]), P.hmask);
        uint64_t h = mix64(tag) & smask;
        for (uint64_t probe = 0; probe <= smask; ++probe) {
            const uint64_t cur = stag[h];
            if (cur == kEmptyTag) return ~0ull;       // never assigned
            if (cur == tag) {
                const uint32_t s_id = sid[h];
                const uint64_t loc = sloc[h];
                if (s_id != kNoId && loc_len(loc) == len &&
                    sd_equal(A.bytes, A.safe, loc_off(loc), B.bytes, B.safe, off, len))
                    return s_id;
                break;                                // tags are unique: the next round's
            }
            h = (h + 1) & smask;
        }
    }
    return ~0ull;
}

// ids[i] = the id of a known string, UINT64_MAX for a miss; bmiss[block] = its misses.
// Requests are thread-contiguous within a block (as k_sd_count), kSdTile per block.
__global__ __launch_bounds__(kSdBlock) void k_sd_resolve(SdBatch B, uint64_t n, SdParams P,
                                                         const uint64_t *__restrict__ stag,
                                                         const uint32_t *__restrict__ sid,
                                                         const uint64_t *__restrict__ sloc, uint64_t smask, SdArena A,
                                                         uint64_t *__restrict__ ids, uint32_t *__restrict__ bmiss) {
    __shared__ uint32_t wsum[kSdBlock / 64];
    constexpr int PER = kSdTile / kSdBlock;
    const uint64_t base = (uint64_t)blockIdx.x * kSdTile;
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const uint64_t i = base + (uint64_t)threadIdx.x * PER + k;
        if (i < n) {
            const uint64_t id = sd_find(B, i, P, stag, sid, sloc, smask, A);
            ids[i] = id;
            c += id == ~0ull;
        }
    }
    uint32_t tot;
    (void)block_excl_scan<kSdBlock>(c, wsum, &tot);
    if (threadIdx.x == 0) bmiss[blockIdx.x] = tot;
}

// Exclusive scan of the per-block miss counts in place; *total = all misses.
__global__ __launch_bounds__(kSdScan) void k_sd_xscan(uint32_t *__restrict__ v, uint32_t nblk,
                                                      uint32_t *__restrict__ total) {
    __shared__ uint32_t wsum[kSdScan / 64];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nblk + kSdScan - 1) / kSdScan;
    uint32_t sum = 0;
    for (uint32_t k = 0; k < per; ++k) {
        const uint32_t j = t * per + k;
        if (j < nblk) sum += v[j];
    }
    uint32_t tot;
    uint32_t run = block_excl_scan<kSdScan>(sum, wsum, &tot);
    for (uint32_t k = 0; k < per; ++k) {
        const uint32_t j = t * per + k;
        if (j < nblk) {
            const uint32_t c = v[j];
            v[j] = run;
            run += c;
        }
    }
    if (t == 0) *total = tot;
}

// The misses in arrival order: list[bmiss[block] + rank in block] = i.
__global__ __launch_bounds__(kSdBlock) void k_sd_compact(uint64_t n, const uint64_t *__restrict__ ids,
                                                         const uint32_t *__restrict__ bmiss,
                                                         uint32_t *__restrict__ list) {
    __shared__ uint32_t wsum[kSdBlock / 64];
    constexpr int PER = kSdTile / kSdBlock;
    const uint64_t base = (uint64_t)blockIdx.x * kSdTile;
    bool miss[PER];
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const uint64_t i = base + (uint64_t)threadIdx.x * PER + k;
        miss[k] = i < n && ids[i] == ~0ull;
        c += miss[k];
    }
    uint32_t tot;
    uint32_t at = bmiss[blockIdx.x] + block_excl_scan<kSdBlock>(c, wsum, &tot);
#pragma unroll
    for (int k = 0; k < PER; ++k)
        if (miss[k]) list[at++] = (uint32_t)(base + (uint64_t)threadIdx.x * PER + k);
}

__global__ void k_sd_init(uint64_t *__restrict__ stag, uint32_t *__restrict__ sid, uint32_t *__restrict__ sfirst,
                          uint64_t nslots) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nslots; j += stride) {
        stag[j] = kEmptyTag;
        sid[j] = kNoId;
        sfirst[j] = kNoId;
    }
}

unsigned sd_grid(uint64_t n, unsigned block, unsigned cap = 8192) {
    const uint64_t g = (n + block - 1) / block;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, cap));
}

// Host hash of the prefix (the seeds of the four rounds derive from it).
uint64_t host_hash(const uint8_t *p, uint32_t len) {
    uint64_t h = mix64(0x243F6A8885A308D3ull ^ ((uint64_t)len * 0x9E3779B97F4A7C15ull));
    for (uint32_t k = 0; 8u * k < len; ++k) {
        uint64_t w = 0;
        for (uint32_t b = 0; b < 8 && 8u * k + b < len; ++b) w |= (uint64_t)p[8u * k + b] << (8 * b);
        h = mix64(h ^ w);
    }
    return h;
}

}  // namespace

struct tbe_string_directory {
    uint64_t capacity = 0, nslots = 0, arena_bytes = 0, arena_alloc = 0;
    int device = 0;
    uint64_t imask = 0;
    uint32_t ish = 0;
    bool used = false;
    SdParams P{};
    uint64_t *stag = nullptr;
    uint32_t *sid = nullptr;
    uint32_t *sfirst = nullptr;
    uint64_t *sloc = nullptr;
    uint64_t *iloc = nullptr;
    uint8_t *arena = nullptr;
    unsigned long long *state = nullptr;   // see k_sd_scan
    // per-batch scratch
    uint64_t tmp_cap = 0;
    uint32_t *slot_of = nullptr;
    uint32_t *list[2] = {nullptr, nullptr};
    uint32_t *list_n = nullptr;            // [kRounds]
    uint32_t *bsum = nullptr, *bbytes = nullptr;
    uint64_t *bbase = nullptr;
    uint32_t *miss = nullptr;              // warm path: the batch's misses, arrival order
    uint32_t *bmiss = nullptr;             // warm path: misses per block (scanned)
    // warm-path choice: 0 auto (the last observed batch's new-key share), 1 full pass, 2 warm
    int mode = 0;
    unsigned long long *h_state = nullptr; // pinned: state[0] after the last assign (async copy)
    hipEvent_t ev_state = nullptr;
    bool state_pending = false;
    unsigned long long last_ids = 0;       // ids at the previous observed copy
    uint64_t since_n = 0;                  // requests assigned since the last copy was enqueued
    uint64_t last_n = 0;                   // requests between the previous copy and the one in flight
    double new_share = 1.0;                // new keys / requests between the last two observed copies
    // host-buffer staging
    uint64_t st_bytes = 0, st_n = 0;
    uint8_t *d_bytes = nullptr;
    uint64_t *d_offs = nullptr, *d_ids = nullptr;
};

namespace {

void sd_free_scratch(tbe_string_directory *d) {
    for (void *p : {(void *)d->slot_of, (void *)d->list[0], (void *)d->list[1], (void *)d->bsum, (void *)d->bbytes,
                    (void *)d->bbase, (void *)d->miss, (void *)d->bmiss})
        if (p) (void)hipFree(p);
    d->slot_of = d->list[0] = d->list[1] = d->bsum = d->bbytes = d->miss = d->bmiss = nullptr;
    d->bbase = nullptr;
    d->tmp_cap = 0;
}

tbe_status sd_scratch(tbe_string_directory *d, uint64_t n) {
    if (n <= d->tmp_cap) return TBE_OK;
    if (hipDeviceSynchronize() != hipSuccess) return TBE_EDEVICE;   // the previous batch may use them
    sd_free_scratch(d);
    const uint64_t cap = std::max<uint64_t>(n, 1u << 16);
    const uint64_t nblk = (cap + kSdTile - 1) / kSdTile;
    if (hipMalloc(&d->slot_of, cap * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&d->list[0], cap * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&d->list[1], cap * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&d->bsum, nblk * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&d->bbytes, nblk * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&d->bbase, nblk * sizeof(uint64_t)) != hipSuccess ||
        hipMalloc(&d->miss, cap * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&d->bmiss, nblk * sizeof(uint32_t)) != hipSuccess) {
        sd_free_scratch(d);
        return TBE_ENOMEM;
    }
    d->tmp_cap = cap;
    return TBE_OK;
}

bool batch_ok(const uint8_t *d_bytes, uint64_t n_bytes, const uint64_t *d_offs, uint64_t n) {
    if (!d_offs || n >= (1ull << 32)) return false;
    if (n_bytes && !d_bytes) return false;
    return (reinterpret_cast<uintptr_t>(d_bytes) & 7u) == 0;
}

}  // namespace

extern "C" {

tbe_status tbe_sdir_create(uint64_t capacity, uint64_t arena_bytes, const char *prefix, uint32_t prefix_len,
                           int32_t device, tbe_string_directory **out) {
    if (!out) return TBE_EINVAL;
    *out = nullptr;
    if (capacity == 0 || capacity > 0xFFFFFFFEull || arena_bytes > (1ull << 46) || (prefix_len && !prefix))
        return TBE_EINVAL;
    tbe_string_directory *d = new (std::nothrow) tbe_string_directory();
    if (!d) return TBE_ENOMEM;
    if (device >= 0) {
        if (hipSetDevice(device) != hipSuccess) { delete d; return TBE_EDEVICE; }
        d->device = device;
    } else if (hipGetDevice(&d->device) != hipSuccess) {
        delete d;
        return TBE_EDEVICE;
    }
    d->capacity = capacity;
    d->arena_bytes = arena_bytes & ~7ull;
    d->arena_alloc = d->arena_bytes + 16;
    uint64_t ns = 1;
    while (ns < 2 * capacity) ns <<= 1;
    d->nslots = ns;
    scramble_params(capacity, d->imask, d->ish);
    const uint64_t ph = host_hash(reinterpret_cast<const uint8_t *>(prefix), prefix_len);
    for (int k = 0; k < kRounds; ++k) d->P.seed[k] = mix64(ph + (uint64_t)(k + 1) * 0x9E3779B97F4A7C15ull);
    d->P.hmask = (1ull << 62) - 1;
    bool ok = hipMalloc(&d->stag, ns * sizeof(uint64_t)) == hipSuccess &&
              hipMalloc(&d->sid, ns * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&d->sfirst, ns * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&d->sloc, ns * sizeof(uint64_t)) == hipSuccess &&
              hipMalloc(&d->iloc, capacity * sizeof(uint64_t)) == hipSuccess &&
              hipMalloc(&d->arena, d->arena_alloc) == hipSuccess &&
              hipMalloc(&d->state, 8 * sizeof(unsigned long long)) == hipSuccess &&
              hipMalloc(&d->list_n, (kRounds + 1) * sizeof(uint32_t)) == hipSuccess &&
              hipHostMalloc(&d->h_state, sizeof(unsigned long long), hipHostMallocDefault) == hipSuccess &&
              hipEventCreateWithFlags(&d->ev_state, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        tbe_sdir_destroy(d);
        return TBE_ENOMEM;
    }
    k_sd_init<<<sd_grid(ns, 256), 256>>>(d->stag, d->sid, d->sfirst, ns);
    if (hipMemset(d->state, 0, 8 * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(d->arena, 0, d->arena_alloc) != hipSuccess ||
        hipMemset(d->iloc, 0, capacity * sizeof(uint64_t)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        tbe_sdir_destroy(d);
        return TBE_EDEVICE;
    }
    *out = d;
    return TBE_OK;
}

void tbe_sdir_destroy(tbe_string_directory *d) {
    if (!d) return;
    (void)hipSetDevice(d->device);
    (void)hipDeviceSynchronize();
    sd_free_scratch(d);
    if (d->h_state) (void)hipHostFree(d->h_state);
    if (d->ev_state) (void)hipEventDestroy(d->ev_state);
    for (void *p : {(void *)d->stag, (void *)d->sid, (void *)d->sfirst, (void *)d->sloc, (void *)d->iloc,
                    (void *)d->arena, (void *)d->state, (void *)d->list_n, (void *)d->d_bytes, (void *)d->d_offs,
                    (void *)d->d_ids})
        if (p) (void)hipFree(p);
    delete d;
}

tbe_status tbe_sdir_set_hash_bits(tbe_string_directory *d, uint32_t bits) {
    if (!d || bits == 0 || bits > 62 || d->used) return TBE_EINVAL;
    d->P.hmask = (bits == 62) ? (1ull << 62) - 1 : (1ull << bits) - 1;
    return TBE_OK;
}

tbe_status tbe_sdir_assign_device(tbe_string_directory *d, const uint8_t *d_bytes, uint64_t n_bytes,
                                  const uint64_t *d_offs, uint64_t n, uint64_t *d_ids, void *stream) {
    if (!d) return TBE_EINVAL;
    if (n == 0) return TBE_OK;
    if (!d_ids || !batch_ok(d_bytes, n_bytes, d_offs, n)) return TBE_EINVAL;
    if (hipSetDevice(d->device) != hipSuccess) return TBE_EDEVICE;
    tbe_status rc = sd_scratch(d, n);
    if (rc != TBE_OK) return rc;
    d->used = true;
    hipStream_t st = (hipStream_t)stream;
    const SdBatch B{d_bytes, d_offs, n_bytes, n_bytes & ~7ull};
    const SdArena A{d->arena, d->arena_alloc & ~7ull};
    unsigned long long *err = d->state + 1;
    if (hipMemsetAsync(d->list_n, 0, (kRounds + 1) * sizeof(uint32_t), st) != hipSuccess) return TBE_EDEVICE;
    const uint64_t smask = d->nslots - 1;
    const uint32_t nblk = (uint32_t)((n + kSdTile - 1) / kSdTile);
    // The warm path pays one lookup pass over the batch to run the assign machinery over
    // its misses only: chosen while the last observed batch brought few new keys (its id
    // count is copied back asynchronously; the choice never waits for it).
    // The copy in flight holds the id count after the batch it followed; last_n counts every
    // request assigned between that copy and the previous one (several batches when copies
    // were still pending), so the share is new ids per request over exactly those batches.
    if (d->state_pending) {
        const hipError_t q = hipEventQuery(d->ev_state);
        if (q == hipSuccess) {
            d->new_share = d->last_n ? (double)(*d->h_state - d->last_ids) / (double)d->last_n : 1.0;
            d->last_ids = *d->h_state;
            d->state_pending = false;
        } else if (q != hipErrorNotReady) {
            // an unreadable copy: forget it, take the full path, and copy again below
            (void)hipGetLastError();
            d->new_share = 1.0;
            d->state_pending = false;
        }
    }
    const bool warm = d->mode == 2 || (d->mode == 0 && d->new_share < kWarmShare);
    const uint32_t *miss = warm ? d->miss : nullptr;
    const uint32_t *miss_n = warm ? d->list_n + kRounds : nullptr;
    if (warm) {
        k_sd_resolve<<<nblk, kSdBlock, 0, st>>>(B, n, d->P, d->stag, d->sid, d->sloc, smask, A, d_ids, d->bmiss);
        k_sd_xscan<<<1, kSdScan, 0, st>>>(d->bmiss, nblk, d->list_n + kRounds);
        k_sd_compact<<<nblk, kSdBlock, 0, st>>>(n, d_ids, d->bmiss, d->miss);
    }
    for (int round = 0; round < kRounds; ++round) {
        const uint32_t *in = round ? d->list[(round - 1) & 1] : miss;
        const uint32_t *in_n = round ? d->list_n + (round - 1) : miss_n;
        uint32_t *nx = (round + 1 < kRounds) ? d->list[round & 1] : nullptr;
        uint32_t *nx_n = (round + 1 < kRounds) ? d->list_n + round : nullptr;
        const unsigned g = in ? (round ? kListGrid : sd_grid(n, kSdBlock)) : sd_grid(n, kSdBlock);
        k_sd_claim<<<g, kSdBlock, 0, st>>>(B, n, in, in_n, (uint32_t)round, d->P, d->stag, d->sid, d->sfirst, smask,
                                           d->slot_of, err);
        k_sd_verify<<<g, kSdBlock, 0, st>>>(B, n, in, in_n, A, d->sid, d->sfirst, d->sloc, d->slot_of, nx, nx_n, err);
    }
    k_sd_count<<<nblk, kSdBlock, 0, st>>>(d_offs, n, d->slot_of, d->sid, d->sfirst, d->bsum, d->bbytes, miss,
                                          miss_n);
    k_sd_scan<<<1, kSdScan, 0, st>>>(d->bsum, d->bbytes, d->bbase, nblk, d->state, d->capacity, d->arena_bytes);
    k_sd_assign<<<nblk, kSdBlock, 0, st>>>(B, n, d->slot_of, d->sid, d->sfirst, d->sloc, d->iloc, d->arena, d->bsum,
                                           d->bbase, d->state, d->capacity, d->arena_bytes, d->imask, d->ish, miss,
                                           miss_n);
    k_sd_gather<<<sd_grid(n, 256), 256, 0, st>>>(d->slot_of, n, d->sid, d_ids, miss, miss_n);
    d->since_n += n;
    if (!d->state_pending) {
        // the id count after this batch, for a later call's choice
        if (hipMemcpyAsync(d->h_state, d->state, sizeof(unsigned long long), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipEventRecord(d->ev_state, st) != hipSuccess)
            return TBE_EDEVICE;
        d->state_pending = true;
        d->last_n = d->since_n;
        d->since_n = 0;
    }
    return hipGetLastError() == hipSuccess ? TBE_OK : TBE_EDEVICE;
}

tbe_status tbe_sdir_set_mode(tbe_string_directory *d, int32_t mode) {
    if (!d || mode < 0 || mode > 2) return TBE_EINVAL;
    d->mode = mode;
    return TBE_OK;
}

tbe_status tbe_sdir_lookup_device(tbe_string_directory *d, const uint8_t *d_bytes, uint64_t n_bytes,
                                  const uint64_t *d_offs, uint64_t n, uint64_t *d_ids, void *stream) {
    if (!d) return TBE_EINVAL;
    if (n == 0) return TBE_OK;
    if (!d_ids || !batch_ok(d_bytes, n_bytes, d_offs, n)) return TBE_EINVAL;
    if (hipSetDevice(d->device) != hipSuccess) return TBE_EDEVICE;
    const SdBatch B{d_bytes, d_offs, n_bytes, n_bytes & ~7ull};
    const SdArena A{d->arena, d->arena_alloc & ~7ull};
    k_sd_lookup<<<sd_grid(n, kSdBlock), kSdBlock, 0, (hipStream_t)stream>>>(B, n, d->P, d->stag, d->sid, d->sloc,
                                                                            d->nslots - 1, A, d_ids);
    return hipGetLastError() == hipSuccess ? TBE_OK : TBE_EDEVICE;
}

tbe_status tbe_sdir_assign(tbe_string_directory *d, const uint8_t *bytes, uint64_t n_bytes, const uint64_t *offs,
                           uint64_t n, uint64_t *ids) {
    if (!d) return TBE_EINVAL;
    if (n == 0) return TBE_OK;
    if (!offs || !ids || (n_bytes && !bytes) || n >= (1ull << 32)) return TBE_EINVAL;
    if (hipSetDevice(d->device) != hipSuccess) return TBE_EDEVICE;
    if (n_bytes > d->st_bytes || n > d->st_n) {
        if (hipDeviceSynchronize() != hipSuccess) return TBE_EDEVICE;
        for (void *p : {(void *)d->d_bytes, (void *)d->d_offs, (void *)d->d_ids})
            if (p) (void)hipFree(p);
        d->d_bytes = nullptr;
        d->d_offs = d->d_ids = nullptr;
        d->st_bytes = d->st_n = 0;
        const uint64_t nb = std::max<uint64_t>(n_bytes, 1u << 16), nn = std::max<uint64_t>(n, 1u << 12);
        if (hipMalloc(&d->d_bytes, nb + 8) != hipSuccess || hipMalloc(&d->d_offs, (nn + 1) * sizeof(uint64_t)) != hipSuccess ||
            hipMalloc(&d->d_ids, nn * sizeof(uint64_t)) != hipSuccess)
            return TBE_ENOMEM;
        d->st_bytes = nb;
        d->st_n = nn;
    }
    if ((n_bytes && hipMemcpy(d->d_bytes, bytes, n_bytes, hipMemcpyHostToDevice) != hipSuccess) ||
        hipMemcpy(d->d_offs, offs, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice) != hipSuccess)
        return TBE_EDEVICE;
    tbe_status rc = tbe_sdir_assign_device(d, d->d_bytes, n_bytes, d->d_offs, n, d->d_ids, nullptr);
    if (rc != TBE_OK) return rc;
    return hipMemcpy(ids, d->d_ids, n * sizeof(uint64_t), hipMemcpyDeviceToHost) == hipSuccess ? TBE_OK : TBE_EDEVICE;
}

tbe_status tbe_sdir_size(tbe_string_directory *d, uint64_t *n_ids) {
    if (!d || !n_ids) return TBE_EINVAL;
    if (hipSetDevice(d->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return TBE_EDEVICE;
    unsigned long long st[2] = {0, 0};
    if (hipMemcpy(st, d->state, sizeof st, hipMemcpyDeviceToHost) != hipSuccess) return TBE_EDEVICE;
    *n_ids = st[0];
    if (st[1] & (kErrRange | kErrRounds | kErrArena | kErrFull)) return TBE_ERANGE;
    return (st[1] & kErrBatch) ? TBE_EINVAL : TBE_OK;
}

tbe_status tbe_sdir_key_of(tbe_string_directory *d, uint64_t id, uint8_t *buf, uint64_t cap, uint64_t *len) {
    if (!d || !len || (cap && !buf) || id >= d->capacity) return TBE_EINVAL;
    if (hipSetDevice(d->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return TBE_EDEVICE;
    uint64_t loc = 0;   // iloc is zero for ids never assigned
    if (hipMemcpy(&loc, d->iloc + id, sizeof loc, hipMemcpyDeviceToHost) != hipSuccess) return TBE_EDEVICE;
    if (!(loc & kLocValid)) return TBE_EINVAL;
    *len = loc_len(loc);
    const uint64_t m = std::min<uint64_t>(loc_len(loc), cap);
    if (m && hipMemcpy(buf, d->arena + loc_off(loc), m, hipMemcpyDeviceToHost) != hipSuccess) return TBE_EDEVICE;
    return TBE_OK;
}

}  // extern "C"
