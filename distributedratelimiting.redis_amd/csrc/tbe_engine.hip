// tbe_engine.hip -- MI355X batched token-bucket engine: kernels, orchestration, C ABI.
//
// Replaces the reference's per-request Redis script round-trip
// (TokenBucket/RedisTokenBucketRateLimiter.cs:63, PartitionedRedisTokenBucketRateLimiter.cs:42)
// with one batched pipeline over an HBM-resident bucket table.  Per batch of n requests
// (arrival order i = 0..n-1):
//
//   bucket b(key) = key >> r_bits  (2^r_bits keys per bucket; 2^11 at 1e8 keys)
//   1. LSD stable partition of the requests by b, P = ceil(bits(b)/8) passes of 8 bits:
//        k_hist / k_hist_dig  per-tile digit histograms (+ running in-block prefix)
//        k_colscan            digit-column scan of the per-block sums -> digit offsets
//        k_scatter_rec        stable local rank (wave ballot-match) -> LDS staging ->
//                             coalesced runs; the last pass writes fold records
//      After the last pass the requests are grouped by bucket, arrival order kept inside.
//   2. k_bscan_lb: first sorted position of every bucket (decoupled look-back).
//   3. k_fold_wide: one workgroup per bucket.  The bucket's 2^r_bits table rows (its
//      slice) are the only state it touches, pulled into LDS by LDS-DMA.  Requests are
//      taken in arrival order, 1536 at a time; every pending request evaluates the script
//      against its key's current row and the key's earliest modifying request commits
//      (speculative rounds, LDS atomicMax election), so per-key order is the reference's
//      serial order.  Dirty lines are written back once.  Sparse batches: k_fold_sparse
//      (one wave per bucket); hot keys: their own runs (k_hot_*).
//   4. k_unscatter: {granted, remaining} back in arrival order through pass 0's
//      permutation (the fold already put each reply at its pass-0 output position).
// DESIGN.md §5 describes every kernel.
//
// Memory-bound integer/byte work plus a little FP64; no MFMA.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/tbe.h"
#include "tbe_device.hpp"
#include "tbe_numfmt.hpp"

#pragma clang fp contract(off)

using namespace tbe;

namespace {

// Non-temporal hints where data is touched once (tools/ablate.py A/B, profiles/
// r01_v10_ablate.log): partition-pass input loads and permutation stores, the
// un-partition passes, the fold's table slices.  NOT the partition passes' record runs
// (their partial lines merge in L2: 50% slower streamed) nor the fold's replies (the
// un-partition gather reuses their lines).  -DTBE_NO_NT turns them off for A/B runs
// (slice loads cached instead: fold 1.17 -> 1.31 ms in round 1).
#ifndef TBE_NO_NT
#define LD_P(p) ld_nt(p)
#define ST_PERM(p, v) st_nt((p), (v))
#define LD_U(p) ld_nt(p)
#define ST_U(p, v) st_nt((p), (v))
#define ST_S(p, v) slot_store_nt((p), (v))
#else
#define LD_P(p) (*(p))
#define ST_PERM(p, v) (*(p) = (v))
#define LD_U(p) (*(p))
#define ST_U(p, v) (*(p) = (v))
#define ST_S(p, v) (*(p) = (v))
#endif
#define LD_F(p) (*(p))
#define ST_F(p, v) (*(p) = (v))

#ifndef TBE_PART_BLOCK
#define TBE_PART_BLOCK 512
#endif
#ifndef TBE_PART_ITEMS
#define TBE_PART_ITEMS 8
#endif
constexpr int kPartBlock = TBE_PART_BLOCK;             // partition workgroup
constexpr int kPartItems = TBE_PART_ITEMS;             // elements per thread per tile
constexpr int kTile = kPartBlock * kPartItems;         // 4096 requests per partition tile
// k_unscatter's own tiles (any size is correct; 8192 keeps each workgroup's gathers in
// the digit runs of two partition tiles)
#ifndef TBE_UN_BLOCK
#define TBE_UN_BLOCK 1024
#endif
#ifndef TBE_UN_ITEMS
#define TBE_UN_ITEMS 8
#endif
constexpr int kUnBlock = TBE_UN_BLOCK;
constexpr int kUnItems = TBE_UN_ITEMS;
constexpr int kUnTile = kUnBlock * kUnItems;
#ifndef TBE_HIST_BLOCKS
#define TBE_HIST_BLOCKS 1024
#endif
constexpr int kMaxHistBlocks = TBE_HIST_BLOCKS;   // k_hist workgroups (each walks consecutive tiles)
static_assert(kMaxHistBlocks % 256 == 0, "k_colscan reads kMaxHistBlocks / 256 blocks per thread");
constexpr int kMaxRBits = 11;                          // <= 2048 rows per bucket (32 KB LDS)

// Hot keys (see the "hot keys" section below for how their runs are decided).
constexpr uint32_t kHotKeysMax = 1024;
#ifndef TBE_HOT_SLOT_BITS
#define TBE_HOT_SLOT_BITS 12
#endif
constexpr uint32_t kHotSlots = 1u << TBE_HOT_SLOT_BITS;   // hash slots: power of two, load <= kHotKeysMax / kHotSlots
static_assert(kHotSlots >= 2 * kHotKeysMax, "hot table load factor <= 1/2");
constexpr uint32_t kHotEmpty = 0xFFFFFFFFu;
constexpr uint32_t kHotMin = 2048;               // requests in one batch that make a key hot
constexpr uint32_t kHotCandMax = 4096;           // nominations kept per batch (the busiest win)

struct HotSet {
    uint32_t count;                  // hot keys in use this batch (index h -> bucket nb + h)
    uint32_t n_cand;                 // nominations for the following batch
    uint32_t key[kHotKeysMax];
    uint64_t cand[kHotCandMax];      // (requests << 32) | key
    uint64_t slot[kHotSlots];        // open-addressing hash table: (index << 32) | key
};

__device__ __forceinline__ uint32_t hot_hash(uint32_t key) { return (key * 0x9E3779B1u) >> (32 - TBE_HOT_SLOT_BITS); }
constexpr uint64_t kHotSlotEmpty = 0xFFFFFFFFFFFFFFFFull;
// The table is two halves of kHotSlots/2 slots (two-choice cuckoo) and a key lives
// at hot_h1 in the first half or hot_h2 in the second, so a probe is two independent LDS
// reads and never a chain.  With linear probing at load 1/4, ~10% of a Zipf batch's
// lookups continued a chain, so nearly every wave of every tile ran the chain loop
// (profiles/r03_ablate_hot_probe.log: the probes cost 0.13 + 0.15 ms over uniform).
constexpr uint32_t kHotHalf = kHotSlots / 2;
__device__ __forceinline__ uint32_t hot_h1(uint32_t key) { return (key * 0x9E3779B1u) >> (33 - TBE_HOT_SLOT_BITS); }
__device__ __forceinline__ uint32_t hot_h2(uint32_t key) {
    uint32_t x = (key ^ (key >> 16)) * 0x85EBCA6Bu;
    x ^= x >> 13;
    return kHotHalf + ((x * 0xC2B2AE35u) >> (33 - TBE_HOT_SLOT_BITS));
}

// Copy a hot set's hash table into LDS (every thread calls; one barrier).  Returns
// whether any key is hot.  (Probing the global table through the caches instead was
// slower, CHANGELOG round 3.)
constexpr uint32_t kHotLds = kHotSlots;   // LDS copy of the table
template <int BLOCK>
__device__ __forceinline__ bool hot_load(const HotSet *__restrict__ hot, uint64_t *slots) {
    const bool any = hot != nullptr && hot->count != 0;
    if (any)
        for (int j = threadIdx.x; j < (int)kHotSlots; j += BLOCK) slots[j] = hot->slot[j];
    __syncthreads();
    return any;
}
// The table the probes read: the workgroup's LDS copy.
__device__ __forceinline__ const uint64_t *hot_table(const HotSet *__restrict__, const uint64_t *lds) {
    return lds;
}

// Partition key of a request: the key itself, or (nb + h) << r_bits for hot key h.
__device__ __forceinline__ uint32_t hot_sortkey(uint32_t key, const uint64_t *slots, uint32_t nb,
                                                int r_bits) {
    const uint64_t v1 = slots[hot_h1(key)], v2 = slots[hot_h2(key)];
    if ((uint32_t)v1 == key) return (nb + (uint32_t)(v1 >> 32)) << r_bits;
    if ((uint32_t)v2 == key) return (nb + (uint32_t)(v2 >> 32)) << r_bits;
    return key;
    uint32_t h = hot_hash(key);
    for (;;) {
        const uint64_t v = slots[h];
        const uint32_t k = (uint32_t)v;
        if (k == key) return (nb + (uint32_t)(v >> 32)) << r_bits;
        if (k == kHotEmpty) return key;
        h = (h + 1) & (kHotSlots - 1);
    }
}

// hot_sortkey for N requests at once: the first probes of all N issue together (LDS
// latency overlaps); the rare collision chains finish one by one.
template <int N, typename KeyT>
__device__ __forceinline__ void hot_sortkeys(const KeyT (&kv)[N], const uint64_t *slots, uint32_t nb,
                                             int r_bits, uint32_t (&sk)[N]) {
    // both probes of 4 requests in flight at a time (8 would spill in the hot histogram)
    constexpr int G = N < 4 ? N : 4;
    static_assert(N % G == 0, "groups of G requests");
#pragma unroll
    for (int g = 0; g < N; g += G) {
        uint64_t v1[G], v2[G];
#pragma unroll
        for (int u = 0; u < G; ++u) {
            v1[u] = slots[hot_h1((uint32_t)kv[g + u])];
            v2[u] = slots[hot_h2((uint32_t)kv[g + u])];
        }
#pragma unroll
        for (int u = 0; u < G; ++u) {
            const uint32_t key = (uint32_t)kv[g + u];
            const bool in1 = (uint32_t)v1[u] == key;
            const uint64_t v = in1 ? v1[u] : v2[u];
            sk[g + u] = (in1 || (uint32_t)v2[u] == key) ? (nb + (uint32_t)(v >> 32)) << r_bits : key;
        }
    }
    return;
    uint64_t v[N];
#pragma unroll
    for (int it = 0; it < N; ++it) v[it] = slots[hot_hash((uint32_t)kv[it])];
#pragma unroll
    for (int it = 0; it < N; ++it) {
        const uint32_t key = (uint32_t)kv[it];
        const uint32_t k = (uint32_t)v[it];
        if (k == key) sk[it] = (nb + (uint32_t)(v[it] >> 32)) << r_bits;
        else if (k == kHotEmpty) sk[it] = key;
        else sk[it] = hot_sortkey(key, slots, nb, r_bits);
    }
}

// ----------------------------------------------------------------------------- kernels
// Per-tile digit histograms.  Block j walks tiles [j*tpb, (j+1)*tpb) in order and
// writes for each tile the exclusive running count per digit within its block
// (tileprefix) and, at the end, the block's totals (blocksum).  Pass 0 also validates
// keys (key < n_keys).  Digits come from the key bits under `kmask` (the low 32 bits, or
// a packed record's key field) exactly as the scatter computes them, so counts stay
// consistent even for an (invalid) key >= 2^32.
// HOT (first pass of a token-bucket batch with hot runs): a hot key's digits come from
// its run's partition key (hot_sortkey), as in k_scatter_rec<true, true>.
//
// 512 threads x 8 keys per tile, and the next tile's keys are loaded while this one is
// counted (the loads, not the LDS counting, bound this kernel).
constexpr int kHBlock = 512;
constexpr int kHItems = kTile / kHBlock;              // 8
#ifndef TBE_HIST_AHEAD
#define TBE_HIST_AHEAD 1                     // tiles of keys in flight ahead of the one counted
#endif
#ifndef TBE_HIST_WAVES
#define TBE_HIST_WAVES 8                     // minimum waves per SIMD (register budget)
#endif
#ifndef TBE_HIST_HOT_WAVES
#define TBE_HIST_HOT_WAVES 6
#endif
template <typename KeyT, bool HOT = false>
__global__ __launch_bounds__(kHBlock, HOT ? TBE_HIST_HOT_WAVES : TBE_HIST_WAVES) void k_hist(const KeyT *__restrict__ keys, uint64_t n,
                                                  int shift, uint32_t tiles_per_blk,
                                                  uint32_t ntiles, uint32_t *__restrict__ tileprefix,
                                                  uint32_t *__restrict__ blocksum, uint64_t n_keys,
                                                  uint32_t *__restrict__ err, int validate,
                                                  uint64_t kmask, const HotSet *__restrict__ hot = nullptr,
                                                  uint32_t nb = 0, int r_bits = 0,
                                                  uint32_t *__restrict__ bcount = nullptr,
                                                  int lowbits = 0, uint32_t nbt = 0,
                                                  uint8_t *__restrict__ dig_out = nullptr) {
    __shared__ uint32_t h8[kDigits * 8];
    __shared__ uint32_t tile_lo[2];
    static_assert(kHBlock == 2 * kDigits && kDigits * 8 == 4 * kHBlock, "two threads per digit; 4 counters each");
    __shared__ uint64_t hs[HOT ? kHotLds : 1];
    const int tid = threadIdx.x;
    const bool dig = tid < kDigits;                  // this thread owns digit `tid`'s totals
    const bool any_hot = HOT && hot_load<kHBlock>(hot, hs);
    const uint32_t t0 = blockIdx.x * tiles_per_blk;
    const uint32_t t1 = min(t0 + tiles_per_blk, ntiles);
    uint32_t run = 0;
    uint32_t acc = 0, acc_lo = 0;   // bucket counting (last pass): this thread's digit
    bool bad = false;
    KeyT kn[kHItems];
#if TBE_HIST_AHEAD >= 2
    KeyT kn2[kHItems];
#endif
    auto load_into = [&](KeyT (&dst)[kHItems], uint32_t t) {
#pragma unroll
        for (int it = 0; it < kHItems; ++it) {
            const uint64_t i = (uint64_t)t * kTile + it * kHBlock + tid;
            dst[it] = (t < t1 && i < n) ? LD_P(keys + i) : (KeyT)0;
        }
    };
    load_into(kn, t0);
#if TBE_HIST_AHEAD >= 2
    load_into(kn2, t0 + 1);
#endif
    for (uint32_t t = t0; t < t1; ++t) {
        KeyT kv[kHItems];
#pragma unroll
        for (int it = 0; it < kHItems; ++it) kv[it] = kn[it];
#if TBE_HIST_AHEAD >= 2
#pragma unroll
        for (int it = 0; it < kHItems; ++it) kn[it] = kn2[it];
        load_into(kn2, t + 2);                       // two tiles in flight while this one is counted
#else
        load_into(kn, t + 1);                        // in flight while this tile is counted
#endif
#pragma unroll
        for (int u = 0; u < 4; ++u) h8[u * kHBlock + tid] = 0;
        __syncthreads();
        const uint64_t base = (uint64_t)t * kTile;
        const uint64_t last = min<uint64_t>(base + kTile, n) - 1;
        uint32_t skv[kHItems];
        if (HOT && any_hot) {
            hot_sortkeys<kHItems>(kv, hot_table(hot, hs), nb, r_bits, skv);
        } else {
#pragma unroll
            for (int it = 0; it < kHItems; ++it) skv[it] = (uint32_t)((uint64_t)kv[it] & kmask);
        }
#pragma unroll
        for (int it = 0; it < kHItems; ++it) {
            const uint64_t i = base + it * kHBlock + tid;
            const bool valid = i < n;
            const uint32_t sk = skv[it];
            const uint32_t d = (sk >> shift) & (kDigits - 1);
            const uint64_t vmask = __ballot(valid);
            const uint32_t d0 = __shfl(d, vmask ? __ffsll((long long)vmask) - 1 : 0, 64);
            if (__all(!valid || d == d0)) {
                // the whole wave on one digit (a hot run's tile): one add
                if (vmask && (vmask & lanemask_lt()) == 0 && valid) atomicAdd(&h8[d0 * 8], (uint32_t)__popcll(vmask));
            } else {
                // 8 copies of each counter: lanes that share a digit (skewed traffic) mostly
                // hit different words instead of serialising on one
                if (valid) atomicAdd(&h8[d * 8 + (tid & 7)], 1u);
            }
            if (dig_out && valid) dig_out[i] = (uint8_t)d;   // pass 0: k_unrank re-ranks from it
            if (valid) {
                bad |= validate && ((uint64_t)kv[it] >= n_keys);
                if (bcount && (i == base || i == last)) {
                    // the tile's first and last bucket low bits (sorted by earlier passes)
                    tile_lo[i == last] = lowbits ? (sk >> r_bits) & ((1u << lowbits) - 1u) : 0u;
                    if (i == base && i == last) tile_lo[0] = tile_lo[1];
                }
            }
        }
        __syncthreads();
        uint32_t c = 0;
        if (dig) {
#pragma unroll
            for (int u = 0; u < 8; ++u) c += h8[tid * 8 + ((u + tid) & 7)];
            tileprefix[(uint64_t)t * kDigits + tid] = run;
            run += c;
        }
        if (bcount) {
            // Last pass: count requests per bucket for the fold's bucket starts.  The
            // previous passes left the requests sorted by the bucket's lower bits, so a
            // tile usually shares them: then its digit histogram is the bucket count,
            // summed here over the block's consecutive tiles and added once per change.
            const uint32_t lo0 = tile_lo[0], lo1 = tile_lo[1];
            if (lo0 == lo1) {
                if (dig) {
                    if (lo0 != acc_lo) {
                        const uint32_t bk = ((uint32_t)tid << lowbits) | acc_lo;
                        if (acc && bk < nbt) atomicAdd(&bcount[bk], acc);
                        acc = 0;
                        acc_lo = lo0;
                    }
                    acc += c;
                }
            } else if (lo1 - lo0 < 8) {
                // the lower bits change inside this tile (at most once per value): count
                // per (lower bits, digit) in LDS, then add each nonzero count once
                __syncthreads();                     // everyone has read its digit count
#pragma unroll
                for (int u = 0; u < 4; ++u) h8[u * kHBlock + tid] = 0;
                __syncthreads();
#pragma unroll
                for (int it = 0; it < kHItems; ++it) {
                    const uint64_t i = base + it * kHBlock + tid;
                    const uint32_t bk = skv[it] >> r_bits;
                    if (i < n) atomicAdd(&h8[((bk & ((1u << lowbits) - 1u)) - lo0) * kDigits + ((bk >> lowbits) & (kDigits - 1))], 1u);
                }
                __syncthreads();
                if (dig) {
                    for (uint32_t u = 0; u <= lo1 - lo0; ++u) {
                        const uint32_t cnt = h8[u * kDigits + tid];
                        const uint32_t bk = ((uint32_t)tid << lowbits) | (lo0 + u);
                        if (cnt && bk < nbt) atomicAdd(&bcount[bk], cnt);
                    }
                }
            } else {
#pragma unroll
                for (int it = 0; it < kHItems; ++it) {
                    const uint64_t i = base + it * kHBlock + tid;
                    const uint32_t bk = skv[it] >> r_bits;
                    if (i < n && bk < nbt) atomicAdd(&bcount[bk], 1u);
                }
            }
        }
        __syncthreads();
    }
    if (bcount && dig) {
        const uint32_t bk = ((uint32_t)tid << lowbits) | acc_lo;
        if (acc && bk < nbt) atomicAdd(&bcount[bk], acc);
    }
    if (dig) blocksum[(uint64_t)blockIdx.x * kDigits + tid] = run;
    if (__any(bad) && (tid & 63) == 0) atomicOr(err, 1u);
}

// Pass 1's histogram (of 2) from the digit stream: pass 0's scatter wrote each request's
// pass-1 digit as one byte in pass 0's output order (dig), so this reads 1 byte per request
// where k_hist reads the 8-byte record.  Same outputs as k_hist's last pass: tileprefix,
// blocksum and the per-bucket counts.  A request's bucket is (pass-1 digit << 8) | its
// pass-0 digit, and the pass-0 digit follows from its position: pass 0's output is sorted
// by it, with digit d starting at the exclusive scan of pass 0's digit totals (dtot0).
// 512 threads x 8 consecutive bytes (one 8-byte load) per 4096-request tile.
__global__ __launch_bounds__(kHBlock, TBE_HIST_WAVES) void k_hist_dig(
    const uint8_t *__restrict__ dig, uint64_t n, uint32_t tiles_per_blk, uint32_t ntiles,
    uint32_t *__restrict__ tileprefix, uint32_t *__restrict__ blocksum,
    const uint32_t *__restrict__ dtot0, uint32_t *__restrict__ bcount, uint32_t nbt) {
    __shared__ uint32_t h8[kDigits * 8];
    __shared__ uint32_t dstart[kDigits + 1];
    __shared__ uint32_t wsum[kHBlock / 64];
    // first and last pass-0 digit of each of the next kHBlock / 2 tiles, found by one
    // binary search per thread instead of two serial ones per tile
    __shared__ uint32_t tlo[kHBlock];
    static_assert(kHBlock == 2 * kDigits && kDigits * 8 == 4 * kHBlock, "two threads per digit; 4 counters each");
    static_assert(kHItems % 8 == 0, "8-byte loads");
    constexpr int kW = kHItems / 8;                  // 8-byte words per thread per tile
    const int tid = threadIdx.x;
    const bool own = tid < kDigits;                  // this thread owns digit `tid`'s totals
    {
        uint32_t all;
        const uint32_t pre = block_excl_scan<kHBlock>(own ? dtot0[tid] : 0u, wsum, &all);
        if (own) dstart[tid] = pre;
        if (tid == 0) dstart[kDigits] = 0xFFFFFFFFu;
    }
    // pass-0 digit of output position i: the last digit whose start is <= i
    auto d0_of = [&](uint32_t i) {
        uint32_t lo = 0, hi = kDigits;               // dstart[lo] <= i < dstart[hi]
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (dstart[mid] <= i) lo = mid;
            else hi = mid;
        }
        return lo;
    };
    const uint32_t t0 = blockIdx.x * tiles_per_blk;
    const uint32_t t1 = min(t0 + tiles_per_blk, ntiles);
    uint32_t run = 0, acc = 0, acc_lo = 0;
    auto load = [&](uint32_t t, uint64_t (&dst)[kW]) {
#pragma unroll
        for (int q = 0; q < kW; ++q) {
            const uint64_t i = (uint64_t)t * kTile + (uint64_t)tid * kHItems + 8 * q;
            uint64_t v = 0;
            if (t < t1 && i + 8 <= n) {
                v = LD_P(reinterpret_cast<const uint64_t *>(dig + i));
            } else if (t < t1) {
                for (int u = 0; i + u < n; ++u) v |= (uint64_t)dig[i + u] << (8 * u);
            }
            dst[q] = v;
        }
    };
    uint64_t vn[kW];
    load(t0, vn);
    __syncthreads();                                 // dstart
    for (uint32_t t = t0; t < t1; ++t) {
        uint64_t vw[kW];
#pragma unroll
        for (int q = 0; q < kW; ++q) vw[q] = vn[q];
        load(t + 1, vn);                             // in flight while this tile is counted
#pragma unroll
        for (int u = 0; u < 4; ++u) h8[u * kHBlock + tid] = 0;
        const uint64_t base = (uint64_t)t * kTile;
        const uint32_t tk = (t - t0) % (kHBlock / 2);
        if (tk == 0) {   // (the previous tile's reads of tlo are behind the loop's last barrier)
            const uint32_t tt = t + (uint32_t)(tid >> 1);
            if (tt < t1) {
                const uint64_t b = (uint64_t)tt * kTile;
                tlo[tid] = d0_of((uint32_t)((tid & 1) ? min<uint64_t>(b + kTile, n) - 1 : b));
            }
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kHItems; ++u) {
            const uint64_t i = base + (uint64_t)tid * kHItems + u;
            const bool valid = i < n;
            const uint32_t d = (uint32_t)(vw[u >> 3] >> (8 * (u & 7))) & (kDigits - 1);
            const uint64_t vmask = __ballot(valid);
            const uint32_t dw = __shfl(d, vmask ? __ffsll((long long)vmask) - 1 : 0, 64);
            if (__all(!valid || d == dw)) {
                if (vmask && (vmask & lanemask_lt()) == 0 && valid) atomicAdd(&h8[dw * 8], (uint32_t)__popcll(vmask));
            } else if (valid) {
                atomicAdd(&h8[d * 8 + (tid & 7)], 1u);
            }
        }
        __syncthreads();
        uint32_t c = 0;
        if (own) {
#pragma unroll
            for (int u = 0; u < 8; ++u) c += h8[tid * 8 + ((u + tid) & 7)];
            tileprefix[(uint64_t)t * kDigits + tid] = run;
            run += c;
        }
        // per-bucket counts, as k_hist's last pass
        const uint32_t lo0 = tlo[2 * tk], lo1 = tlo[2 * tk + 1];
        if (lo0 == lo1) {
            if (own) {
                if (lo0 != acc_lo) {
                    const uint32_t bk = ((uint32_t)tid << kDigitBits) | acc_lo;
                    if (acc && bk < nbt) atomicAdd(&bcount[bk], acc);
                    acc = 0;
                    acc_lo = lo0;
                }
                acc += c;
            }
        } else if (lo1 - lo0 < 8) {
            __syncthreads();                         // everyone has read its digit count
#pragma unroll
            for (int u = 0; u < 4; ++u) h8[u * kHBlock + tid] = 0;
            __syncthreads();
#pragma unroll
            for (int u = 0; u < kHItems; ++u) {
                const uint64_t i = base + (uint64_t)tid * kHItems + u;
                if (i >= n) continue;
                uint32_t lo = 0;
                for (uint32_t x = 1; x <= lo1 - lo0; ++x) lo += dstart[lo0 + x] <= (uint32_t)i;
                const uint32_t d = (uint32_t)(vw[u >> 3] >> (8 * (u & 7))) & (kDigits - 1);
                atomicAdd(&h8[lo * kDigits + d], 1u);
            }
            __syncthreads();
            if (own) {
                for (uint32_t u = 0; u <= lo1 - lo0; ++u) {
                    const uint32_t cnt = h8[u * kDigits + tid];
                    const uint32_t bk = ((uint32_t)tid << kDigitBits) | (lo0 + u);
                    if (cnt && bk < nbt) atomicAdd(&bcount[bk], cnt);
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < kHItems; ++u) {
                const uint64_t i = base + (uint64_t)tid * kHItems + u;
                if (i >= n) continue;
                const uint32_t bk = (((uint32_t)(vw[u >> 3] >> (8 * (u & 7))) & (kDigits - 1)) << kDigitBits) | d0_of((uint32_t)i);
                if (bk < nbt) atomicAdd(&bcount[bk], 1u);
            }
        }
        __syncthreads();
    }
    if (own) {
        const uint32_t bk = ((uint32_t)tid << kDigitBits) | acc_lo;
        if (acc && bk < nbt) atomicAdd(&bcount[bk], acc);
        blocksum[(uint64_t)blockIdx.x * kDigits + tid] = run;
    }
}

// Digit-column scan, one workgroup per digit d: blockprefix[j][d] = number of digit-d
// elements in blocks < j; digit_total[d] = all of them.  The digit bases (exclusive scan
// of digit_total) are formed by each consumer workgroup itself.
__global__ __launch_bounds__(kBlock) void k_colscan(const uint32_t *__restrict__ blocksum,
                                                    uint32_t nblk,
                                                    uint32_t *__restrict__ blockprefix,
                                                    uint32_t *__restrict__ digit_total) {
    __shared__ uint32_t wsum[kWaves];
    const int d = blockIdx.x, tid = threadIdx.x;
    constexpr int PER = kMaxHistBlocks / kBlock;   // blocks per thread
    uint32_t c[PER], s = 0;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const uint32_t j = tid * PER + u;
        c[u] = (j < nblk) ? blocksum[(uint64_t)j * kDigits + d] : 0u;
        s += c[u];
    }
    uint32_t total;
    uint32_t pre = block_excl_scan<kBlock>(s, wsum, &total);
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const uint32_t j = tid * PER + u;
        if (j < nblk) blockprefix[(uint64_t)j * kDigits + d] = pre;
        pre += c[u];
    }
    if (tid == 0) digit_total[d] = total;
}

// goff[d] = global output position of this tile's first digit-d element.
template <int BLOCK>
__device__ __forceinline__ void tile_offsets(uint32_t tile, uint32_t tiles_per_blk,
                                             const uint32_t *__restrict__ tileprefix,
                                             const uint32_t *__restrict__ blockprefix,
                                             const uint32_t *__restrict__ digit_total,
                                             uint32_t *goff, uint32_t *wsum) {
    const int tid = threadIdx.x;
    uint32_t tot = (tid < kDigits) ? digit_total[tid] : 0u;
    uint32_t all;
    const uint32_t base = block_excl_scan<BLOCK>(tot, wsum, &all);
    if (tid < kDigits)
        goff[tid] = base + blockprefix[(uint64_t)(tile / tiles_per_blk) * kDigits + tid] +
                    tileprefix[(uint64_t)tile * kDigits + tid];
}

// Stable partition of one tile by digit d = (key >> shift) & 255.  Payload travels as
// SoA {key u32, permits i32, ts i64}; it is staged through LDS in two 8-byte rounds so
// each digit's run leaves the workgroup as one contiguous, coalesced write.
// IDX: also carry each request's arrival index (queueing kind: it becomes the request
// id of a queued entry); pass 0 generates it (iin == nullptr).
template <typename KeyIn, bool IDX, bool TS = true>
__global__ __launch_bounds__(kPartBlock) void k_scatter(
    const KeyIn *__restrict__ kin, const int32_t *__restrict__ pin, const int64_t *__restrict__ tin,
    const uint32_t *__restrict__ iin, uint64_t n, int shift, const uint32_t *__restrict__ tileprefix,
    const uint32_t *__restrict__ blockprefix, const uint32_t *__restrict__ digit_total,
    uint32_t tiles_per_blk, uint32_t *__restrict__ kout, int32_t *__restrict__ pout,
    int64_t *__restrict__ tout, uint32_t *__restrict__ iout, uint32_t *__restrict__ perm,
    uint32_t *__restrict__ err, int validate) {
    __shared__ RankLds<kPartBlock> L;
    __shared__ uint32_t goff[kDigits];
    // staging buffer; during ranking it holds the per-(round, wave, digit) counts
    __shared__ uint64_t stage[kTile];
    static_assert(kPartItems * (kPartBlock / 64) * kDigits * 2 <= kTile * 8, "cnt fits in stage");

    const int tid = threadIdx.x;
    const uint32_t tile = xcd_swizzle(blockIdx.x, gridDim.x);
    const uint64_t base = (uint64_t)tile * kTile;
    const int nvalid = (int)min<uint64_t>(kTile, n - base);

    // Issue every load of the tile up front; the payload waits in registers while the
    // ranks are computed.
    uint32_t key[kPartItems], lpos[kPartItems];
    int32_t pm[kPartItems];
    int64_t tv[kPartItems];
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int e = it * kPartBlock + tid;
        const bool v = e < nvalid;
        key[it] = v ? (uint32_t)kin[base + e] : 0u;
        pm[it] = v ? pin[base + e] : 0;
        tv[it] = (v && TS) ? tin[base + e] : 0;
    }
    tile_offsets<kPartBlock>(tile, tiles_per_blk, tileprefix, blockprefix, digit_total, goff, L.wsum);
    rank_tile<kPartBlock, kPartItems>(key, shift, nvalid, L, reinterpret_cast<uint16_t *>(stage), lpos);
    __syncthreads();   // the counts in `stage` are dead from here on

    bool bad = false;
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int e = it * kPartBlock + tid;
        if (e < nvalid) {
            const uint32_t d = (key[it] >> shift) & (kDigits - 1);
            bad |= validate && (pm[it] < 0 || tv[it] < 0);
            stage[lpos[it]] = ((uint64_t)key[it] << 32) | (uint32_t)pm[it];
            // where input element e goes: the inverse pass is a plain gather through it
            perm[base + e] = goff[d] + lpos[it] - L.lstart[d];
        }
    }
    __syncthreads();
    uint32_t gpos[kPartItems];
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int j = it * kPartBlock + tid;
        if (j < nvalid) {
            const uint64_t s = stage[j];
            const uint32_t k = (uint32_t)(s >> 32);
            const uint32_t d = (k >> shift) & (kDigits - 1);
            gpos[it] = goff[d] + (uint32_t)j - L.lstart[d];
            kout[gpos[it]] = k;
            pout[gpos[it]] = (int32_t)(uint32_t)s;
        }
    }
    if (TS) {
        __syncthreads();
#pragma unroll
        for (int it = 0; it < kPartItems; ++it) {
            const int e = it * kPartBlock + tid;
            if (e < nvalid) stage[lpos[it]] = (uint64_t)tv[it];
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < kPartItems; ++it) {
            const int j = it * kPartBlock + tid;
            if (j < nvalid) tout[gpos[it]] = (int64_t)stage[j];
        }
    }
    if (IDX) {
        uint32_t *stage32 = reinterpret_cast<uint32_t *>(stage);
        uint32_t iv[kPartItems];
#pragma unroll
        for (int it = 0; it < kPartItems; ++it) {
            const int e = it * kPartBlock + tid;
            iv[it] = (e < nvalid) ? (iin ? iin[base + e] : (uint32_t)(base + e)) : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < kPartItems; ++it) {
            const int e = it * kPartBlock + tid;
            if (e < nvalid) stage32[lpos[it]] = iv[it];
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < kPartItems; ++it) {
            const int j = it * kPartBlock + tid;
            if (j < nvalid) iout[gpos[it]] = stage32[j];
        }
    }
    if (validate && __any(bad) && (tid & 63) == 0) atomicOr(err, 1u);
}

// bstart = exclusive scan of the per-bucket counts k_hist's last pass gathered;
// bstart[nbt] = the batch size.  One 1024-thread workgroup over rows of 16384 buckets:
// a coalesced load into LDS, each thread scans its 16 consecutive counts, one block
// scan of the thread sums, and a coalesced store back through LDS.
constexpr int kScanPer = 16;
// dlist (sparse batches): dlist[0] = the number of ordinary buckets (< nb) with at least
// wide_min requests, dlist[1..] their ids (any order): k_fold_wide's whole grid then walks
// only those, and k_fold_sparse takes the rest.
__global__ __launch_bounds__(1024) void k_bscan(const uint32_t *__restrict__ bcount, uint32_t nbt,
                                                uint32_t *__restrict__ bstart, uint32_t nb = 0,
                                                uint32_t wide_min = 0, uint32_t *__restrict__ dlist = nullptr) {
    // row-major [1024][kScanPer] padded to kScanPer + 1 words per thread: a thread's 16
    // consecutive counts no longer sit 16 words apart from its neighbours' (bank conflicts)
    __shared__ uint32_t tile[1024 * (kScanPer + 1)];
    auto pad = [](uint32_t j) { return (j / kScanPer) * (kScanPer + 1) + (j % kScanPer); };
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t n_dense;
    if (threadIdx.x == 0) n_dense = 0;
    const uint32_t t = threadIdx.x;
    constexpr uint32_t kRow = 1024 * kScanPer;
    constexpr int kGroup = 4;   // rows whose loads are all issued before the first is scanned
    uint32_t carry = 0;
    for (uint32_t g0 = 0; g0 < nbt; g0 += kGroup * kRow) {
        uint32_t ld[kGroup][kScanPer];
#pragma unroll
        for (int r = 0; r < kGroup; ++r)
#pragma unroll
            for (int k = 0; k < kScanPer; ++k) {
                const uint32_t j = g0 + r * kRow + k * 1024 + t;
                ld[r][k] = j < nbt ? bcount[j] : 0u;
            }
#pragma unroll
        for (int r = 0; r < kGroup; ++r) {
            const uint32_t r0 = g0 + r * kRow;
            if (r0 >= nbt) break;                      // uniform across the block
#pragma unroll
            for (int k = 0; k < kScanPer; ++k) tile[pad(k * 1024 + t)] = ld[r][k];
            __syncthreads();
            uint32_t v[kScanPer], sum = 0;
#pragma unroll
            for (int k = 0; k < kScanPer; ++k) {
                v[k] = tile[t * (kScanPer + 1) + k];
                sum += v[k];
            }
            if (dlist) {
#pragma unroll
                for (int k = 0; k < kScanPer; ++k) {
                    const uint32_t bk = r0 + t * kScanPer + k;
                    if (bk < nb && v[k] >= wide_min) dlist[1 + atomicAdd(&n_dense, 1u)] = bk;
                }
            }
            uint32_t total;
            uint32_t pre = carry + block_excl_scan<1024>(sum, wsum, &total);
#pragma unroll
            for (int k = 0; k < kScanPer; ++k) {
                tile[t * (kScanPer + 1) + k] = pre;
                pre += v[k];
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kScanPer; ++k) {
                const uint32_t j = r0 + k * 1024 + t;
                if (j < nbt) bstart[j] = tile[pad(k * 1024 + t)];
            }
            carry += total;
            __syncthreads();
        }
    }
    if (t == 0) bstart[nbt] = carry;
    if (dlist) {
        __syncthreads();
        if (t == 0) dlist[0] = n_dense;
    }
}

// Bucket starts of a dense batch by decoupled look-back (round 5): k_bscan is one
// workgroup walking ~50K counts (17-21 us per config-B batch, latency-bound).  Here each
// 1024-thread workgroup scans 4096 consecutive counts, publishes its total tagged with the
// batch number (flags[blk] = tag << 32 | total; no reset between batches), and one wave
// sums the totals of every earlier workgroup once they are published.  Workgroups are
// dispatched in index order, so an earlier one is always running or done: the wait ends.
constexpr int kBsPer = 4;
constexpr uint32_t kBsTile = 1024u * kBsPer;
constexpr uint32_t kBsMaxBlocks = 64;        // nb_total <= 2^16 buckets (two 8-bit passes)
// Sparse batches also list their dense buckets (dlist, as k_bscan; dlist[0] was zeroed with
// the counts): one global atomic per dense bucket, of which a sparse batch has few.
__global__ __launch_bounds__(1024) void k_bscan_lb(const uint32_t *__restrict__ bcount, uint32_t nbt,
                                                   uint32_t *__restrict__ bstart,
                                                   unsigned long long *__restrict__ flags, uint32_t tag,
                                                   uint32_t nb = 0, uint32_t wide_min = 0,
                                                   uint32_t *__restrict__ dlist = nullptr) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t excl;
    const uint32_t t = threadIdx.x, blk = blockIdx.x;
    const uint32_t b0 = blk * kBsTile + t * kBsPer;
    uint32_t v[kBsPer];
#pragma unroll
    for (int k = 0; k < kBsPer; ++k) v[k] = (b0 + k < nbt) ? bcount[b0 + k] : 0u;
    if (dlist) {
#pragma unroll
        for (int k = 0; k < kBsPer; ++k)
            if (b0 + k < nb && v[k] >= wide_min) dlist[1 + atomicAdd(dlist, 1u)] = b0 + k;
    }
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < kBsPer; ++k) sum += v[k];
    uint32_t total;
    const uint32_t pre = block_excl_scan<1024>(sum, wsum, &total);
    if (t == 0)
        __hip_atomic_store(&flags[blk], ((unsigned long long)tag << 32) | total, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (t < 64) {
        uint32_t acc = 0;
        for (uint32_t j0 = 0; j0 < blk; j0 += 64) {
            const uint32_t j = j0 + t;
            uint32_t val = 0;
            if (j < blk) {
                unsigned long long f;
                do {
                    f = __hip_atomic_load(&flags[j], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                } while ((uint32_t)(f >> 32) != tag);
                val = (uint32_t)f;
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) val += __shfl_xor(val, o, 64);
            acc += val;
        }
        if (t == 0) excl = acc;
    }
    __syncthreads();
    uint32_t run = excl + pre;
#pragma unroll
    for (int k = 0; k < kBsPer; ++k) {
        if (b0 + k < nbt) bstart[b0 + k] = run;
        run += v[k];
    }
    if (blk == gridDim.x - 1 && t == 0) bstart[nbt] = excl + total;
}

// Packed request records (token-bucket kind).  When the key, a permit code and a
// 32-bit time offset fit one u64, the partition passes and the fold move one 8-byte
// record per request instead of {key u32, permits i32, ts i64}:
//
//   bits [0, kb)            key (< n_keys <= 2^kb)
//   bits [kb, kb+pb)        permit code min(permits, TokenLimit + 1): x <= TokenLimit
//                           always (TB:221), so every larger request is decided, and
//                           leaves the state, exactly like TokenLimit + 1 (TB:224)
//   bit  kb+pb              escape
//   bits [kb+pb+1, 64)      ts - base  (base = ts[0] of the batch - 2^(wb-1)), or, with
//                           the escape bit, the arrival index: the fold then reads the
//                           request's timestamp from the caller's array
//
// wb = 64 - kb - pb - 1 >= 32, so a batch whose timestamps lie within +-35 minutes of
// its first one never escapes.
struct PackFmt {
    uint64_t kmask;     // (1 << kb) - 1
    int32_t kb;
    int32_t pb;
    int32_t pc_max;     // TokenLimit + 1
    int32_t wb;
    // Narrow pass-0 records (round 5; token bucket, two passes, fold records, digit stream):
    // pass 0 writes a u32 per request -- row within the bucket (rb bits), permit code,
    // escape, ts - base0 (w0 = 32 - rb - pb - 1 bits, base0 = ts[0] - 2^(w0-1)) -- beside
    // the one-byte digit stream that already carries the pass-1 digit; the pass-0 digit is
    // the record's position.  An escaped request (time outside the window) also writes its
    // timestamp to a side array at its pass-0 output position, where the fold finds it.
    // 4 + 1 bytes instead of 8 + 1 written by pass 0 and read by pass 1.
    int32_t n0;         // 1: pass 0 writes narrow records
    int32_t rb;         // row bits (r_bits) of a narrow record
    int32_t w0;         // time-offset bits of a narrow record
};
__device__ __forceinline__ int64_t pack_base32(const int64_t *__restrict__ ts, const PackFmt &F) {
    return ts[0] - ((int64_t)1 << (F.w0 - 1));
}
// A narrow pass-0 record from the partition key (row = its low rb bits); *esc: the time did
// not fit and goes to the side array.
__device__ __forceinline__ uint32_t pack_rec32(uint32_t pkey, int32_t p, int64_t ts, int64_t tbase, const PackFmt &F,
                                               bool &esc) {
    const uint32_t pc = (uint32_t)(p < 0 ? 0 : (p > F.pc_max ? F.pc_max : p));
    const uint64_t d = (uint64_t)ts - (uint64_t)tbase;
    const bool fits = ts >= tbase && (d >> F.w0) == 0;
    esc = !fits;
    return (pkey & ((1u << F.rb) - 1u)) | (pc << F.rb) | ((uint32_t)!fits << (F.rb + F.pb)) |
           (fits ? (uint32_t)d << (F.rb + F.pb + 1) : 0u);
}
__device__ __forceinline__ int64_t pack_base(const int64_t *__restrict__ ts, const PackFmt &F) {
    return ts[0] - ((int64_t)1 << (F.wb - 1));
}
// req_time_rel's base for a batch (TimeBase): 2^31 us (~35 min) below its first
// timestamp, so that request times up to ~35 min above it and stored row times up to ~35
// min below it take the 32-bit path.  Not pack_base: with wb > 32 (few keys or a small
// TokenLimit, e.g. config D's wb = 33) that sits 2^32 us below, every request lies beyond
// req_time_rel's window and the whole fold took req_time's 64-bit path.
#ifndef TBE_REL_BASE
#define TBE_REL_BASE 1                       // 0: pack_base, as before round 6 (A/B)
#endif
__device__ __forceinline__ int64_t rel_base(const int64_t *__restrict__ ts, const PackFmt &F) {
#if TBE_REL_BASE
    (void)F;
    const int64_t b = ts[0] - ((int64_t)1 << 31);
    return b > 0 ? b : 0;
#else
    return pack_base(ts, F);
#endif
}
__device__ __forceinline__ uint64_t pack_rec(uint64_t key, int32_t p, int64_t ts, uint64_t idx,
                                             int64_t tbase, const PackFmt &F) {
    const uint64_t pc = (uint64_t)(p < 0 ? 0 : (p > F.pc_max ? F.pc_max : p));
    const uint64_t d = (uint64_t)ts - (uint64_t)tbase;
    const bool fits = ts >= tbase && (d >> F.wb) == 0;
    const uint64_t pay = fits ? d : idx;
    return (key & F.kmask) | (pc << F.kb) | ((uint64_t)!fits << (F.kb + F.pb)) |
           (pay << (F.kb + F.pb + 1));
}
__device__ __forceinline__ void unpack_rec(uint64_t rec, const int64_t *__restrict__ ts_orig,
                                           int64_t tbase, const PackFmt &F, uint32_t &key,
                                           int32_t &p, int64_t &ts) {
    key = (uint32_t)(rec & F.kmask);
    p = (int32_t)((rec >> F.kb) & ((1ull << F.pb) - 1));
    const uint64_t pay = rec >> (F.kb + F.pb + 1);
    ts = ((rec >> (F.kb + F.pb)) & 1) ? ts_orig[pay] : (int64_t)((uint64_t)tbase + pay);
}

// Fold records (token-bucket kind, packed, >= 2 partition passes).  The last pass writes,
// instead of a PackFmt record and its permutation, what the fold and the hot runs need:
//
//   bits [0, rb)              row within the bucket (the key field's low r_bits)
//   bits [rb, rb+pb)          permit code (as PackFmt)
//   bit  rb+pb                escape
//   bits [rb+pb+1, +pw)       the request's position in the last pass's INPUT (the previous
//                             pass's output): its reply goes there, so the last pass needs
//                             no permutation and no un-partition pass of its own
//   bits [rb+pb+1+pw, 64)     ts - base1 (tw bits, base1 = ts[0] - 2^(tw-1)); with the
//                             escape bit: unused, and the fold takes the request's time from
//                             the previous pass's record at that position
//
// pw = ceil_log2(batch), tw = 64 - rb - pb - 1 - pw (config B: 22 bits, +-2.1 s around the
// batch's first request; the batch spans 10 ms).  Used when tw >= 8.
struct FoldFmt {
    int32_t on;
    int32_t n0;             // pass 0 wrote narrow records: an escaped record's time is rec0[pos] itself
    int32_t rb, pb, pw, tw;
    uint32_t nb;            // ordinary buckets
    uint32_t region_bits;   // 8 * (passes - 1): buckets with equal low region_bits share a reply region
    uint32_t n_hi;          // ceil(nb / 2^region_bits)
};
__device__ __forceinline__ int64_t fold_base(const int64_t *__restrict__ ts, const FoldFmt &G) {
    return ts[0] - ((int64_t)1 << (G.tw - 1));
}
__device__ __forceinline__ uint64_t fold_rec(uint64_t rec0, uint32_t pos, int64_t tbase0, int64_t tbase1,
                                             const PackFmt &F, const FoldFmt &G) {
    const uint64_t row = rec0 & ((1ull << G.rb) - 1);
    const uint64_t pc = (rec0 >> F.kb) & ((1ull << F.pb) - 1);
    const bool esc0 = (rec0 >> (F.kb + F.pb)) & 1;
    const int64_t ts = (int64_t)((uint64_t)tbase0 + (rec0 >> (F.kb + F.pb + 1)));
    const uint64_t d = (uint64_t)ts - (uint64_t)tbase1;
    const bool fits = !esc0 && ts >= tbase1 && (d >> G.tw) == 0;
    return row | (pc << G.rb) | ((uint64_t)!fits << (G.rb + G.pb)) | ((uint64_t)pos << (G.rb + G.pb + 1)) |
           ((fits ? d : 0ull) << (G.rb + G.pb + 1 + G.pw));
}
__device__ __forceinline__ uint64_t fold_rec32(uint32_t r32, uint32_t pos, int64_t tbase0, int64_t tbase1,
                                               const PackFmt &F, const FoldFmt &G) {
    const uint64_t row = r32 & ((1u << F.rb) - 1u);
    const uint64_t pc = (r32 >> F.rb) & ((1u << F.pb) - 1u);
    const bool esc0 = (r32 >> (F.rb + F.pb)) & 1u;
    const int64_t ts = (int64_t)((uint64_t)tbase0 + (uint64_t)(r32 >> (F.rb + F.pb + 1)));
    const uint64_t d = (uint64_t)ts - (uint64_t)tbase1;
    const bool fits = !esc0 && ts >= tbase1 && (d >> G.tw) == 0;
    return row | (pc << G.rb) | ((uint64_t)!fits << (G.rb + G.pb)) | ((uint64_t)pos << (G.rb + G.pb + 1)) |
           ((fits ? d : 0ull) << (G.rb + G.pb + 1 + G.pw));
}
// Decode a fold record: row, permit code, time (escaped: through the previous pass's
// record `rec0[pos]`, itself possibly escaped to the caller's ts array) and reply position.
__device__ __forceinline__ void unfold_rec(uint64_t rec, const FoldFmt &G, int64_t tbase1,
                                           const uint64_t *__restrict__ rec0, const int64_t *__restrict__ ts_orig,
                                           int64_t tbase0, const PackFmt &F, uint32_t &row, int32_t &p,
                                           int64_t &ts, uint32_t &pos) {
    row = (uint32_t)(rec & ((1ull << G.rb) - 1));
    p = (int32_t)((rec >> G.rb) & ((1ull << G.pb) - 1));
    pos = (uint32_t)((rec >> (G.rb + G.pb + 1)) & ((1ull << G.pw) - 1));
    if ((rec >> (G.rb + G.pb)) & 1) {
        if (G.n0) {
            ts = (int64_t)rec0[pos];   // the side array of narrow pass-0 records' escaped times
        } else {
            uint32_t k;
            int32_t p0;
            unpack_rec(rec0[pos], ts_orig, tbase0, F, k, p0, ts);
        }
    } else {
        ts = (int64_t)((uint64_t)tbase1 + (rec >> (G.rb + G.pb + 1 + G.pw)));
    }
}
// The fold's bucket for this workgroup.  With fold records the replies of all buckets
// that share their low region_bits land in one region of the previous pass's output (256
// KB of one-byte replies at config B); the buckets of a region are dealt to one XCD
// (workgroups b and b + 8 share one) and run there together, so that XCD's L2 merges their
// scattered one-byte reply stores into whole lines.  Workgroups past the last bucket exit.
__device__ __forceinline__ uint32_t fold_bucket_at(const FoldFmt &G, uint32_t blk) {
    if (!G.on) return blk;
    const uint32_t x = blk & 7u, s = blk >> 3;
    const uint32_t j = s / G.n_hi, hi = s - j * G.n_hi;
    return (hi << G.region_bits) | (x + 8u * j);
}
__device__ __forceinline__ uint32_t fold_bucket(const FoldFmt &G) { return fold_bucket_at(G, blockIdx.x); }
// Any record of the fold's input: (row, permit code, time, reply position).
__device__ __forceinline__ void fold_input(uint64_t rec, uint32_t q, const FoldFmt &G, int64_t tbase1,
                                           const uint64_t *__restrict__ rec0, const int64_t *__restrict__ ts_orig,
                                           int64_t tbase0, const PackFmt &F, uint32_t rmask, uint32_t &row,
                                           int32_t &p, int64_t &ts, uint32_t &pos) {
    if (G.on) {
        unfold_rec(rec, G, tbase1, rec0, ts_orig, tbase0, F, row, p, ts, pos);
    } else {
        uint32_t k;
        unpack_rec(rec, ts_orig, tbase0, F, k, p, ts);
        row = k & rmask;
        pos = q;
    }
}

// Stable partition pass over packed records (see k_scatter; one 8-byte LDS staging
// round instead of two).  FIRST: read the caller's arrays, validate permits and
// timestamps, and pack; otherwise read the previous pass's records.
// HOT (with FIRST): a hot key's record carries its run's partition key (hot_sortkey)
// in the key field.
// IDX (queueing kind): each request's arrival index travels beside its record (a second,
// 4-byte staging round); pass 0 generates it.
// NOTS (approximate kind, FIRST): no timestamps -- every record takes the escape form,
// so its payload field carries the arrival index.
// LAST (token-bucket kind, the last of >= 2 passes): write fold records (FoldFmt) -- each
// element's position in this pass's input rides along -- and no permutation; `tin` is
// then the caller's timestamps (for the record bases).
// TBE_SCATTER0_WAVES (A/B): minimum waves per SIMD of the first pass (which holds the
// caller's three columns of its 8 requests per thread in registers: 108 VGPRs, 4 waves)
#ifndef TBE_BSCAN_LB
#define TBE_BSCAN_LB 1                       // bucket starts by decoupled look-back; 0: one workgroup (A/B)
#endif
#ifndef TBE_NARROW0
#define TBE_NARROW0 1                        // narrow pass-0 records (PackFmt::n0); 0: A/B
#endif
#ifndef TBE_SCATTER0_WAVES
#define TBE_SCATTER0_WAVES 1
#endif
template <bool FIRST, bool HOT = false, bool IDX = false, bool NOTS = false, bool LAST = false>
__global__ __launch_bounds__(kPartBlock, FIRST ? TBE_SCATTER0_WAVES : 1) void k_scatter_rec(
    const uint64_t *__restrict__ kin, const int32_t *__restrict__ pin, const int64_t *__restrict__ tin,
    const uint64_t *__restrict__ rin, uint64_t n, int shift, PackFmt F,
    const uint32_t *__restrict__ tileprefix, const uint32_t *__restrict__ blockprefix,
    const uint32_t *__restrict__ digit_total, uint32_t tiles_per_blk, uint64_t *__restrict__ rout,
    uint32_t *__restrict__ perm, uint32_t *__restrict__ err, const HotSet *__restrict__ hot = nullptr,
    uint32_t nb = 0, int r_bits = 0, const uint32_t *__restrict__ iin = nullptr,
    uint32_t *__restrict__ iout = nullptr, FoldFmt G = FoldFmt{}, uint8_t *__restrict__ dig_next = nullptr,
    const uint8_t *__restrict__ din = nullptr, int64_t *__restrict__ ts0 = nullptr) {
    static_assert(!(FIRST && LAST), "fold records come from a pass after the first");
    // narrow pass-0 records (F.n0): FIRST writes u32 records (+ escaped times to ts0), LAST
    // reads them with the pass-1 digit from the digit stream `din`; the LDS stage then holds
    // record | digit(s) << 32, since the record no longer carries the key.  The queueing
    // kind (IDX) keeps its arrival index beside them; the approximate kind (NOTS) has no
    // time: its narrow record is row | permit code (round 6)
    const bool n0 = F.n0 != 0;
    __shared__ RankLds<kPartBlock> L;
    __shared__ uint32_t goff[kDigits];
    __shared__ uint64_t stage[kTile];
    __shared__ uint16_t stage_e[LAST ? kTile : 1];   // LAST: each staged record's input element
    __shared__ uint64_t hs[HOT ? kHotLds : 1];
    static_assert(kPartItems * (kPartBlock / 64) * kDigits * 2 <= kTile * 8, "cnt fits in stage");

    const int tid = threadIdx.x;
    const uint32_t tile = xcd_swizzle(blockIdx.x, gridDim.x);
    const uint64_t base = (uint64_t)tile * kTile;
    const int nvalid = (int)min<uint64_t>(kTile, n - base);

    uint64_t rec[kPartItems];
    uint32_t key[kPartItems], lpos[kPartItems];
    bool bad = false;
    bool any_hot = false;
    int64_t tv_keep[FIRST ? kPartItems : 1];   // narrow records: escaped times go to ts0
    if (FIRST) {
        uint64_t kv[kPartItems];
        int32_t pv[kPartItems];
        int64_t tv[kPartItems];
#pragma unroll
        for (int it = 0; it < kPartItems; ++it) {
            const int e = wb_elem<kPartBlock, kPartItems>(it);   // wave-blocked tile order
            const bool v = e < nvalid;
            kv[it] = v ? LD_P(kin + base + e) : 0ull;
            pv[it] = v ? LD_P(pin + base + e) : 0;
            tv[it] = NOTS ? -1 : (v ? LD_P(tin + base + e) : 0);
        }
        // the table fill overlaps the tile loads above
        any_hot = HOT && hot_load<kPartBlock>(hot, hs);
        const int64_t tbase = NOTS ? 0 : (n0 ? pack_base32(tin, F) : pack_base(tin, F));
        uint32_t skv[kPartItems];
        if (HOT && any_hot) {
            hot_sortkeys<kPartItems>(kv, hot_table(hot, hs), nb, r_bits, skv);
        } else {
#pragma unroll
            for (int it = 0; it < kPartItems; ++it) skv[it] = (uint32_t)(kv[it] & F.kmask);
        }
#pragma unroll
        for (int it = 0; it < kPartItems; ++it) {
            const int e = wb_elem<kPartBlock, kPartItems>(it);   // wave-blocked tile order
            bad |= (e < nvalid) && (pv[it] < 0 || (!NOTS && tv[it] < 0));
            if (n0) {
                bool esc = false;
                const uint32_t r32 =
                    NOTS ? (skv[it] & ((1u << F.rb) - 1u)) |
                               ((uint32_t)(pv[it] < 0 ? 0 : (pv[it] > F.pc_max ? F.pc_max : pv[it])) << F.rb)
                         : pack_rec32(skv[it], pv[it], tv[it], tbase, F, esc);
                // stage: record | pass-0 digit << 32 | pass-1 digit << 40; escape flag in bit 48
                rec[it] = (uint64_t)r32 | ((uint64_t)((skv[it] >> shift) & (kDigits - 1)) << 32) |
                          ((uint64_t)((skv[it] >> (shift + kDigitBits)) & (kDigits - 1)) << 40) |
                          ((uint64_t)esc << 48);
            } else {
                rec[it] = pack_rec(skv[it], pv[it], tv[it], base + e, tbase, F);
            }
            key[it] = skv[it];
            tv_keep[FIRST ? it : 0] = tv[it];
        }
    } else {
        if (n0) {
            const uint32_t *rin32 = reinterpret_cast<const uint32_t *>(rin);
            uint8_t dv[kPartItems];
#pragma unroll
            for (int it = 0; it < kPartItems; ++it) {
                const int e = wb_elem<kPartBlock, kPartItems>(it);   // wave-blocked tile order
                rec[it] = (e < nvalid) ? (uint64_t)LD_P(rin32 + base + e) : 0ull;
                dv[it] = (e < nvalid) ? din[base + e] : (uint8_t)0;
            }
#pragma unroll
            for (int it = 0; it < kPartItems; ++it) {
                key[it] = (uint32_t)dv[it] << shift;
                rec[it] |= (uint64_t)dv[it] << 32;
            }
        } else {
#pragma unroll
            for (int it = 0; it < kPartItems; ++it) {
                const int e = wb_elem<kPartBlock, kPartItems>(it);   // wave-blocked tile order
                rec[it] = (e < nvalid) ? LD_P(rin + base + e) : 0ull;
                key[it] = (uint32_t)(rec[it] & F.kmask);
            }
        }
    }
    tile_offsets<kPartBlock>(tile, tiles_per_blk, tileprefix, blockprefix, digit_total, goff, L.wsum);
    rank_tile_wb<kPartBlock, kPartItems>(key, shift, nvalid, L, reinterpret_cast<uint32_t *>(stage), lpos);
    int64_t tbase0 = 0, tbase1 = 0;
    if (LAST && tin) {   // (the approximate kind has no timestamps: its records all escape)
        tbase0 = n0 ? pack_base32(tin, F) : pack_base(tin, F);
        tbase1 = fold_base(tin, G);
    }
    __syncthreads();   // the counts in `stage` are dead from here on
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int e = wb_elem<kPartBlock, kPartItems>(it);   // wave-blocked tile order
        if (e < nvalid) {
            const uint32_t d = (key[it] >> shift) & (kDigits - 1);
            stage[lpos[it]] = n0 ? (rec[it] & 0x0000FFFFFFFFFFFFull) : rec[it];
            if (LAST)
                stage_e[lpos[it]] = (uint16_t)e;
            else if (perm)   // (null: k_unrank recomputes the positions)
                ST_PERM(perm + base + e, goff[d] + lpos[it] - L.lstart[d]);
            if (FIRST && n0 && ((rec[it] >> 48) & 1u))   // escaped: its time beside its position
                ts0[goff[d] + lpos[it] - L.lstart[d]] = tv_keep[FIRST ? it : 0];
        }
    }
    __syncthreads();
    uint32_t gpos[kPartItems];
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int j = it * kPartBlock + tid;
        if (j < nvalid) {
            const uint64_t s = stage[j];
            const uint32_t d = n0 ? (uint32_t)(s >> 32) & (kDigits - 1)
                                  : ((uint32_t)(s & F.kmask) >> shift) & (kDigits - 1);
            gpos[it] = goff[d] + (uint32_t)j - L.lstart[d];
            // runs merge in L2: keep cached
            if (n0 && !LAST)
                reinterpret_cast<uint32_t *>(rout)[gpos[it]] = (uint32_t)s;
            else if (n0)
                rout[gpos[it]] = fold_rec32((uint32_t)s, (uint32_t)(base + stage_e[j]), tbase0, tbase1, F, G);
            else
                rout[gpos[it]] = LAST ? fold_rec(s, (uint32_t)(base + stage_e[j]), tbase0, tbase1, F, G) : s;
            // the next pass's digit, one byte beside the record (k_hist_dig reads these)
            if (!LAST && dig_next)
                dig_next[gpos[it]] = n0 ? (uint8_t)(s >> 40)
                                        : (uint8_t)(((uint32_t)(s & F.kmask) >> (shift + kDigitBits)) & (kDigits - 1));
        }
    }
    if (IDX) {
        uint32_t *stage32 = reinterpret_cast<uint32_t *>(stage);
        uint32_t iv[kPartItems];
#pragma unroll
        for (int it = 0; it < kPartItems; ++it) {
            const int e = wb_elem<kPartBlock, kPartItems>(it);   // wave-blocked tile order
            iv[it] = (e < nvalid) ? (FIRST ? (uint32_t)(base + e) : iin[base + e]) : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < kPartItems; ++it) {
            const int e = wb_elem<kPartBlock, kPartItems>(it);   // wave-blocked tile order
            if (e < nvalid) stage32[lpos[it]] = iv[it];
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < kPartItems; ++it) {
            const int j = it * kPartBlock + tid;
            if (j < nvalid) iout[gpos[it]] = stage32[j];
        }
    }
    if (FIRST && __any(bad) && (tid & 63) == 0) atomicOr(err, 1u);
}

// Decide every request of one bucket (see file header).  res[q] is the packed reply of
// sorted request q (bit 31 granted, bits 0-30 remaining).
//
// The bucket's R table rows live in LDS as stored ({v, t_us}, 16 B) plus the row's
// field t as f64 (ft, TB:203 applied to t_us), derived once when a request first
// touches the row and replaced by the request's own new_t on a grant.  A dense bucket
// (>= R/8 requests) pulls its whole 16*R-byte slice with coalesced loads, issued
// together with its first chunk of requests, and writes it back whole; a sparse one
// pulls and writes back only the rows it touches.  Requests go in chunks of 2048
// (arrival order): each computes its state-independent times in parallel, then
// speculative rounds (below) decide them.  Replies stay in registers and leave as one
// coalesced store per chunk.
constexpr int kFoldBlock = 512;
constexpr int kFoldPer = 4;                                 // requests per thread per chunk
constexpr int kFoldChunk = kFoldBlock * kFoldPer;           // 2048
constexpr int kMaxRows = 1 << kMaxRBits;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void slot_store_nt(Slot *p, const Slot &s) {
    u32x4 v;
    __builtin_memcpy(&v, &s, sizeof v);
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
}

// 16 bytes per lane from global memory straight into LDS (global_load_lds_dwordx4, nt):
// the LDS destination is the wave-uniform `lds_wave` + 16 * lane.  A barrier alone does
// NOT wait for it: every issuing wave runs lds_dma_wait() before the __syncthreads() that
// publishes the slice to the workgroup.
typedef __attribute__((address_space(1))) const void gvoid_t;
typedef __attribute__((address_space(3))) void lvoid_t;
__device__ __forceinline__ void lds_dma16(const void *src, void *lds_wave) {
    __builtin_amdgcn_global_load_lds((gvoid_t *)src, (lvoid_t *)lds_wave, 16, 0, 2);
}
// LDS-DMA loads count against vmcnt, not lgkmcnt: a workgroup barrier's release fence
// alone need not wait for them, so every barrier that publishes a DMA'd slice is
// preceded by this explicit wait for this wave's outstanding vector-memory loads.
__device__ __forceinline__ void lds_dma_wait() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// A token-bucket reply is {granted, trunc(new_v)} with 0 <= trunc(new_v) <= TokenLimit.
// When TokenLimit <= 127 it travels as one byte (bit 7 granted, bits 0-6 remaining)
// through the fold and the un-partition passes instead of four.
__device__ __forceinline__ void put_reply(uint32_t *res, uint32_t q, uint32_t rep, uint32_t narrow) {
    if (narrow)
        reinterpret_cast<uint8_t *>(res)[q] = (uint8_t)(((rep >> 24) & 0x80u) | (rep & 0x7Fu));
    else
        res[q] = rep;
}

// Write-back filter of a dense slice: a deny writes nothing (TB:225-236), so only the
// 128-byte lines holding a modified row go back to HBM, each whole (8 rows of 16 B;
// `dirty` has one bit per row, and a bucket's first row starts a line).  A sparse slice
// writes its modified rows one by one (the rows beside them were never loaded).
__device__ __forceinline__ bool row_line_dirty(const uint32_t *dirty, uint32_t j) {
    return ((dirty[j >> 5] >> (j & 24u)) & 0xFFu) != 0;
}
__device__ __forceinline__ bool row_dirty(const uint32_t *dirty, uint32_t j) {
    return (dirty[j >> 5] >> (j & 31u)) & 1u;
}

// Shape of k_fold_wide (profiles/r02_ablate_wide*.log): 512 threads x 2 requests per
// chunk, the rows' field t derived per evaluation instead of cached, a 256-entry pending
// list: 49.9 KB of LDS and 80 VGPRs, so three workgroups (24 waves) share a CU.  The
// fold is latency-bound; against two workgroups of 4 requests per thread with a cached
// field t (74.5 KB, 128 VGPRs) it takes 1.05 instead of 1.20 ms per config-B batch
// (0.92 instead of 1.09 in the denial-dominated steady state).
#ifndef TBE_WIDE_BLOCK
#define TBE_WIDE_BLOCK 512
#endif
#ifndef TBE_WIDE_PER
#define TBE_WIDE_PER 3
#endif
#ifndef TBE_WIDE_WAVES
#define TBE_WIDE_WAVES 6                     // minimum waves per SIMD (register budget)
#endif
#ifndef TBE_WIDE_TAIL
#define TBE_WIDE_TAIL 512
#endif
constexpr int kWideBlock = TBE_WIDE_BLOCK;
constexpr int kWidePer = TBE_WIDE_PER;
constexpr int kWideChunk = kWideBlock * kWidePer;
constexpr int kWideTail = TBE_WIDE_TAIL;
#ifndef TBE_WIDE_SOLO
#define TBE_WIDE_SOLO 1                      // the last rounds in wave 0 alone (0: whole workgroup, A/B)
#endif
constexpr uint32_t kWideSolo = TBE_WIDE_SOLO ? 64u : 0u;   // pending requests the solo wave takes
#ifndef TBE_FOLD_PREFETCH
#define TBE_FOLD_PREFETCH 384                // blocks ahead whose slice k_fold_wide touches (0: off)
#endif
#ifndef TBE_QFOLD_PREFETCH
#define TBE_QFOLD_PREFETCH 0                 // A/B: the same for k_fold_q
#endif
#ifndef TBE_AFOLD_PREFETCH
#define TBE_AFOLD_PREFETCH 0                 // A/B: the same for k_fold_a
#endif
#ifndef TBE_FOLD_PREFETCH_MIN
#define TBE_FOLD_PREFETCH_MIN 1024           // ... by workgroups whose bucket has this many requests
#endif
#ifndef TBE_WIDE_MIN_SHIFT
#define TBE_WIDE_MIN_SHIFT 11
#endif
// Which buckets k_fold_wide takes is decided per launch (wide_min, fold_wide_min below):
// the buckets of at least `wide_min` requests.  k_fold_wide pulls its whole 16*R-byte
// slice by LDS-DMA, k_fold_sparse only the rows a bucket touches.
//  - Dense batches (at least R/32 requests per bucket on average: configs B and C):
//    every nonempty bucket (wide_min = R >> kWideMinShift = 1 at R = 2048).  On a Zipf
//    slice, whose buckets hold fewer requests once the hot keys run apart, the wide fold's
//    24 waves per CU beat the workgroup-per-bucket gather fold's 12 (round 2, R/32: config
//    C fold 0.89 -> 0.69 ms; R/2 .. R/2048 measured, profiles/r02_ablate_wide_threshold*.log);
//    round 3 gave it every bucket (profiles/r03_ablate_hot_wide_walk.log), and round 5
//    removed that gather fold (k_fold_sparse took its sparse buckets).
//  - Sparse batches (fewer than R/8 requests per bucket on average, e.g. 2^20 requests over
//    1e8 keys, ~21 per bucket): k_fold_wide only for the buckets of at least R/8 requests
//    (the list k_bscan_lb builds); the others go one wave each to k_fold_sparse, which
//    gathers just their rows instead of the whole slice (a dense-only fold
//    reads the whole 1.6 GB table for a batch that touches 16 MB of it).
constexpr int kWideMinShift = TBE_WIDE_MIN_SHIFT;
// (A tail walk -- the requests still pending after round 1 counting-sorted by row, each
// row's run decided by one thread -- was slower here: config B fold 0.77 -> 0.88 ms,
// profiles/r03_ablate_hot_wide_walk.log; removed in round 5.)
static_assert(kWideChunk <= 4096 && kWideTail <= kWideBlock, "election tags and tail list");
// The rows' field t (TB:203 of the stored t_us), derived per evaluation (a copy cached in
// LDS cost occupancy and was slower, profiles/r02_ablate_wide*.log)
#define WIDE_FT_GET(j, srow) req_time_rel((srow).t_us == kAbsent ? 0 : (srow).t_us, TB, 0).new_t
#define WIDE_FT_SET(j, v) ((void)0)

// Buckets of >= wide_min requests (every nonempty bucket of a dense batch), shaped as above
// (three workgroups per CU, chunks of 1536 requests).  k_fold_sparse takes the other buckets.
template <bool PACKED>
__global__ __launch_bounds__(kWideBlock, TBE_WIDE_WAVES) void k_fold_wide(
    const uint32_t *__restrict__ skeys, const int32_t *__restrict__ sperm,
    const int64_t *__restrict__ sts, const uint64_t *__restrict__ srec,
    const int64_t *__restrict__ ts_orig, PackFmt F, const uint32_t *__restrict__ bstart,
    int r_bits, uint64_t n_keys, Slot *__restrict__ table, TbParams P,
    uint32_t *__restrict__ res, const uint32_t *__restrict__ err, HotSet *__restrict__ hot_next,
    uint32_t narrow, uint32_t wide_min, FoldFmt G, const uint64_t *__restrict__ rec0,
    const uint32_t *__restrict__ dlist = nullptr) {
    __shared__ Slot row[kMaxRows];
    // aux: requests per row in buckets that may hold a hot key (hcnt), otherwise the
    // compact list of requests still pending after round 1 (t_*)
    // A pending entry is 16 bytes (row | local id << 16, permits, timestamp); its request
    // times are recomputed per round rather than stored, so 512 entries fit in 8 KB.
    __shared__ uint64_t aux[kWideTail * 2 + kWideTail / 2];
    __shared__ uint32_t wsum[kWideBlock / 64];
    uint32_t *hcnt = reinterpret_cast<uint32_t *>(aux);
    uint32_t *t_kl_lid = reinterpret_cast<uint32_t *>(aux);
    int32_t *t_pm = reinterpret_cast<int32_t *>(aux) + kWideTail;
    int64_t *t_ts = reinterpret_cast<int64_t *>(aux) + kWideTail;
    uint32_t *t_pos = reinterpret_cast<uint32_t *>(aux + kWideTail * 2);   // reply positions
    static_assert(kWideTail * 2 * 8 >= kMaxRows * 4, "hcnt fits in aux");
    __shared__ uint32_t own[kMaxRows];
    __shared__ uint32_t loaded[kMaxRows / 32];
    __shared__ uint32_t dirty[kMaxRows / 32];

    const int tid = threadIdx.x;
    // sparse batch: the dense buckets k_bscan listed (dlist); otherwise this block's bucket
    if (dlist && blockIdx.x >= dlist[0]) return;
    const uint32_t b = dlist ? dlist[1 + blockIdx.x] : fold_bucket(G);
    if (G.on && b >= G.nb) return;
    const uint32_t R = 1u << r_bits;
    const uint32_t rmask = R - 1;
    const uint64_t row0 = (uint64_t)b << r_bits;
    const uint32_t nrows = (uint32_t)min<uint64_t>(R, n_keys - row0);
    Slot *__restrict__ rows = table + row0;
    constexpr int kRowsPerThread = (kMaxRows + kWideBlock - 1) / kWideBlock;
    // The slice goes HBM -> LDS directly (LDS-DMA, streaming policy): no VGPRs held for it,
    // so none of the loop invariants spill at this peak.  Rows past nrows get a copy of the
    // last row; no request reaches them and they are never written.
    auto slice_dma = [&]() {
#pragma unroll
        for (int u = 0; u < kRowsPerThread; ++u) {
#if defined(TBE_FOLD_COPY_ONLY) && defined(TBE_COPY_ROWS)
            if (u * kWideBlock >= (TBE_COPY_ROWS)) break;   // A/B: a 3/4 slice
#endif
            const uint32_t j = tid + u * kWideBlock;
            lds_dma16(rows + (j < nrows ? j : nrows - 1), &row[u * kWideBlock + (tid & ~63)]);
        }
    };
    if (*err) return;
    const uint32_t s = bstart[b], e = bstart[b + 1];
    if (s == e) return;
    // Buckets with >= wide_min requests only (k_fold_sparse takes the others): the whole slice
    // is pulled in (LDS-DMA) and only its dirty lines are written back.
    if (e - s < wide_min) return;
    const bool dense = true;
    const int64_t tbase = PACKED ? pack_base(ts_orig, F) : 0;
    const int64_t tbase1 = G.on ? fold_base(ts_orig, G) : 0;
    const TimeBase TB = time_base(PACKED ? rel_base(ts_orig, F) : 0, P.ttl_ms);   // fast request times (req_time_rel)
    const bool count_hot = hot_next != nullptr && (e - s) >= kHotMin;

    uint32_t kl[kWidePer];
    int32_t pm[kWidePer];
    int64_t tsv[kWidePer];
    uint32_t pos[kWidePer];   // where each request's reply goes (FoldFmt), or its sorted position
    uint32_t pend = 0;
    auto load_chunk = [&](uint32_t c) {
        pend = 0;
#pragma unroll
        for (int r = 0; r < kWidePer; ++r) {
            const uint32_t q = c + r * kWideBlock + tid;
            kl[r] = 0;
            pm[r] = 0;
            tsv[r] = 0;
            pos[r] = q;
            if (q < e) {
                if (PACKED) {
                    fold_input(LD_F(srec + q), q, G, tbase1, rec0, ts_orig, tbase, F, rmask, kl[r], pm[r],
                               tsv[r], pos[r]);
                } else {
                    kl[r] = skeys[q] & rmask;
                    pm[r] = sperm[q];
                    tsv[r] = sts[q];
                }
                pend |= 1u << r;
            }
        }
    };

#if TBE_FOLD_PREFETCH
    uint32_t pf_sink = 0;
#endif
    load_chunk(s);   // in flight together with the dense slice
    if (dense) slice_dma();
    for (uint32_t j = tid; j < (R + 31) / 32; j += kWideBlock) {
        loaded[j] = 0;
        dirty[j] = 0;
    }
#ifdef TBE_FOLD_COPY_ONLY
    // A/B floor (not a decision path): the fold's memory traffic without its rounds --
    // records and slice in, the whole slice and one reply per request out
    __syncthreads();
    for (uint32_t c = s; c < e; c += kWideChunk) {
        if (c != s) load_chunk(c);
#pragma unroll
        for (int r = 0; r < kWidePer; ++r)
            if (pend & (1u << r)) put_reply(res, pos[r], kl[r] ^ (uint32_t)pm[r] ^ (uint32_t)tsv[r], narrow);
    }
#ifndef TBE_COPY_ROWS
#define TBE_COPY_ROWS kMaxRows   // A/B: rows per slice written back (3/4: the bytes of 12-byte rows)
#endif
    for (uint32_t j = tid; j < nrows && j < (uint32_t)(TBE_COPY_ROWS); j += kWideBlock) ST_S(rows + j, row[j]);
    return;
#endif

    for (uint32_t c = s; c < e; c += kWideChunk) {
        if (c != s) load_chunk(c);
        for (uint32_t j = tid; j < R; j += kWideBlock) own[j] = 0;
        if (count_hot && c == s)
            for (uint32_t j = tid; j < R; j += kWideBlock) hcnt[j] = 0;
        lds_dma_wait();    // (first chunk) this wave's slice DMA landed
        __syncthreads();   // own[] reset, bitmaps and (first chunk) dense slice visible
#if TBE_FOLD_PREFETCH
        // Touch one word per 128-B line of the slice and of the records of the workgroup
        // TBE_FOLD_PREFETCH blocks later (the same XCD), so that its loads find them in L2 or
        // the Infinity Cache; issued after this slice landed, and waited for only at the
        // barrier before this workgroup's write-back.  384 blocks = half of the 768
        // workgroups in flight: config B fold 0.93 -> 0.85 ms; 768 -> 0.90, 1536 -> 0.93
        // (profiles/r04d_ablate_perm0_prefetch.log)
        if (c == s && e - s >= TBE_FOLD_PREFETCH_MIN) {
            const uint32_t fblk = blockIdx.x + TBE_FOLD_PREFETCH;
            const uint32_t fb = fold_bucket_at(G, fblk);
            if (fblk < gridDim.x && (!G.on || fb < G.nb)) {
                const uint32_t fs = bstart[fb], fe = bstart[fb + 1];
                if (fe - fs >= wide_min && fe > fs) {
                    if (tid < (int)(kMaxRows / 8)) {
                        const uint64_t fr = ((uint64_t)fb << r_bits) + (uint64_t)tid * 8u;
                        if (fr < n_keys) pf_sink = reinterpret_cast<const uint32_t *>(table + fr)[0];
                    } else if (PACKED) {
                        const uint32_t q = fs + (uint32_t)(tid - kMaxRows / 8) * 16u;
                        if (q < fe) pf_sink = (uint32_t)srec[q];
                    }
                }
            }
        }
#endif
        if (count_hot) {
#pragma unroll
            for (int r = 0; r < kWidePer; ++r)
                if (pend & (1u << r)) atomicAdd(&hcnt[kl[r]], 1u);
        }
        uint32_t rep[kWidePer];
#pragma unroll
        for (int r = 0; r < kWidePer; ++r) rep[r] = 0;
        // Speculative rounds.  Every pending request evaluates the script
        // against its key's current row.  An evaluation that does not modify the row (a
        // deny without expiry) leaves it as it found it, so the key's pending requests up
        // to its earliest modifying one are decided by this round's evaluations; that
        // earliest one commits the row it computed and later ones wait for the next
        // round.  A key whose requests in the chunk all deny settles in one round.
        // Election slot: (round << 12) | (4095 - local id); the max is the key's earliest
        // modifier of the newest round, so no reset between rounds.  Workgroup-uniform
        // loops: every thread runs every round and the only exits are __syncthreads_or.
        auto eval_slots = [&](uint32_t round, Slot (&nrow)[kWidePer]) {
#pragma unroll
            for (int r = 0; r < kWidePer; ++r) {
                nrow[r] = Slot{0.0, 0};
                if (pend & (1u << r)) {
                    nrow[r] = row[kl[r]];
                    bool m;
                    // request times recomputed per evaluation (registers: three slots)
                    const ReqTime rqr = PACKED ? req_time_rel(tsv[r], TB, P.ttl_ms) : req_time(tsv[r], P.ttl_ms);
                    rep[r] = tb_step_ft(nrow[r], WIDE_FT_GET(kl[r], nrow[r]), pm[r], rqr, P, m);
                    if (m) atomicMax(&own[kl[r]], (round << 12) | (4095u - (uint32_t)(r * kWideBlock + tid)));
                }
            }
        };
        auto resolve_slots = [&](uint32_t round, const Slot (&nrow)[kWidePer]) {
#pragma unroll
            for (int r = 0; r < kWidePer; ++r) {
                if (!(pend & (1u << r))) continue;
                const uint32_t tag = (round << 12) | (4095u - (uint32_t)(r * kWideBlock + tid));
                const uint32_t o = own[kl[r]];
                if ((o >> 12) != round || o < tag) {
                    pend &= ~(1u << r);             // before the key's first modifier: decided
                } else if (o == tag) {
                    row[kl[r]] = nrow[r];           // the row this round's evaluation produced
                    WIDE_FT_SET(kl[r], rq[r].new_t);        // its field t (unused while absent)
                    atomicOr(&dirty[kl[r] >> 5], 1u << (kl[r] & 31));
                    pend &= ~(1u << r);
                }
            }
        };
        {
            Slot nrow[kWidePer];
            eval_slots(1u, nrow);
            __syncthreads();
            resolve_slots(1u, nrow);
        }
        // Round 1 settles every key's first request.  The few left pending move to a
        // compact list (one per thread) so later rounds evaluate one request per thread
        // instead of every slot of every lane.
#ifdef TBE_FOLD_R1_ONLY
        pend = 0;   // A/B timing only (wrong replies): the cost of the rounds after round 1
#endif
        uint32_t n_tail;
        const uint32_t tail_at = block_excl_scan<kWideBlock>(__popc(pend), wsum, &n_tail);
        uint32_t keep = ~0u;                     // slots whose reply this thread stores
        if (n_tail != 0 && n_tail <= kWideTail && !count_hot) {
            uint32_t at = tail_at;
#pragma unroll
            for (int r = 0; r < kWidePer; ++r) {
                if (pend & (1u << r)) {
                    t_kl_lid[at] = kl[r] | ((uint32_t)(r * kWideBlock + tid) << 16);
                    t_pm[at] = pm[r];
                    t_ts[at] = tsv[r];
                    t_pos[at] = pos[r];
                    ++at;
                }
            }
            keep = ~pend;
            pend = 0;
            __syncthreads();
            bool tp = (uint32_t)tid < n_tail;
            uint32_t tkl = 0, tlid = 0, trep = 0, tpos = 0;
            int32_t tpm = 0;
            int64_t tts = 0;
            ReqTime trq{0.0, 0, 0};
            auto take = [&](uint32_t at) {
                tkl = t_kl_lid[at] & 0xFFFFu;
                tlid = t_kl_lid[at] >> 16;
                tpm = t_pm[at];
                tts = t_ts[at];
                tpos = t_pos[at];
                trq = PACKED ? req_time_rel(tts, TB, P.ttl_ms) : req_time(tts, P.ttl_ms);
            };
            if (tp) take(tid);
            // Each round settles at least the first pending request of every row; when the
            // survivors fit in fewer waves they are packed to the front of the list, so
            // later rounds run on fewer waves (the fold is VALU-issue bound).
            uint32_t in_use = n_tail;
            uint32_t round = 2;
            while (in_use > kWideSolo) {   // block-uniform
                const uint32_t tag = (round << 12) | (4095u - tlid);
                Slot nr = Slot{0.0, 0};
                if (tp) {
                    nr = row[tkl];
                    bool m;
                    trep = tb_step_ft(nr, WIDE_FT_GET(tkl, nr), tpm, trq, P, m);
                    if (m) atomicMax(&own[tkl], tag);
                }
                __syncthreads();
                if (tp) {
                    const uint32_t o = own[tkl];
                    if ((o >> 12) != round || o < tag) {
                        tp = false;
                    } else if (o == tag) {
                        row[tkl] = nr;
                        WIDE_FT_SET(tkl, trq.new_t);
                        atomicOr(&dirty[tkl >> 5], 1u << (tkl & 31));
                        tp = false;
                    }
                    if (!tp) put_reply(res, tpos, trep, narrow);
                }
                ++round;
                const uint64_t bal = __ballot(tp);
                if ((tid & 63) == 0) wsum[tid >> 6] = (uint32_t)__popcll(bal);
                __syncthreads();
                uint32_t off = 0, left = 0;
#pragma unroll
                for (int w = 0; w < kWideBlock / 64; ++w) {
                    const uint32_t cw = wsum[w];
                    off += (w < (tid >> 6)) ? cw : 0u;
                    left += cw;
                }
                if (left == 0) {
                    in_use = 0;
                    break;
                }
                if ((left + 63) / 64 < (in_use + 63) / 64) {
                    if (tp) {
                        const uint32_t at = off + (uint32_t)__popcll(bal & lanemask_lt());
                        t_kl_lid[at] = tkl | (tlid << 16);
                        t_pm[at] = tpm;
                        t_ts[at] = tts;
                        t_pos[at] = tpos;
                    }
                    __syncthreads();
                    tp = (uint32_t)tid < left;
                    if (tp) take(tid);
                    in_use = left;
                }
            }
#if TBE_WIDE_SOLO
            // The last rounds hold at most one wave of pending requests, all in wave 0 (list
            // positions < 64): that wave finishes them alone, ordered by its own LDS accesses
            // (a wave's LDS operations complete in issue order) instead of two workgroup
            // barriers per round that every wave would run.  The others wait at the barrier
            // below.
            if (in_use != 0) {   // block-uniform
                if (tid < 64) {
                    for (;; ++round) {
                        const uint32_t tag = (round << 12) | (4095u - tlid);
                        Slot nr = Slot{0.0, 0};
                        if (tp) {
                            nr = row[tkl];
                            bool m;
                            trep = tb_step_ft(nr, WIDE_FT_GET(tkl, nr), tpm, trq, P, m);
                            if (m) atomicMax(&own[tkl], tag);
                        }
                        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        if (tp) {
                            const uint32_t o = own[tkl];
                            if ((o >> 12) != round || o < tag) {
                                tp = false;
                            } else if (o == tag) {
                                row[tkl] = nr;
                                WIDE_FT_SET(tkl, trq.new_t);
                                atomicOr(&dirty[tkl >> 5], 1u << (tkl & 31));
                                tp = false;
                            }
                            if (!tp) put_reply(res, tpos, trep, narrow);
                        }
                        if (!__any(tp)) break;
                        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                    }
                }
                __syncthreads();   // rows and own[] settled before the next chunk or the write-back
            }
#endif
        } else if (n_tail != 0) {
            // More pending requests than the list holds, or its space holds hcnt: the slots
            // settle one window of local ids at a time (slot r = ids [r*B, r*B+B)).  A key's
            // pending requests in slot r follow all of its requests in earlier slots, which
            // have settled, so each window is a valid order on its own; a round holds one
            // evaluated row per thread instead of kWidePer (no spilled registers).  The round
            // number keeps growing across windows, so own[] needs no reset.
            uint32_t round = 2;
#pragma unroll
            for (int r = 0; r < kWidePer; ++r) {
                const uint32_t bit = 1u << r;
                const uint32_t tag_lo = 4095u - (uint32_t)(r * kWideBlock + tid);
                if (!__syncthreads_or(pend & bit)) continue;
                for (;; ++round) {
                    const uint32_t tag = (round << 12) | tag_lo;
                    Slot nr = Slot{0.0, 0};
                    if (pend & bit) {
                        nr = row[kl[r]];
                        bool m;
                        const ReqTime rqr = PACKED ? req_time_rel(tsv[r], TB, P.ttl_ms) : req_time(tsv[r], P.ttl_ms);
                        rep[r] = tb_step_ft(nr, WIDE_FT_GET(kl[r], nr), pm[r], rqr, P, m);
                        if (m) atomicMax(&own[kl[r]], tag);
                    }
                    __syncthreads();
                    if (pend & bit) {
                        const uint32_t o = own[kl[r]];
                        if ((o >> 12) != round || o < tag) {
                            pend &= ~bit;
                        } else if (o == tag) {
                            row[kl[r]] = nr;
                            WIDE_FT_SET(kl[r], rq[r].new_t);
                            atomicOr(&dirty[kl[r] >> 5], 1u << (kl[r] & 31));
                            pend &= ~bit;
                        }
                    }
                    if (!__syncthreads_or(pend & bit)) {
                        ++round;
                        break;
                    }
                }
            }
        }
#pragma unroll
        for (int r = 0; r < kWidePer; ++r) {
            const uint32_t q = c + r * kWideBlock + tid;
            if (q < e && (keep & (1u << r))) put_reply(res, pos[r], rep[r], narrow);
        }
    }
    __syncthreads();
    // dirty lines stream out (non-temporal: 12% faster fold, profiles/r01_v10_ablate.log)
    for (uint32_t j = tid; j < nrows; j += kWideBlock)
        if (row_line_dirty(dirty, j)) ST_S(rows + j, row[j]);
    if (count_hot) {
        // nominate this bucket's hot keys for their own runs in the next batch
        for (uint32_t j = tid; j < nrows; j += kWideBlock) {
            if (hcnt[j] >= kHotMin) {
                const uint32_t at = atomicAdd(&hot_next->n_cand, 1u);
                if (at < kHotCandMax) hot_next->cand[at] = ((uint64_t)hcnt[j] << 32) | (uint32_t)(row0 + j);
            }
        }
    }
#if TBE_FOLD_PREFETCH
    if (wide_min == 0xFFFFFFFFu) res[s] = pf_sink;   // never (this kernel returned above): keeps the touches
#endif
}

constexpr int64_t kRowWindow = (int64_t)1 << 31;          // k_drain's time base: rows up to ~35 min older

// Field t of a stored row (TB:203 applied to t_us; only used while the key is present).
__device__ __forceinline__ double field_t(int64_t t_us, const TimeBase &B) {
    return req_time_rel(t_us == kAbsent ? 0 : t_us, B, 0).new_t;
}

// Sparse buckets of a sparse batch (fewer than wide_min requests; 2^20 requests over 1e8
// keys put ~21 in each of 48,829 buckets): ONE WAVE per bucket, no LDS.  A workgroup per
// bucket (k_fold) spent its time on dispatch and on the serial latency of its few loads --
// 48,829 workgroups at 3 per CU, 0.38 ms for a 2^20 batch -- while a wave needs nothing a
// workgroup has: its <= 64 requests of a chunk are one per lane, the lanes of one key are
// found by ballot-matching the 11 row bits, and the key's first lane (the earliest: a
// bucket's requests are in arrival order) walks the key's requests in lane order, which
// is the reference's serial order (TB:202-238 per request).  Waves stride over the
// buckets, and each wave fetches the bounds of all its buckets with one load per lane.
// A bucket of more than 64 requests goes in chunks of 64; a key's row written back by one
// chunk is re-read by the next after a workgroup-scope fence.
constexpr int kSpBlock = 256;
constexpr int kSpWaves = kSpBlock / 64;
template <bool PACKED>
__global__ __launch_bounds__(kSpBlock) void k_fold_sparse(
    const uint32_t *__restrict__ skeys, const int32_t *__restrict__ sperm,
    const int64_t *__restrict__ sts, const uint64_t *__restrict__ srec,
    const int64_t *__restrict__ ts_orig, PackFmt F, const uint32_t *__restrict__ bstart,
    int r_bits, uint64_t n_keys, Slot *__restrict__ table, TbParams P,
    uint32_t *__restrict__ res, const uint32_t *__restrict__ err, uint32_t narrow, uint32_t wide_min,
    FoldFmt G, const uint64_t *__restrict__ rec0, uint32_t n_walk) {
    if (*err) return;
    const int lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * kSpWaves + (threadIdx.x >> 6);
    const uint32_t nwaves = gridDim.x * kSpWaves;
    const uint32_t rmask = (1u << r_bits) - 1u;
    const int64_t tbase = PACKED ? pack_base(ts_orig, F) : 0;
    const int64_t tbase1 = G.on ? fold_base(ts_orig, G) : 0;
    const TimeBase TB = time_base(PACKED ? rel_base(ts_orig, F) : -1, P.ttl_ms);
    const uint64_t lt = lanemask_lt();
    for (uint32_t bb0 = wave; bb0 < n_walk; bb0 += nwaves * 64u) {
        // the bounds of this wave's next 64 buckets: lane j holds bucket bb0 + j * nwaves
        const uint32_t my_bb = bb0 + (uint32_t)lane * nwaves;
        uint32_t my_b = 0xFFFFFFFFu, my_s = 0, my_e = 0;
        if (my_bb < n_walk) {
            my_b = fold_bucket_at(G, my_bb);
            if (!G.on || my_b < G.nb) {
                my_s = bstart[my_b];
                my_e = bstart[my_b + 1];
            }
        }
        uint64_t work = __ballot(my_e > my_s && my_e - my_s < wide_min);
        while (work) {
            const int j = __ffsll((long long)work) - 1;
            work &= work - 1;
            const uint32_t b = __shfl(my_b, j, 64);
            const uint32_t s = __shfl(my_s, j, 64), e = __shfl(my_e, j, 64);
            Slot *__restrict__ rows = table + ((uint64_t)b << r_bits);
            for (uint32_t c = s; c < e; c += 64) {
                // the previous chunk's row stores are visible to this wave's loads below: a
                // workgroup-scope fence (the stores complete; the CU's L1 is write-through).
                // An agent-scope one would also write back this XCD's L2 per chunk: a 2^22
                // batch (two chunks per bucket) took 2.4 ms in this kernel that way.
                if (c != s) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                const uint32_t q = c + (uint32_t)lane;
                const bool v = q < e;
                uint32_t kl = 0, pos = q;
                int32_t pm = 0;
                int64_t tsv = 0;
                if (v) {
                    if (PACKED) {
                        fold_input(LD_F(srec + q), q, G, tbase1, rec0, ts_orig, tbase, F, rmask, kl, pm, tsv, pos);
                    } else {
                        kl = skeys[q] & rmask;
                        pm = sperm[q];
                        tsv = sts[q];
                    }
                }
                // lanes of the same key (row): ballot-match the row bits
                uint64_t peers = __ballot(v);
                for (int bit = 0; bit < r_bits; ++bit) {
                    const bool x = (kl >> bit) & 1u;
                    const uint64_t m = __ballot(x);
                    peers &= x ? m : ~m;
                }
                const bool leader = v && (peers & lt) == 0;   // the key's earliest request here
                Slot st = Slot{0.0, 0};
                if (leader) st = rows[kl];
                uint64_t todo = leader ? peers : 0ull;
                bool mod = false;
                while (__any(todo != 0ull)) {
                    const int m = todo ? __ffsll((long long)todo) - 1 : lane;
                    const int32_t pm_m = __shfl(pm, m, 64);
                    const int64_t ts_m = __shfl(tsv, m, 64);
                    const uint32_t pos_m = __shfl(pos, m, 64);
                    if (todo) {
                        const ReqTime rq = PACKED ? req_time_rel(ts_m, TB, P.ttl_ms) : req_time(ts_m, P.ttl_ms);
                        bool md;
                        const uint32_t rep = tb_step_ft(st, field_t(st.t_us, TB), pm_m, rq, P, md);
                        mod |= md;
                        put_reply(res, pos_m, rep, narrow);
                        todo &= todo - 1;
                    }
                }
                if (leader && mod) rows[kl] = st;
            }
        }
    }
}

// Inverse of one k_scatter pass: out[i] = in[perm[i]] with perm the positions that pass
// wrote (runs of ~32 consecutive positions per digit and tile, so the gather coalesces).
// FINAL: unpack into granted/status (u8) and remaining (i32) in arrival order.
// WAIT: queueing-kind reply packing (see pack_wait).
constexpr uint32_t kRemNone = 0x3FFFFFFFu;
__device__ __forceinline__ uint32_t pack_wait(uint32_t status, bool evaluated, uint32_t rem) {
    return (status << 30) | (evaluated ? (rem & kRemNone) : kRemNone);
}
// Queueing kind with TokenLimit <= 62: one byte, status in bits 6-7 and remaining in bits
// 0-5 (63 = no script call), through the fold and the un-partition passes.
constexpr uint32_t kRemNone8 = 63u;
// Queueing and approximate kinds with TokenLimit <= 16382 (remaining / AvailableTokens
// never exceeds TokenLimit): two bytes, status in bits 14-15 and the count in bits 0-13
// (16383 = no script call).
constexpr uint32_t kRemNone16 = 0x3FFFu;
// rw: reply width code of the wait kinds -- 1 one byte, 2 two bytes, otherwise four.
__device__ __forceinline__ void put_wait(uint32_t *res, uint32_t q, uint32_t status, bool evaluated, uint32_t rem,
                                         uint32_t rw) {
    if (rw == 1)
        reinterpret_cast<uint8_t *>(res)[q] = (uint8_t)((status << 6) | (evaluated ? (rem & 63u) : kRemNone8));
    else if (rw == 2)
        reinterpret_cast<uint16_t *>(res)[q] =
            (uint16_t)((status << 14) | (evaluated ? (rem & kRemNone16) : kRemNone16));
    else
        res[q] = pack_wait(status, evaluated, rem);
}
// A four-byte wait reply (pack_wait) in the two-byte form.
__device__ __forceinline__ uint16_t wait16(uint32_t v) {
    const uint32_t rem = v & kRemNone;
    return (uint16_t)(((v >> 30) << 14) | (rem == kRemNone ? kRemNone16 : (rem & kRemNone16)));
}

template <bool FINAL, bool WAIT, int W = 4>
__global__ __launch_bounds__(kUnBlock) void k_unscatter(uint64_t n, const uint32_t *__restrict__ perm,
                                                          const uint32_t *__restrict__ res_in,
                                                          uint32_t *__restrict__ res_out,
                                                          uint8_t *__restrict__ granted,
                                                          int32_t *__restrict__ remaining,
                                                          const uint32_t *__restrict__ err = nullptr,
                                                          uint32_t *__restrict__ sticky = nullptr) {
    // One workgroup per 8192 positions, XCD-aware like k_scatter: the tile's gathers land
    // in the digit runs of the partition tiles it covers, which stay in this XCD's L2.
    const int tid = threadIdx.x;
    // the batch's last kernel carries k_sticky's work (every kernel that sets err ran before)
    if (sticky && blockIdx.x == 0 && tid == 0 && *err) *sticky = 1u;
    const uint32_t tile = xcd_swizzle(blockIdx.x, gridDim.x);
    const uint64_t base = (uint64_t)tile * kUnTile;
    const int nvalid = (int)min<uint64_t>(kUnTile, n - base);
    uint32_t pv[kUnItems], r[kUnItems];
#pragma unroll
    for (int it = 0; it < kUnItems; ++it) {
        const int e = it * kUnBlock + tid;
        pv[it] = (e < nvalid) ? LD_U(perm + base + e) : 0u;
    }
#pragma unroll
    for (int it = 0; it < kUnItems; ++it) {
        const int e = it * kUnBlock + tid;
        r[it] = (e < nvalid) ? (W == 1 ? (uint32_t)reinterpret_cast<const uint8_t *>(res_in)[pv[it]]
                                : W == 2 ? (uint32_t)reinterpret_cast<const uint16_t *>(res_in)[pv[it]]
                                         : res_in[pv[it]])
                             : 0u;
    }
#pragma unroll
    for (int it = 0; it < kUnItems; ++it) {
        const int e = it * kUnBlock + tid;
        if (e >= nvalid) continue;
        const uint64_t i = base + e;
        if (FINAL && WAIT && W == 1) {
            ST_U(granted + i, (uint8_t)(r[it] >> 6));
            const uint32_t rem = r[it] & 63u;
            ST_U(remaining + i, (rem == kRemNone8) ? -1 : (int32_t)rem);
        } else if (FINAL && WAIT && W == 2) {
            ST_U(granted + i, (uint8_t)(r[it] >> 14));
            const uint32_t rem = r[it] & kRemNone16;
            ST_U(remaining + i, (rem == kRemNone16) ? -1 : (int32_t)rem);
        } else if (FINAL && WAIT) {
            ST_U(granted + i, (uint8_t)(r[it] >> 30));
            const uint32_t rem = r[it] & kRemNone;
            ST_U(remaining + i, (rem == kRemNone) ? -1 : (int32_t)rem);
        } else if (FINAL && W == 1) {
            ST_U(granted + i, (uint8_t)(r[it] >> 7));
            ST_U(remaining + i, (int32_t)(r[it] & 0x7Fu));
        } else if (FINAL) {
            ST_U(granted + i, (uint8_t)(r[it] >> 31));
            ST_U(remaining + i, (int32_t)(r[it] & 0x7FFFFFFFu));
        } else if (W == 1) {
            ST_U(reinterpret_cast<uint8_t *>(res_out) + i, (uint8_t)r[it]);
        } else if (W == 2) {
            ST_U(reinterpret_cast<uint16_t *>(res_out) + i, (uint16_t)r[it]);
        } else {
            ST_U(res_out + i, r[it]);
        }
    }
}

// Final un-partition of the token-bucket kind without a stored permutation.  Pass 0 put
// request i of tile t at goff_t[d] + (its stable rank among the tile's digit-d requests),
// d = its pass-0 digit.  That position is recomputed here per partition tile -- the same
// tile, the same wave-blocked ranking (rank_tile_wb) of the same digits, which k_hist's
// first pass stored as one byte per request, and the same tile offsets -- so pass 0 writes
// no 4-byte permutation and this pass reads one byte per request instead of four:
// granted[i], remaining[i] = reply at that position.  W: reply width (1 or 4 bytes).
template <int W, bool WAIT = false>
__global__ __launch_bounds__(kPartBlock) void k_unrank(uint64_t n, const uint8_t *__restrict__ digit,
                                                       const uint32_t *__restrict__ tileprefix,
                                                       const uint32_t *__restrict__ blockprefix,
                                                       const uint32_t *__restrict__ digit_total,
                                                       uint32_t tiles_per_blk, const uint32_t *__restrict__ res_in,
                                                       uint8_t *__restrict__ granted,
                                                       int32_t *__restrict__ remaining) {
    __shared__ RankLds<kPartBlock> L;
    __shared__ uint32_t goff[kDigits];
    __shared__ uint32_t wcnt[(kPartBlock / 64) * kDigits];
    const uint32_t tile = xcd_swizzle(blockIdx.x, gridDim.x);
    const uint64_t base = (uint64_t)tile * kTile;
    const int nvalid = (int)min<uint64_t>(kTile, n - base);
    uint32_t dg[kPartItems], lpos[kPartItems];
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int e = wb_elem<kPartBlock, kPartItems>(it);
        dg[it] = e < nvalid ? (uint32_t)LD_U(digit + base + e) : 0u;
    }
    tile_offsets<kPartBlock>(tile, tiles_per_blk, tileprefix, blockprefix, digit_total, goff, L.wsum);
    rank_tile_wb<kPartBlock, kPartItems>(dg, 0, nvalid, L, wcnt, lpos);
    uint32_t r[kPartItems];
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int e = wb_elem<kPartBlock, kPartItems>(it);
        const uint32_t q = goff[dg[it]] + lpos[it] - L.lstart[dg[it]];
        r[it] = e < nvalid ? (W == 1   ? (uint32_t)reinterpret_cast<const uint8_t *>(res_in)[q]
                              : W == 2 ? (uint32_t)reinterpret_cast<const uint16_t *>(res_in)[q]
                                       : res_in[q])
                           : 0u;
    }
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int e = wb_elem<kPartBlock, kPartItems>(it);
        if (e >= nvalid) continue;
        const uint64_t i = base + e;
        if (WAIT && W == 1) {            // status, remaining (put_wait forms)
            ST_U(granted + i, (uint8_t)(r[it] >> 6));
            const uint32_t rem = r[it] & 63u;
            ST_U(remaining + i, (rem == kRemNone8) ? -1 : (int32_t)rem);
        } else if (WAIT && W == 2) {
            ST_U(granted + i, (uint8_t)(r[it] >> 14));
            const uint32_t rem = r[it] & kRemNone16;
            ST_U(remaining + i, (rem == kRemNone16) ? -1 : (int32_t)rem);
        } else if (WAIT) {
            ST_U(granted + i, (uint8_t)(r[it] >> 30));
            const uint32_t rem = r[it] & kRemNone;
            ST_U(remaining + i, (rem == kRemNone) ? -1 : (int32_t)rem);
        } else if (W == 1) {             // granted, remaining (put_reply forms)
            ST_U(granted + i, (uint8_t)(r[it] >> 7));
            ST_U(remaining + i, (int32_t)(r[it] & 0x7Fu));
        } else {
            ST_U(granted + i, (uint8_t)(r[it] >> 31));
            ST_U(remaining + i, (int32_t)(r[it] & 0x7FFFFFFFu));
        }
    }
}

// ----------------------------------------------------------------------------- hot keys
// Skewed traffic (SURVEY.md §8d config C, §7 hard part iii).  A key that takes at least
// kHotMin requests of one batch becomes "hot" for the next batch: the first partition
// pass gives its requests a bucket of their own (id nb + h, past the nb ordinary
// buckets), so after the partition they form one run, in arrival order, instead of
// filling one ordinary bucket's serial rounds.  A run is cut into segments of kSeg
// requests:
//   k_hot_summary  (parallel)  per segment: the latest timestamp and the smallest permit
//                              code in it;
//   k_hot_chain    (one workgroup per run) walks the segments in order carrying the
//                  key's row S.  The script's decision is monotone in the request time
//                  and in the permits: x never decreases with a later TIME (TB:218-221),
//                  a request grants whenever a larger one does (TB:224), and passive
//                  expiry only starts at a later time.  So if a segment's extreme request
//                  (latest time, fewest permits) would leave S unmodified, every request
//                  of the segment does: the segment passes S through.  Segments that may
//                  modify S are decided here, serially, with the fold's speculative
//                  rounds;
//   k_hot_replies  (parallel)  decides every request of a pass-through segment against
//                              the S it saw.
// Which keys are hot only changes speed, never a decision.
constexpr int kSegBlock = kFoldBlock;
constexpr int kSegItems = 16;   // (8: no faster, 4: slower; profiles/r05u_ablate_hot_segments.log)
constexpr uint32_t kSeg = kSegBlock * kSegItems;  // 8192 requests per run segment

struct SegSummary {
    int64_t max_ts;
    int32_t min_p;
    uint32_t pad;
};
struct SegState {
    Slot s;          // the run's row when the segment starts
    double ft;       // its field t
    uint32_t pass;   // 0: k_hot_chain decided the segment; 1: no request of it modifies s and
                     // k_hot_replies decides it; 2: the same, already decided by k_hot_summary<true>
    uint32_t pad;
};


// segbase[h] = first segment of run h; segbase[kHotKeysMax] = all segments (the scan
// k_hot_summary's workgroups do, workgroup 0 publishing it).
// Run h of segment j: the last h with segbase[h] <= j.
__device__ __forceinline__ uint32_t seg_run(const uint32_t *segbase, uint32_t j) {
    uint32_t lo = 0, hi = kHotKeysMax;   // segbase[lo] <= j < segbase[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (segbase[mid] <= j) lo = mid;
        else hi = mid;
    }
    return lo;
}

// SPEC (the form launched): also decide the segment here when it passes the run's
// row as it stands before the batch (S0, table[key]) through -- the test k_hot_chain makes
// first, on the same summary -- so in the steady state, where a run's segments all pass
// (a hot key is mostly denied), k_hot_replies reads the run a second time only behind a
// segment that modified the row.
template <bool SPEC>
__global__ __launch_bounds__(kSegBlock) void k_hot_summary(
    const uint64_t *__restrict__ srec, const int64_t *__restrict__ ts_orig, PackFmt F,
    const uint32_t *__restrict__ bstart, uint32_t nb, uint32_t *segbase,
    SegSummary *__restrict__ summ, const uint32_t *__restrict__ err, FoldFmt G, const uint64_t *__restrict__ rec0,
    const HotSet *__restrict__ hot = nullptr, const Slot *__restrict__ table = nullptr, TbParams P = TbParams{},
    uint32_t *__restrict__ res = nullptr, uint32_t narrow = 0, uint32_t plan = 0) {
    __shared__ int64_t wts[kSegBlock / 64];
    __shared__ int32_t wp[kSegBlock / 64];
    __shared__ uint32_t pass_s0;
    __shared__ uint32_t sb[kHotKeysMax + 1];
    __shared__ uint32_t sbw[kSegBlock / 64];
    if (*err) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (plan) {
        // the runs' segment scan, done by every workgroup (1024 run lengths from the bucket
        // starts); workgroup 0 publishes segbase for k_hot_chain and k_hot_replies
        static_assert(kHotKeysMax == 2 * kSegBlock, "two runs per thread");
        const uint32_t cnt = hot->count;
        uint32_t ns[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const uint32_t h = 2 * tid + u;
            ns[u] = h < cnt ? (bstart[nb + h + 1] - bstart[nb + h] + kSeg - 1) / kSeg : 0u;
        }
        uint32_t all;
        const uint32_t pre = block_excl_scan<kSegBlock>(ns[0] + ns[1], sbw, &all);
        sb[2 * tid] = pre;
        sb[2 * tid + 1] = pre + ns[0];
        if (tid == 0) sb[kHotKeysMax] = all;
        __syncthreads();
        if (blockIdx.x == 0) {
            for (uint32_t j = tid; j <= kHotKeysMax; j += kSegBlock) segbase[j] = sb[j];
        }
        segbase = sb;
    }
    const uint32_t total = segbase[kHotKeysMax];
    const int64_t tbase = pack_base(ts_orig, F);
    const int64_t tbase1 = G.on ? fold_base(ts_orig, G) : 0;
    const TimeBase TB = time_base(rel_base(ts_orig, F), P.ttl_ms);
    for (uint32_t j = blockIdx.x; j < total; j += gridDim.x) {
        const uint32_t h = seg_run(segbase, j);
        const uint32_t a = bstart[nb + h] + (j - segbase[h]) * kSeg;
        const uint32_t b = min(a + kSeg, bstart[nb + h + 1]);
        int64_t mx = INT64_MIN;
        int32_t mn = INT32_MAX;
        // the run's row before the batch, in flight with the records (SPEC)
        const Slot s0 = SPEC ? table[hot->key[h]] : Slot{0.0, 0};
        uint64_t rv[kSegItems];   // every record of the segment in flight at once
#pragma unroll
        for (int it = 0; it < kSegItems; ++it) {
            const uint32_t q = a + it * kSegBlock + tid;
            rv[it] = q < b ? srec[q] : 0ull;
        }
#pragma unroll
        for (int it = 0; it < kSegItems; ++it) {
            const uint32_t q = a + it * kSegBlock + tid;
            if (q >= b) continue;
            uint32_t k, pos;
            int32_t p;
            int64_t ts;
            fold_input(rv[it], q, G, tbase1, rec0, ts_orig, tbase, F, 0u, k, p, ts, pos);
            mx = max(mx, ts);
            mn = min(mn, p);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            mx = max(mx, (int64_t)__shfl_xor((long long)mx, o, 64));
            mn = min(mn, __shfl_xor(mn, o, 64));
        }
        if (lane == 0) {
            wts[w] = mx;
            wp[w] = mn;
        }
        __syncthreads();
        if (tid == 0) {
            for (int u = 1; u < kSegBlock / 64; ++u) {
                mx = max(mx, wts[u]);
                mn = min(mn, wp[u]);
            }
            summ[j] = SegSummary{mx, mn, 0u};
        }
        if (SPEC) {
            const double ft0 = new_t_of(s0.t_us == kAbsent ? 0 : s0.t_us);
            if (tid == 0) {
                Slot c = s0;
                bool m;
                (void)tb_step_ft(c, ft0, mn, req_time(mx, P.ttl_ms), P, m);
                pass_s0 = m ? 0u : 1u;
            }
            __syncthreads();
            if (pass_s0) {
#pragma unroll
                for (int it = 0; it < kSegItems; ++it) {
                    const uint32_t q = a + it * kSegBlock + tid;
                    if (q >= b) continue;
                    uint32_t k, pos;
                    int32_t p;
                    int64_t ts;
                    fold_input(rv[it], q, G, tbase1, rec0, ts_orig, tbase, F, 0u, k, p, ts, pos);
                    Slot c = s0;
                    bool m;
                    put_reply(res, pos, tb_step_ft(c, ft0, p, req_time_rel(ts, TB, P.ttl_ms), P, m), narrow);
                }
            }
        }
        __syncthreads();
    }
}

// One workgroup per run (see the section comment).
__global__ __launch_bounds__(kSegBlock) void k_hot_chain(
    const uint64_t *__restrict__ srec, const int64_t *__restrict__ ts_orig, PackFmt F,
    const uint32_t *__restrict__ bstart, uint32_t nb, const HotSet *__restrict__ hot,
    HotSet *__restrict__ hot_next, const uint32_t *__restrict__ segbase,
    const SegSummary *__restrict__ summ, SegState *__restrict__ sst, Slot *__restrict__ table,
    TbParams P, uint32_t *__restrict__ res, const uint32_t *__restrict__ err, uint32_t narrow, FoldFmt G,
    const uint64_t *__restrict__ rec0, uint32_t spec) {
    __shared__ Slot S;
    __shared__ double ftS;
    __shared__ uint32_t first, own;
    if (*err) return;
    const uint32_t h = blockIdx.x;
    if (h >= hot->count) return;
    const int tid = threadIdx.x;
    const uint32_t key = hot->key[h];
    const uint32_t s0 = bstart[nb + h], e0 = bstart[nb + h + 1];
    if (s0 == e0) return;
    const uint32_t j0 = segbase[h], nseg = segbase[h + 1] - j0;
    const int64_t tbase = pack_base(ts_orig, F);
    const int64_t tbase1 = G.on ? fold_base(ts_orig, G) : 0;
    const TimeBase TB = time_base(rel_base(ts_orig, F), P.ttl_ms);
    if (tid == 0) {
        S = table[key];
        ftS = new_t_of(S.t_us == kAbsent ? 0 : S.t_us);
    }
    __syncthreads();
    bool touched = false;
    uint32_t cur = 0;
    while (cur < nseg) {
        // the first segment at or after `cur` that may modify S
        const Slot s = S;
        const double ft = ftS;
        uint32_t f = nseg;
        for (uint32_t u = cur + tid; u < nseg; u += kSegBlock) {
            const SegSummary sm = summ[j0 + u];
            Slot c = s;
            bool m;
            (void)tb_step_ft(c, ft, sm.min_p, req_time(sm.max_ts, P.ttl_ms), P, m);
            if (m) {
                f = u;
                break;
            }
        }
        if (tid == 0) first = nseg;
        __syncthreads();
        atomicMin(&first, f);
        __syncthreads();
        f = first;
        // pass = 1: k_hot_replies decides the segment; 2: k_hot_summary<true> already did
        // (it passes the run's initial row through, which only the segments before the
        // first modifying one see)
        const uint32_t pv = (spec && !touched) ? 2u : 1u;
        for (uint32_t u = cur + tid; u < f; u += kSegBlock) sst[j0 + u] = SegState{s, ft, pv, 0u};
        if (f == nseg) break;
        if (tid == 0) sst[j0 + f].pass = 0u;
        touched = true;
        // decide segment f here, 2048 requests at a time, in speculative rounds
        const uint32_t a = s0 + f * kSeg, b = min(a + kSeg, e0);
        for (uint32_t c = a; c < b; c += kFoldChunk) {
            int32_t pm[kFoldPer];
            ReqTime rq[kFoldPer];
            uint32_t rep[kFoldPer], pos[kFoldPer], pend = 0;
#pragma unroll
            for (int r = 0; r < kFoldPer; ++r) {
                const uint32_t q = c + r * kSegBlock + tid;
                int64_t ts = 0;
                pm[r] = 0;
                rep[r] = 0;
                pos[r] = q;
                if (q < b) {
                    uint32_t k;
                    fold_input(srec[q], q, G, tbase1, rec0, ts_orig, tbase, F, 0u, k, pm[r], ts, pos[r]);
                    pend |= 1u << r;
                }
                rq[r] = req_time_rel(ts, TB, P.ttl_ms);
            }
            if (tid == 0) own = 0;
            __syncthreads();
            for (uint32_t round = 1;; ++round) {
                const Slot sc = S;
                const double fc = ftS;
                Slot nrow[kFoldPer];
#pragma unroll
                for (int r = 0; r < kFoldPer; ++r) {
                    nrow[r] = sc;
                    if (pend & (1u << r)) {
                        bool m;
                        rep[r] = tb_step_ft(nrow[r], fc, pm[r], rq[r], P, m);
                        if (m) atomicMax(&own, (round << 12) | (4095u - (uint32_t)(r * kSegBlock + tid)));
                    }
                }
                __syncthreads();
                const uint32_t o = own;
#pragma unroll
                for (int r = 0; r < kFoldPer; ++r) {
                    if (!(pend & (1u << r))) continue;
                    const uint32_t tag = (round << 12) | (4095u - (uint32_t)(r * kSegBlock + tid));
                    if ((o >> 12) != round || o < tag) {
                        pend &= ~(1u << r);
                    } else if (o == tag) {
                        S = nrow[r];
                        ftS = rq[r].new_t;
                        pend &= ~(1u << r);
                    }
                }
                if (!__syncthreads_or(pend != 0)) break;
            }
#pragma unroll
            for (int r = 0; r < kFoldPer; ++r) {
                const uint32_t q = c + r * kSegBlock + tid;
                if (q < b) put_reply(res, pos[r], rep[r], narrow);
            }
        }
        __syncthreads();
        cur = f + 1;
    }
    if (tid == 0) {
        if (touched) table[key] = S;
        if (e0 - s0 >= kHotMin / 2) {                 // still hot: nominate again
            const uint32_t at = atomicAdd(&hot_next->n_cand, 1u);
            if (at < kHotCandMax) hot_next->cand[at] = ((uint64_t)(e0 - s0) << 32) | key;
        }
    }
}

// Replies of the pass-through segments: each request against the row its segment saw.
__global__ __launch_bounds__(kSegBlock) void k_hot_replies(
    const uint64_t *__restrict__ srec, const int64_t *__restrict__ ts_orig, PackFmt F,
    const uint32_t *__restrict__ bstart, uint32_t nb, const uint32_t *__restrict__ segbase,
    const SegState *__restrict__ sst, TbParams P, uint32_t *__restrict__ res,
    const uint32_t *__restrict__ err, uint32_t narrow, FoldFmt G, const uint64_t *__restrict__ rec0) {
    if (*err) return;
    const int tid = threadIdx.x;
    const uint32_t total = segbase[kHotKeysMax];
    const int64_t tbase = pack_base(ts_orig, F);
    const int64_t tbase1 = G.on ? fold_base(ts_orig, G) : 0;
    const TimeBase TB = time_base(rel_base(ts_orig, F), P.ttl_ms);
    for (uint32_t j = blockIdx.x; j < total; j += gridDim.x) {
        const SegState st = sst[j];
        if (st.pass != 1u) continue;
        const uint32_t h = seg_run(segbase, j);
        const uint32_t a = bstart[nb + h] + (j - segbase[h]) * kSeg;
        const uint32_t b = min(a + kSeg, bstart[nb + h + 1]);
        uint64_t rv[kSegItems];   // every record of the segment in flight at once
#pragma unroll
        for (int it = 0; it < kSegItems; ++it) {
            const uint32_t q = a + it * kSegBlock + tid;
            rv[it] = q < b ? srec[q] : 0ull;
        }
#pragma unroll
        for (int it = 0; it < kSegItems; ++it) {
            const uint32_t q = a + it * kSegBlock + tid;
            if (q >= b) continue;
            uint32_t k, pos;
            int32_t p;
            int64_t ts;
            fold_input(rv[it], q, G, tbase1, rec0, ts_orig, tbase, F, 0u, k, p, ts, pos);
            Slot c = st.s;
            bool m;
            put_reply(res, pos, tb_step_ft(c, st.ft, p, req_time_rel(ts, TB, P.ttl_ms), P, m), narrow);
        }
    }
}

// The next batch's hot set from this batch's nominations (one 1024-thread workgroup):
// the `cap` busiest nominated keys (bitonic sort of the nominations, descending by
// their request counts), then their hash table.
__global__ __launch_bounds__(1024) void k_hot_update(HotSet *__restrict__ next, uint32_t cap,
                                                     const uint32_t *__restrict__ err) {
    __shared__ uint64_t c[kHotCandMax];
    // The nominations are consumed here: n_cand restarts at 0 for the fold that next
    // nominates into this set (three batches later), so no separate reset is launched.
    if (*err) {
        if (threadIdx.x == 0) next->n_cand = 0;
        return;
    }
    const uint32_t t = threadIdx.x;
    const uint32_t nc = min(next->n_cand, kHotCandMax);
    for (uint32_t j = t; j < kHotCandMax; j += 1024) c[j] = j < nc ? next->cand[j] : 0ull;
    for (uint32_t j = t; j < kHotSlots; j += 1024) next->slot[j] = kHotSlotEmpty;
    __syncthreads();
    if (t == 0) next->n_cand = 0;
    for (uint32_t k = 2; nc > cap && k <= kHotCandMax; k <<= 1) {   // select only when over capacity
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = t; i < kHotCandMax; i += 1024) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const uint64_t a = c[i], b = c[l];
                    const bool desc = (i & k) == 0;
                    if (desc ? (a < b) : (a > b)) {
                        c[i] = b;
                        c[l] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
    const uint32_t nh = min(nc, cap);
    // Two-choice placement in LDS (c is reused as the table once every thread holds its
    // key): a CAS into the key's first-half slot, else its second-half slot; the few keys
    // that lose both (~1% at load 1/4) are placed by thread 0 with cuckoo kicks.  A key
    // that still finds no slot after kCuckooKicks moves stays out of the table: its requests
    // take their ordinary buckets and its run is empty (speed only, never a decision).
    static_assert(kHotSlots <= kHotCandMax, "the cuckoo table reuses c[kHotCandMax] as its kHotSlots slots");
    __shared__ uint64_t left[64];
    __shared__ uint32_t n_left;
    const uint32_t key = t < nh ? (uint32_t)c[t] : 0u;
    __syncthreads();
    for (uint32_t j = t; j < kHotSlots; j += 1024) c[j] = kHotSlotEmpty;
    if (t == 0) n_left = 0;
    __syncthreads();
    if (t < nh) {
        next->key[t] = key;
        const unsigned long long mine = ((unsigned long long)t << 32) | key;
        unsigned long long *tab = reinterpret_cast<unsigned long long *>(c);
        const unsigned long long o1 = atomicCAS(&tab[hot_h1(key)], kHotSlotEmpty, mine);
        if (o1 != kHotSlotEmpty && (uint32_t)o1 != key) {
            const unsigned long long o2 = atomicCAS(&tab[hot_h2(key)], kHotSlotEmpty, mine);
            if (o2 != kHotSlotEmpty && (uint32_t)o2 != key) {
                const uint32_t at = atomicAdd(&n_left, 1u);
                if (at < 64) left[at] = mine;
            }
        }
    }
    __syncthreads();
    if (t == 0) {
        constexpr int kCuckooKicks = 64;
        for (uint32_t l = 0; l < min(n_left, 64u); ++l) {
            uint64_t cur = left[l];
            const uint32_t k0 = (uint32_t)cur;
            if ((uint32_t)c[hot_h1(k0)] == k0 || (uint32_t)c[hot_h2(k0)] == k0) continue;   // a duplicate placed since
            uint32_t at = hot_h1(k0);
            for (int m = 0; m < kCuckooKicks && cur != kHotSlotEmpty; ++m) {
                const uint64_t old = c[at];
                c[at] = cur;
                cur = old;
                if (cur == kHotSlotEmpty) break;
                const uint32_t k = (uint32_t)cur;
                at = (at == hot_h1(k)) ? hot_h2(k) : hot_h1(k);
            }
        }
    }
    __syncthreads();
    for (uint32_t j = t; j < kHotSlots; j += 1024) next->slot[j] = c[j];
    if (t == 0) next->count = nh;
}

constexpr uint64_t kHotSampleMin = 65536;   // estimated requests of a batch that make a key hot (k_hot_sample)

// Every batch is sampled (rounds 3-4 sampled only an engine's first
// two batches): a key that turns hot in a running engine would otherwise fill one ordinary
// bucket for the two batches its fold nomination takes, and that workgroup walks its
// millions of requests (~27 ms at config C's hottest key).  One 1024-thread workgroup, on
// the partition stream before the batch's first histogram:
//   1. S requests (hot_sample_n: n / 8192 clamped to [1024, 8192], so that a key at the
//      threshold is expected >= 8 times), one per stratum of the batch at a hashed offset,
//      counted in an LDS hash (key << 32 | count per slot, bounded probing: a sample that
//      finds no slot is dropped -- speed only);
//   2. every key estimated at >= kHotSampleMin requests of the batch that its hot set lacks
//      is appended to the set (new run index, cuckoo placement in an LDS copy of the table,
//      over the dead sample slots), up to the set's capacity -- fold nominations fill at
//      most cap - kHotSampleReserve of it;
//   3. only if a key was added, the table goes back to global memory.
// No 64-bit division anywhere (the strata are n / S apart, offsets by multiply-high): the
// first version's three per sample, and its 16,384 samples probing 8,192 slots, made it a
// 54 us kernel (profiles/r05n_*).  Which keys run apart only changes speed, never a decision.
constexpr uint32_t kHsSlots = 16384;
constexpr uint32_t kHsSampleMax = 8192;
constexpr int kHsProbes = 8;
constexpr uint32_t kHsNewMax = 256;   // config C: ~71 keys above kHotSampleMin at cold start
constexpr unsigned long long kHsEmpty = ~0ull;
__device__ __forceinline__ uint32_t hot_sample_n(uint64_t n) {
    return (uint32_t)min<uint64_t>(kHsSampleMax, max<uint64_t>(1024, n >> 13));
}
__global__ __launch_bounds__(1024) void k_hot_sample(const uint64_t *__restrict__ keys, uint64_t n,
                                                     uint64_t n_keys, HotSet *__restrict__ hot, uint32_t cap) {
    __shared__ unsigned long long sl[kHsSlots];   // the sample counts, then the hot table
    __shared__ uint64_t newk[kHsNewMax];
    __shared__ uint32_t nnew, count;
    static_assert(kHotSlots <= kHsSlots, "the hot table fits over the sample slots");
    const uint32_t t = threadIdx.x;
    const uint32_t S = hot_sample_n(n);
    if (n < S) return;                        // (launched for n >= kHotSampleMin only)
    if (t == 0) {
        nnew = 0;
        count = hot->count;
    }
    for (uint32_t j = t; j < kHsSlots; j += 1024) sl[j] = kHsEmpty;
    // one request from each of S strata of `step` requests, at a hashed offset inside the
    // stratum: a fixed stride would alias with periodic traffic (a key at every 10th
    // position is never sampled at stride 4096).  All of a thread's loads are issued before
    // any is used.
    const uint64_t step = n / S;             // < 2^32: the offset is a 32 x 32-bit multiply-high
    constexpr int kPerThread = kHsSampleMax / 1024;
    uint64_t kv[kPerThread];
#pragma unroll
    for (int j = 0; j < kPerThread; ++j) {
        const uint32_t i = t + 1024u * j;
        kv[j] = ~0ull;
        if (i < S) {
            uint32_t hx = (i + 0x9E3779B9u) * 0x85EBCA6Bu;
            hx ^= hx >> 13;
            hx *= 0xC2B2AE35u;
            hx ^= hx >> 16;
            kv[j] = keys[(uint64_t)i * step + (((uint64_t)hx * step) >> 32)];
        }
    }
    __syncthreads();                          // slots cleared
#pragma unroll
    for (int j = 0; j < kPerThread; ++j) {
        const uint64_t key = kv[j];
        if (key >= n_keys || key >= 0xFFFFFFFFull) continue;   // invalid keys fail the batch anyway
        const uint32_t k = (uint32_t)key;
        uint32_t h = (k * 0x9E3779B1u) >> (32 - 14);
        static_assert(kHsSlots == 1u << 14, "14-bit sample slots");
        for (int probe = 0; probe < kHsProbes; ++probe) {
            const unsigned long long old = atomicCAS(&sl[h], kHsEmpty, ((unsigned long long)k << 32) | 1ull);
            if (old == kHsEmpty) break;
            if ((uint32_t)(old >> 32) == k) {
                atomicAdd(&sl[h], 1ull);
                break;
            }
            h = (h + 1) & (kHsSlots - 1);
        }
    }
    __syncthreads();
    // estimated requests c * n / S >= kHotSampleMin, and not yet in the set
    for (uint32_t j = t; j < kHsSlots; j += 1024) {
        const unsigned long long v = sl[j];
        if (v == kHsEmpty || (uint64_t)(uint32_t)v * n < kHotSampleMin * S) continue;
        const uint32_t k = (uint32_t)(v >> 32);
        if (count && ((uint32_t)hot->slot[hot_h1(k)] == k || (uint32_t)hot->slot[hot_h2(k)] == k)) continue;
        const uint32_t at = atomicAdd(&nnew, 1u);
        if (at < kHsNewMax) newk[at] = k;
    }
    __syncthreads();
    if (nnew == 0) return;                    // workgroup-uniform
    uint64_t *tab = reinterpret_cast<uint64_t *>(sl);
    for (uint32_t j = t; j < kHotSlots; j += 1024) tab[j] = count ? hot->slot[j] : kHotSlotEmpty;
    __syncthreads();
    if (t == 0) {
        uint32_t cnt = count;
        for (uint32_t u = 0; u < min(nnew, kHsNewMax) && cnt < cap; ++u) {
            const uint32_t key = (uint32_t)newk[u];
            hot->key[cnt] = key;
            uint64_t cur = ((uint64_t)cnt << 32) | key;
            ++cnt;
            uint32_t at = hot_h1(key);
            if (tab[at] != kHotSlotEmpty && tab[hot_h2(key)] == kHotSlotEmpty) at = hot_h2(key);
            // cuckoo kicks; an entry left without a slot keeps its run index and runs empty
            for (int m = 0; m < 64 && cur != kHotSlotEmpty; ++m) {
                const uint64_t old = tab[at];
                tab[at] = cur;
                cur = old;
                if (cur == kHotSlotEmpty) break;
                const uint32_t k = (uint32_t)cur;
                at = (at == hot_h1(k)) ? hot_h2(k) : hot_h1(k);
            }
        }
        count = cnt;
    }
    __syncthreads();
    for (uint32_t j = t; j < kHotSlots; j += 1024) hot->slot[j] = tab[j];
    if (t == 0) hot->count = count;
}

// ----------------------------------------------------------------------------- queueing kind
// Per-key queue header (u64): bits 0-15 head, 16-31 count, 32-63 qsum (= _queueCount).
// Ring entry (u64): bits 16-63 request id, 0-15 permits.  Ring of key k: ring[k*C .. k*C+C).
struct QParams {
    int32_t token_limit;
    int32_t queue_limit;
    int32_t order;       // 0 OldestFirst, 1 NewestFirst
    uint32_t cap;        // ring entries per key (max(1, QueueLimit))
    int32_t wait;        // 1 = WaitAsyncCore (may queue), 0 = AcquireCore (lease or fail)
    uint32_t ai_base;    // added to eviction causes (a chunk's offset in its host batch)
    int64_t id_base;     // request id of arrival index 0 of this batch
};
__device__ __forceinline__ uint64_t qh_pack(uint32_t head, uint32_t cnt, int64_t qsum) {
    return (uint64_t)(head & 0xFFFFu) | ((uint64_t)(cnt & 0xFFFFu) << 16) | ((uint64_t)qsum << 32);
}
// Stored width of a queue header (round 6).  With QueueLimit <= kQh32MaxLimit the header is
// kept in 32 bits -- head 10 bits, count 11, queued permits 11: every queued entry holds >= 1
// permit (a zero-permit wait is granted at once, Q:153) and the queued permits never exceed
// QueueLimit (Q:92), so head, count and permits are all <= QueueLimit -- which halves the
// header bytes the fold reads and writes back.  Kernels work on the 64-bit form (qh_pack):
// qh_widen on every load, qh_store<HW> on every store.
#ifndef TBE_QH32
#define TBE_QH32 1                           // 0: 64-bit headers always (A/B)
#endif
constexpr uint32_t kQh32MaxLimit = 1024;
__host__ __device__ inline uint64_t qh_widen(uint64_t h) { return h; }
__host__ __device__ inline uint64_t qh_widen(uint32_t h) {
    return (uint64_t)(h & 0x3FFu) | ((uint64_t)((h >> 10) & 0x7FFu) << 16) | ((uint64_t)(h >> 21) << 32);
}
template <typename HW>
__host__ __device__ inline HW qh_store(uint64_t h);
template <>
__host__ __device__ inline uint64_t qh_store<uint64_t>(uint64_t h) { return h; }
template <>
__host__ __device__ inline uint32_t qh_store<uint32_t>(uint64_t h) {
    return (uint32_t)(h & 0x3FFu) | ((uint32_t)((h >> 16) & 0x7FFu) << 10) | ((uint32_t)(h >> 32) << 21);
}

// k_fold_q's shape: 768 threads x 2 requests (79 VGPRs, 56.8 KB of LDS), two workgroups
// (24 waves) per CU; against 512 x 4 (128 VGPRs, 16 waves) the config-D fold takes 1.91
// instead of 2.04 ms (profiles/r02_ablate_q.log).
#ifndef TBE_Q_BLOCK
#define TBE_Q_BLOCK 768
#endif
#ifndef TBE_Q_ITEMS
#define TBE_Q_ITEMS 2
#endif
#ifndef TBE_Q_WAVES
#define TBE_Q_WAVES 6
#endif
constexpr int kQBlock = TBE_Q_BLOCK;               // k_fold_q workgroup
constexpr int kQItems = TBE_Q_ITEMS;
constexpr int kQChunk = kQBlock * kQItems;         // 2048 requests per chunk
// One request of one key (WaitAsyncCore Q:67-134 / TryLeaseUnsynchronized Q:136-165)
// against the key's row `st` and queue header `hdr`; `kr` is the key's ring.  Sets the
// reply fields and ORs smod / hmod when the row / header changed.
__device__ __forceinline__ void q_step(Slot &st, uint64_t &hdr, bool &smod, bool &hmod, int32_t p, const ReqTime &rq,
                                       const TimeBase &TB, uint32_t ai, uint64_t *__restrict__ kr, const TbParams &P,
                                       const QParams &Q,
                                       uint32_t *__restrict__ ev_cause, int64_t *__restrict__ ev_id,
                                       uint32_t *__restrict__ ev_count, uint32_t ev_cap, uint32_t &status,
                                       uint32_t &rem, bool &evaluated) {
    uint32_t head = (uint32_t)(hdr & 0xFFFFu), cnt = (uint32_t)((hdr >> 16) & 0xFFFFu);
    int64_t qsum = (int64_t)(hdr >> 32);
    rem = 0;
    evaluated = false;
    if (p > Q.token_limit) {                                   // Q:70-73
        status = TBE_WAIT_REJECTED;
        return;
    }
    bool granted = false;
    if (p == 0 || !(cnt > 0 && Q.order == 0)) {                // Q:153
        bool m;
        const double ft = req_time_rel(st.t_us == kAbsent ? 0 : st.t_us, TB, 0).new_t;   // the row's field t
        const uint32_t reply = tb_step_ft(st, ft, p, rq, P, m);
        smod |= m;
        evaluated = true;
        granted = (reply >> 31) != 0;
        rem = reply & 0x7FFFFFFFu;
    }
    if (granted) {
        status = TBE_WAIT_GRANTED;
        return;
    }
    if (!Q.wait) {
        status = TBE_WAIT_FAILED;                              // TryLease only
        return;
    }
    if ((int64_t)Q.queue_limit - qsum < p) {                   // Q:92
        if (!(Q.order == 1 && p <= Q.queue_limit)) {
            status = TBE_WAIT_FAILED;                          // Q:113
            return;
        }
        while ((int64_t)Q.queue_limit - qsum < p) {            // Q:94-109
            const uint64_t ent = kr[head];
            const uint32_t at = atomicAdd(ev_count, 1u);
            if (at < ev_cap) {
                ev_cause[at] = ai + Q.ai_base;
                ev_id[at] = (int64_t)(ent >> 16);
            }
            qsum -= (int64_t)(ent & 0xFFFFu);
            head = (head + 1 == Q.cap) ? 0 : head + 1;
            --cnt;
        }
    }
    uint32_t tail = head + cnt;                                // Q:117-132
    if (tail >= Q.cap) tail -= Q.cap;
#if defined(TBE_Q_RING_SECTOR_AB)
    {   // A/B timing only (wrong queues): a whole aligned 32-byte sector per enqueue, so
        // the store needs no read-modify-write below L2
        typedef uint64_t u64x4 __attribute__((ext_vector_type(4)));
        const uint64_t v = ((uint64_t)(Q.id_base + ai) << 16) | (uint32_t)p;
        *reinterpret_cast<u64x4 *>(kr + (tail & ~3u)) = u64x4{v, v, v, v};
    }
#elif !defined(TBE_Q_NO_RING_WRITE)
    kr[tail] = ((uint64_t)(Q.id_base + ai) << 16) | (uint32_t)p;
#else
    (void)kr;   // A/B timing only (wrong queues): the cost of the ring stores
#endif
    ++cnt;
    qsum += p;
    hdr = qh_pack(head, cnt, qsum);
    hmod = true;
    status = TBE_WAIT_QUEUED;
}

// One key's share of a replenish tick (Q:237-271): grant the head (OldestFirst) or tail
// (NewestFirst) entry while the script grants at the tick.  Every queued entry holds >= 1
// permit, so when one permit is denied the entry is too, with the same state change (a
// denial only ever deletes a lapsed key): a one-permit probe decides that case without
// reading the ring.  WRITE = false counts the grants and changes nothing; WRITE = true
// applies them to (st, h) and logs them at at, at + 1, ... (key << 16 | drain position,
// request id, remaining).  Both forms take the same decisions, so a count pass followed by
// one reservation per workgroup and a writing pass logs exactly the grants -- one global
// atomic per workgroup instead of one per grant (a single log counter shared by every
// grant of the tick serialised them: 23M grants took 15 ms).
struct DrainLog {
    uint64_t *keyseq;
    int64_t *id;
    int32_t *rem;
    uint32_t cap;
};
// The row's field t as tb_step derives it, by req_time_rel against the batch's time base
// (rows of recent grants take its 32-bit path; any other falls back to req_time).
#ifndef TBE_TICK_FT
#define TBE_TICK_FT 1                        // 0: tb_step's own 64-bit derivation (A/B)
#endif
__device__ __forceinline__ uint32_t tick_step(Slot &row, int32_t permits, const ReqTime &rq, const TimeBase &TB,
                                              const TbParams &P, bool &modified) {
#if TBE_TICK_FT
    return tb_step_ft(row, req_time_rel(row.t_us == kAbsent ? 0 : row.t_us, TB, 0).new_t, permits, rq, P, modified);
#else
    (void)TB;
    return tb_step(row, permits, rq, P, modified);
#endif
}
template <bool WRITE>
__device__ __forceinline__ uint32_t drain_key(uint64_t key, Slot &st, uint64_t &h, bool &smod,
                                              const uint64_t *__restrict__ kr, const ReqTime &rqT, const TimeBase &TB,
                                              const TbParams &P, const QParams &Q, const DrainLog &L, uint32_t at) {
    uint32_t cnt = (uint32_t)((h >> 16) & 0xFFFFu);
    if (cnt == 0) return 0;
    uint32_t head = (uint32_t)(h & 0xFFFFu);
    int64_t qsum = (int64_t)(h >> 32);
    Slot s = st;
    bool m_any = false;
    uint32_t seq = 0;
    while (cnt > 0) {
        {
            Slot probe = s;
            bool pm;
            if (!(tick_step(probe, 1, rqT, TB, P, pm) >> 31)) {
                s = probe;
                m_any |= pm;
                break;
            }
        }
        uint32_t idx = head;
        if (Q.order == 1) {
            idx = head + cnt - 1;
            if (idx >= Q.cap) idx -= Q.cap;
        }
        const uint64_t ent = kr[idx];
        const int32_t p = (int32_t)(ent & 0xFFFFu);
        bool m;
        const uint32_t reply = tick_step(s, p, rqT, TB, P, m);
        m_any |= m;
        if (!(reply >> 31)) break;
        if (WRITE && at + seq < L.cap) {
            L.keyseq[at + seq] = (key << 16) | seq;
            L.id[at + seq] = (int64_t)(ent >> 16);
            L.rem[at + seq] = (int32_t)(reply & 0x7FFFFFFFu);
        }
        ++seq;
        qsum -= p;
        if (Q.order == 0) head = (head + 1 == Q.cap) ? 0 : head + 1;
        --cnt;
    }
    if (WRITE) {
        st = s;
        if (seq) h = qh_pack(head, cnt, qsum);
    }
    smod |= m_any;   // (WRITE = false: whether the writing pass would change the row)
    return seq;
}

// A replenish tick fused into a queue batch (tbe_wait_batch_tick_device): after the
// batch's requests, every key of the bucket is drained at `ts` exactly as k_drain does,
// on the rows and headers already in LDS.  ts < 0: no tick.
struct QTick {
    int64_t ts;
    uint64_t *keyseq;
    int64_t *id;
    int32_t *rem;
    uint32_t *count;
    uint32_t cap;
};

// (Deciding each row's requests in one thread after an LDS counting sort, instead of
// election rounds, was parity-equal but slower: config-D fold 3.11 against 2.41 ms,
// profiles/r02_ablate_qwalk.log; removed in round 5.)
// Tail walk (round 3): after the first owner round, the requests still pending (a key's
// second, third, ... request of the chunk; about a third of config D's) are sorted by row
// in LDS and each row's run is decided by one thread in arrival order -- no further
// workgroup-wide rounds.  Taken when at most kQTail requests are pending and no row has
// more than kQTailRun of them; otherwise the rounds go on.  Same decisions as the rounds:
// each key's requests are still taken in arrival order, and keys are independent.
#ifndef TBE_Q_TAIL_WALK
#define TBE_Q_TAIL_WALK 1
#endif
constexpr uint32_t kQTail = kQBlock;     // one pending request per thread at most
constexpr uint32_t kQTailRun = 32;       // longest run a walking thread sorts and decides

// WaitAsyncCore (Q:67-134) for every request of one bucket, in arrival order per key:
// the same bucket/chunk/owner-round structure as k_fold, plus the key's queue header in
// LDS and its ring in HBM.  A ring entry written in one round and read (evicted) in a
// later round of the same workgroup is ordered by the round's __syncthreads
// (workgroup-scope fence; one CU, one vector L1).
// PACKED: requests arrive as packed records (PackFmt; permit code min(p, TokenLimit + 1),
// which leaves REJECTED exactly where p > TokenLimit) beside their arrival indices.
template <bool PACKED, typename HW>
__global__ __launch_bounds__(kQBlock, TBE_Q_WAVES) void k_fold_q(
    const uint32_t *__restrict__ skeys, const int32_t *__restrict__ sperm,
    const int64_t *__restrict__ sts, const uint32_t *__restrict__ sidx,
    const uint64_t *__restrict__ srec, const int64_t *__restrict__ ts_orig, PackFmt F,
    const uint32_t *__restrict__ bstart, int r_bits, uint64_t n_keys, Slot *__restrict__ table,
    HW *__restrict__ qhdr, uint64_t *__restrict__ ring, TbParams P, QParams Q,
    uint32_t *__restrict__ res, uint32_t *__restrict__ ev_cause, int64_t *__restrict__ ev_id,
    uint32_t *__restrict__ ev_count, uint32_t ev_cap, const uint32_t *__restrict__ err, uint32_t narrow,
    QTick T, FoldFmt G, const uint64_t *__restrict__ rec0) {
    __shared__ __attribute__((aligned(16))) Slot slot[1 << kMaxRBits];   // LDS-DMA destinations
    __shared__ __attribute__((aligned(16))) HW qh[1 << kMaxRBits];
    __shared__ uint32_t own[1 << kMaxRBits];      // election slots, or the walk's row counts / starts
    __shared__ uint32_t loaded[(1 << kMaxRBits) / 32];
    __shared__ uint32_t dirty[(1 << kMaxRBits) / 32];    // rows modified (smod)
    __shared__ uint32_t hdirty[(1 << kMaxRBits) / 32];   // queue headers modified (hmod)
#if TBE_Q_TAIL_WALK
    __shared__ uint32_t tw_e[kQTail];             // row | chunk index << 16
    __shared__ int32_t tw_pm[kQTail];
    __shared__ int64_t tw_ts[kQTail];
    __shared__ uint32_t tw_ai[kQTail];
    __shared__ uint32_t tw_pos[kQTail];           // reply positions
    __shared__ uint16_t tw_sorted[kQTail];        // tail entries by row
    __shared__ uint32_t tw_sum[kQBlock / 64];
    __shared__ uint32_t tw_max;
#endif

    if (*err) return;
    const int tid = threadIdx.x;
    const uint32_t b = fold_bucket(G);
    if (G.on && b >= G.nb) return;
    const uint32_t s = bstart[b], e = bstart[b + 1];
    const bool tick = T.ts >= 0;
    if (s == e && !tick) return;
    const uint32_t R = 1u << r_bits;
    const uint32_t rmask = R - 1;
    const uint64_t row0 = (uint64_t)b << r_bits;
    const uint32_t nrows = (uint32_t)min<uint64_t>(R, n_keys - row0);
    Slot *__restrict__ rows = table + row0;
    HW *__restrict__ hrows = qhdr + row0;

    // A dense bucket (>= R/8 requests: nearly every 128-byte line of its slice is touched)
    // pulls its whole slice of rows and queue headers with coalesced loads and writes it
    // back whole; a sparse one gathers and writes back only the rows it touches.
    const bool dense = tick || (e - s) >= (R >> 3);   // a tick drains every row
    const int64_t tbase = PACKED ? pack_base(ts_orig, F) : 0;
    const int64_t tbase1 = G.on ? fold_base(ts_orig, G) : 0;
    const TimeBase TB = time_base(PACKED ? rel_base(ts_orig, F) : 0, P.ttl_ms);   // fast request / row times (req_time_rel)
    if (dense) {
        // The slice goes HBM -> LDS directly (LDS-DMA, streaming policy): no VGPRs held for
        // it.  Rows one per lane; headers two per lane (16 B), the header array being padded
        // to an even row count.  Rows past nrows get copies of the last ones; no request
        // reaches them and they are never written back.
        constexpr int kRPT = (kMaxRows + kQBlock - 1) / kQBlock;
#pragma unroll
        for (int u = 0; u < kRPT; ++u) {
            const uint32_t wbase = u * kQBlock + (tid & ~63);   // wave-uniform
            if (wbase < R) {
                const uint32_t j = tid + u * kQBlock;
                lds_dma16(rows + (j < nrows ? j : nrows - 1), &slot[wbase]);
            }
        }
        constexpr uint32_t kHPL = 16 / sizeof(HW);   // headers per 16-byte lane load
        constexpr int kHPT = (kMaxRows / kHPL + kQBlock - 1) / kQBlock;
        const uint32_t ngrp = (nrows + kHPL - 1) / kHPL;   // (the header array is padded to kHPL)
#pragma unroll
        for (int u = 0; u < kHPT; ++u) {
            const uint32_t wbase = u * kQBlock + (tid & ~63);   // group index of lane 0
            if (kHPL * wbase < R) {
                const uint32_t pj = tid + u * kQBlock;
                lds_dma16(hrows + kHPL * (pj < ngrp ? pj : ngrp - 1), &qh[kHPL * wbase]);
            }
        }
    }
    for (uint32_t j = tid; j < (R + 31) / 32; j += kQBlock) {
        loaded[j] = dense ? ~0u : 0u;
        dirty[j] = 0;
        hdirty[j] = 0;
    }
    lds_dma_wait();    // this wave's slice and header DMA landed
    __syncthreads();
#if TBE_QFOLD_PREFETCH
    // as k_fold_wide: touch the rows, queue headers and records of the workgroup
    // TBE_QFOLD_PREFETCH blocks later (same XCD); waited for at the write-back barrier
    uint32_t pf_sink = 0;
    if (e - s >= TBE_FOLD_PREFETCH_MIN) {
        const uint32_t fblk = blockIdx.x + TBE_QFOLD_PREFETCH;
        const uint32_t fb = fold_bucket_at(G, fblk);
        if (fblk < gridDim.x && (!G.on || fb < G.nb)) {
            const uint32_t fs = bstart[fb], fe = bstart[fb + 1];
            const uint64_t frow = (uint64_t)fb << r_bits;
            if (fe > fs && frow < n_keys) {
                const uint32_t fn = (uint32_t)min<uint64_t>(R, n_keys - frow);
                const uint32_t t = (uint32_t)tid;
                if (t < kMaxRows / 8) {
                    if (t * 8u < fn) pf_sink = reinterpret_cast<const uint32_t *>(table + frow + t * 8u)[0];
                } else if (t < kMaxRows / 8 + kMaxRows / 16) {
                    const uint32_t h = (t - kMaxRows / 8) * 16u;
                    if (h < fn) pf_sink = reinterpret_cast<const uint32_t *>(qhdr + frow + h)[0];
                } else if (PACKED) {
                    const uint32_t q = fs + (t - kMaxRows / 8 - kMaxRows / 16) * 16u;
                    if (q < fe) pf_sink = (uint32_t)srec[q];
                }
            }
        }
    }
#endif

    for (uint32_t c = s; c < e; c += kQChunk) {
        uint32_t kl[kQItems], ai[kQItems], pos[kQItems];
        int32_t pm[kQItems];
        int64_t ts[kQItems];
        uint32_t pend = 0;
#pragma unroll
        for (int r = 0; r < kQItems; ++r) {
            const uint32_t q = c + r * kQBlock + tid;
            pos[r] = q;
            if (q < e) {
                if (PACKED) {
                    fold_input(srec[q], q, G, tbase1, rec0, ts_orig, tbase, F, rmask, kl[r], pm[r], ts[r], pos[r]);
                } else {
                    kl[r] = skeys[q] & rmask;
                    pm[r] = sperm[q];
                    ts[r] = sts[q];
                }
                ai[r] = sidx[q];
                pend |= 1u << r;
            } else {
                kl[r] = 0; pm[r] = 0; ts[r] = 0; ai[r] = 0;
            }
        }
        for (uint32_t j = tid; j < R; j += kQBlock) own[j] = 0;   // election slots of this chunk
        uint32_t mine = 0;   // rows this thread gathers (a sparse bucket's first touch)
        if (!dense) {        // (a dense slice is all loaded)
#pragma unroll
            for (int r = 0; r < kQItems; ++r) {
                if (pend & (1u << r)) {
                    const uint32_t bit = 1u << (kl[r] & 31);
                    const uint32_t old = atomicOr(&loaded[kl[r] >> 5], bit);
                    if (!(old & bit)) mine |= 1u << r;
                }
            }
        }
        if (mine) {
            Slot tmp[kQItems];
            HW th[kQItems];
#pragma unroll
            for (int r = 0; r < kQItems; ++r) {
                tmp[r] = Slot{0.0, 0};
                th[r] = 0;
                if (mine & (1u << r)) { tmp[r] = rows[kl[r]]; th[r] = hrows[kl[r]]; }
            }
#pragma unroll
            for (int r = 0; r < kQItems; ++r)
                if (mine & (1u << r)) { slot[kl[r]] = tmp[r]; qh[kl[r]] = th[r]; }
        }
        __syncthreads();   // claimed rows and headers visible
        // Owner rounds: each key's earliest pending request wins an election slot tagged
        // (round << 12) | (4095 - chunk index) by atomicMax, so a newer round's tag beats
        // every older one and the slots need no reset between rounds (two barriers per
        // round).  Slots are zeroed at each chunk start.
        for (uint32_t round = 1;; ++round) {
#pragma unroll
            for (int r = 0; r < kQItems; ++r)
                if (pend & (1u << r)) atomicMax(&own[kl[r]], (round << 12) | (4095u - (uint32_t)(r * kQBlock + tid)));
            __syncthreads();
            uint32_t won = 0;
#pragma unroll
            for (int r = 0; r < kQItems; ++r) {
                if (!((pend & (1u << r)) &&
                      own[kl[r]] == ((round << 12) | (4095u - (uint32_t)(r * kQBlock + tid)))))
                    continue;
                won |= 1u << r;
                Slot st = slot[kl[r]];
                uint64_t h = qh_widen(qh[kl[r]]);
                bool smod = false, hmod = false, evaluated;
                uint32_t status, rem;
                // request times derived by the winner (not held across rounds: registers)
                const ReqTime rqr = req_time_rel(ts[r], TB, P.ttl_ms);
                q_step(st, h, smod, hmod, pm[r], rqr, TB, ai[r], ring + (row0 + kl[r]) * (uint64_t)Q.cap, P, Q,
                       ev_cause, ev_id, ev_count, ev_cap, status, rem, evaluated);
                put_wait(res, pos[r], status, evaluated, rem, narrow);
                if (smod) slot[kl[r]] = st;
                if (hmod) qh[kl[r]] = qh_store<HW>(h);
                if (smod) atomicOr(&dirty[kl[r] >> 5], 1u << (kl[r] & 31));
                if (hmod) atomicOr(&hdirty[kl[r] >> 5], 1u << (kl[r] & 31));
            }
            pend &= ~won;
#ifdef TBE_Q_R1_ONLY
            pend = 0;   // A/B timing only (wrong replies): the cost of the rounds after round 1
#endif
#if TBE_Q_TAIL_WALK
            if (round == 1) {
                uint32_t n_tail;
                const uint32_t at0 = block_excl_scan<kQBlock>(__popc(pend), tw_sum, &n_tail);
                if (n_tail == 0) break;                       // block-uniform
                if (n_tail <= kQTail) {
                    // the pending requests, compacted (entry i = the i-th pending request)
                    uint32_t at = at0;
#pragma unroll
                    for (int r = 0; r < kQItems; ++r) {
                        if (pend & (1u << r)) {
                            tw_e[at] = kl[r] | ((uint32_t)(r * kQBlock + tid) << 16);
                            tw_pm[at] = pm[r];
                            tw_ts[at] = ts[r];
                            tw_ai[at] = ai[r];
                            tw_pos[at] = pos[r];
                            ++at;
                        }
                    }
                    for (uint32_t j = tid; j < R; j += kQBlock) own[j] = 0;   // round-1 tags are read
                    if (tid == 0) tw_max = 0;
                    __syncthreads();
                    // counting sort by row: rank within the row, row starts, placement
                    const bool te = (uint32_t)tid < n_tail;
                    uint32_t trow = 0, trk = 0;
                    if (te) {
                        trow = tw_e[tid] & 0xFFFFu;
                        trk = atomicAdd(&own[trow], 1u);
                    }
                    __syncthreads();
                    {
                        constexpr uint32_t RPT = (kMaxRows + kQBlock - 1) / kQBlock;
                        uint32_t cn[RPT], sum = 0, mx = 0;
#pragma unroll
                        for (uint32_t u = 0; u < RPT; ++u) {
                            const uint32_t j = tid * RPT + u;
                            cn[u] = j < R ? own[j] : 0u;
                            sum += cn[u];
                            mx = cn[u] > mx ? cn[u] : mx;
                        }
                        uint32_t tot;
                        uint32_t st0 = block_excl_scan<kQBlock>(sum, tw_sum, &tot);
#pragma unroll
                        for (uint32_t u = 0; u < RPT; ++u) {
                            const uint32_t j = tid * RPT + u;
                            if (j < R) own[j] = st0;
                            st0 += cn[u];
                        }
                        if (mx) atomicMax(&tw_max, mx);
                    }
                    __syncthreads();
                    if (te) tw_sorted[own[trow] + trk] = (uint16_t)tid;
                    __syncthreads();
                    if (tw_max <= kQTailRun) {
                        // thread t takes sorted position t; the first position of a row's run
                        // walks the run
                        if (te) {
                            const uint32_t e0 = tw_sorted[tid];
                            const uint32_t row = tw_e[e0] & 0xFFFFu;
                            const uint32_t start = own[row];
                            if ((uint32_t)tid == start) {
                                const uint32_t stop = (row + 1 < R) ? own[row + 1] : n_tail;
                                // arrival order inside the run (insertion sort by chunk index)
                                for (uint32_t x = start + 1; x < stop; ++x) {
                                    const uint16_t v = tw_sorted[x];
                                    const uint32_t vl = tw_e[v] >> 16;
                                    uint32_t y = x;
                                    while (y > start && (tw_e[tw_sorted[y - 1]] >> 16) > vl) {
                                        tw_sorted[y] = tw_sorted[y - 1];
                                        --y;
                                    }
                                    tw_sorted[y] = v;
                                }
                                Slot st = slot[row];
                                uint64_t h = qh_widen(qh[row]);
                                bool smod = false, hmod = false;
                                uint64_t *__restrict__ kr = ring + (row0 + row) * (uint64_t)Q.cap;
                                for (uint32_t x = start; x < stop; ++x) {
                                    const uint32_t en = tw_sorted[x];
                                    uint32_t status, rem;
                                    bool evaluated;
                                    const ReqTime rq1 = req_time_rel(tw_ts[en], TB, P.ttl_ms);
                                    q_step(st, h, smod, hmod, tw_pm[en], rq1, TB, tw_ai[en], kr, P, Q, ev_cause, ev_id,
                                           ev_count, ev_cap, status, rem, evaluated);
                                    put_wait(res, tw_pos[en], status, evaluated, rem, narrow);
                                }
                                if (smod) {
                                    slot[row] = st;
                                    atomicOr(&dirty[row >> 5], 1u << (row & 31));
                                }
                                if (hmod) {
                                    qh[row] = qh_store<HW>(h);
                                    atomicOr(&hdirty[row >> 5], 1u << (row & 31));
                                }
                            }
                        }
                        __syncthreads();   // the chunk's rows are settled before the next chunk
                        break;             // block-uniform (tw_max)
                    }
                    // a long run: the rounds go on from the list (the round-1 registers of the
                    // pending requests are reloaded, so they need not live through the walk;
                    // own[] holds row starts < 2 << 12, below every tag of round 2 on)
                    {
                        uint32_t at1 = at0;
#pragma unroll
                        for (int r = 0; r < kQItems; ++r) {
                            if (pend & (1u << r)) {
                                kl[r] = tw_e[at1] & 0xFFFFu;
                                pm[r] = tw_pm[at1];
                                ts[r] = tw_ts[at1];
                                ai[r] = tw_ai[at1];
                                pos[r] = tw_pos[at1];
                                ++at1;
                            }
                        }
                    }
                }
            }
#endif
            if (!__syncthreads_or(pend != 0)) break;
        }
    }
    __syncthreads();
#ifdef TBE_Q_TICK_SKIP
    if (false) {   // A/B timing only (wrong queues): the cost of the fused tick's drain
#else
    if (tick) {
#endif
        // The fused replenish tick (Q:237-271, as k_drain) on the rows and headers in LDS:
        // count this workgroup's grants, reserve them in the log with one atomic, then
        // drain and log (drain_key).
        const ReqTime rqT = req_time(T.ts, P.ttl_ms);
        const DrainLog L{T.keyseq, T.id, T.rem, T.cap};
        constexpr uint32_t kRowsPer = (kMaxRows + kQBlock - 1) / kQBlock;
        static_assert(kRowsPer <= 32, "one bit per row of this thread");
        uint32_t mine = 0;
        // rows whose writing pass changes something: it grants, or its one-permit probe
        // lapsed the key (passive expiry); every other row's writing pass is a no-op, and
        // in config D's steady state (ticks that grant nothing) that is every row
        uint32_t need = 0;
#pragma unroll
        for (uint32_t u = 0; u < kRowsPer; ++u) {
            const uint32_t j = tid + u * kQBlock;
            if (j < nrows) {
                Slot st = slot[j];
                uint64_t h = qh_widen(qh[j]);
                bool sm = false;
                const uint32_t g = drain_key<false>(row0 + j, st, h, sm, ring + (row0 + j) * (uint64_t)Q.cap, rqT, TB, P,
                                                    Q, L, 0);
                mine += g;
                if (g || sm) need |= 1u << u;
            }
        }
        uint32_t total;
        __shared__ uint32_t tick_wsum[kQBlock / 64];
        const uint32_t off = block_excl_scan<kQBlock>(mine, tick_wsum, &total);
        __shared__ uint32_t log_base;
        if (tid == 0) log_base = total ? atomicAdd(T.count, total) : 0u;
        __syncthreads();
        uint32_t at = log_base + off;
#pragma unroll
        for (uint32_t u = 0; u < kRowsPer; ++u) {
            const uint32_t j = tid + u * kQBlock;
            if ((need >> u) & 1u) {
                Slot st = slot[j];
                uint64_t h = qh_widen(qh[j]);
                const uint64_t h0 = h;
                bool smod = false;
                const uint32_t g = drain_key<true>(row0 + j, st, h, smod, ring + (row0 + j) * (uint64_t)Q.cap, rqT, TB, P,
                                                   Q, L, at);
                at += g;
                if (smod) slot[j] = st;
                if (h != h0) qh[j] = qh_store<HW>(h);
                if (smod) atomicOr(&dirty[j >> 5], 1u << (j & 31));
                if (h != h0) atomicOr(&hdirty[j >> 5], 1u << (j & 31));
            }
        }
        __syncthreads();
    }
    // dense: whole dirty lines of rows (8 per line) and of headers (16 per line).  Rows and
    // headers keep separate dirty bits: in config D's steady state nearly every request
    // queues or fails, which changes a header but not the row, and one shared bit wrote
    // the whole 1.6 GB row table back every batch.
    for (uint32_t j = tid; j < nrows; j += kQBlock) {
        if (dense ? row_line_dirty(dirty, j) : row_dirty(dirty, j)) ST_S(rows + j, slot[j]);
        const bool hline = sizeof(HW) == 8 ? ((hdirty[j >> 5] >> (j & 16u)) & 0xFFFFu) != 0   // 16 per line
                                           : hdirty[j >> 5] != 0;                            // 32 per line
        if (dense ? hline : row_dirty(hdirty, j)) ST_U(hrows + j, qh[j]);
    }
#if TBE_QFOLD_PREFETCH
    if (n_keys == 0) res[s] = pf_sink;   // never (no engine has 0 keys): keeps the touches
#endif
}

// One replenish tick (Q:237-271) over every key: drain the head (OldestFirst) or tail
// (NewestFirst) while the acquire script grants.  One thread per key.  Grants are logged
// as (key, drain position, request id, remaining); the host orders them by key.
template <typename HW>
__global__ __launch_bounds__(kBlock) void k_drain(
    uint64_t n_keys, Slot *__restrict__ table, HW *__restrict__ qhdr,
    const uint64_t *__restrict__ ring, TbParams P, QParams Q, int64_t ts_us,
    uint64_t *__restrict__ log_keyseq, int64_t *__restrict__ log_id, int32_t *__restrict__ log_rem,
    uint32_t *__restrict__ log_count, uint32_t log_cap) {
    __shared__ uint32_t wsum[kWaves];
    __shared__ uint32_t log_base;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const ReqTime rqT = req_time(ts_us, P.ttl_ms);
    const TimeBase TB = time_base(ts_us > kRowWindow ? ts_us - kRowWindow : 0, 0);   // rows' field t (tick_step)
    const DrainLog L{log_keyseq, log_id, log_rem, log_cap};
    // block-uniform trip count (the log reservation below is a block-wide scan)
    for (uint64_t k0 = (uint64_t)blockIdx.x * kBlock; k0 < n_keys; k0 += stride) {
        const uint64_t key = k0 + threadIdx.x;
        const bool valid = key < n_keys;
        uint64_t h = valid ? qh_widen(qhdr[key]) : 0ull;
        const bool queued = ((h >> 16) & 0xFFFFu) != 0;
        Slot st = (valid && queued) ? table[key] : Slot{0.0, 0};
        const uint64_t *__restrict__ kr = ring + key * (uint64_t)Q.cap;
        bool sm = false;
        Slot st0 = st;
        uint64_t h0 = h;
        const uint32_t mine = queued ? drain_key<false>(key, st0, h0, sm, kr, rqT, TB, P, Q, L, 0) : 0u;
        uint32_t total;
        const uint32_t off = block_excl_scan<kBlock>(mine, wsum, &total);
        if (threadIdx.x == 0) log_base = total ? atomicAdd(log_count, total) : 0u;
        __syncthreads();
        if (queued && (mine != 0 || sm)) {   // (else the writing pass is a no-op)
            bool smod = false;
            const uint64_t hb = h;
            drain_key<true>(key, st, h, smod, kr, rqT, TB, P, Q, L, log_base + off);
            if (smod) table[key] = st;
            if (h != hb) qhdr[key] = qh_store<HW>(h);
        }
        __syncthreads();   // log_base is rewritten by the next trip
    }
}

// ----------------------------------------------------------------------------- approximate kind
// One client's local tier per key (A:36-37, A:84-214), the global tier replica per key
// (the sync script's Redis hash {v, p, t}, A:241-270) and the per-key queue ring.
struct ALocal {
    int32_t cap;     // (int)Math.Ceiling((TokenLimit - _globalThrottleScore) / _instanceCountEstimate)
    int32_t local;   // _localThrottleScore
    uint16_t qsum;   // _queueCount (<= QueueLimit <= 65535)
    uint16_t zc;     // zero-permit registrations in the queue (<= AParams.zero_slots)
    uint32_t hc;     // ring head (bits 0-15) | count (bits 16-31)
};
struct AClient {
    double est;      // _instanceCountEstimate
    int32_t global;  // _globalThrottleScore
    int32_t pad;
};
struct AParams {
    int32_t token_limit;
    int32_t queue_limit;
    int32_t order;          // 0 OldestFirst, 1 NewestFirst
    uint32_t cap;           // ring entries per key: max(1, QueueLimit) + zero_slots
    int64_t id_base;
    int32_t wait;           // 1: WaitAsyncCore (A:116-183), 0: AcquireCore (A:84-113)
    int32_t zero_slots;     // ring entries a key may give to zero-permit registrations
    uint32_t ai_base;       // added to eviction causes (a chunk's offset in its host batch)
    uint32_t pad;
    double decay_rate;      // FillRatePerSecond (A:224 decay_rate)
    double period_s;        // ReplenishmentPeriod.TotalSeconds (A:443)
};
constexpr int64_t kApproxTtlMs = 86400LL * 1000;   // EXPIRE 86400 (A:268)

__device__ __forceinline__ int32_t wrap_sub(int32_t a, int32_t b) {
    return (int32_t)((uint32_t)a - (uint32_t)b);
}
__device__ __forceinline__ int32_t avail_of(const ALocal &a) {       // A:37
    const int32_t d = wrap_sub(a.cap, a.local);
    return d > 0 ? d : 0;
}
// C# (int)double on x64: truncation; NaN and out-of-range give int.MinValue.
__device__ __forceinline__ int32_t dotnet_to_int(double x) {
    if (!(x > -2147483649.0 && x < 2147483648.0)) return INT32_MIN;
    return (int32_t)x;
}

// WaitAsyncCore / AcquireCore of one client for every request of one bucket, per key in
// arrival order (same bucket/chunk/round structure as k_fold; no timestamps: the local
// tier never reads the clock).  Reply: pack_wait(status, true, AvailableTokens after).
// Round 3 tried two replacements for the owner rounds, both decided the same and both were
// slower on config E (profiles/r03_ablate_approx_fold.log): a walk of each key's run by one
// thread after an LDS counting sort (fold 1.22 against 0.76 ms), and deciding whole runs at
// once when all of a key's requests in the chunk lease (A:191-209; 0.91 ms: the sort, the run
// sums and the registers they spill cost more than the rounds they save).
// Requests per thread per chunk (A/B: a larger chunk means fewer chunks per bucket and
// fewer owner rounds in total, at more registers).
#ifndef TBE_A_PER
#define TBE_A_PER 4
#endif
constexpr int kAPer = TBE_A_PER;
constexpr int kAChunk = kFoldBlock * kAPer;
static_assert(kAChunk <= 4096, "election tags");
#ifndef TBE_A_WAVES
#define TBE_A_WAVES 6                        // minimum waves per SIMD: 80 VGPRs, 3 workgroups per CU
                                             // (0.867 -> 0.688 ms, profiles/r02_ablate_queue_dma_approx_waves.log)
#endif
template <bool PACKED>
__global__ __launch_bounds__(kFoldBlock, TBE_A_WAVES) void k_fold_a(
    const uint32_t *__restrict__ skeys, const int32_t *__restrict__ sperm,
    const uint32_t *__restrict__ sidx, const uint64_t *__restrict__ srec, PackFmt F,
    const uint32_t *__restrict__ bstart, int r_bits,
    uint64_t n_keys, ALocal *__restrict__ alocal, uint64_t *__restrict__ ring, AParams A,
    uint32_t *__restrict__ res, uint32_t *__restrict__ ev_cause, int64_t *__restrict__ ev_id,
    uint32_t *__restrict__ ev_count, uint32_t ev_cap, const uint32_t *__restrict__ err, uint32_t rw, FoldFmt G,
    const uint64_t *__restrict__ rec0) {
    __shared__ ALocal sl[kMaxRows];
    __shared__ uint32_t own[kMaxRows];
    __shared__ uint32_t rbuf[kAChunk];
    __shared__ uint32_t loaded[kMaxRows / 32];
    __shared__ uint32_t dirty[kMaxRows / 32];

    if (*err) return;
    const int tid = threadIdx.x;
    const uint32_t b = fold_bucket(G);
    if (G.on && b >= G.nb) return;
    const uint32_t s = bstart[b], e = bstart[b + 1];
    if (s == e) return;
    const uint32_t R = 1u << r_bits;
    const uint32_t rmask = R - 1;
    const uint64_t row0 = (uint64_t)b << r_bits;
    const uint32_t nrows = (uint32_t)min<uint64_t>(R, n_keys - row0);
    ALocal *__restrict__ rows = alocal + row0;
    // A dense bucket (>= R/8 requests: config E has ~13,700 per bucket) pulls its whole
    // local-tier slice with coalesced streaming loads and writes it back whole; a sparse one
    // gathers the rows it touches.  (Round 1 dropped this variant after a wrong result that
    // the rebuilt variant does not reproduce -- DESIGN.md §5 "Streaming hints".)
    const bool dense = (e - s) >= (R >> 3);
    if (dense) {
        // HBM -> LDS directly (LDS-DMA, streaming policy; rows past nrows get a copy of
        // the last row, which nothing reads or writes back)
        constexpr int kRPT = (kMaxRows + kFoldBlock - 1) / kFoldBlock;
#pragma unroll
        for (int u = 0; u < kRPT; ++u) {
            const uint32_t j = tid + u * kFoldBlock;
            if (u * kFoldBlock < (int)R) lds_dma16(rows + (j < nrows ? j : nrows - 1), &sl[u * kFoldBlock + (tid & ~63)]);
        }
    }
    for (uint32_t j = tid; j < (R + 31) / 32; j += kFoldBlock) {
        loaded[j] = dense ? ~0u : 0u;
        dirty[j] = 0;
    }
#if TBE_AFOLD_PREFETCH
    uint32_t pf_sink = 0;
#endif
    for (uint32_t c = s; c < e; c += kAChunk) {
        for (uint32_t j = tid; j < R; j += kFoldBlock) own[j] = 0;
        uint32_t kl[kAPer];
        int32_t pm[kAPer];
        uint32_t pend = 0;
#pragma unroll
        for (int r = 0; r < kAPer; ++r) {
            const uint32_t q = c + r * kFoldBlock + tid;
            kl[r] = 0; pm[r] = 0;
            if (q < e) {
                if (PACKED) {   // key | permit code | escape | arrival index (k_scatter_rec NOTS),
                                // or a fold record: row | permit code | escape | reply position
                    const uint64_t rec = srec[q];
                    kl[r] = (uint32_t)rec & rmask;
                    pm[r] = (int32_t)((rec >> (G.on ? G.rb : F.kb)) & ((1ull << F.pb) - 1));
                } else {
                    kl[r] = skeys[q] & rmask;
                    pm[r] = sperm[q];
                }
                pend |= 1u << r;
            }
        }
        // a request's arrival index is read again where it queues or evicts (rare): not
        // held across the rounds (registers).  With fold records it is the payload of the
        // previous pass's record at the reply position.
        auto reply_pos = [&](uint32_t q) -> uint32_t {
            return G.on ? (uint32_t)((srec[q] >> (G.rb + G.pb + 1)) & ((1ull << G.pw) - 1)) : q;
        };
        auto arrival = [&](int r) -> uint32_t {
            const uint32_t q = c + r * kFoldBlock + tid;
            if (!PACKED) return sidx[q];
            return (uint32_t)((G.on ? rec0[reply_pos(q)] : srec[q]) >> (F.kb + F.pb + 1));
        };
        lds_dma_wait();    // (first chunk) this wave's slice DMA landed
        __syncthreads();
#if TBE_AFOLD_PREFETCH
        // as k_fold_wide: touch the local-tier slice and records of the workgroup
        // TBE_AFOLD_PREFETCH blocks later (same XCD); waited for at the write-back barrier
        if (c == s && e - s >= TBE_FOLD_PREFETCH_MIN) {
            const uint32_t fblk = blockIdx.x + TBE_AFOLD_PREFETCH;
            const uint32_t fb = fold_bucket_at(G, fblk);
            if (fblk < gridDim.x && (!G.on || fb < G.nb)) {
                const uint32_t fs = bstart[fb], fe = bstart[fb + 1];
                const uint64_t frow = (uint64_t)fb << r_bits;
                if (fe > fs && frow < n_keys) {
                    const uint32_t fn = (uint32_t)min<uint64_t>(R, n_keys - frow);
                    const uint32_t t = (uint32_t)tid;
                    if (t < kMaxRows / 8) {
                        if (t * 8u < fn) pf_sink = reinterpret_cast<const uint32_t *>(alocal + frow + t * 8u)[0];
                    } else if (PACKED) {
                        const uint32_t q = fs + (t - kMaxRows / 8) * 16u;
                        if (q < fe) pf_sink = (uint32_t)srec[q];
                    }
                }
            }
        }
#endif
        uint32_t mine = 0;
#pragma unroll
        for (int r = 0; r < kAPer; ++r) {
            if (pend & (1u << r)) {
                const uint32_t bit = 1u << (kl[r] & 31);
                if (!(atomicOr(&loaded[kl[r] >> 5], bit) & bit)) mine |= 1u << r;
            }
        }
        if (mine) {   // sparse buckets only (a dense slice is all loaded)
            ALocal tmp[kAPer];
#pragma unroll
            for (int r = 0; r < kAPer; ++r) {
                tmp[r] = ALocal{0, 0, 0, 0, 0u};
                if (mine & (1u << r)) tmp[r] = rows[kl[r]];
            }
#pragma unroll
            for (int r = 0; r < kAPer; ++r)
                if (mine & (1u << r)) sl[kl[r]] = tmp[r];
        }
        __syncthreads();
        for (uint32_t round = 1;; ++round) {
#pragma unroll
            for (int r = 0; r < kAPer; ++r)
                if (pend & (1u << r))
                    atomicMax(&own[kl[r]], (round << 12) | (4095u - (uint32_t)(r * kFoldBlock + tid)));
            __syncthreads();
#pragma unroll
            for (int r = 0; r < kAPer; ++r) {
                const uint32_t tag = (round << 12) | (4095u - (uint32_t)(r * kFoldBlock + tid));
                if (!((pend & (1u << r)) && own[kl[r]] == tag)) continue;
                pend &= ~(1u << r);
                ALocal a = sl[kl[r]];
                const int32_t p = pm[r];
                uint32_t status;
                bool modified = false, evaluated = true;
                const int32_t avail = avail_of(a);
                if (p > A.token_limit) {                                   // A:87-90 / A:119-122
                    status = TBE_WAIT_REJECTED;
                    evaluated = false;
                } else if (p == 0 && (avail > 0 || !A.wait)) {            // A:93-102 / A:127-130
                    status = (avail > 0) ? TBE_WAIT_GRANTED : TBE_WAIT_FAILED;
                } else if (p == 0) {
                    // WaitAsync(0) while throttled: TryLease fails (A:191, availableTokens
                    // != 0) and QueueLimit - _queueCount < 0 never holds (A:141), so the
                    // registration queues with Count 0 (A:166-181) and completes at the
                    // next drain that reaches it (A:474: AvailableTokens >= 0).  The
                    // reference bounds such registrations by nothing; the ring gives each
                    // key zero_slots of them, beyond which the wait fails.
                    if (a.zc < A.zero_slots) {
                        uint32_t head = a.hc & 0xFFFFu, cnt = a.hc >> 16;
                        uint32_t tail = head + cnt;
                        if (tail >= A.cap) tail -= A.cap;
                        ring[(row0 + kl[r]) * (uint64_t)A.cap + tail] = (uint64_t)(A.id_base + arrival(r)) << 16;
                        a.hc = (head & 0xFFFFu) | ((cnt + 1) << 16);
                        a.zc = (uint16_t)(a.zc + 1);
                        modified = true;
                        status = TBE_WAIT_QUEUED;
                    } else {
                        status = TBE_WAIT_FAILED;
                    }
                } else if (avail >= p && avail != 0 && (a.qsum == 0 || A.order == 1)) {  // A:191-209
                    a.local = (int32_t)((uint32_t)a.local + (uint32_t)p);
                    modified = true;
                    status = TBE_WAIT_GRANTED;
                } else if (!A.wait) {
                    status = TBE_WAIT_FAILED;                              // A:111
                } else {
                    uint32_t head = a.hc & 0xFFFFu, cnt = a.hc >> 16;
                    uint64_t *__restrict__ kr = ring + (row0 + kl[r]) * (uint64_t)A.cap;
                    bool fail = false;
                    if ((int64_t)A.queue_limit - a.qsum < p) {             // A:141
                        if (A.order == 1 && p <= A.queue_limit) {          // A:143-158
                            while ((int64_t)A.queue_limit - a.qsum < p) {
                                const uint64_t ent = kr[head];
                                const uint32_t at = atomicAdd(ev_count, 1u);
                                if (at < ev_cap) {
                                    ev_cause[at] = arrival(r) + A.ai_base;
                                    ev_id[at] = (int64_t)(ent >> 16);
                                }
                                a.qsum = (uint16_t)(a.qsum - (uint32_t)(ent & 0xFFFFu));
                                if ((ent & 0xFFFFu) == 0) a.zc = (uint16_t)(a.zc - 1);   // DequeueHead takes it too
                                head = (head + 1 == A.cap) ? 0 : head + 1;
                                --cnt;
                            }
                        } else {
                            fail = true;                                   // A:159-163
                        }
                    }
                    if (fail) {
                        status = TBE_WAIT_FAILED;
                    } else {                                               // A:166-181
                        uint32_t tail = head + cnt;
                        if (tail >= A.cap) tail -= A.cap;
                        kr[tail] = ((uint64_t)(A.id_base + arrival(r)) << 16) | (uint32_t)p;
                        ++cnt;
                        a.qsum = (uint16_t)(a.qsum + (uint32_t)p);
                        status = TBE_WAIT_QUEUED;
                    }
                    a.hc = (head & 0xFFFFu) | (cnt << 16);
                    modified = true;
                }
                rbuf[r * kFoldBlock + tid] = pack_wait(status, evaluated, (uint32_t)avail_of(a));
                if (modified) {
                    sl[kl[r]] = a;
                    atomicOr(&dirty[kl[r] >> 5], 1u << (kl[r] & 31));
                }
            }
#ifdef TBE_A_R1_ONLY
            pend = 0;   // A/B timing only (wrong replies): the cost of the rounds after round 1
#endif
            if (!__syncthreads_or(pend != 0)) break;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kAPer; ++r) {
            const uint32_t q = c + r * kFoldBlock + tid;
            if (q < e) {
                const uint32_t at = PACKED ? reply_pos(q) : q;
                if (rw == 2) reinterpret_cast<uint16_t *>(res)[at] = wait16(rbuf[r * kFoldBlock + tid]);
                else res[at] = rbuf[r * kFoldBlock + tid];
            }
        }
    }
    __syncthreads();
    for (uint32_t j = tid; j < nrows; j += kFoldBlock) {
        if (dense) {
            u32x4 v;
            __builtin_memcpy(&v, &sl[j], sizeof v);
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(rows + j));
        } else if (dirty[j >> 5] & (1u << (j & 31))) {
            rows[j] = sl[j];
        }
    }
#if TBE_AFOLD_PREFETCH
    if (n_keys == 0) res[s] = pf_sink;   // never (no engine has 0 keys): keeps the touches
#endif
}

// A:430-435: count = _localThrottleScore; _localThrottleScore = 0, for every key.
__global__ __launch_bounds__(kBlock) void k_approx_collect(uint64_t n_keys, ALocal *__restrict__ alocal,
                                                           int32_t *__restrict__ counts) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x; k < n_keys; k += stride) {
        counts[k] = alocal[k].local;
        alocal[k].local = 0;
    }
}

// One refresh epoch (A:412-508) for every key: replay the n_clients sync-script calls
// (A:241-270) in client order, client r at ts + r*stagger with count all[r][k], on this
// engine's replica of the global tier (every engine replays the same calls, so the
// replicas stay bit-identical); take client `my`'s reply (A:440-443: (int)v', and the
// period through Lua "%.14g" and double.Parse); then drain the queue (A:462-501).
__global__ __launch_bounds__(kBlock) void k_approx_sync(
    uint64_t n_keys, ALocal *__restrict__ alocal, AClient *__restrict__ aclient,
    double *__restrict__ gv, double *__restrict__ gp, int64_t *__restrict__ gt,
    const uint64_t *__restrict__ ring, AParams A, const int32_t *__restrict__ all_counts,
    uint32_t n_clients, uint32_t my, int64_t ts_us, int64_t stagger_us,
    uint64_t *__restrict__ log_keyseq, int64_t *__restrict__ log_id, int32_t *__restrict__ log_rem,
    uint32_t *__restrict__ log_count, uint32_t log_cap, uint32_t write_client) {
    // the sync times (TIME at A:241-242) of the first clients are the same for every key
    constexpr uint32_t kSyncTimes = 64;
    __shared__ ReqTime crq[kSyncTimes];
    if (threadIdx.x < min(n_clients, kSyncTimes))
        crq[threadIdx.x] = req_time(ts_us + (int64_t)threadIdx.x * stagger_us, kApproxTtlMs);
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x; k < n_keys; k += stride) {
        // all_counts == nullptr: one client that collects here (A:430-435 fused into the
        // epoch: the local count is swapped to 0 and used as this client's count)
        ALocal a = alocal[k];
        const int32_t own = a.local;
        if (!all_counts) a.local = 0;
        double v = gv[k], p = gp[k];
        int64_t t = gt[k];
        int32_t my_global = 0;
        double my_period = 0.0;
        for (uint32_t r = 0; r < n_clients; ++r) {
            const int64_t ts = ts_us + (int64_t)r * stagger_us;
            const ReqTime rq = r < kSyncTimes ? crq[r] : req_time(ts, kApproxTtlMs);   // A:241-242
            const bool present = (t != kAbsent) && !(t < rq.exp_lt);          // EXPIRE 86400 (A:268)
            const double pv = present ? v : 0.0;                              // A:247-252
            const double pp = present ? p : 0.0;
            const double pt = present ? new_t_of(t) : rq.new_t;
            const double dt = lua_max(0.0, rq.new_t - pt);                    // A:255
            const double decay = dt * A.decay_rate;
            const double nv = lua_max(0.0, pv - decay) +
                              (double)(all_counts ? all_counts[(uint64_t)r * n_keys + k] : own);   // A:258
            const double a8 = pp * 0.8;                                       // A:262
            const double b2 = dt * 0.2;
            const double np = a8 + b2;
            v = nv;                                                           // A:265
            p = np;
            t = ts;
            if (r == my) {
                my_global = (int32_t)(int64_t)nv;                             // A:270 -> A:441
                my_period = round_trip_14g(np);                               // A:270 -> A:442
            }
        }
        gv[k] = v;
        gp[k] = p;
        gt[k] = t;
        // A:443: Math.Max(1, Math.Round(P / period)); P / 0 = +inf
        const double q = A.period_s / my_period;
        const double rnd = __builtin_rint(q);
        const double est = (rnd != rnd) ? rnd : (rnd > 1.0 ? rnd : 1.0);
        // The client view {est, global} only answers queries (the lease path reads the cap
        // derived from it).  With one client it is a function of the tier row just written
        // (k_aclient_derive), so it is derived when asked for instead of written here: 16 of
        // the 96 bytes per key of config E's refresh (round 6).
        if (write_client) {
            AClient ac;
            ac.est = est;
            ac.global = my_global;
            ac.pad = 0;
            aclient[k] = ac;
        }
        const double lim = (double)wrap_sub(A.token_limit, my_global) / est;
        a.cap = dotnet_to_int(__builtin_ceil(lim));
        // drain (A:467-501)
        uint32_t head = a.hc & 0xFFFFu, cnt = a.hc >> 16, seq = 0;
        const uint64_t *__restrict__ kr = ring + k * (uint64_t)A.cap;
        while (cnt > 0) {
            uint32_t idx = head;
            if (A.order == 1) {
                idx = head + cnt - 1;
                if (idx >= A.cap) idx -= A.cap;
            }
            const uint64_t ent = kr[idx];
            const int32_t c = (int32_t)(ent & 0xFFFFu);
            if (avail_of(a) < c) break;                                  // A:474 (Count 0: always)
            a.qsum = (uint16_t)(a.qsum - (uint32_t)c);
            if (c == 0) a.zc = (uint16_t)(a.zc - 1);
            a.local = (int32_t)((uint32_t)a.local + (uint32_t)c);
            if (A.order == 0) head = (head + 1 == A.cap) ? 0 : head + 1;
            --cnt;
            const uint32_t at = atomicAdd(log_count, 1u);
            if (at < log_cap) {
                log_keyseq[at] = (k << 16) | seq;
                log_id[at] = (int64_t)(ent >> 16);
                log_rem[at] = avail_of(a);
            }
            ++seq;
        }
        a.hc = (head & 0xFFFFu) | (cnt << 16);
        alocal[k] = a;
    }
}

// The client view of keys [first, first + count) after a one-client sync: exactly what
// k_approx_sync computes for r == my when the client's sync is the last (A:441-443).
__global__ __launch_bounds__(kBlock) void k_aclient_derive(uint64_t first, uint64_t count, const double *__restrict__ gv,
                                                           const double *__restrict__ gp, AClient *__restrict__ aclient,
                                                           double period_s) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < count; i += (uint64_t)gridDim.x * kBlock) {
        const uint64_t k = first + i;
        const int32_t my_global = (int32_t)(int64_t)gv[k];
        const double my_period = round_trip_14g(gp[k]);
        const double q = period_s / my_period;
        const double rnd = __builtin_rint(q);
        AClient ac;
        ac.est = (rnd != rnd) ? rnd : (rnd > 1.0 ? rnd : 1.0);
        ac.global = my_global;
        ac.pad = 0;
        aclient[k] = ac;
    }
}

__global__ void k_init_approx(uint64_t n_keys, ALocal *__restrict__ alocal, AClient *__restrict__ aclient,
                              double *__restrict__ gv, double *__restrict__ gp, int64_t *__restrict__ gt,
                              int32_t token_limit) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_keys; k += stride) {
        alocal[k] = ALocal{token_limit, 0, 0, 0, 0u};  // global 0, est 1 -> cap = TokenLimit
        aclient[k] = AClient{1.0, 0, 0};
        gv[k] = 0.0;
        gp[k] = 0.0;
        gt[k] = kAbsent;
    }
}

__global__ void k_init_table(Slot *__restrict__ table, uint64_t n_keys, double cap) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = i; k < n_keys; k += stride) table[k] = Slot{cap, kAbsent};
}

__global__ void k_sticky(const uint32_t *__restrict__ err, uint32_t *__restrict__ sticky) {
    if (threadIdx.x == 0 && *err) *sticky = 1u;
}

// Entries in all queues: qhdr count bits (queueing kind) or ALocal.hc count bits
// (approximate kind).  Re-establishes the host's count after device-pointer batches.
template <typename HW>
__global__ __launch_bounds__(kBlock) void k_count_queued(uint64_t n_keys, const HW *__restrict__ qhdr,
                                                        const ALocal *__restrict__ alocal,
                                                        unsigned long long *__restrict__ out) {
    __shared__ unsigned long long part[kBlock / 64];
    unsigned long long c = 0;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x; k < n_keys; k += stride)
        c += qhdr ? ((qh_widen(qhdr[k]) >> 16) & 0xFFFFu) : ((alocal[k].hc >> 16) & 0xFFFFu);
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += part[w];
        if (t) atomicAdd(out, t);
    }
}

// ----------------------------------------------------------------------------- host side
enum Stage { ST_HIST = 0, ST_COLSCAN, ST_SCATTER, ST_BOUNDS, ST_FOLD, ST_UNSCATTER, ST_HOT, ST_COUNT };

struct PassBufs {
    uint64_t *rec = nullptr;     // pass output, packed records (token bucket, PackFmt)
    uint32_t *keys = nullptr;    // pass output (u32 keys)
    int32_t *permits = nullptr;
    int64_t *ts = nullptr;
    uint32_t *idx = nullptr;     // arrival index (queueing kind only)
    uint32_t *perm = nullptr;    // output position of each input element of the pass
    uint32_t *tileprefix = nullptr;
    uint32_t *blockprefix = nullptr;
    uint32_t *digit_total = nullptr;
};

// Everything one batch owns while it is in flight: the partition passes' output, the
// replies before unscatter, the bucket starts and the batch's error flag.  A token-bucket
// engine keeps two, so batch b+1 can be partitioned while batch b is folded.
struct Workspace {
    uint64_t cap_n = 0;
    std::vector<PassBufs> pass;
    uint32_t *blocksum = nullptr;
    uint32_t *res[2] = {nullptr, nullptr};
    uint32_t *bstart = nullptr;
    uint32_t *bcount = nullptr;   // requests per bucket of the batch
    uint32_t *dlist = nullptr;    // sparse batches: count + ids of the dense buckets (k_bscan)
    unsigned long long *bsflags = nullptr;   // k_bscan_lb's published totals (tagged per launch)
    uint32_t bs_tag = 0;          // tag of bsflags' last k_bscan_lb launch (0: the zeroed state)
    bool bs_fresh = false;        // bsflags just allocated: zeroed on the batch's stream first
    uint8_t *dig0 = nullptr;      // each request's pass-0 digit (k_unrank re-ranks from it)
    uint8_t *dig1 = nullptr;      // pass 1's digit of pass 0's output, in that order (k_hist_dig)
    int64_t *ts0 = nullptr;       // narrow pass-0 records: escaped requests' times at their pass-0 position
    uint32_t *err = nullptr;      // the batch's invalid-request flag
    hipEvent_t hot_done = nullptr;   // pipelined: k_hot_update of the last batch on this workspace
    bool hot_pending = false;
    uint32_t *segbase = nullptr;  // hot runs
    SegSummary *summ = nullptr;
    SegState *sst = nullptr;
    hipEvent_t done = nullptr;    // recorded after the batch's last kernel
    bool used = false;
};

inline int ceil_log2(uint64_t x) {
    int b = 0;
    while ((1ull << b) < x) ++b;
    return b;
}

}  // namespace

struct tbe_engine {
    tbe_config cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    TbParams params{};
    int r_bits = 0;          // bucket = key >> r_bits
    uint32_t nbuckets = 0;   // ceil(n_keys / 2^r_bits)
    int passes = 0;          // 8-bit LSD passes over the bucket id
    bool packed = false;     // token bucket and queueing kinds: passes move packed u64 records (PackFmt)
    bool narrow = false;     // one-byte replies: token bucket (packed, TokenLimit <= 127, put_reply),
                             // queueing kind (TokenLimit <= 62, put_wait)
    bool medium = false;     // two-byte replies: queueing and approximate kinds, TokenLimit <= 16382
    // reply width code of the wait kinds' folds (put_wait): 1, 2 or 4 (as 0) bytes
    uint32_t wait_rw() const { return narrow ? 1u : (medium ? 2u : 0u); }
    PackFmt pf{};
    // fold records (FoldFmt): the last of >= 2 passes writes them, the fold and the hot runs
    // put each reply straight into the previous pass's order, and that pass's un-partition
    // and permutation disappear (token bucket, packed; TBE_FLAG_UNSCATTER_ALL turns it off)
    bool foldrec = false;
    // k_unrank (TBE_FLAG_RERANK, A/B): the final un-partition recomputes pass 0's positions
    // from one-byte digits, so pass 0 writes no permutation (packed records)
    bool unrank = false;
    // digit stream (packed, 2 passes): pass 0 also writes each request's pass-1 digit as a
    // byte in its output order, and pass 1's histogram (k_hist_dig) reads 1 byte per
    // request instead of 8 (TBE_FLAG_HIST_RECORDS: off)
    bool dig1 = false;
    // narrow pass-0 records (PackFmt::n0): token bucket, packed, two passes, fold records and
    // the digit stream, and at least 8 time-offset bits left in 32
    bool n0 = false;
    // hot runs (token bucket, packed): bucket ids [nbuckets, nb_total) belong to hot keys.
    // Batch b is partitioned by hot[b % 3] and nominates into hot[(b + 2) % 3], so the set
    // batch b+1 is partitioned by was complete before batch b's fold began.
    uint32_t hot_cap = 0;
    uint32_t nb_total = 0;
    HotSet *hot[3] = {nullptr, nullptr, nullptr};
    uint64_t nbatch = 0;
    Slot *table = nullptr;
    // queueing kind
    QParams qp{};
    uint64_t *qhdr = nullptr;      // per-key queue header (32-bit words when qh32: qh_store)
    bool qh32 = false;             // queue headers stored 32 bits wide (QueueLimit <= kQh32MaxLimit)
    uint64_t *ring = nullptr;      // per-key rings of qp.cap entries
    uint64_t queued_total = 0;     // entries in all queues (host-side count)
    // After a device-pointer wait batch or drain the host cannot see how many entries
    // were queued or drained: queued_total is then an upper bound (queued_exact false)
    // until a host-buffer call recounts the queues on the device (sync_queued).
    bool queued_exact = true;
    bool ev_pending = false;       // the eviction log of a device wait batch is unread
    unsigned long long *qcount = nullptr;
    uint32_t *ev_cause = nullptr;  // eviction log of the last wait batch
    int64_t *ev_id = nullptr;
    uint64_t ev_cap = 0;
    uint64_t *log_keyseq = nullptr;  // refresh grant log
    int64_t *log_id = nullptr;
    int32_t *log_rem = nullptr;
    uint64_t log_cap = 0;
    uint32_t *counters = nullptr;  // [0] eviction count, [1] refresh log count
    // approximate kind
    AParams ap{};
    ALocal *alocal = nullptr;
    AClient *aclient = nullptr;
    bool aclient_lazy = false;    // the last sync had one client: aclient is derived on demand
    double *gv = nullptr, *gp = nullptr;
    int64_t *gt = nullptr;
    int32_t *acounts = nullptr;   // tbe_approx_refresh's own count buffer (single client)
    int wait_mode = 1;
    QTick qtick{-1, nullptr, nullptr, nullptr, nullptr, 0};   // tbe_wait_batch_tick_device
    std::vector<std::pair<uint64_t, int64_t>> evicted;              // (cause, id), sorted
    std::vector<std::tuple<uint64_t, int64_t, int32_t>> drained;     // (key, id, rem)

    // Batch workspaces.  Pipelined (token bucket): batch b uses ws[b % 2]; its partition
    // passes run on `pstream`, its fold, hot runs and unscatter on `stream`, so the next
    // batch's partition overlaps this batch's fold.  Other kinds use ws[0] on one stream.
    Workspace ws[2];
    int ws_cur = 0;
    bool pipeline = false;
    hipStream_t pstream = nullptr;
    hipStream_t hstream = nullptr;   // pipelined with hot runs: k_hot_update
    hipEvent_t ev_in = nullptr, ev_part = nullptr, ev_out = nullptr, ev_hot = nullptr;
    uint32_t *sticky = nullptr;      // set by any skipped batch until tbe_synchronize reads it
    uint32_t *last_err = nullptr;    // the error flag of the last enqueued batch
    // host-buffer path staging
    hipStream_t cin = nullptr, cout = nullptr;   // chunked pinned path: copy-in / copy-out streams
    hipStream_t cin2 = nullptr;                  // second copy-in stream (TBE_CIN_STREAMS == 2)
    std::vector<hipEvent_t> ev_chunk2;
    std::vector<hipEvent_t> ev_chunk;            // per-chunk copy-in done
    uint64_t stage_cap = 0;
    uint64_t *d_keys = nullptr;
    int32_t *d_permits = nullptr;
    int64_t *d_ts = nullptr;
    uint8_t *d_granted = nullptr;
    int32_t *d_remaining = nullptr;

    // Stage timing (TBE_FLAG_STAGE_TIMING): an event pair per stage per batch, recorded
    // on the launch stream without any host synchronisation; read in tbe_stage_times.
    bool timing = false;
    uint32_t timing_mask = 0;   // stages that record events (bit s: stage s)
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    std::vector<std::pair<int, size_t>> ev_marks;   // (stage, index of start event)
    int open_stage = -1;
    std::string last_error = "ok";
};

// Calls f with the queue headers typed by their stored width (uint32_t* or uint64_t*).
template <typename F>
static void with_qhdr(tbe_engine *e, F &&f) {
    if (e->qh32) f(reinterpret_cast<uint32_t *>(e->qhdr));
    else f(e->qhdr);
}

namespace {

tbe_status fail(tbe_engine *e, tbe_status st, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (e) e->last_error = buf;
    return st;
}

#define HIP_TRY(e, expr)                                                                    \
    do {                                                                                    \
        hipError_t _rc = (expr);                                                            \
        if (_rc != hipSuccess)                                                              \
            return fail((e), _rc == hipErrorOutOfMemory ? TBE_ENOMEM : TBE_EDEVICE,         \
                        "%s failed: %s", #expr, hipGetErrorString(_rc));                    \
    } while (0)

template <typename T>
void dfree(T *&p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

void free_workspace(Workspace &w) {
    if (w.used && w.done) (void)hipEventSynchronize(w.done);   // its last batch has finished
    if (w.hot_pending && w.hot_done) (void)hipEventSynchronize(w.hot_done);
    w.hot_pending = false;
    for (auto &pb : w.pass) {
        dfree(pb.rec);
        dfree(pb.keys);
        dfree(pb.permits);
        dfree(pb.ts);
        dfree(pb.idx);
        dfree(pb.perm);
        dfree(pb.tileprefix);
        dfree(pb.blockprefix);
        dfree(pb.digit_total);
    }
    w.pass.clear();
    dfree(w.blocksum);
    dfree(w.summ);
    dfree(w.sst);
    dfree(w.segbase);
    dfree(w.res[0]);
    dfree(w.res[1]);
    dfree(w.bstart);
    dfree(w.bcount);
    w.err = nullptr;   // (the word after the bucket counts)
    w.dlist = nullptr;   // (after err)
    dfree(w.bsflags);
    dfree(w.dig0);
    dfree(w.dig1);
    dfree(w.ts0);
    w.cap_n = 0;
    w.used = false;
}

void free_staging(tbe_engine *e) {
    dfree(e->d_keys);
    dfree(e->d_permits);
    dfree(e->d_ts);
    dfree(e->d_granted);
    dfree(e->d_remaining);
    e->stage_cap = 0;
}

void tiles_for(uint64_t n, uint32_t &ntiles, uint32_t &nblk, uint32_t &tpb) {
    ntiles = (uint32_t)((n + kTile - 1) / kTile);
    tpb = (ntiles + kMaxHistBlocks - 1) / kMaxHistBlocks;
    if (tpb == 0) tpb = 1;
    nblk = (ntiles + tpb - 1) / tpb;
}

tbe_status ensure_workspace(tbe_engine *e, Workspace &w, uint64_t n) {
    if (n <= w.cap_n) return TBE_OK;
    free_workspace(w);
    uint64_t cap = std::max<uint64_t>(n, 1u << 16);
    uint32_t ntiles, nblk, tpb;
    tiles_for(cap, ntiles, nblk, tpb);
    w.pass.resize(e->passes);
    for (auto &pb : w.pass) {
        if (e->packed) {
            HIP_TRY(e, hipMalloc(&pb.rec, cap * sizeof(uint64_t)));
        } else {
            HIP_TRY(e, hipMalloc(&pb.keys, cap * sizeof(uint32_t)));
            HIP_TRY(e, hipMalloc(&pb.permits, cap * sizeof(int32_t)));
            HIP_TRY(e, hipMalloc(&pb.ts, cap * sizeof(int64_t)));
        }
        HIP_TRY(e, hipMalloc(&pb.perm, cap * sizeof(uint32_t)));
        if (e->cfg.kind != TBE_KIND_TOKEN_BUCKET) HIP_TRY(e, hipMalloc(&pb.idx, cap * sizeof(uint32_t)));
        HIP_TRY(e, hipMalloc(&pb.tileprefix, (uint64_t)ntiles * kDigits * sizeof(uint32_t)));
        HIP_TRY(e, hipMalloc(&pb.blockprefix, (uint64_t)kMaxHistBlocks * kDigits * sizeof(uint32_t)));
        HIP_TRY(e, hipMalloc(&pb.digit_total, kDigits * sizeof(uint32_t)));
    }
    HIP_TRY(e, hipMalloc(&w.blocksum, (uint64_t)kMaxHistBlocks * kDigits * sizeof(uint32_t)));
    if (e->hot_cap) {
        const uint64_t segs = cap / kSeg + kHotKeysMax + 1;
        HIP_TRY(e, hipMalloc(&w.summ, segs * sizeof(SegSummary)));
        HIP_TRY(e, hipMalloc(&w.sst, segs * sizeof(SegState)));
        HIP_TRY(e, hipMalloc(&w.segbase, (kHotKeysMax + 1) * sizeof(uint32_t)));
    }
    HIP_TRY(e, hipMalloc(&w.res[0], cap * sizeof(uint32_t)));
    HIP_TRY(e, hipMalloc(&w.res[1], cap * sizeof(uint32_t)));
    HIP_TRY(e, hipMalloc(&w.bstart, ((uint64_t)e->nb_total + 1) * sizeof(uint32_t)));
    // the batch's error flag is the word after its bucket counts and the dense-bucket list
    // (sparse batches) follows it: one memset clears the counts, the flag and the list's count
    HIP_TRY(e, hipMalloc(&w.bcount, ((uint64_t)e->nb_total + 2 + e->nbuckets) * sizeof(uint32_t)));
    w.err = w.bcount + e->nb_total;
    w.dlist = w.bcount + e->nb_total + 1;
    // k_bscan_lb's flags are zeroed on the stream of the first batch that uses them
    // (run_batch), not with a device-wide synchronisation here
    HIP_TRY(e, hipMalloc(&w.bsflags, kBsMaxBlocks * sizeof(unsigned long long)));
    w.bs_fresh = true;
    w.bs_tag = 0;
    if (e->unrank) HIP_TRY(e, hipMalloc(&w.dig0, cap));
    if (e->dig1) HIP_TRY(e, hipMalloc(&w.dig1, cap));
    if (e->n0 && e->cfg.kind != TBE_KIND_APPROXIMATE) HIP_TRY(e, hipMalloc(&w.ts0, cap * sizeof(int64_t)));
    w.cap_n = cap;
    return TBE_OK;
}

tbe_status ensure_host_staging(tbe_engine *e, uint64_t n) {
    // Staging for the host-buffer entry points (each such call synchronises before it returns).
    if (n <= e->stage_cap) return TBE_OK;
    free_staging(e);
    const uint64_t cap = std::max<uint64_t>(n, 1u << 16);
    HIP_TRY(e, hipMalloc(&e->d_keys, cap * sizeof(uint64_t)));
    HIP_TRY(e, hipMalloc(&e->d_permits, cap * sizeof(int32_t)));
    HIP_TRY(e, hipMalloc(&e->d_ts, cap * sizeof(int64_t)));
    HIP_TRY(e, hipMalloc(&e->d_granted, cap * sizeof(uint8_t)));
    HIP_TRY(e, hipMalloc(&e->d_remaining, cap * sizeof(int32_t)));
    e->stage_cap = cap;
    return TBE_OK;
}

hipEvent_t next_event(tbe_engine *e) {
    if (e->ev_used == e->ev_pool.size()) {
        hipEvent_t ev = nullptr;
        if (hipEventCreate(&ev) != hipSuccess) return nullptr;
        e->ev_pool.push_back(ev);
    }
    return e->ev_pool[e->ev_used++];
}
inline void stage_begin(tbe_engine *e, int s, hipStream_t st) {
    if (!e->timing || !((e->timing_mask >> s) & 1u)) return;
    const size_t idx = e->ev_used;
    hipEvent_t a = next_event(e), b = next_event(e);
    if (!a || !b) return;
    (void)hipEventRecord(a, st);
    e->ev_marks.emplace_back(s, idx);
    (void)b;
}
inline void stage_end(tbe_engine *e, int s, hipStream_t st) {
    if (!e->timing || e->ev_marks.empty() || e->ev_marks.back().first != s) return;
    (void)hipEventRecord(e->ev_pool[e->ev_marks.back().second + 1], st);
}

// The token-bucket fold's density gate (see kWideMinShift): k_fold_wide takes the buckets
// of at least the returned number of requests, k_fold_sparse the rest (a sparse batch: the
// returned number is above 1).  Dense batches give every nonempty bucket to k_fold_wide;
// sparse ones only the buckets of >= R/8 requests.
#ifndef TBE_SPARSE_GATE_SHIFT
#define TBE_SPARSE_GATE_SHIFT 3              // sparse batch: fewer than R >> this requests per bucket
#endif
uint32_t fold_wide_min(const tbe_engine *e, uint64_t n) {
    const uint32_t R = 1u << e->r_bits;
    const uint32_t all = std::max(1u, R >> kWideMinShift);
    if (n >= (uint64_t)e->nbuckets * std::max(1u, R >> TBE_SPARSE_GATE_SHIFT)) return all;
    return std::max(all, R >> 3);
}

#ifndef TBE_HOT_SPARSE_MIN_LOG2
#define TBE_HOT_SPARSE_MIN_LOG2 20           // sparse batches below 2^this take no hot-key runs
#endif
// Run slots the per-batch sampler keeps free of fold nominations (k_hot_sample)
inline uint32_t hot_reserve_host(uint32_t cap) { return std::min(32u, cap / 4u); }

// Fold records for a batch of n requests: the reply position takes ceil_log2(n) bits, the
// time offset what is left (>= 8 bits, else the plain records).  tbe_batch_format reports it.
FoldFmt batch_fold_fmt(const tbe_engine *e, uint64_t n) {
    FoldFmt G{};
    if (!e->foldrec) return G;
    const bool approx = e->cfg.kind == TBE_KIND_APPROXIMATE;
    const int pw = std::max(1, ceil_log2(n));
    const int tw = 64 - e->r_bits - e->pf.pb - 1 - pw;
    if (tw >= (approx ? 1 : 8)) {   // (the approximate kind's records carry no time)
        G.on = 1;
        // approximate kind: narrow pass-0 records only in batches that cannot queue, whose
        // fold never reads an arrival index (k_fold_a's arrival())
        G.n0 = (e->n0 && !(approx && e->wait_mode)) ? 1 : 0;
        G.rb = e->r_bits;
        G.pb = e->pf.pb;
        G.pw = pw;
        G.tw = tw;
        G.nb = e->nbuckets;
        G.region_bits = (uint32_t)(kDigitBits * (e->passes - 1));
        G.n_hi = (uint32_t)(((uint64_t)e->nbuckets + (1ull << G.region_bits) - 1) >> G.region_bits);
    }
    return G;
}

// Enqueue the whole pipeline for one device-resident batch.  `caller` is the stream the
// inputs were produced on and the replies are awaited on; NULL: the inputs are complete
// at the call and the replies are ordered on the engine's stream.
//
// Pipelined engines (token bucket) split a batch over two streams: the partition passes
// and the bucket starts run on pstream (sp), the fold, hot runs and unscatter, the only
// kernels that touch the table, on the engine's stream (sf).  Batch b+1's partition then
// runs while batch b is folded: it reads only its inputs, its own workspace (free once
// batch b-1 is done) and hot[(b+1) % 3] (complete since batch b-1's hot update).
tbe_status run_batch(tbe_engine *e, const uint64_t *keys, const int32_t *permits,
                     const int64_t *ts, uint64_t n, uint8_t *granted, int32_t *remaining,
                     hipStream_t caller, int64_t id_base = 0, hipEvent_t in_ready = nullptr,
                     hipStream_t out_stream = nullptr, uint32_t ai_base = 0) {
    const bool approx = e->cfg.kind == TBE_KIND_APPROXIMATE;
    const bool wait = e->cfg.kind != TBE_KIND_TOKEN_BUCKET;   // status-packed replies
    if (n == 0) return TBE_OK;
    if (n >= (1ull << 32)) return fail(e, TBE_EINVAL, "batch of %llu requests exceeds 2^32-1",
                                       (unsigned long long)n);
    if (e->packed && !approx && !ts) return fail(e, TBE_EINVAL, "null timestamps");
    const bool pipe = e->pipeline;
    Workspace &w = e->ws[pipe ? e->ws_cur : 0];
    tbe_status rc = ensure_workspace(e, w, n);
    if (rc != TBE_OK) return rc;
    uint32_t ntiles, nblk, tpb;
    tiles_for(n, ntiles, nblk, tpb);
    hipStream_t sf = caller ? caller : e->stream, sp = sf;
    if (pipe) {
        sf = e->stream;
        sp = e->pstream;
        if (in_ready) {               // chunked host-buffer path: this chunk's copy-in
            HIP_TRY(e, hipStreamWaitEvent(sp, in_ready, 0));
        } else if (caller) {
            HIP_TRY(e, hipEventRecord(e->ev_in, caller));
            HIP_TRY(e, hipStreamWaitEvent(sp, e->ev_in, 0));
        }
        if (w.used) HIP_TRY(e, hipStreamWaitEvent(sp, w.done, 0));
        if (w.hot_pending) HIP_TRY(e, hipStreamWaitEvent(sp, w.hot_done, 0));   // this batch's hot set
    } else if (in_ready) {            // chunked host-buffer path (queueing / approximate)
        HIP_TRY(e, hipStreamWaitEvent(sf, in_ready, 0));
    }
    HIP_TRY(e, hipMemsetAsync(w.bcount, 0, ((uint64_t)e->nb_total + 2) * sizeof(uint32_t), sp));   // + err, dlist[0]
    if (w.bs_fresh) {
        HIP_TRY(e, hipMemsetAsync(w.bsflags, 0, kBsMaxBlocks * sizeof(unsigned long long), sp));
        w.bs_fresh = false;
    }

    const uint64_t kmask = e->packed ? e->pf.kmask : ~0ull;
    const FoldFmt G = batch_fold_fmt(e, n);
    // narrow pass-0 records only with this batch's fold records; the folds then find an
    // escaped request's time in ts0 (FoldFmt::n0)
    PackFmt pf = e->pf;
    pf.n0 = G.n0;
    const uint64_t *rec0 = G.on ? (G.n0 ? reinterpret_cast<const uint64_t *>(w.ts0) : w.pass[e->passes - 2].rec)
                                : nullptr;
    const bool unrank = e->unrank;
    const unsigned fold_grid = G.on ? (unsigned)((1ull << G.region_bits) * G.n_hi) : e->nbuckets;
    // token bucket: a sparse batch's dense buckets are listed for k_fold_wide, the rest go to
    // one wave each (k_fold_sparse)
    const uint32_t tb_wmin = (!approx && !wait) ? fold_wide_min(e, n) : 1u;
    const bool sparse_tb = tb_wmin > 1u;
    // hot runs: see tbe_engine::hot.  Not in a sparse batch below 2^20 requests (the
    // micro-batch regime): there a key busy enough to matter fills one dense bucket, which
    // k_fold_wide takes whole, and the hot machinery (the sampler, four launches) costs more
    // than it saves -- uniform 2^18: 0.10 ms per batch without, Zipf 2^20: 0.44 with against
    // 0.68 without (profiles/r05q_ablate_hot_sparse.log).  Which keys are hot never changes
    // a decision; the hot sets keep their contents for the next batch that runs them.
    const bool hot_on = e->hot_cap && !(sparse_tb && n < (1ull << TBE_HOT_SPARSE_MIN_LOG2));
    HotSet *hot = hot_on ? e->hot[e->nbatch % 3] : nullptr;
    HotSet *hot_next = hot_on ? e->hot[(e->nbatch + 2) % 3] : nullptr;
    // every batch: its dominant keys join its own hot set (k_hot_sample)
    if (hot && n >= kHotSampleMin) k_hot_sample<<<1, 1024, 0, sp>>>(keys, n, e->cfg.n_keys, hot, e->hot_cap);
    for (int p = 0; p < e->passes; ++p) {
        const int shift = e->r_bits + kDigitBits * p;
        PassBufs &out = w.pass[p];
        stage_begin(e, ST_HIST, sp);
        // the last pass also counts requests per bucket (k_bscan turns them into bstart)
        uint32_t *bc = (p == e->passes - 1) ? w.bcount : nullptr;
        const int lowbits = kDigitBits * p;
        uint8_t *dig = (p == 0 && unrank) ? w.dig0 : nullptr;
        uint8_t *dnext = (p == 0 && e->dig1) ? w.dig1 : nullptr;   // pass 1's digits (k_hist_dig)
        if (p == 0 && hot)
            k_hist<uint64_t, true><<<nblk, kHBlock, 0, sp>>>(keys, n, shift, tpb, ntiles, out.tileprefix,
                                                             w.blocksum, e->cfg.n_keys, w.err, 1, kmask,
                                                             hot, e->nbuckets, e->r_bits, bc, lowbits,
                                                             e->nb_total, dig);
        else if (p == 0)
            k_hist<uint64_t><<<nblk, kHBlock, 0, sp>>>(keys, n, shift, tpb, ntiles, out.tileprefix,
                                                       w.blocksum, e->cfg.n_keys, w.err, 1, kmask,
                                                       nullptr, e->nbuckets, e->r_bits, bc, lowbits,
                                                       e->nb_total, dig);
        else if (e->dig1 && p == 1)
            k_hist_dig<<<nblk, kHBlock, 0, sp>>>(w.dig1, n, tpb, ntiles, out.tileprefix, w.blocksum,
                                                 w.pass[0].digit_total, bc, e->nb_total);
        else if (e->packed)
            k_hist<uint64_t><<<nblk, kHBlock, 0, sp>>>(w.pass[p - 1].rec, n, shift, tpb, ntiles,
                                                       out.tileprefix, w.blocksum, e->cfg.n_keys,
                                                       w.err, 0, kmask, nullptr, e->nbuckets,
                                                       e->r_bits, bc, lowbits, e->nb_total);
        else
            k_hist<uint32_t><<<nblk, kHBlock, 0, sp>>>(w.pass[p - 1].keys, n, shift, tpb, ntiles,
                                                       out.tileprefix, w.blocksum, e->cfg.n_keys,
                                                       w.err, 0, kmask, nullptr, e->nbuckets,
                                                       e->r_bits, bc, lowbits, e->nb_total);
        stage_end(e, ST_HIST, sp);
        stage_begin(e, ST_COLSCAN, sp);
        k_colscan<<<kDigits, kBlock, 0, sp>>>(w.blocksum, nblk, out.blockprefix, out.digit_total);
        stage_end(e, ST_COLSCAN, sp);
        stage_begin(e, ST_SCATTER, sp);
        if (e->packed && approx && p == 0)
            k_scatter_rec<true, false, false, true><<<ntiles, kPartBlock, 0, sp>>>(
                keys, permits, nullptr, nullptr, n, shift, pf, out.tileprefix, out.blockprefix,
                out.digit_total, tpb, out.rec, unrank ? nullptr : out.perm, w.err, nullptr, 0, 0, nullptr,
                nullptr, FoldFmt{}, dnext);
        else if (e->packed && approx && G.on && p == e->passes - 1)
            k_scatter_rec<false, false, false, false, true><<<ntiles, kPartBlock, 0, sp>>>(
                nullptr, nullptr, nullptr, w.pass[p - 1].rec, n, shift, pf, out.tileprefix,
                out.blockprefix, out.digit_total, tpb, out.rec, nullptr, w.err, nullptr, 0, 0, nullptr,
                nullptr, G, nullptr, w.dig1);
        else if (e->packed && approx)
            k_scatter_rec<false><<<ntiles, kPartBlock, 0, sp>>>(
                nullptr, nullptr, nullptr, w.pass[p - 1].rec, n, shift, e->pf, out.tileprefix,
                out.blockprefix, out.digit_total, tpb, out.rec, out.perm, w.err);
        else if (e->packed && wait && p == 0)
            k_scatter_rec<true, false, true><<<ntiles, kPartBlock, 0, sp>>>(
                keys, permits, ts, nullptr, n, shift, pf, out.tileprefix, out.blockprefix,
                out.digit_total, tpb, out.rec, unrank ? nullptr : out.perm, w.err, nullptr, 0, 0, nullptr, out.idx,
                FoldFmt{}, dnext, nullptr, w.ts0);
        else if (e->packed && wait && G.on && p == e->passes - 1)
            k_scatter_rec<false, false, true, false, true><<<ntiles, kPartBlock, 0, sp>>>(
                nullptr, nullptr, ts, w.pass[p - 1].rec, n, shift, pf, out.tileprefix,
                out.blockprefix, out.digit_total, tpb, out.rec, nullptr, w.err, nullptr, 0, 0,
                w.pass[p - 1].idx, out.idx, G, nullptr, w.dig1);
        else if (e->packed && wait)
            k_scatter_rec<false, false, true><<<ntiles, kPartBlock, 0, sp>>>(
                nullptr, nullptr, nullptr, w.pass[p - 1].rec, n, shift, e->pf, out.tileprefix,
                out.blockprefix, out.digit_total, tpb, out.rec, out.perm, w.err, nullptr, 0, 0,
                w.pass[p - 1].idx, out.idx);
        else if (e->packed && p == 0 && hot)
            k_scatter_rec<true, true><<<ntiles, kPartBlock, 0, sp>>>(
                keys, permits, ts, nullptr, n, shift, pf, out.tileprefix, out.blockprefix,
                out.digit_total, tpb, out.rec, unrank ? nullptr : out.perm, w.err, hot, e->nbuckets, e->r_bits,
                nullptr, nullptr, FoldFmt{}, dnext, nullptr, w.ts0);
        else if (e->packed && p == 0)
            k_scatter_rec<true><<<ntiles, kPartBlock, 0, sp>>>(
                keys, permits, ts, nullptr, n, shift, pf, out.tileprefix, out.blockprefix,
                out.digit_total, tpb, out.rec, unrank ? nullptr : out.perm, w.err, nullptr, 0, 0, nullptr,
                nullptr, FoldFmt{}, dnext, nullptr, w.ts0);
        else if (e->packed && G.on && p == e->passes - 1)
            k_scatter_rec<false, false, false, false, true><<<ntiles, kPartBlock, 0, sp>>>(
                nullptr, nullptr, ts, w.pass[p - 1].rec, n, shift, pf, out.tileprefix,
                out.blockprefix, out.digit_total, tpb, out.rec, nullptr, w.err, nullptr, 0, 0, nullptr,
                nullptr, G, nullptr, w.dig1, nullptr);
        else if (e->packed)
            k_scatter_rec<false><<<ntiles, kPartBlock, 0, sp>>>(
                nullptr, nullptr, nullptr, w.pass[p - 1].rec, n, shift, e->pf, out.tileprefix,
                out.blockprefix, out.digit_total, tpb, out.rec, out.perm, w.err);
        else if (approx && p == 0)
            k_scatter<uint64_t, true, false><<<ntiles, kPartBlock, 0, sp>>>(
                keys, permits, nullptr, nullptr, n, shift, out.tileprefix, out.blockprefix,
                out.digit_total, tpb, out.keys, out.permits, nullptr, out.idx, out.perm, w.err, 1);
        else if (approx)
            k_scatter<uint32_t, true, false><<<ntiles, kPartBlock, 0, sp>>>(
                w.pass[p - 1].keys, w.pass[p - 1].permits, nullptr, w.pass[p - 1].idx, n, shift,
                out.tileprefix, out.blockprefix, out.digit_total, tpb, out.keys, out.permits, nullptr,
                out.idx, out.perm, w.err, 0);
        else if (p == 0 && !wait)
            k_scatter<uint64_t, false><<<ntiles, kPartBlock, 0, sp>>>(
                keys, permits, ts, nullptr, n, shift, out.tileprefix, out.blockprefix,
                out.digit_total, tpb, out.keys, out.permits, out.ts, nullptr, out.perm, w.err, 1);
        else if (p == 0)
            k_scatter<uint64_t, true><<<ntiles, kPartBlock, 0, sp>>>(
                keys, permits, ts, nullptr, n, shift, out.tileprefix, out.blockprefix,
                out.digit_total, tpb, out.keys, out.permits, out.ts, out.idx, out.perm, w.err, 1);
        else if (!wait)
            k_scatter<uint32_t, false><<<ntiles, kPartBlock, 0, sp>>>(
                w.pass[p - 1].keys, w.pass[p - 1].permits, w.pass[p - 1].ts, nullptr, n, shift,
                out.tileprefix, out.blockprefix, out.digit_total, tpb, out.keys, out.permits,
                out.ts, nullptr, out.perm, w.err, 0);
        else
            k_scatter<uint32_t, true><<<ntiles, kPartBlock, 0, sp>>>(
                w.pass[p - 1].keys, w.pass[p - 1].permits, w.pass[p - 1].ts, w.pass[p - 1].idx,
                n, shift, out.tileprefix, out.blockprefix, out.digit_total, tpb, out.keys,
                out.permits, out.ts, out.idx, out.perm, w.err, 0);
        stage_end(e, ST_SCATTER, sp);
    }
    const PassBufs &sorted = w.pass[e->passes - 1];
    stage_begin(e, ST_BOUNDS, sp);
    const uint32_t bs_blocks = (e->nb_total + kBsTile - 1) / kBsTile;
    if (TBE_BSCAN_LB && bs_blocks <= kBsMaxBlocks) {
        // a fresh tag per launch on these flags, taken here: a batch that
        // failed between its launch and the end of run_batch cannot hand its tag on
        if (++w.bs_tag == 0) {   // 2^32 launches: back to the zeroed state
            HIP_TRY(e, hipMemsetAsync(w.bsflags, 0, kBsMaxBlocks * sizeof(unsigned long long), sp));
            w.bs_tag = 1;
        }
        k_bscan_lb<<<bs_blocks, 1024, 0, sp>>>(w.bcount, e->nb_total, w.bstart, w.bsflags, w.bs_tag,
                                               e->nbuckets, tb_wmin, sparse_tb ? w.dlist : nullptr);
    }
    else if (sparse_tb)
        k_bscan<<<1, 1024, 0, sp>>>(w.bcount, e->nb_total, w.bstart, e->nbuckets, tb_wmin, w.dlist);
    else
        k_bscan<<<1, 1024, 0, sp>>>(w.bcount, e->nb_total, w.bstart);
    stage_end(e, ST_BOUNDS, sp);
    if (pipe) {
        HIP_TRY(e, hipEventRecord(e->ev_part, sp));
        HIP_TRY(e, hipStreamWaitEvent(sf, e->ev_part, 0));
    }
    // hot_next->n_cand was reset by the k_hot_update that consumed its last nominations
    stage_begin(e, ST_FOLD, sf);
    if (approx) {
        AParams a = e->ap;
        a.id_base = id_base;
        a.wait = e->wait_mode;
        a.ai_base = ai_base;
        if (e->packed)
            k_fold_a<true><<<fold_grid, kFoldBlock, 0, sf>>>(
                nullptr, nullptr, nullptr, sorted.rec, e->pf, w.bstart, e->r_bits, e->cfg.n_keys, e->alocal,
                e->ring, a, w.res[0], e->ev_cause, e->ev_id, e->counters,
                (uint32_t)std::min<uint64_t>(e->ev_cap, 0xFFFFFFFFu), w.err, e->wait_rw(), G, rec0);
        else
            k_fold_a<false><<<e->nbuckets, kFoldBlock, 0, sf>>>(
                sorted.keys, sorted.permits, sorted.idx, nullptr, e->pf, w.bstart, e->r_bits, e->cfg.n_keys,
                e->alocal, e->ring, a, w.res[0], e->ev_cause, e->ev_id, e->counters,
                (uint32_t)std::min<uint64_t>(e->ev_cap, 0xFFFFFFFFu), w.err, e->wait_rw(), G, rec0);
    } else if (wait) {
        QParams q = e->qp;
        q.id_base = id_base;
        q.wait = e->wait_mode;
        q.ai_base = ai_base;
        with_qhdr(e, [&](auto *qh) {
            using HW = std::remove_pointer_t<decltype(qh)>;
            if (e->packed)
                k_fold_q<true, HW><<<fold_grid, kQBlock, 0, sf>>>(
                    nullptr, nullptr, nullptr, sorted.idx, sorted.rec, ts, e->pf, w.bstart, e->r_bits,
                    e->cfg.n_keys, e->table, qh, e->ring, e->params, q, w.res[0], e->ev_cause, e->ev_id,
                    e->counters, (uint32_t)std::min<uint64_t>(e->ev_cap, 0xFFFFFFFFu), w.err, e->wait_rw(),
                    e->qtick, G, rec0);
            else
                k_fold_q<false, HW><<<e->nbuckets, kQBlock, 0, sf>>>(
                    sorted.keys, sorted.permits, sorted.ts, sorted.idx, nullptr, nullptr, e->pf, w.bstart,
                    e->r_bits, e->cfg.n_keys, e->table, qh, e->ring, e->params, q, w.res[0], e->ev_cause,
                    e->ev_id, e->counters, (uint32_t)std::min<uint64_t>(e->ev_cap, 0xFFFFFFFFu), w.err,
                    e->wait_rw(), e->qtick, G, rec0);
        });
    } else if (sparse_tb) {
        // sparse batch: at most n / wmin buckets are dense (k_bscan listed them); one wave per
        // other bucket
        const unsigned dgrid = (unsigned)std::min<uint64_t>(e->nbuckets, n / tb_wmin + 1);
        const uint32_t walk = e->packed ? fold_grid : e->nbuckets;
        const unsigned sgrid = (unsigned)std::min<uint64_t>((walk + kSpWaves - 1) / kSpWaves, 2048);
        if (e->packed) {
            k_fold_wide<true><<<dgrid, kWideBlock, 0, sf>>>(
                nullptr, nullptr, nullptr, sorted.rec, ts, e->pf, w.bstart, e->r_bits, e->cfg.n_keys,
                e->table, e->params, w.res[0], w.err, hot_next, e->narrow ? 1u : 0u, tb_wmin, G, rec0, w.dlist);
            k_fold_sparse<true><<<sgrid, kSpBlock, 0, sf>>>(
                nullptr, nullptr, nullptr, sorted.rec, ts, e->pf, w.bstart, e->r_bits, e->cfg.n_keys,
                e->table, e->params, w.res[0], w.err, e->narrow ? 1u : 0u, tb_wmin, G, rec0, walk);
        } else {
            k_fold_wide<false><<<dgrid, kWideBlock, 0, sf>>>(
                sorted.keys, sorted.permits, sorted.ts, nullptr, nullptr, e->pf, w.bstart, e->r_bits,
                e->cfg.n_keys, e->table, e->params, w.res[0], w.err, nullptr, 0u, tb_wmin, G, rec0, w.dlist);
            k_fold_sparse<false><<<sgrid, kSpBlock, 0, sf>>>(
                sorted.keys, sorted.permits, sorted.ts, nullptr, nullptr, e->pf, w.bstart, e->r_bits,
                e->cfg.n_keys, e->table, e->params, w.res[0], w.err, 0u, tb_wmin, G, rec0, walk);
        }
    } else if (e->packed) {   // a dense batch: k_fold_wide takes every bucket
        k_fold_wide<true><<<fold_grid, kWideBlock, 0, sf>>>(
            nullptr, nullptr, nullptr, sorted.rec, ts, e->pf, w.bstart, e->r_bits, e->cfg.n_keys,
            e->table, e->params, w.res[0], w.err, hot_next, e->narrow ? 1u : 0u, tb_wmin, G, rec0);
    } else {
        k_fold_wide<false><<<e->nbuckets, kWideBlock, 0, sf>>>(
            sorted.keys, sorted.permits, sorted.ts, nullptr, nullptr, e->pf, w.bstart, e->r_bits,
            e->cfg.n_keys, e->table, e->params, w.res[0], w.err, nullptr, 0u, tb_wmin, G, rec0);
    }
    stage_end(e, ST_FOLD, sf);
    if (hot) {
        // runs of this batch's hot keys, after the fold (which may write back a hot key's
        // unchanged row as part of its bucket's slice), then the hot set of batch b+2
        stage_begin(e, ST_HOT, sf);
        const unsigned sgrid = (unsigned)std::min<uint64_t>(1024, n / kSeg + e->hot_cap);
        // (the summary kernel also scans the run lengths into the runs' first segments)
        k_hot_summary<true><<<sgrid, kSegBlock, 0, sf>>>(sorted.rec, ts, e->pf, w.bstart, e->nbuckets,
                                                             w.segbase, w.summ, w.err, G, rec0, hot, e->table,
                                                             e->params, w.res[0], e->narrow ? 1u : 0u, 1u);
        k_hot_chain<<<e->hot_cap, kSegBlock, 0, sf>>>(sorted.rec, ts, e->pf, w.bstart, e->nbuckets, hot,
                                                      hot_next, w.segbase, w.summ, w.sst, e->table,
                                                      e->params, w.res[0], w.err, e->narrow ? 1u : 0u, G, rec0,
                                                      1u);
        k_hot_replies<<<sgrid, kSegBlock, 0, sf>>>(sorted.rec, ts, e->pf, w.bstart, e->nbuckets,
                                                   w.segbase, w.sst, e->params, w.res[0], w.err, e->narrow ? 1u : 0u,
                                                   G, rec0);
        if (pipe) {
            // The next-but-one batch's hot set, on a stream of its own beside this batch's
            // un-partition; batch b+2 (same workspace) waits for it before its partition.
            HIP_TRY(e, hipEventRecord(e->ev_hot, sf));
            HIP_TRY(e, hipStreamWaitEvent(e->hstream, e->ev_hot, 0));
            k_hot_update<<<1, 1024, 0, e->hstream>>>(hot_next, e->hot_cap - hot_reserve_host(e->hot_cap), w.err);
            HIP_TRY(e, hipEventRecord(w.hot_done, e->hstream));
            w.hot_pending = true;
        } else {
            k_hot_update<<<1, 1024, 0, sf>>>(hot_next, e->hot_cap - hot_reserve_host(e->hot_cap), w.err);
        }
        stage_end(e, ST_HOT, sf);
    }
    stage_begin(e, ST_UNSCATTER, sf);
    const unsigned untiles = (unsigned)((n + kUnTile - 1) / kUnTile);
    int cur = 0;
    // with fold records the replies are already in pass passes-2's output order
    for (int p = e->passes - (G.on ? 2 : 1); p >= 1; --p) {
        if (e->narrow && !approx)
            k_unscatter<false, false, 1><<<untiles, kUnBlock, 0, sf>>>(n, w.pass[p].perm, w.res[cur],
                                                                   w.res[cur ^ 1], nullptr, nullptr);
        else if (e->medium)
            k_unscatter<false, false, 2><<<untiles, kUnBlock, 0, sf>>>(n, w.pass[p].perm, w.res[cur],
                                                                   w.res[cur ^ 1], nullptr, nullptr);
        else
            k_unscatter<false, false><<<untiles, kUnBlock, 0, sf>>>(n, w.pass[p].perm, w.res[cur],
                                                                    w.res[cur ^ 1], nullptr, nullptr);
        cur ^= 1;
    }
#define TBE_UNRANK(...)                                                                             \
    __VA_ARGS__<<<ntiles, kPartBlock, 0, sf>>>(n, w.dig0, w.pass[0].tileprefix, w.pass[0].blockprefix, \
                                               w.pass[0].digit_total, tpb, w.res[cur], granted, remaining)
    if (unrank && !wait && e->narrow)
        TBE_UNRANK(k_unrank<1>);
    else if (unrank && !wait)
        TBE_UNRANK(k_unrank<4>);
    else if (unrank && e->narrow)
        TBE_UNRANK(k_unrank<1, true>);
    else if (unrank && e->medium)
        TBE_UNRANK(k_unrank<2, true>);
    else if (unrank)
        TBE_UNRANK(k_unrank<4, true>);
#undef TBE_UNRANK
    else if (e->narrow && !wait && !approx)
        k_unscatter<true, false, 1><<<untiles, kUnBlock, 0, sf>>>(n, w.pass[0].perm, w.res[cur],
                                                                  nullptr, granted, remaining,
            w.err, e->sticky);
    else if (wait && e->narrow)
        k_unscatter<true, true, 1><<<untiles, kUnBlock, 0, sf>>>(n, w.pass[0].perm, w.res[cur],
                                                                 nullptr, granted, remaining,
            w.err, e->sticky);
    else if (wait && e->medium)
        k_unscatter<true, true, 2><<<untiles, kUnBlock, 0, sf>>>(n, w.pass[0].perm, w.res[cur],
                                                                 nullptr, granted, remaining,
            w.err, e->sticky);
    else if (wait)
        k_unscatter<true, true><<<untiles, kUnBlock, 0, sf>>>(n, w.pass[0].perm, w.res[cur],
                                                              nullptr, granted, remaining,
            w.err, e->sticky);
    else
        k_unscatter<true, false><<<untiles, kUnBlock, 0, sf>>>(n, w.pass[0].perm, w.res[cur],
                                                               nullptr, granted, remaining,
            w.err, e->sticky);
    stage_end(e, ST_UNSCATTER, sf);
    if (unrank) k_sticky<<<1, 64, 0, sf>>>(w.err, e->sticky);   // (otherwise the final unscatter did it)
    HIP_TRY(e, hipGetLastError());
    if (pipe) {
        HIP_TRY(e, hipEventRecord(w.done, sf));
        w.used = true;
        hipStream_t outs = out_stream ? out_stream : caller;
        if (outs && outs != sf) {
            HIP_TRY(e, hipEventRecord(e->ev_out, sf));
            HIP_TRY(e, hipStreamWaitEvent(outs, e->ev_out, 0));
        }
        e->ws_cur ^= 1;
    } else if (out_stream && out_stream != sf) {
        HIP_TRY(e, hipEventRecord(e->ev_out, sf));
        HIP_TRY(e, hipStreamWaitEvent(out_stream, e->ev_out, 0));
    }
    e->last_err = w.err;
    ++e->nbatch;
    return TBE_OK;
}

}  // namespace

// ============================================================================= C ABI
// Resident state is allocated with plain hipMalloc.  (Round 5 allocated the rings with
// hipExtMallocWithFlags(..., hipDeviceMallocContiguous) for 0.24 ms of config D, and queue
// and approximate engines created after another engine had been freed then gave wrong
// replies on some boxes; that flag is not among those hip_runtime_api.h documents for
// hipExtMallocWithFlags, and the engine no longer uses it.  CHANGELOG round 6.)
template <typename T>
hipError_t dalloc(T **p, size_t bytes) {
    return hipMalloc(reinterpret_cast<void **>(p), bytes);
}

extern "C" {

double tbe_fill_rate(int32_t tokens_per_period, int64_t replenishment_period_ticks) {
    const double total_seconds = (double)replenishment_period_ticks / 10000000.0;
    return (double)tokens_per_period / total_seconds;
}

static thread_local std::string g_create_error = "no error";

static tbe_status create_fail(tbe_status st, const char *msg) {
    g_create_error = msg;
    return st;
}

tbe_status tbe_create(const tbe_config *config, tbe_engine **out_engine) {
    if (!out_engine) return create_fail(TBE_EINVAL, "out_engine is NULL");
    *out_engine = nullptr;
    // struct_size versions the config: a caller built against the round-1 header (which
    // ended at max_batch) passes the shorter size, and the fields it lacks read as 0.
    constexpr size_t kConfigV1 = offsetof(tbe_config, zero_wait_slots);
    if (!config || config->struct_size < kConfigV1)
        return create_fail(TBE_EINVAL, "config is NULL or struct_size too small");
    tbe_config c_in;
    std::memset(&c_in, 0, sizeof c_in);
    std::memcpy(&c_in, config, std::min<size_t>(config->struct_size, sizeof c_in));
    const tbe_config &c = c_in;
    if (c.kind != TBE_KIND_TOKEN_BUCKET && c.kind != TBE_KIND_QUEUEING &&
        c.kind != TBE_KIND_APPROXIMATE)
        return create_fail(TBE_EINVAL, "unknown kind");
    if (c.kind != TBE_KIND_TOKEN_BUCKET) {
        if (c.queue_limit < 0 || c.queue_limit > 0xFFFF)                            // Q ctor
            return create_fail(TBE_EINVAL, "QueueLimit must lie in [0, 65535]");
        if (c.queue_order != 0 && c.queue_order != 1)
            return create_fail(TBE_EINVAL, "QueueProcessingOrder must be OldestFirst (0) or NewestFirst (1)");
        if (c.token_limit >= (int32_t)kRemNone)                                     // reply packing
            return create_fail(TBE_EINVAL, "TokenLimit must be < 2^30 - 1 for queueing limiters");
        if (c.zero_wait_slots < 0 || (c.kind == TBE_KIND_QUEUEING && c.zero_wait_slots != 0) ||
            std::max(1, c.queue_limit) + c.zero_wait_slots > 0xFFFF)
            return create_fail(TBE_EINVAL, "zero_wait_slots must be >= 0 (approximate kind only) with "
                                           "max(1, QueueLimit) + zero_wait_slots <= 65535");
    }
    if (c.n_keys == 0 || c.n_keys > (1ull << 32))
        return create_fail(TBE_EINVAL, "n_keys must lie in [1, 2^32]");
    if (c.token_limit <= 0 || c.tokens_per_period <= 0)                       // TB:29-32
        return create_fail(TBE_EINVAL, "Both TokenLimit and TokensPerPeriod must be set to values greater than 0.");
    if (c.replenishment_period_ticks <= 0)                                    // TB:34-37 (+ "inf")
        return create_fail(TBE_EINVAL, "ReplenishmentPeriod must be greater than TimeSpan.Zero");
    const double rate = tbe_fill_rate(c.tokens_per_period, c.replenishment_period_ticks);
    if (!std::isfinite(rate) || !(rate > 0.0)) return create_fail(TBE_EINVAL, "fill rate is not finite and positive");

    tbe_engine *e = new (std::nothrow) tbe_engine();
    if (!e) return create_fail(TBE_ENOMEM, "host allocation failed");
    e->cfg = c;
    e->params.cap = (double)c.token_limit;
    e->params.rate = rate;
    {
        // TB:234: math.ceil(math.min(math.max(capacity / fill_rate, 1), 31536000))
        double q = (double)c.token_limit / rate;
        q = (1.0 > q) ? 1.0 : q;
        q = (31536000.0 < q) ? 31536000.0 : q;
        e->params.ttl_ms = (int64_t)std::ceil(q) * 1000;
    }
    const int kb = ceil_log2(c.n_keys);
    e->r_bits = std::min(kMaxRBits, std::max(4, kb - 10));
    e->nbuckets = (uint32_t)((c.n_keys + (1ull << e->r_bits) - 1) >> e->r_bits);
    const int bbits = ceil_log2(e->nbuckets);
    e->passes = std::max(1, (bbits + kDigitBits - 1) / kDigitBits);
    e->timing = (c.flags & (TBE_FLAG_STAGE_TIMING | TBE_FLAG_FOLD_TIMING)) != 0;
    e->timing_mask = (c.flags & TBE_FLAG_STAGE_TIMING) ? ~0u : (1u << ST_FOLD);
    {
        // Packed records need key + permit code + a >= 32-bit time offset + escape bit.
        // Hot runs (token bucket, packed) take bucket ids past the ordinary ones that the
        // passes' digits already cover, and widen the key field to those ids.
        int pbits = 0;
        while (pbits < 32 && ((int64_t)1 << pbits) <= (int64_t)c.token_limit + 1) ++pbits;
        auto layout = [&](uint32_t hot_cap) {
            const uint64_t span = std::max<uint64_t>(c.n_keys, ((uint64_t)e->nbuckets + hot_cap) << e->r_bits);
            const int kbits = std::max(1, ceil_log2(span));
            e->pf.kb = kbits;
            e->pf.pb = pbits;
            e->pf.kmask = (kbits >= 64) ? ~0ull : ((1ull << kbits) - 1);
            e->pf.pc_max = (c.token_limit == INT32_MAX) ? INT32_MAX : c.token_limit + 1;
            e->pf.wb = 64 - kbits - pbits - 1;
            return e->pf.wb >= 32 && kbits <= 32 && (c.flags & TBE_FLAG_NO_PACK) == 0;
        };
        uint32_t hot_cap = 0;
        if ((c.flags & TBE_FLAG_NO_HOT) == 0 && c.kind == TBE_KIND_TOKEN_BUCKET) {
            const uint64_t room = (1ull << (kDigitBits * e->passes)) - e->nbuckets;
            hot_cap = (uint32_t)std::min<uint64_t>(kHotKeysMax, room);
            if (hot_cap < 16) hot_cap = 0;
        }
        e->packed = hot_cap && layout(hot_cap);
        if (!e->packed) {
            hot_cap = 0;
            e->packed = layout(0);
        }
        e->hot_cap = hot_cap;
        e->nb_total = e->nbuckets + hot_cap;
        e->foldrec = e->packed && e->passes >= 2 && (c.flags & TBE_FLAG_UNSCATTER_ALL) == 0;
        e->unrank = e->packed && (c.flags & TBE_FLAG_UNSCATTER_ALL) == 0 && (c.flags & TBE_FLAG_RERANK) != 0;
        e->dig1 = e->packed && e->passes == 2 && (c.flags & TBE_FLAG_HIST_RECORDS) == 0;
        {
            const int w0 = 32 - e->r_bits - pbits - 1;
            // token bucket and queueing kinds: the time offset needs >= 8 bits; the approximate
            // kind's narrow record is row | permit code (no time), used by batches that cannot
            // queue (AcquireCore: no arrival index is ever read, batch_fold_fmt)
            e->n0 = TBE_NARROW0 && e->dig1 && e->foldrec &&
                    (c.kind == TBE_KIND_APPROXIMATE ? e->r_bits + pbits + 1 <= 32 : w0 >= 8);
            e->pf.n0 = 0;                  // per batch (run_batch): only with this batch's fold records
            e->pf.rb = e->r_bits;
            e->pf.w0 = w0;
        }
        e->narrow = (c.flags & TBE_FLAG_NO_NARROW) == 0 &&
                    ((e->packed && c.kind == TBE_KIND_TOKEN_BUCKET && c.token_limit <= 127) ||
                     (c.kind == TBE_KIND_QUEUEING && c.token_limit <= 62));
        e->medium = (c.flags & TBE_FLAG_NO_NARROW) == 0 && !e->narrow && c.token_limit <= (int32_t)kRemNone16 - 1 &&
                    (c.kind == TBE_KIND_QUEUEING || c.kind == TBE_KIND_APPROXIMATE);
    }

    auto bail = [&](tbe_status st) {
        tbe_destroy(e);
        return create_fail(st, st == TBE_ENOMEM ? "device allocation failed" : "HIP device error");
    };
    if (c.device >= 0) {
        if (hipSetDevice(c.device) != hipSuccess) return bail(TBE_EDEVICE);
        e->device = c.device;
    } else if (hipGetDevice(&e->device) != hipSuccess) {
        return bail(TBE_EDEVICE);
    }
    e->pipeline = c.kind == TBE_KIND_TOKEN_BUCKET && (c.flags & TBE_FLAG_NO_PIPELINE) == 0;
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(TBE_EDEVICE);
    e->own_stream = true;
    if (e->pipeline && hipStreamCreateWithFlags(&e->pstream, hipStreamNonBlocking) != hipSuccess)
        return bail(TBE_EDEVICE);
    if (e->pipeline && hipStreamCreateWithFlags(&e->hstream, hipStreamNonBlocking) != hipSuccess)
        return bail(TBE_EDEVICE);
    for (hipEvent_t *ev : {&e->ev_in, &e->ev_part, &e->ev_out, &e->ev_hot, &e->ws[0].done, &e->ws[1].done,
                           &e->ws[0].hot_done, &e->ws[1].hot_done})
        if (hipEventCreateWithFlags(ev, hipEventDisableTiming) != hipSuccess) return bail(TBE_EDEVICE);
    // Every resident buffer is allocated before any initialisation is enqueued, and every
    // one is then initialised on e->stream -- the rings and the headers' pad entry too, though
    // no decision reads a ring entry the engine did not write -- so a new engine never sees
    // bytes an earlier allocation left (tests/test_gpu_recreate.py).
    const uint64_t qhdr_n = (c.n_keys + 3) & ~3ull;   // k_fold_q loads headers 16 bytes per lane
    uint64_t ring_n = 0;
    if (dalloc(&e->table, c.n_keys * sizeof(Slot)) != hipSuccess) return bail(TBE_ENOMEM);
    if (e->hot_cap)
        for (auto &hs : e->hot)
            if (dalloc(&hs, sizeof(HotSet)) != hipSuccess) return bail(TBE_ENOMEM);
    if (dalloc(&e->sticky, sizeof(uint32_t)) != hipSuccess) return bail(TBE_ENOMEM);
    if (c.kind == TBE_KIND_QUEUEING) {
        e->qp.token_limit = c.token_limit;
        e->qp.queue_limit = c.queue_limit;
        e->qp.order = c.queue_order;
        e->qp.cap = (uint32_t)std::max(1, c.queue_limit);
        ring_n = c.n_keys * (uint64_t)e->qp.cap;
        e->qh32 = TBE_QH32 && (uint32_t)c.queue_limit <= kQh32MaxLimit;
        if (dalloc(&e->qhdr, qhdr_n * (e->qh32 ? sizeof(uint32_t) : sizeof(uint64_t))) != hipSuccess)
            return bail(TBE_ENOMEM);
    } else if (c.kind == TBE_KIND_APPROXIMATE) {
        e->ap.token_limit = c.token_limit;
        e->ap.queue_limit = c.queue_limit;
        e->ap.order = c.queue_order;
        e->ap.zero_slots = c.zero_wait_slots;
        e->ap.cap = (uint32_t)(std::max(1, c.queue_limit) + c.zero_wait_slots);
        e->ap.decay_rate = rate;
        e->ap.period_s = (double)c.replenishment_period_ticks / 10000000.0;
        ring_n = c.n_keys * (uint64_t)e->ap.cap;
        if (dalloc(&e->alocal, c.n_keys * sizeof(ALocal)) != hipSuccess) return bail(TBE_ENOMEM);
        if (dalloc(&e->aclient, c.n_keys * sizeof(AClient)) != hipSuccess) return bail(TBE_ENOMEM);
        if (dalloc(&e->gv, c.n_keys * sizeof(double)) != hipSuccess) return bail(TBE_ENOMEM);
        if (dalloc(&e->gp, c.n_keys * sizeof(double)) != hipSuccess) return bail(TBE_ENOMEM);
        if (dalloc(&e->gt, c.n_keys * sizeof(int64_t)) != hipSuccess) return bail(TBE_ENOMEM);
    }
    if (ring_n) {
        if (dalloc(&e->ring, ring_n * sizeof(uint64_t)) != hipSuccess) return bail(TBE_ENOMEM);
        if (dalloc(&e->counters, 2 * sizeof(uint32_t)) != hipSuccess) return bail(TBE_ENOMEM);
    }
    for (int i = 0; i < (e->pipeline ? 2 : 1); ++i)
        if (c.max_batch && ensure_workspace(e, e->ws[i], c.max_batch) != TBE_OK) return bail(TBE_ENOMEM);
    // initialisation, in order on the engine's stream
    hipError_t ie = hipSuccess;
    auto zero = [&](void *p, size_t bytes) {
        if (p && ie == hipSuccess) ie = hipMemsetAsync(p, 0, bytes, e->stream);
    };
    for (auto &hs : e->hot) zero(hs, sizeof(HotSet));
    zero(e->sticky, sizeof(uint32_t));
    zero(e->qhdr, qhdr_n * (e->qh32 ? sizeof(uint32_t) : sizeof(uint64_t)));
    zero(e->ring, ring_n * sizeof(uint64_t));
    zero(e->counters, 2 * sizeof(uint32_t));
    for (auto &w : e->ws)
        if (w.bsflags && w.bs_fresh) {
            zero(w.bsflags, kBsMaxBlocks * sizeof(unsigned long long));
            w.bs_fresh = false;
        }
    if (ie != hipSuccess) return bail(TBE_EDEVICE);
    k_init_table<<<2048, 256, 0, e->stream>>>(e->table, c.n_keys, e->params.cap);
    if (c.kind == TBE_KIND_APPROXIMATE)
        k_init_approx<<<2048, 256, 0, e->stream>>>(c.n_keys, e->alocal, e->aclient, e->gv, e->gp, e->gt,
                                                   c.token_limit);
    if (hipGetLastError() != hipSuccess) return bail(TBE_EDEVICE);
    if (hipStreamSynchronize(e->stream) != hipSuccess) return bail(TBE_EDEVICE);
    *out_engine = e;
    return TBE_OK;
}

void tbe_destroy(tbe_engine *e) {
    if (!e) return;
    if (e->pstream) (void)hipStreamSynchronize(e->pstream);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->hstream) (void)hipStreamSynchronize(e->hstream);
    for (hipStream_t s2 : {e->cin, e->cout, e->cin2})
        if (s2) (void)hipStreamSynchronize(s2);
    free_workspace(e->ws[0]);
    free_workspace(e->ws[1]);
    free_staging(e);
    dfree(e->table);
    dfree(e->alocal);
    dfree(e->aclient);
    dfree(e->gv);
    dfree(e->gp);
    dfree(e->gt);
    dfree(e->acounts);
    dfree(e->qhdr);
    dfree(e->ring);
    dfree(e->counters);
    dfree(e->qcount);
    dfree(e->ev_cause);
    dfree(e->ev_id);
    dfree(e->log_keyseq);
    dfree(e->log_id);
    dfree(e->log_rem);
    dfree(e->sticky);
    for (auto &hs : e->hot) dfree(hs);
    for (auto &ev : e->ev_pool)
        if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : {e->ev_in, e->ev_part, e->ev_out, e->ev_hot, e->ws[0].done, e->ws[1].done,
                          e->ws[0].hot_done, e->ws[1].hot_done})
        if (ev) (void)hipEventDestroy(ev);
    if (e->pstream) (void)hipStreamDestroy(e->pstream);
    if (e->hstream) (void)hipStreamDestroy(e->hstream);
    for (hipEvent_t ev : e->ev_chunk)
        if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : e->ev_chunk2)
        if (ev) (void)hipEventDestroy(ev);
    for (hipStream_t s2 : {e->cin, e->cout, e->cin2})
        if (s2) (void)hipStreamDestroy(s2);
    if (e->own_stream && e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

const char *tbe_last_error(const tbe_engine *e) {
    return e ? e->last_error.c_str() : g_create_error.c_str();
}

// ---- the host-buffer path from page-locked buffers (tbe_alloc_host), chunked so that
// PCIe copies overlap the decisions: every chunk's copy-in is enqueued up front on one
// copy stream, each chunk is decided as a sub-batch as soon as its copy lands (sub-batches
// in arrival order are the same serial order as one batch), and its replies go back on a
// second copy stream while later chunks are decided.  The whole batch is validated on
// the host first (several threads), so an invalid batch still changes nothing.
static constexpr uint64_t kHostChunk = 1ull << 22;

static bool host_pinned(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();   // pageable memory is not an error worth keeping
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

static bool host_validate(const tbe_engine *e, const uint64_t *keys, const int32_t *permits, const int64_t *ts,
                          uint64_t n) {
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    std::vector<char> bad(nt, 0);
    const uint64_t nk = e->cfg.n_keys;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            const uint64_t a = n * t / nt, b = n * (t + 1) / nt;
            bool x = false;
            if (ts)
                for (uint64_t i = a; i < b; ++i) x |= (keys[i] >= nk) | (permits[i] < 0) | (ts[i] < 0);
            else
                for (uint64_t i = a; i < b; ++i) x |= (keys[i] >= nk) | (permits[i] < 0);
            bad[t] = x;
        });
    for (auto &x : th) x.join();
    for (char b : bad)
        if (b) return false;
    return true;
}

// Copy a page-locked batch in, chunk by chunk, in chunk order; ev_chunk[c] fires when
// chunk c is on the device.  With TBE_CIN_STREAMS == 2 the timestamps travel on a second
// copy stream (another DMA queue) beside the keys and permits.
#ifndef TBE_CIN_STREAMS
#define TBE_CIN_STREAMS 1
#endif
static tbe_status copy_in_chunks(tbe_engine *e, const uint64_t *keys, const int32_t *permits, const int64_t *ts,
                                 uint64_t n, uint64_t nch) {
    if (!e->cin) {
        HIP_TRY(e, hipStreamCreateWithFlags(&e->cin, hipStreamNonBlocking));
        HIP_TRY(e, hipStreamCreateWithFlags(&e->cout, hipStreamNonBlocking));
    }
    const bool two = TBE_CIN_STREAMS == 2 && ts;
    if (two && !e->cin2) HIP_TRY(e, hipStreamCreateWithFlags(&e->cin2, hipStreamNonBlocking));
    while (e->ev_chunk.size() < nch) {
        hipEvent_t ev = nullptr;
        HIP_TRY(e, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        e->ev_chunk.push_back(ev);
    }
    while (two && e->ev_chunk2.size() < nch) {
        hipEvent_t ev = nullptr;
        HIP_TRY(e, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        e->ev_chunk2.push_back(ev);
    }
    for (uint64_t c = 0; c < nch; ++c) {
        const uint64_t o = c * kHostChunk, m = std::min(kHostChunk, n - o);
        if (two) {
            HIP_TRY(e, hipMemcpyAsync(e->d_ts + o, ts + o, m * sizeof(int64_t), hipMemcpyHostToDevice, e->cin2));
            HIP_TRY(e, hipEventRecord(e->ev_chunk2[c], e->cin2));
        }
        HIP_TRY(e, hipMemcpyAsync(e->d_keys + o, keys + o, m * sizeof(uint64_t), hipMemcpyHostToDevice, e->cin));
        HIP_TRY(e, hipMemcpyAsync(e->d_permits + o, permits + o, m * sizeof(int32_t), hipMemcpyHostToDevice, e->cin));
        if (ts && !two)
            HIP_TRY(e, hipMemcpyAsync(e->d_ts + o, ts + o, m * sizeof(int64_t), hipMemcpyHostToDevice, e->cin));
        if (two) HIP_TRY(e, hipStreamWaitEvent(e->cin, e->ev_chunk2[c], 0));
        HIP_TRY(e, hipEventRecord(e->ev_chunk[c], e->cin));
    }
    return TBE_OK;
}

static tbe_status acquire_chunked(tbe_engine *e, const uint64_t *keys, const int32_t *permits, const int64_t *ts,
                                  uint64_t n, uint8_t *granted, int32_t *remaining) {
    const uint64_t nch = (n + kHostChunk - 1) / kHostChunk;
    {
        tbe_status rc = copy_in_chunks(e, keys, permits, ts, n, nch);
        if (rc != TBE_OK) return rc;
    }
    if (!host_validate(e, keys, permits, ts, n)) {   // overlaps the first copies
        HIP_TRY(e, hipStreamSynchronize(e->cin));
        return fail(e, TBE_EINVAL, "invalid request in batch (key >= n_keys, permits < 0 or ts < 0)");
    }
    for (uint64_t c = 0; c < nch; ++c) {
        const uint64_t o = c * kHostChunk, m = std::min(kHostChunk, n - o);
        tbe_status rc = run_batch(e, e->d_keys + o, e->d_permits + o, e->d_ts + o, m, e->d_granted + o,
                                  e->d_remaining + o, nullptr, 0, e->ev_chunk[c], e->cout);
        if (rc != TBE_OK) return rc;
        HIP_TRY(e, hipMemcpyAsync(granted + o, e->d_granted + o, m, hipMemcpyDeviceToHost, e->cout));
        HIP_TRY(e, hipMemcpyAsync(remaining + o, e->d_remaining + o, m * sizeof(int32_t), hipMemcpyDeviceToHost,
                                  e->cout));
    }
    HIP_TRY(e, hipStreamSynchronize(e->cout));
    return TBE_OK;
}

tbe_status tbe_acquire_batch(tbe_engine *e, const uint64_t *keys, const int32_t *permits,
                             const int64_t *ts_us, uint64_t n, uint8_t *granted,
                             int32_t *remaining) {
    if (!e) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_TOKEN_BUCKET) return fail(e, TBE_EINVAL, "not a token-bucket engine");
    if (n == 0) return TBE_OK;
    if (!keys || !permits || !ts_us || !granted || !remaining)
        return fail(e, TBE_EINVAL, "null buffer");
    HIP_TRY(e, hipSetDevice(e->device));
    tbe_status rc = ensure_host_staging(e, n);
    if (rc != TBE_OK) return rc;
    if (e->pipeline && n >= 2 * kHostChunk && host_pinned(keys) && host_pinned(permits) &&
        host_pinned(ts_us) && host_pinned(granted) && host_pinned(remaining))
        return acquire_chunked(e, keys, permits, ts_us, n, granted, remaining);
    hipStream_t st = e->stream;
    HIP_TRY(e, hipMemcpyAsync(e->d_keys, keys, n * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    HIP_TRY(e, hipMemcpyAsync(e->d_permits, permits, n * sizeof(int32_t), hipMemcpyHostToDevice, st));
    HIP_TRY(e, hipMemcpyAsync(e->d_ts, ts_us, n * sizeof(int64_t), hipMemcpyHostToDevice, st));
    rc = run_batch(e, e->d_keys, e->d_permits, e->d_ts, n, e->d_granted, e->d_remaining, st);
    if (rc != TBE_OK) return rc;
    uint32_t flag = 0;
    HIP_TRY(e, hipMemcpyAsync(&flag, e->last_err, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(e, hipMemcpyAsync(granted, e->d_granted, n, hipMemcpyDeviceToHost, st));
    HIP_TRY(e, hipMemcpyAsync(remaining, e->d_remaining, n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(e, hipStreamSynchronize(st));
    if (flag) {
        HIP_TRY(e, hipMemsetAsync(e->sticky, 0, sizeof(uint32_t), st));
        HIP_TRY(e, hipStreamSynchronize(st));
        return fail(e, TBE_EINVAL, "invalid request in batch (key >= n_keys, permits < 0 or ts < 0)");
    }
    return TBE_OK;
}

tbe_status tbe_acquire_batch_device(tbe_engine *e, const uint64_t *d_keys, const int32_t *d_permits,
                                    const int64_t *d_ts_us, uint64_t n, uint8_t *d_granted,
                                    int32_t *d_remaining, void *stream) {
    if (!e) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_TOKEN_BUCKET) return fail(e, TBE_EINVAL, "not a token-bucket engine");
    if (n == 0) return TBE_OK;
    if (!d_keys || !d_permits || !d_ts_us || !d_granted || !d_remaining)
        return fail(e, TBE_EINVAL, "null buffer");
    HIP_TRY(e, hipSetDevice(e->device));
    return run_batch(e, d_keys, d_permits, d_ts_us, n, d_granted, d_remaining, (hipStream_t)stream);
}

tbe_status tbe_alloc_host(uint64_t bytes, void **out) {
    if (!out) return TBE_EINVAL;
    *out = nullptr;
    if (bytes == 0) return TBE_OK;
    const hipError_t rc = hipHostMalloc(out, bytes, hipHostMallocDefault);
    if (rc != hipSuccess) {
        *out = nullptr;
        return rc == hipErrorOutOfMemory ? TBE_ENOMEM : TBE_EDEVICE;
    }
    return TBE_OK;
}

void tbe_free_host(void *p) {
    if (p) (void)hipHostFree(p);
}

tbe_status tbe_synchronize(tbe_engine *e) {
    if (!e) return TBE_EINVAL;
    HIP_TRY(e, hipSetDevice(e->device));
    HIP_TRY(e, hipDeviceSynchronize());
    uint32_t sticky = 0;
    HIP_TRY(e, hipMemcpy(&sticky, e->sticky, sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (sticky) {
        HIP_TRY(e, hipMemset(e->sticky, 0, sizeof(uint32_t)));
        return fail(e, TBE_EINVAL, "an enqueued batch held an invalid request and was skipped");
    }
    return TBE_OK;
}

tbe_status tbe_query(tbe_engine *e, uint64_t key, int64_t ts_us, double *v, double *t,
                     int32_t *present) {
    if (!e || !v || !t || !present) return TBE_EINVAL;
    if (key >= e->cfg.n_keys) return fail(e, TBE_EINVAL, "key out of range");
    HIP_TRY(e, hipSetDevice(e->device));
    Slot s;
    HIP_TRY(e, hipMemcpyAsync(&s, e->table + key, sizeof(Slot), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    *present = 0;
    *v = 0.0;
    *t = 0.0;
    if (s.t_us == kAbsent) return TBE_OK;
    if (ts_us >= 0 && (ts_us / 1000) > (s.t_us / 1000) + e->params.ttl_ms) return TBE_OK;
    *present = 1;
    *v = s.v;
    const int64_t sec = s.t_us / 1000000, usec = s.t_us - sec * 1000000;
    *t = (double)sec + ((double)usec / 1000000.0);
    return TBE_OK;
}

tbe_status tbe_export_state(tbe_engine *e, uint64_t first, uint64_t count, double *v, int64_t *t_us) {
    if (!e || !v || !t_us) return TBE_EINVAL;
    if (first > e->cfg.n_keys || count > e->cfg.n_keys - first)
        return fail(e, TBE_EINVAL, "range out of bounds");
    if (count == 0) return TBE_OK;
    HIP_TRY(e, hipSetDevice(e->device));
    std::vector<Slot> tmp(count);
    HIP_TRY(e, hipMemcpyAsync(tmp.data(), e->table + first, count * sizeof(Slot),
                              hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    for (uint64_t i = 0; i < count; ++i) {
        v[i] = tmp[i].v;
        t_us[i] = tmp[i].t_us;
    }
    return TBE_OK;
}

// Ring entries of all keys: the most any sequence of batches can leave queued.
static uint64_t ring_entries(const tbe_engine *e) {
    const uint32_t cap = e->cfg.kind == TBE_KIND_APPROXIMATE ? e->ap.cap : e->qp.cap;
    return e->cfg.n_keys * (uint64_t)cap;
}

// Host-buffer calls size their logs from queued_total; after device-pointer batches it is
// only an upper bound, so count the queues on the device once (all streams drained first:
// device batches may have run on caller streams).
static tbe_status sync_queued(tbe_engine *e) {
    if (e->queued_exact) return TBE_OK;
    HIP_TRY(e, hipDeviceSynchronize());
    if (!e->qcount) HIP_TRY(e, hipMalloc(&e->qcount, sizeof(unsigned long long)));
    hipStream_t st = e->stream;
    HIP_TRY(e, hipMemsetAsync(e->qcount, 0, sizeof(unsigned long long), st));
    const uint64_t blocks = std::min<uint64_t>((e->cfg.n_keys + kBlock - 1) / kBlock, 8192);
    if (e->cfg.kind == TBE_KIND_QUEUEING)
        with_qhdr(e, [&](auto *qh) {
            k_count_queued<<<(unsigned)blocks, kBlock, 0, st>>>(e->cfg.n_keys, qh, e->alocal, e->qcount);
        });
    else
        k_count_queued<<<(unsigned)blocks, kBlock, 0, st>>>(e->cfg.n_keys, (const uint64_t *)nullptr, e->alocal,
                                                            e->qcount);
    HIP_TRY(e, hipGetLastError());
    unsigned long long q = 0;
    HIP_TRY(e, hipMemcpyAsync(&q, e->qcount, sizeof q, hipMemcpyDeviceToHost, st));
    HIP_TRY(e, hipStreamSynchronize(st));
    e->queued_total = q;
    e->queued_exact = true;
    return TBE_OK;
}

// Device-pointer variant of status_batch: the whole batch stays in HBM, nothing is
// synchronised.  Evictions (NewestFirst waits only) go to the engine's eviction log, read
// lazily by tbe_evicted; its capacity n + queued_total bounds them (every eviction
// removes an entry queued before the batch or by it).
static tbe_status status_batch_device(tbe_engine *e, const uint64_t *d_keys, const int32_t *d_permits,
                                      const int64_t *d_ts, uint64_t n, int64_t id_base,
                                      uint8_t *d_status, int32_t *d_remaining, void *stream) {
    e->evicted.clear();
    e->ev_pending = false;
    if (n == 0) return TBE_OK;
    if (!d_keys || !d_permits || !d_status || !d_remaining) return fail(e, TBE_EINVAL, "null buffer");
    if (id_base < 0 || (uint64_t)id_base + n > (1ull << 47))
        return fail(e, TBE_EINVAL, "request ids must lie in [0, 2^47)");
    HIP_TRY(e, hipSetDevice(e->device));
    const int32_t order = e->cfg.kind == TBE_KIND_APPROXIMATE ? e->ap.order : e->qp.order;
    const bool may_evict = e->wait_mode == 1 && order == 1;
    if (may_evict) {
        const uint64_t need_ev = e->queued_total + n;
        if (need_ev > e->ev_cap) {
            dfree(e->ev_cause);
            dfree(e->ev_id);
            e->ev_cap = 0;
            HIP_TRY(e, hipMalloc(&e->ev_cause, need_ev * sizeof(uint32_t)));
            HIP_TRY(e, hipMalloc(&e->ev_id, need_ev * sizeof(int64_t)));
            e->ev_cap = need_ev;
        }
    }
    hipStream_t st = stream ? (hipStream_t)stream : e->stream;
    HIP_TRY(e, hipMemsetAsync(e->counters, 0, sizeof(uint32_t), st));
    tbe_status rc = run_batch(e, d_keys, d_permits, d_ts, n, d_status, d_remaining, st, id_base);
    if (rc != TBE_OK) return rc;
    e->ev_pending = may_evict;
    if (e->wait_mode == 1) {
        e->queued_total = std::min<uint64_t>(e->queued_total + n, ring_entries(e));
        e->queued_exact = false;
    }
    return TBE_OK;
}

tbe_status tbe_import_state(tbe_engine *e, uint64_t first, uint64_t count, const double *v,
                            const int64_t *t_us) {
    if (!e) return TBE_EINVAL;
    if (e->cfg.kind == TBE_KIND_APPROXIMATE) return fail(e, TBE_EINVAL, "not a token-bucket engine");
    if (first > e->cfg.n_keys || count > e->cfg.n_keys - first)
        return fail(e, TBE_EINVAL, "range out of bounds");
    if (count == 0) return TBE_OK;
    if (!v || !t_us) return fail(e, TBE_EINVAL, "null buffer");
    std::vector<Slot> tmp(count);
    for (uint64_t i = 0; i < count; ++i) {
        if (t_us[i] != kAbsent && t_us[i] < 0) return fail(e, TBE_EINVAL, "t_us < 0");
        tmp[i] = t_us[i] == kAbsent ? Slot{e->params.cap, kAbsent} : Slot{v[i], t_us[i]};
    }
    HIP_TRY(e, hipSetDevice(e->device));
    HIP_TRY(e, hipDeviceSynchronize());   // after every enqueued batch, whatever its stream
    HIP_TRY(e, hipMemcpy(e->table + first, tmp.data(), count * sizeof(Slot), hipMemcpyHostToDevice));
    return TBE_OK;
}

static tbe_status status_batch(tbe_engine *e, const uint64_t *keys, const int32_t *permits,
                               const int64_t *ts_us, uint64_t n, int64_t id_base, uint8_t *status,
                               int32_t *remaining, uint64_t *n_evicted);

tbe_status tbe_wait_batch(tbe_engine *e, const uint64_t *keys, const int32_t *permits,
                          const int64_t *ts_us, uint64_t n, int64_t id_base, uint8_t *status,
                          int32_t *remaining, uint64_t *n_evicted) {
    if (!e || !n_evicted) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_QUEUEING) return fail(e, TBE_EINVAL, "not a queueing engine");
    if (n && !ts_us) return fail(e, TBE_EINVAL, "null buffer");
    e->wait_mode = 1;
    return status_batch(e, keys, permits, ts_us, n, id_base, status, remaining, n_evicted);
}

tbe_status tbe_queue_attempt_batch(tbe_engine *e, const uint64_t *keys, const int32_t *permits,
                                   const int64_t *ts_us, uint64_t n, uint8_t *status,
                                   int32_t *remaining) {
    if (!e) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_QUEUEING) return fail(e, TBE_EINVAL, "not a queueing engine");
    if (n && !ts_us) return fail(e, TBE_EINVAL, "null buffer");
    uint64_t n_ev = 0;
    e->wait_mode = 0;
    return status_batch(e, keys, permits, ts_us, n, 0, status, remaining, &n_ev);
}

tbe_status tbe_approx_acquire_batch(tbe_engine *e, const uint64_t *keys, const int32_t *permits,
                                    uint64_t n, int32_t wait, int64_t id_base, uint8_t *status,
                                    int32_t *available, uint64_t *n_evicted) {
    if (!e || !n_evicted) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_APPROXIMATE) return fail(e, TBE_EINVAL, "not an approximate engine");
    e->wait_mode = wait ? 1 : 0;
    return status_batch(e, keys, permits, nullptr, n, id_base, status, available, n_evicted);
}

tbe_status tbe_wait_batch_device(tbe_engine *e, const uint64_t *d_keys, const int32_t *d_permits,
                                 const int64_t *d_ts_us, uint64_t n, int64_t id_base, int32_t wait,
                                 uint8_t *d_status, int32_t *d_remaining, void *stream) {
    if (!e) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_QUEUEING) return fail(e, TBE_EINVAL, "not a queueing engine");
    if (n && !d_ts_us) return fail(e, TBE_EINVAL, "null buffer");
    e->wait_mode = wait ? 1 : 0;
    return status_batch_device(e, d_keys, d_permits, d_ts_us, n, id_base, d_status, d_remaining, stream);
}

tbe_status tbe_approx_acquire_batch_device(tbe_engine *e, const uint64_t *d_keys, const int32_t *d_permits,
                                           uint64_t n, int32_t wait, int64_t id_base, uint8_t *d_status,
                                           int32_t *d_available, void *stream) {
    if (!e) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_APPROXIMATE) return fail(e, TBE_EINVAL, "not an approximate engine");
    e->wait_mode = wait ? 1 : 0;
    return status_batch_device(e, d_keys, d_permits, nullptr, n, id_base, d_status, d_available, stream);
}

// Host-buffer queue / approximate batch from page-locked buffers: chunks of kHostChunk
// requests, copy-in on cin, decide on the engine stream, copy-out on cout, so copies
// overlap the decisions (as acquire_chunked).  The batch is validated on the host before
// anything is applied; chunk c's request ids and eviction causes are offset by c's
// position, so the result is the unchunked call's.
static tbe_status status_chunked(tbe_engine *e, const uint64_t *keys, const int32_t *permits, const int64_t *ts,
                                 uint64_t n, int64_t id_base, uint8_t *status, int32_t *remaining,
                                 uint32_t *nev) {
    const uint64_t nch = (n + kHostChunk - 1) / kHostChunk;
    {
        tbe_status rc = copy_in_chunks(e, keys, permits, ts, n, nch);
        if (rc != TBE_OK) return rc;
    }
    if (!host_validate(e, keys, permits, ts, n)) {
        HIP_TRY(e, hipStreamSynchronize(e->cin));
        return fail(e, TBE_EINVAL, "invalid request in batch (key >= n_keys, permits < 0 or ts < 0)");
    }
    HIP_TRY(e, hipMemsetAsync(e->counters, 0, sizeof(uint32_t), e->stream));
    for (uint64_t c = 0; c < nch; ++c) {
        const uint64_t o = c * kHostChunk, m = std::min(kHostChunk, n - o);
        tbe_status rc = run_batch(e, e->d_keys + o, e->d_permits + o, ts ? e->d_ts + o : nullptr, m,
                                  e->d_granted + o, e->d_remaining + o, nullptr, id_base + (int64_t)o,
                                  e->ev_chunk[c], e->cout, (uint32_t)o);
        if (rc != TBE_OK) return rc;
        HIP_TRY(e, hipMemcpyAsync(status + o, e->d_granted + o, m, hipMemcpyDeviceToHost, e->cout));
        HIP_TRY(e, hipMemcpyAsync(remaining + o, e->d_remaining + o, m * sizeof(int32_t), hipMemcpyDeviceToHost,
                                  e->cout));
    }
    HIP_TRY(e, hipMemcpyAsync(nev, e->counters, sizeof(uint32_t), hipMemcpyDeviceToHost, e->cout));
    HIP_TRY(e, hipStreamSynchronize(e->cout));
    return TBE_OK;
}

static tbe_status status_batch(tbe_engine *e, const uint64_t *keys, const int32_t *permits,
                               const int64_t *ts_us, uint64_t n, int64_t id_base, uint8_t *status,
                               int32_t *remaining, uint64_t *n_evicted) {
    *n_evicted = 0;
    e->evicted.clear();
    e->ev_pending = false;
    if (n == 0) return TBE_OK;
    if (!keys || !permits || !status || !remaining) return fail(e, TBE_EINVAL, "null buffer");
    {
        tbe_status qrc = sync_queued(e);
        if (qrc != TBE_OK) return qrc;
    }
    if (id_base < 0 || (uint64_t)id_base + n > (1ull << 47))
        return fail(e, TBE_EINVAL, "request ids must lie in [0, 2^47)");
    HIP_TRY(e, hipSetDevice(e->device));
    tbe_status rc = ensure_host_staging(e, n);
    if (rc != TBE_OK) return rc;
    // Evictions in one batch are bounded by the entries queued before it plus n.
    const uint64_t need_ev = e->queued_total + n;
    if (need_ev > e->ev_cap) {
        dfree(e->ev_cause);
        dfree(e->ev_id);
        e->ev_cap = 0;
        HIP_TRY(e, hipMalloc(&e->ev_cause, need_ev * sizeof(uint32_t)));
        HIP_TRY(e, hipMalloc(&e->ev_id, need_ev * sizeof(int64_t)));
        e->ev_cap = need_ev;
    }
    hipStream_t st = e->stream;
    uint32_t flag = 0, nev = 0;
    if (n >= 2 * kHostChunk && host_pinned(keys) && host_pinned(permits) && (!ts_us || host_pinned(ts_us)) &&
        host_pinned(status) && host_pinned(remaining)) {
        rc = status_chunked(e, keys, permits, ts_us, n, id_base, status, remaining, &nev);
        if (rc != TBE_OK) return rc;
    } else {
        HIP_TRY(e, hipMemsetAsync(e->counters, 0, sizeof(uint32_t), st));
        HIP_TRY(e, hipMemcpyAsync(e->d_keys, keys, n * sizeof(uint64_t), hipMemcpyHostToDevice, st));
        HIP_TRY(e, hipMemcpyAsync(e->d_permits, permits, n * sizeof(int32_t), hipMemcpyHostToDevice, st));
        if (ts_us)
            HIP_TRY(e, hipMemcpyAsync(e->d_ts, ts_us, n * sizeof(int64_t), hipMemcpyHostToDevice, st));
        rc = run_batch(e, e->d_keys, e->d_permits, ts_us ? e->d_ts : nullptr, n, e->d_granted,
                       e->d_remaining, st, id_base);
        if (rc != TBE_OK) return rc;
        HIP_TRY(e, hipMemcpyAsync(&flag, e->last_err, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        HIP_TRY(e, hipMemcpyAsync(&nev, e->counters, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        HIP_TRY(e, hipMemcpyAsync(status, e->d_granted, n, hipMemcpyDeviceToHost, st));
        HIP_TRY(e, hipMemcpyAsync(remaining, e->d_remaining, n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        HIP_TRY(e, hipStreamSynchronize(st));
    }
    if (flag) {
        HIP_TRY(e, hipMemsetAsync(e->sticky, 0, sizeof(uint32_t), st));
        HIP_TRY(e, hipStreamSynchronize(st));
        return fail(e, TBE_EINVAL, "invalid request in batch (key >= n_keys, permits < 0 or ts < 0)");
    }
    if (nev) {
        std::vector<uint32_t> cause(nev);
        std::vector<int64_t> id(nev);
        HIP_TRY(e, hipMemcpy(cause.data(), e->ev_cause, nev * sizeof(uint32_t), hipMemcpyDeviceToHost));
        HIP_TRY(e, hipMemcpy(id.data(), e->ev_id, nev * sizeof(int64_t), hipMemcpyDeviceToHost));
        e->evicted.resize(nev);
        for (uint32_t i = 0; i < nev; ++i) e->evicted[i] = {cause[i], id[i]};
        std::sort(e->evicted.begin(), e->evicted.end());
    }
    uint64_t queued = 0;
    for (uint64_t i = 0; i < n; ++i) queued += status[i] == TBE_WAIT_QUEUED;
    e->queued_total = e->queued_total + queued - nev;
    *n_evicted = nev;
    return TBE_OK;
}

tbe_status tbe_evicted(tbe_engine *e, uint64_t *cause_index, int64_t *request_id, uint64_t capacity,
                       uint64_t *n_written) {
    if (!e || !n_written) return TBE_EINVAL;
    if (e->ev_pending) {   // the last batch was a device-pointer wait batch
        HIP_TRY(e, hipSetDevice(e->device));
        HIP_TRY(e, hipDeviceSynchronize());
        uint32_t nev = 0;
        HIP_TRY(e, hipMemcpy(&nev, e->counters, sizeof(uint32_t), hipMemcpyDeviceToHost));
        if (nev > e->ev_cap) return fail(e, TBE_EDEVICE, "eviction log overflow");
        std::vector<uint32_t> cause(nev);
        std::vector<int64_t> id(nev);
        if (nev) {
            HIP_TRY(e, hipMemcpy(cause.data(), e->ev_cause, nev * sizeof(uint32_t), hipMemcpyDeviceToHost));
            HIP_TRY(e, hipMemcpy(id.data(), e->ev_id, nev * sizeof(int64_t), hipMemcpyDeviceToHost));
        }
        e->evicted.resize(nev);
        for (uint32_t i = 0; i < nev; ++i) e->evicted[i] = {cause[i], id[i]};
        std::sort(e->evicted.begin(), e->evicted.end());
        e->ev_pending = false;
    }
    const uint64_t m = std::min<uint64_t>(capacity, e->evicted.size());
    if (m && (!cause_index || !request_id)) return fail(e, TBE_EINVAL, "null buffer");
    for (uint64_t i = 0; i < m; ++i) {
        cause_index[i] = e->evicted[i].first;
        request_id[i] = e->evicted[i].second;
    }
    *n_written = m;
    return TBE_OK;
}

tbe_status tbe_refresh(tbe_engine *e, int64_t ts_us, uint64_t *n_granted) {
    if (!e || !n_granted) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_QUEUEING) return fail(e, TBE_EINVAL, "not a queueing engine");
    if (ts_us < 0) return fail(e, TBE_EINVAL, "ts_us < 0");
    *n_granted = 0;
    e->drained.clear();
    HIP_TRY(e, hipSetDevice(e->device));
    {
        tbe_status qrc = sync_queued(e);
        if (qrc != TBE_OK) return qrc;
    }
    if (e->queued_total == 0) return TBE_OK;
    if (e->queued_total > e->log_cap) {
        dfree(e->log_keyseq);
        dfree(e->log_id);
        dfree(e->log_rem);
        e->log_cap = 0;
        HIP_TRY(e, hipMalloc(&e->log_keyseq, e->queued_total * sizeof(uint64_t)));
        HIP_TRY(e, hipMalloc(&e->log_id, e->queued_total * sizeof(int64_t)));
        HIP_TRY(e, hipMalloc(&e->log_rem, e->queued_total * sizeof(int32_t)));
        e->log_cap = e->queued_total;
    }
    hipStream_t st = e->stream;
    HIP_TRY(e, hipMemsetAsync(e->counters + 1, 0, sizeof(uint32_t), st));
    const uint64_t blocks = std::min<uint64_t>((e->cfg.n_keys + kBlock - 1) / kBlock, 8192);
    with_qhdr(e, [&](auto *qh) {
        k_drain<<<(unsigned)blocks, kBlock, 0, st>>>(e->cfg.n_keys, e->table, qh, e->ring, e->params, e->qp, ts_us,
                                                    e->log_keyseq, e->log_id, e->log_rem, e->counters + 1,
                                                    (uint32_t)std::min<uint64_t>(e->log_cap, 0xFFFFFFFFu));
    });
    HIP_TRY(e, hipGetLastError());
    uint32_t cnt = 0;
    HIP_TRY(e, hipMemcpyAsync(&cnt, e->counters + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(e, hipStreamSynchronize(st));
    if (cnt) {
        std::vector<uint64_t> ks(cnt);
        std::vector<int64_t> id(cnt);
        std::vector<int32_t> rem(cnt);
        HIP_TRY(e, hipMemcpy(ks.data(), e->log_keyseq, cnt * sizeof(uint64_t), hipMemcpyDeviceToHost));
        HIP_TRY(e, hipMemcpy(id.data(), e->log_id, cnt * sizeof(int64_t), hipMemcpyDeviceToHost));
        HIP_TRY(e, hipMemcpy(rem.data(), e->log_rem, cnt * sizeof(int32_t), hipMemcpyDeviceToHost));
        std::vector<uint32_t> order(cnt);
        for (uint32_t i = 0; i < cnt; ++i) order[i] = i;
        std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return ks[a] < ks[b]; });
        e->drained.resize(cnt);
        for (uint32_t i = 0; i < cnt; ++i)
            e->drained[i] = std::make_tuple(ks[order[i]] >> 16, id[order[i]], rem[order[i]]);
    }
    e->queued_total -= cnt;
    *n_granted = cnt;
    return TBE_OK;
}

tbe_status tbe_refresh_bound(tbe_engine *e, uint64_t *bound) {
    if (!e || !bound) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_QUEUEING) return fail(e, TBE_EINVAL, "not a queueing engine");
    // every drained entry holds >= 1 permit (zero-permit requests are never queued) and a
    // tick grants at most TokenLimit tokens per key
    const uint64_t per_key = std::min<uint64_t>(e->qp.cap, (uint64_t)std::max(e->qp.token_limit, 1));
    *bound = std::min<uint64_t>(e->queued_total, e->cfg.n_keys * per_key);
    return TBE_OK;
}

tbe_status tbe_refresh_device(tbe_engine *e, int64_t ts_us, uint64_t *d_keyseq, int64_t *d_request_id,
                              int32_t *d_remaining, uint64_t capacity, uint32_t *d_count, void *stream) {
    if (!e || !d_count) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_QUEUEING) return fail(e, TBE_EINVAL, "not a queueing engine");
    if (ts_us < 0) return fail(e, TBE_EINVAL, "ts_us < 0");
    uint64_t bound = 0;
    tbe_status rc = tbe_refresh_bound(e, &bound);
    if (rc != TBE_OK) return rc;
    if (capacity < bound || bound > 0xFFFFFFFFull)
        return fail(e, TBE_EINVAL, "drain log capacity %llu below the bound %llu (tbe_refresh_bound)",
                    (unsigned long long)capacity, (unsigned long long)bound);
    if (bound && (!d_keyseq || !d_request_id || !d_remaining)) return fail(e, TBE_EINVAL, "null buffer");
    HIP_TRY(e, hipSetDevice(e->device));
    e->drained.clear();
    hipStream_t st = stream ? (hipStream_t)stream : e->stream;
    HIP_TRY(e, hipMemsetAsync(d_count, 0, sizeof(uint32_t), st));
    if (bound == 0) return TBE_OK;   // nothing queued
    const uint64_t blocks = std::min<uint64_t>((e->cfg.n_keys + kBlock - 1) / kBlock, 8192);
    with_qhdr(e, [&](auto *qh) {
        k_drain<<<(unsigned)blocks, kBlock, 0, st>>>(e->cfg.n_keys, e->table, qh, e->ring, e->params, e->qp, ts_us,
                                                    d_keyseq, d_request_id, d_remaining, d_count,
                                                    (uint32_t)std::min<uint64_t>(capacity, 0xFFFFFFFFu));
    });
    HIP_TRY(e, hipGetLastError());
    e->queued_exact = false;   // queued_total stays an upper bound
    return TBE_OK;
}

tbe_status tbe_wait_batch_tick_device(tbe_engine *e, const uint64_t *d_keys, const int32_t *d_permits,
                                      const int64_t *d_ts_us, uint64_t n, int64_t id_base, int32_t wait,
                                      uint8_t *d_status, int32_t *d_remaining, int64_t tick_ts_us,
                                      uint64_t *d_keyseq, int64_t *d_request_id, int32_t *d_log_remaining,
                                      uint64_t capacity, uint32_t *d_count, void *stream) {
    if (!e || !d_count) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_QUEUEING) return fail(e, TBE_EINVAL, "not a queueing engine");
    if (tick_ts_us < 0) return fail(e, TBE_EINVAL, "tick_ts_us < 0");
    if (n == 0) return tbe_refresh_device(e, tick_ts_us, d_keyseq, d_request_id, d_log_remaining, capacity,
                                          d_count, stream);
    if (!d_ts_us) return fail(e, TBE_EINVAL, "null buffer");
    // the drain log bound after this batch's possible enqueues (tbe_refresh_bound)
    const uint64_t per_key = std::min<uint64_t>(e->qp.cap, (uint64_t)std::max(e->qp.token_limit, 1));
    const uint64_t queued_after = wait ? std::min<uint64_t>(e->queued_total + n, ring_entries(e)) : e->queued_total;
    const uint64_t bound = std::min<uint64_t>(queued_after, e->cfg.n_keys * per_key);
    if (capacity < bound || bound > 0xFFFFFFFFull)
        return fail(e, TBE_EINVAL, "drain log capacity %llu below the bound %llu (tbe_refresh_bound after the batch)",
                    (unsigned long long)capacity, (unsigned long long)bound);
    if (bound && (!d_keyseq || !d_request_id || !d_log_remaining)) return fail(e, TBE_EINVAL, "null buffer");
    HIP_TRY(e, hipSetDevice(e->device));
    hipStream_t st = stream ? (hipStream_t)stream : e->stream;
    HIP_TRY(e, hipMemsetAsync(d_count, 0, sizeof(uint32_t), st));
    e->wait_mode = wait ? 1 : 0;
    e->qtick = QTick{tick_ts_us, d_keyseq, d_request_id, d_log_remaining, d_count,
                     (uint32_t)std::min<uint64_t>(capacity, 0xFFFFFFFFu)};
    const tbe_status rc = status_batch_device(e, d_keys, d_permits, d_ts_us, n, id_base, d_status, d_remaining, stream);
    e->qtick = QTick{-1, nullptr, nullptr, nullptr, nullptr, 0};
    if (rc != TBE_OK) return rc;
    e->drained.clear();
    e->queued_exact = false;   // queued_total stays an upper bound
    return TBE_OK;
}

tbe_status tbe_approx_collect(tbe_engine *e, int32_t *d_counts, void *stream) {
    if (!e || !d_counts) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_APPROXIMATE) return fail(e, TBE_EINVAL, "not an approximate engine");
    HIP_TRY(e, hipSetDevice(e->device));
    hipStream_t st = stream ? (hipStream_t)stream : e->stream;
    const uint64_t blocks = std::min<uint64_t>((e->cfg.n_keys + kBlock - 1) / kBlock, 8192);
    k_approx_collect<<<(unsigned)blocks, kBlock, 0, st>>>(e->cfg.n_keys, e->alocal, d_counts);
    HIP_TRY(e, hipGetLastError());
    HIP_TRY(e, hipStreamSynchronize(st));
    return TBE_OK;
}

static tbe_status approx_sync(tbe_engine *e, const int32_t *d_all_counts, uint32_t n_clients,
                              uint32_t my_client, int64_t ts_us, int64_t stagger_us, uint64_t *n_granted,
                              hipStream_t producer = nullptr);
tbe_status tbe_approx_sync(tbe_engine *e, const int32_t *d_all_counts, uint32_t n_clients,
                           uint32_t my_client, int64_t ts_us, int64_t stagger_us, uint64_t *n_granted) {
    if (!e || !d_all_counts || !n_granted) return TBE_EINVAL;
    return approx_sync(e, d_all_counts, n_clients, my_client, ts_us, stagger_us, n_granted);
}
tbe_status tbe_approx_sync_stream(tbe_engine *e, const int32_t *d_all_counts, uint32_t n_clients,
                                  uint32_t my_client, int64_t ts_us, int64_t stagger_us, void *stream,
                                  uint64_t *n_granted) {
    if (!e || !d_all_counts || !n_granted) return TBE_EINVAL;
    return approx_sync(e, d_all_counts, n_clients, my_client, ts_us, stagger_us, n_granted, (hipStream_t)stream);
}
// d_all_counts == nullptr: a single client whose collect runs inside the sync kernel.
// producer != nullptr: the counts are written by work enqueued on that stream (e.g. the
// collective that exchanged them); the sync kernel is ordered after it by an event.
static tbe_status approx_sync(tbe_engine *e, const int32_t *d_all_counts, uint32_t n_clients,
                              uint32_t my_client, int64_t ts_us, int64_t stagger_us, uint64_t *n_granted,
                              hipStream_t producer) {
    if (!e || !n_granted) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_APPROXIMATE) return fail(e, TBE_EINVAL, "not an approximate engine");
    if (n_clients == 0 || my_client >= n_clients || ts_us < 0 || stagger_us < 0)
        return fail(e, TBE_EINVAL, "bad sync arguments");
    *n_granted = 0;
    e->drained.clear();
    HIP_TRY(e, hipSetDevice(e->device));
    if (producer && producer != e->stream) {
        HIP_TRY(e, hipEventRecord(e->ev_in, producer));
        HIP_TRY(e, hipStreamWaitEvent(e->stream, e->ev_in, 0));
    }
    {
        tbe_status qrc = sync_queued(e);
        if (qrc != TBE_OK) return qrc;
    }
    const uint64_t need = std::max<uint64_t>(e->queued_total, 1);
    if (need > e->log_cap) {
        dfree(e->log_keyseq);
        dfree(e->log_id);
        dfree(e->log_rem);
        e->log_cap = 0;
        HIP_TRY(e, hipMalloc(&e->log_keyseq, need * sizeof(uint64_t)));
        HIP_TRY(e, hipMalloc(&e->log_id, need * sizeof(int64_t)));
        HIP_TRY(e, hipMalloc(&e->log_rem, need * sizeof(int32_t)));
        e->log_cap = need;
    }
    hipStream_t st = e->stream;
    HIP_TRY(e, hipMemsetAsync(e->counters + 1, 0, sizeof(uint32_t), st));
    const uint64_t blocks = std::min<uint64_t>((e->cfg.n_keys + kBlock - 1) / kBlock, 8192);
    k_approx_sync<<<(unsigned)blocks, kBlock, 0, st>>>(
        e->cfg.n_keys, e->alocal, e->aclient, e->gv, e->gp, e->gt, e->ring, e->ap, d_all_counts,
        n_clients, my_client, ts_us, stagger_us, e->log_keyseq, e->log_id, e->log_rem, e->counters + 1,
        (uint32_t)std::min<uint64_t>(e->log_cap, 0xFFFFFFFFu), n_clients != 1 ? 1u : 0u);
    HIP_TRY(e, hipGetLastError());
    e->aclient_lazy = n_clients == 1;
    uint32_t cnt = 0;
    HIP_TRY(e, hipMemcpyAsync(&cnt, e->counters + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(e, hipStreamSynchronize(st));
    if (cnt) {
        std::vector<uint64_t> ks(cnt);
        std::vector<int64_t> id(cnt);
        std::vector<int32_t> rem(cnt);
        HIP_TRY(e, hipMemcpy(ks.data(), e->log_keyseq, cnt * sizeof(uint64_t), hipMemcpyDeviceToHost));
        HIP_TRY(e, hipMemcpy(id.data(), e->log_id, cnt * sizeof(int64_t), hipMemcpyDeviceToHost));
        HIP_TRY(e, hipMemcpy(rem.data(), e->log_rem, cnt * sizeof(int32_t), hipMemcpyDeviceToHost));
        std::vector<uint32_t> order(cnt);
        for (uint32_t i = 0; i < cnt; ++i) order[i] = i;
        std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return ks[a] < ks[b]; });
        e->drained.resize(cnt);
        for (uint32_t i = 0; i < cnt; ++i)
            e->drained[i] = std::make_tuple(ks[order[i]] >> 16, id[order[i]], rem[order[i]]);
    }
    e->queued_total -= cnt;
    *n_granted = cnt;
    return TBE_OK;
}

tbe_status tbe_approx_refresh(tbe_engine *e, int64_t ts_us, uint64_t *n_granted) {
    if (!e || !n_granted) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_APPROXIMATE) return fail(e, TBE_EINVAL, "not an approximate engine");
    if (ts_us < 0) return fail(e, TBE_EINVAL, "ts_us < 0");
    HIP_TRY(e, hipSetDevice(e->device));
    return approx_sync(e, nullptr, 1, 0, ts_us, 0, n_granted);
}

tbe_status tbe_approx_query(tbe_engine *e, uint64_t key, int32_t *local, int32_t *global_score,
                            double *est, int32_t *available, uint32_t *queued) {
    if (!e || !local || !global_score || !est || !available || !queued) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_APPROXIMATE) return fail(e, TBE_EINVAL, "not an approximate engine");
    if (key >= e->cfg.n_keys) return fail(e, TBE_EINVAL, "key out of range");
    HIP_TRY(e, hipSetDevice(e->device));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    ALocal a;
    AClient c;
    if (e->aclient_lazy) {   // (idempotent: the value a one-client sync would have written)
        k_aclient_derive<<<1, kBlock, 0, e->stream>>>(key, 1, e->gv, e->gp, e->aclient, e->ap.period_s);
        HIP_TRY(e, hipGetLastError());
        HIP_TRY(e, hipStreamSynchronize(e->stream));
    }
    HIP_TRY(e, hipMemcpy(&a, e->alocal + key, sizeof a, hipMemcpyDeviceToHost));
    HIP_TRY(e, hipMemcpy(&c, e->aclient + key, sizeof c, hipMemcpyDeviceToHost));
    *local = a.local;
    *global_score = c.global;
    *est = c.est;
    const int32_t d = (int32_t)((uint32_t)a.cap - (uint32_t)a.local);
    *available = d > 0 ? d : 0;
    *queued = a.hc >> 16;
    return TBE_OK;
}

tbe_status tbe_approx_export_state(tbe_engine *e, uint64_t first, uint64_t count, double *v, double *p,
                                   int64_t *t_us) {
    if (!e) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_APPROXIMATE) return fail(e, TBE_EINVAL, "not an approximate engine");
    if (first > e->cfg.n_keys || count > e->cfg.n_keys - first)
        return fail(e, TBE_EINVAL, "range out of bounds");
    if (count == 0) return TBE_OK;
    if (!v || !p || !t_us) return fail(e, TBE_EINVAL, "null buffer");
    HIP_TRY(e, hipSetDevice(e->device));
    HIP_TRY(e, hipDeviceSynchronize());   // after every enqueued batch and sync, whatever its stream
    HIP_TRY(e, hipMemcpy(v, e->gv + first, count * sizeof(double), hipMemcpyDeviceToHost));
    HIP_TRY(e, hipMemcpy(p, e->gp + first, count * sizeof(double), hipMemcpyDeviceToHost));
    HIP_TRY(e, hipMemcpy(t_us, e->gt + first, count * sizeof(int64_t), hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < count; ++i)
        if (t_us[i] == kAbsent) v[i] = p[i] = 0.0;   // absent: the sync script's default {0, 0}
    return TBE_OK;
}

tbe_status tbe_approx_import_state(tbe_engine *e, uint64_t first, uint64_t count, const double *v,
                                   const double *p, const int64_t *t_us) {
    if (!e) return TBE_EINVAL;
    if (e->cfg.kind != TBE_KIND_APPROXIMATE) return fail(e, TBE_EINVAL, "not an approximate engine");
    if (first > e->cfg.n_keys || count > e->cfg.n_keys - first)
        return fail(e, TBE_EINVAL, "range out of bounds");
    if (count == 0) return TBE_OK;
    if (!v || !p || !t_us) return fail(e, TBE_EINVAL, "null buffer");
    std::vector<double> tv(count), tp(count);
    for (uint64_t i = 0; i < count; ++i) {
        if (t_us[i] != kAbsent && t_us[i] < 0) return fail(e, TBE_EINVAL, "t_us < 0");
        tv[i] = t_us[i] == kAbsent ? 0.0 : v[i];
        tp[i] = t_us[i] == kAbsent ? 0.0 : p[i];
    }
    HIP_TRY(e, hipSetDevice(e->device));
    HIP_TRY(e, hipDeviceSynchronize());
    if (e->aclient_lazy) {
        // the client views still follow from the tier rows this import overwrites: write them
        const uint64_t blocks = std::min<uint64_t>((e->cfg.n_keys + kBlock - 1) / kBlock, 8192);
        k_aclient_derive<<<(unsigned)blocks, kBlock, 0, e->stream>>>(0, e->cfg.n_keys, e->gv, e->gp, e->aclient,
                                                                     e->ap.period_s);
        HIP_TRY(e, hipGetLastError());
        HIP_TRY(e, hipStreamSynchronize(e->stream));
        e->aclient_lazy = false;
    }
    HIP_TRY(e, hipMemcpy(e->gv + first, tv.data(), count * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(e, hipMemcpy(e->gp + first, tp.data(), count * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(e, hipMemcpy(e->gt + first, t_us, count * sizeof(int64_t), hipMemcpyHostToDevice));
    return TBE_OK;
}

tbe_status tbe_refresh_log(tbe_engine *e, uint64_t *keys, int64_t *request_id, int32_t *remaining,
                           uint64_t capacity, uint64_t *n_written) {
    if (!e || !n_written) return TBE_EINVAL;
    const uint64_t m = std::min<uint64_t>(capacity, e->drained.size());
    if (m && (!keys || !request_id || !remaining)) return fail(e, TBE_EINVAL, "null buffer");
    for (uint64_t i = 0; i < m; ++i) {
        keys[i] = std::get<0>(e->drained[i]);
        request_id[i] = std::get<1>(e->drained[i]);
        remaining[i] = std::get<2>(e->drained[i]);
    }
    *n_written = m;
    return TBE_OK;
}

tbe_status tbe_queue_of(tbe_engine *e, uint64_t key, int64_t *request_id, int32_t *permits,
                        uint32_t capacity, uint32_t *count) {
    if (!e || !count) return TBE_EINVAL;
    if (e->cfg.kind == TBE_KIND_TOKEN_BUCKET) return fail(e, TBE_EINVAL, "engine has no queues");
    if (key >= e->cfg.n_keys) return fail(e, TBE_EINVAL, "key out of range");
    HIP_TRY(e, hipSetDevice(e->device));
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    const uint32_t rcap = e->cfg.kind == TBE_KIND_QUEUEING ? e->qp.cap : e->ap.cap;
    uint32_t head = 0, cnt = 0;
    if (e->cfg.kind == TBE_KIND_QUEUEING) {
        uint64_t h = 0;
        if (e->qh32) {
            uint32_t h32 = 0;
            HIP_TRY(e, hipMemcpy(&h32, reinterpret_cast<uint32_t *>(e->qhdr) + key, sizeof h32, hipMemcpyDeviceToHost));
            h = qh_widen(h32);
        } else {
            HIP_TRY(e, hipMemcpy(&h, e->qhdr + key, sizeof(uint64_t), hipMemcpyDeviceToHost));
        }
        head = (uint32_t)(h & 0xFFFFu);
        cnt = (uint32_t)((h >> 16) & 0xFFFFu);
    } else {
        ALocal a;
        HIP_TRY(e, hipMemcpy(&a, e->alocal + key, sizeof a, hipMemcpyDeviceToHost));
        head = a.hc & 0xFFFFu;
        cnt = a.hc >> 16;
    }
    std::vector<uint64_t> ent(rcap);
    HIP_TRY(e, hipMemcpy(ent.data(), e->ring + key * (uint64_t)rcap, rcap * sizeof(uint64_t),
                         hipMemcpyDeviceToHost));
    if (cnt && (!request_id || !permits) && capacity) return fail(e, TBE_EINVAL, "null buffer");
    for (uint32_t j = 0; j < cnt && j < capacity; ++j) {
        const uint64_t x = ent[(head + j) % rcap];
        request_id[j] = (int64_t)(x >> 16);
        permits[j] = (int32_t)(x & 0xFFFFu);
    }
    *count = cnt;
    return TBE_OK;
}

// CancelQueueState.TrySetCanceled (Q:480-506, A:531-557) for cancels grouped into runs of
// one key (the host sorts them stably by key): one thread per run applies its cancels in
// call order.  A found entry leaves the ring at once, the later entries close up behind
// it (order kept), count -1 and qsum (_queueCount) -= its permits.  The reference instead
// leaves a canceled registration in its deque until the drain reaches it, where it
// consumes tokens and A:489 adds its count back a second time; a
// bounded ring cannot hold entries that no longer count against QueueLimit.
extern "C++" {   // (inside the C ABI's extern "C" block: a template needs C++ linkage)
template <typename HW>
__global__ __launch_bounds__(256) void k_cancel(
    const uint64_t *__restrict__ ckeys, const int64_t *__restrict__ cids,
    const uint32_t *__restrict__ run_start, uint32_t n_runs, int32_t approx,
    HW *__restrict__ qhdr, ALocal *__restrict__ alocal, uint64_t *__restrict__ ring,
    uint32_t cap, uint8_t *__restrict__ hit) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_runs) return;
    const uint32_t c0 = run_start[r], c1 = run_start[r + 1];
    const uint64_t key = ckeys[c0];
    uint32_t head, cnt;
    int64_t qsum;
    ALocal a{};
    if (approx) {
        a = alocal[key];
        head = a.hc & 0xFFFFu;
        cnt = a.hc >> 16;
        qsum = a.qsum;
    } else {
        const uint64_t h = qh_widen(qhdr[key]);
        head = (uint32_t)(h & 0xFFFFu);
        cnt = (uint32_t)((h >> 16) & 0xFFFFu);
        qsum = (int64_t)(h >> 32);
    }
    uint64_t *__restrict__ kr = ring + key * (uint64_t)cap;
    bool changed = false;
    for (uint32_t c = c0; c < c1; ++c) {
        const int64_t id = cids[c];
        uint32_t j = 0;
        if (id < 0) j = cnt;   // never a request id: not queued
        while (j < cnt && (int64_t)(kr[(head + j) % cap] >> 16) != id) ++j;
        if (j == cnt) {
            hit[c] = 0;
            continue;
        }
        qsum -= (int64_t)(kr[(head + j) % cap] & 0xFFFFu);
        if (approx && (kr[(head + j) % cap] & 0xFFFFu) == 0) a.zc = (uint16_t)(a.zc - 1);
        for (; j + 1 < cnt; ++j) kr[(head + j) % cap] = kr[(head + j + 1) % cap];
        --cnt;
        hit[c] = 1;
        changed = true;
    }
    if (!changed) return;
    if (approx) {
        a.qsum = (uint16_t)qsum;
        a.hc = (head & 0xFFFFu) | (cnt << 16);
        alocal[key] = a;
    } else {
        qhdr[key] = qh_store<HW>(qh_pack(head, cnt, qsum));
    }
}
}   // extern "C++"

tbe_status tbe_queue_cancel(tbe_engine *e, const uint64_t *keys, const int64_t *request_ids,
                            uint64_t n, uint8_t *cancelled, uint64_t *n_cancelled) {
    if (!e || !n_cancelled) return TBE_EINVAL;
    *n_cancelled = 0;
    if (e->cfg.kind == TBE_KIND_TOKEN_BUCKET) return fail(e, TBE_EINVAL, "engine has no queues");
    if (n == 0) return TBE_OK;
    if (!keys || !request_ids || !cancelled) return fail(e, TBE_EINVAL, "null buffer");
    if (n >= (1ull << 31)) return fail(e, TBE_EINVAL, "batch too large");
    for (uint64_t i = 0; i < n; ++i)
        if (keys[i] >= e->cfg.n_keys) return fail(e, TBE_EINVAL, "key out of range");
    std::vector<uint32_t> ord(n);
    for (uint32_t i = 0; i < (uint32_t)n; ++i) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return keys[x] < keys[y]; });
    std::vector<uint64_t> ck(n);
    std::vector<int64_t> ci(n);
    std::vector<uint32_t> runs;
    for (uint64_t c = 0; c < n; ++c) {
        ck[c] = keys[ord[c]];
        ci[c] = request_ids[ord[c]];
        if (c == 0 || ck[c] != ck[c - 1]) runs.push_back((uint32_t)c);
    }
    const uint32_t n_runs = (uint32_t)runs.size();
    runs.push_back((uint32_t)n);
    // one scratch allocation: keys | ids | run starts | hits
    const size_t off_ids = n * sizeof(uint64_t), off_runs = off_ids + n * sizeof(int64_t);
    const size_t off_hit = off_runs + runs.size() * sizeof(uint32_t), bytes = off_hit + n;
    struct Scratch {
        char *p = nullptr;
        ~Scratch() { dfree(p); }
    } s;
    HIP_TRY(e, hipSetDevice(e->device));
    HIP_TRY(e, hipDeviceSynchronize());   // after every enqueued batch, whatever its stream
    HIP_TRY(e, hipMalloc(&s.p, bytes));
    HIP_TRY(e, hipMemcpy(s.p, ck.data(), off_ids, hipMemcpyHostToDevice));
    HIP_TRY(e, hipMemcpy(s.p + off_ids, ci.data(), n * sizeof(int64_t), hipMemcpyHostToDevice));
    HIP_TRY(e, hipMemcpy(s.p + off_runs, runs.data(), runs.size() * sizeof(uint32_t),
                         hipMemcpyHostToDevice));
    const bool approx = e->cfg.kind == TBE_KIND_APPROXIMATE;
    const uint32_t rcap = approx ? e->ap.cap : e->qp.cap;
    with_qhdr(e, [&](auto *qh) {
        k_cancel<<<(n_runs + 255) / 256, 256, 0, e->stream>>>(
            (const uint64_t *)s.p, (const int64_t *)(s.p + off_ids), (const uint32_t *)(s.p + off_runs),
            n_runs, approx ? 1 : 0, qh, e->alocal, e->ring, rcap, (uint8_t *)(s.p + off_hit));
    });
    HIP_TRY(e, hipGetLastError());
    HIP_TRY(e, hipStreamSynchronize(e->stream));
    std::vector<uint8_t> hit(n);
    HIP_TRY(e, hipMemcpy(hit.data(), s.p + off_hit, n, hipMemcpyDeviceToHost));
    uint64_t m = 0;
    for (uint64_t c = 0; c < n; ++c) {
        cancelled[ord[c]] = hit[c];
        m += hit[c];
    }
    e->queued_total -= std::min(e->queued_total, m);
    *n_cancelled = m;
    return TBE_OK;
}

tbe_status tbe_layout(const tbe_engine *e, uint32_t *passes, uint32_t *r_bits, uint32_t *packed) {
    if (!e || !passes || !r_bits || !packed) return TBE_EINVAL;
    *passes = (uint32_t)e->passes;
    *r_bits = (uint32_t)e->r_bits;
    *packed = (e->packed ? 1u : 0u) | (e->hot_cap ? 2u : 0u) | (e->pipeline ? 4u : 0u) |
              (e->narrow ? 8u : 0u) | (e->medium ? 16u : 0u) | (e->foldrec ? 32u : 0u) |
              (e->dig1 ? 64u : 0u) | (e->unrank ? 128u : 0u) | (e->n0 ? 256u : 0u) | (e->qh32 ? 512u : 0u);
    return TBE_OK;
}

tbe_status tbe_batch_format(const tbe_engine *e, uint64_t n, uint32_t *out, uint32_t n_out) {
    if (!e || !out || n_out < 8) return TBE_EINVAL;
    const FoldFmt G = batch_fold_fmt(e, n);
    out[0] = (uint32_t)e->passes;
    out[1] = (uint32_t)G.on;
    out[2] = (uint32_t)G.pw;                       // reply-position bits of a fold record
    out[3] = (uint32_t)G.tw;                       // time-offset bits of a fold record
    out[4] = (uint32_t)e->pf.kb;                   // pass-0 record: key bits
    out[5] = (uint32_t)e->pf.pb;                   // permit-code bits
    out[6] = (uint32_t)(G.n0 ? e->pf.w0 : e->pf.wb);   // pass-0 time-offset bits (narrow records: w0)
    out[7] = (uint32_t)e->r_bits;
    if (n_out > 8) {   // 1: a sparse token-bucket batch (k_fold_sparse + listed dense buckets, no hot runs)
        const bool tb = e->cfg.kind == TBE_KIND_TOKEN_BUCKET;
        out[8] = (tb && fold_wide_min(e, n) > 1u) ? 1u : 0u;
    }
    return TBE_OK;
}

tbe_status tbe_stage_times(tbe_engine *e, double *out, uint32_t n_out, uint32_t *n_written) {
    if (!e || !out || !n_written) return TBE_EINVAL;
    double ms_sum[ST_COUNT] = {};
    if (!e->ev_marks.empty()) {
        HIP_TRY(e, hipSetDevice(e->device));
        HIP_TRY(e, hipEventSynchronize(e->ev_pool[e->ev_marks.back().second + 1]));
        for (const auto &m : e->ev_marks) {
            float ms = 0.f;
            HIP_TRY(e, hipEventElapsedTime(&ms, e->ev_pool[m.second], e->ev_pool[m.second + 1]));
            ms_sum[m.first] += ms;
        }
    }
    e->ev_marks.clear();
    e->ev_used = 0;
    const uint32_t m = std::min<uint32_t>(n_out, ST_COUNT);
    for (uint32_t i = 0; i < m; ++i) out[i] = ms_sum[i];
    *n_written = m;
    return TBE_OK;
}

}  // extern "C"
