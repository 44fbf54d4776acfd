// tbe_device.hpp -- device-side building blocks of the batched token-bucket engine
// (gfx950 / CDNA4, wave64).  Included by tbe_engine.hip only.
//
// The decision arithmetic restates the reference acquire script
// (TokenBucket/RedisTokenBucketRateLimiter.cs, "TB" in SURVEY.md) line by line in
// IEEE binary64 with contraction disabled (this file is compiled with
// -ffp-contract=off and carries `#pragma clang fp contract(off)`): the script's
// `prev.v + (delta_t * fill_rate)` is a multiply THEN an add, two roundings, never
// an FMA (SURVEY.md §7 hard part (i)).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace tbe {

constexpr int kBlock = 256;            // 4 waves of 64
constexpr int kWaves = kBlock / 64;
constexpr int kDigitBits = 8;
constexpr int kDigits = 1 << kDigitBits;
constexpr int64_t kAbsent = INT64_MIN;  // t of a key never granted (or reset)

// One bucket-table row: Redis hash {v, t} of one key (TB:230), 16 B, AoS so that a
// key's state is one dwordx4 access.
struct __attribute__((aligned(16))) Slot {
    double v;      // field v
    int64_t t_us;  // injected TIME of the last grant; field t = new_t_of(t_us)
};

// ----------------------------------------------------------------- Lua / Redis semantics
// Lua 5.1 math.max / math.min keep the FIRST argument unless a later one is strictly
// better (lmathlib.c); the ternaries below reproduce that, including -0.0 and NaN.
__device__ __forceinline__ double lua_max(double a, double b) { return (b > a) ? b : a; }
__device__ __forceinline__ double lua_min(double a, double b) { return (b < a) ? b : a; }

// TB:202-203: new_t = now[1] + (now[2] / 1000000) over Redis TIME = (sec, usec).
// One correctly rounded f64 division (hipcc's default IEEE div sequence), one add.
__device__ __forceinline__ double new_t_of(int64_t ts_us) {
    const int64_t sec = ts_us / 1000000;
    const int64_t usec = ts_us - sec * 1000000;
    return (double)sec + ((double)usec / 1000000.0);
}

struct TbParams {
    double cap;       // Lua `capacity` (TB:184), TokenLimit as f64
    double rate;      // Lua `fill_rate` (TB:185), FillRatePerSecond bits
    int64_t ttl_ms;   // EXPIRE seconds (TB:234) * 1000
};

// One evaluation of the acquire script against the state held in `s` (TB:202-238).
// Returns the packed reply: bit 31 = success (TB:224/238), bits 0-30 = trunc(new_v)
// (TB:238 -> RESP integer -> TB:73).  Writes s on success only (TB:225-236).
__device__ __forceinline__ uint32_t tb_acquire(Slot &s, int32_t permits, int64_t ts_us,
                                               const TbParams &P, bool &granted) {
    const double new_t = new_t_of(ts_us);
    // HGETALL (TB:210) with Redis passive expiry: the key lapses when the command-time
    // snapshot (ms) exceeds grant_ms + ttl (EXPIRE at TB:235).
    const bool present = (s.t_us != kAbsent) && !((ts_us / 1000) > (s.t_us / 1000) + P.ttl_ms);
    const double pv = present ? s.v : P.cap;              // TB:211-215
    const double pt = present ? new_t_of(s.t_us) : new_t;
    const double delta_t = lua_max(0.0, new_t - pt);      // TB:218
    const double fill = delta_t * P.rate;                 // TB:221: mul ...
    double x = lua_max(0.0, lua_min(P.cap, pv + fill));   // ... then add (never fused)
    const double p = (double)permits;
    granted = x >= p;                                     // TB:224
    if (granted) {
        x = x - p;                                        // TB:227
        s.v = x;                                          // TB:230 HSET v, t
        s.t_us = ts_us;
    }
    return (granted ? 0x80000000u : 0u) | (uint32_t)(int32_t)x;   // {success, new_v}
}

// ----------------------------------------------------------------- wave / block helpers
__device__ __forceinline__ uint64_t lanemask_lt() {
    const int lane = threadIdx.x & 63;
    return (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
}

// Exclusive scan of one value per thread over a 256-thread block; *total gets the sum.
// `wsum` is 4 words of LDS.  Contains two barriers.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t *wsum, uint32_t *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t v = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    if (lane == 63) wsum[w] = v;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int j = 0; j < kWaves; ++j) {
        const uint32_t s = wsum[j];
        pre += (j < w) ? s : 0u;
        tot += s;
    }
    *total = tot;
    __syncthreads();
    return pre + v - x;
}

// Stable local ranking of a tile of kBlock*ITEMS elements by an 8-bit digit.
// Element e = it*kBlock + threadIdx.x (striped, so global loads coalesce); tile order
// is e order.  Produces, for every valid element, its position `lpos` in the tile
// sorted stably by digit, and lstart[d] = first position of digit d.
//   1. per (it, wave): ballot-match the 8 digit bits -> in-wave rank + wave count
//   2. per digit: exclusive scan of the counts over (it, wave) in tile order
//   3. block scan of the digit totals -> lstart
// LDS: cnt[ITEMS*kWaves*kDigits] u16, lstart[kDigits] u32, wsum[4] u32.
template <int ITEMS>
__device__ __forceinline__ void rank_tile(const uint32_t (&dig)[ITEMS], int nvalid, uint16_t *cnt,
                                          uint32_t *lstart, uint32_t *wsum,
                                          uint32_t (&lpos)[ITEMS]) {
    const int tid = threadIdx.x, w = tid >> 6;
    uint32_t *cnt32 = reinterpret_cast<uint32_t *>(cnt);
    for (int i = tid; i < ITEMS * kWaves * kDigits / 2; i += kBlock) cnt32[i] = 0;
    __syncthreads();
    const uint64_t lt = lanemask_lt();
    uint32_t wrank[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const int e = it * kBlock + tid;
        const bool valid = e < nvalid;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < kDigitBits; ++b) {
            const bool bit = (dig[it] >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        wrank[it] = (uint32_t)__popcll(peers & lt);
        if (valid && wrank[it] == 0)
            cnt[(it * kWaves + w) * kDigits + dig[it]] = (uint16_t)__popcll(peers);
    }
    __syncthreads();
    {
        const int d = tid;  // kBlock == kDigits: one digit column per thread
        uint32_t s = 0;
#pragma unroll 8
        for (int j = 0; j < ITEMS * kWaves; ++j) {
            const uint32_t c = cnt[j * kDigits + d];
            cnt[j * kDigits + d] = (uint16_t)s;
            s += c;
        }
        uint32_t total;
        lstart[d] = block_excl_scan(s, wsum, &total);
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const int e = it * kBlock + tid;
        lpos[it] = (e < nvalid)
                       ? lstart[dig[it]] + cnt[(it * kWaves + w) * kDigits + dig[it]] + wrank[it]
                       : 0u;
    }
}

}  // namespace tbe
