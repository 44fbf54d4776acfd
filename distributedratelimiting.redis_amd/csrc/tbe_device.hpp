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

// Split an injected timestamp (us, >= 0, < 2^53) into Redis TIME's (sec, usec):
// an f64 estimate of ts/1e6 is off by at most one, fixed by one integer correction
// (tests/test_fastdiv.py checks the identity with the same operations).
__device__ __forceinline__ void split_ts(int64_t ts_us, int64_t &sec, int64_t &usec) {
    int64_t s = (int64_t)((double)ts_us * 1e-6);
    int64_t r = ts_us - s * 1000000;
    if (r < 0) {
        s -= 1;
        r += 1000000;
    } else if (r >= 1000000) {
        s += 1;
        r -= 1000000;
    }
    sec = s;
    usec = r;
}

// TB:202-203: new_t = now[1] + (now[2] / 1000000).  The quotient usec / 1e6 is the
// IEEE-correctly-rounded one: q0 = u * fl(1e-6), r = fma(-q0, 1e6, u), q = fma(r,
// fl(1e-6), q0) equals u / 1e6 for EVERY u in [0, 1e6) (checked exhaustively,
// tests/test_fastdiv.py).  Then one rounded add, as in Lua.
__device__ __forceinline__ double new_t_of(int64_t ts_us) {
    int64_t sec, usec;
    split_ts(ts_us, sec, usec);
    const double x = (double)usec;
    const double rcp = 1.0 / 1000000.0;
    const double q0 = x * rcp;
    const double r = __builtin_fma(-q0, 1000000.0, x);
    const double q = __builtin_fma(r, rcp, q0);
    return (double)sec + q;
}

struct TbParams {
    double cap;       // Lua `capacity` (TB:184), TokenLimit as f64
    double rate;      // Lua `fill_rate` (TB:185), FillRatePerSecond bits
    int64_t ttl_ms;   // EXPIRE seconds (TB:234) * 1000
};

// Everything of one request that does not depend on bucket state, computed in
// parallel before the per-key serial order is resolved.
struct ReqTime {
    double new_t;    // TB:203
    int64_t exp_lt;  // passive expiry: a stored grant time t_us < exp_lt has lapsed
    int64_t ts;      // the injected TIME itself: what a grant stores
};
// Redis lapses a key when the command's millisecond snapshot ms = ts / 1000 exceeds
// grant_ms + ttl_ms (EXPIRE at TB:235), grant_ms = t_us / 1000.  For t_us >= 0 and
// integer X, floor(t_us / 1000) < X iff t_us < 1000 X, so the test is one compare:
// t_us < 1000 * (ms - ttl_ms).
__device__ __forceinline__ ReqTime req_time(int64_t ts_us, int64_t ttl_ms) {
    ReqTime r;
    r.new_t = new_t_of(ts_us);
    r.exp_lt = (ts_us / 1000 - ttl_ms) * 1000;
    r.ts = ts_us;
    return r;
}

// The same quantities for timestamps close above a base: a batch's timestamps lie in a
// window of well under 2^32 us above its packed-record base, so (sec, usec) and the
// millisecond snapshot follow from the base's own split plus 32-bit arithmetic on the
// delta.  The results are identical to req_time's: sec = sec0 + (usec0 + d) / 1e6,
// usec = (usec0 + d) % 1e6, ts / 1000 = m0 + (r0 + d) / 1000, and new_t is formed from
// (sec, usec) by the same operations as new_t_of.  Timestamps outside the window (or a
// base that does not split) take req_time.
struct TimeBase {
    int64_t tbase;
    int64_t e0;        // 1000 * (tbase / 1000 - ttl_ms)
    uint32_t sec0;     // tbase / 1e6
    uint32_t usec0;    // tbase % 1e6
    uint32_t r0;       // tbase % 1000
    uint32_t ok;
};
constexpr uint64_t kRelMax = 0xFFFFFFFFull - 1000000ull;   // usec0 + d and r0 + d stay in u32
__host__ __device__ inline TimeBase time_base(int64_t tbase, int64_t ttl_ms) {
    TimeBase b{tbase, 0, 0, 0, 0, 0};
    if (tbase < 0) return b;
    const int64_t sec0 = tbase / 1000000;
    if (sec0 > (int64_t)0xFFFFFFFFll - 10000) return b;   // sec0 + (u32 / 1e6) fits in u32
    b.sec0 = (uint32_t)sec0;
    b.usec0 = (uint32_t)(tbase - sec0 * 1000000);
    b.r0 = (uint32_t)(tbase % 1000);
    b.e0 = (tbase / 1000 - ttl_ms) * 1000;
    b.ok = 1;
    return b;
}
__device__ __forceinline__ ReqTime req_time_rel(int64_t ts_us, const TimeBase &B, int64_t ttl_ms) {
    const uint64_t d = (uint64_t)ts_us - (uint64_t)B.tbase;
    if (!B.ok || ts_us < B.tbase || d > kRelMax) return req_time(ts_us, ttl_ms);
    const uint32_t u = B.usec0 + (uint32_t)d;
    const uint32_t s1 = u / 1000000u;
    const uint32_t usec = u - s1 * 1000000u;
    const uint32_t sec = B.sec0 + s1;
    const double x = (double)usec;
    const double rcp = 1.0 / 1000000.0;
    const double q0 = x * rcp;
    const double r = __builtin_fma(-q0, 1000000.0, x);
    const double q = __builtin_fma(r, rcp, q0);
    ReqTime rt;
    rt.new_t = (double)sec + q;
    rt.exp_lt = B.e0 + (int64_t)((B.r0 + (uint32_t)d) / 1000u) * 1000;
    rt.ts = ts_us;
    return rt;
}

// One evaluation of the acquire script (TB:202-238) on a key's stored row {v, t_us}
// (the Redis hash {v, t}), with the row's field t supplied by the caller as ft =
// new_t_of(row.t_us) (ignored while the key is absent).  Returns the packed reply: bit
// 31 = success (TB:224/238), bits 0-30 = trunc(new_v) (TB:238 -> RESP integer ->
// TB:73).  `modified` is set when the row changed: on a grant (HSET, TB:225-236) and
// when Redis' passive expiry deleted the key on access (the HGETALL at TB:210 finds it
// lapsed), which happens even if the request is then denied.  A call that leaves
// `modified` false leaves the row exactly as it found it.
__device__ __forceinline__ uint32_t tb_step_ft(Slot &row, double ft, int32_t permits,
                                               const ReqTime &rq, const TbParams &P, bool &modified) {
    const bool had = row.t_us != kAbsent;
    // EXPIRE at TB:235 lapses when the command-time snapshot (ms) exceeds grant_ms + ttl.
    const bool expired = had && row.t_us < rq.exp_lt;
    const bool present = had && !expired;
    const double pv = present ? row.v : P.cap;                          // TB:211-215
    const double pt = present ? ft : rq.new_t;
    const double delta_t = lua_max(0.0, rq.new_t - pt);                 // TB:218
    const double fill = delta_t * P.rate;                               // TB:221: mul ...
    double x = lua_max(0.0, lua_min(P.cap, pv + fill));                 // ... then add (never fused)
    const double p = (double)permits;
    const bool granted = x >= p;                                        // TB:224
    if (granted) {
        x = x - p;                                                      // TB:227
        row.v = x;                                                      // TB:230 HSET v, t
        row.t_us = rq.ts;
    } else if (expired) {
        row.v = P.cap;                                                  // deleted by passive expiry
        row.t_us = kAbsent;
    }
    modified = granted || expired;
    return (granted ? 0x80000000u : 0u) | (uint32_t)(int32_t)x;         // {success, new_v}
}

// The same, deriving field t from the row itself.
__device__ __forceinline__ uint32_t tb_step(Slot &row, int32_t permits, const ReqTime &rq,
                                            const TbParams &P, bool &modified) {
    const double ft = new_t_of(row.t_us == kAbsent ? 0 : row.t_us);
    return tb_step_ft(row, ft, permits, rq, P, modified);
}

__device__ __forceinline__ uint32_t tb_acquire(Slot &s, int32_t permits, int64_t ts_us,
                                               const TbParams &P, bool &modified) {
    return tb_step(s, permits, req_time(ts_us, P.ttl_ms), P, modified);
}

// ----------------------------------------------------------------- streaming memory hints
// Non-temporal loads/stores for data touched once per kernel (table slices, pass records,
// permutations, replies): they stream through the caches instead of displacing lines
// that other waves are still reusing.
template <typename T>
__device__ __forceinline__ T ld_nt(const T *p) { return __builtin_nontemporal_load(p); }
template <typename T>
__device__ __forceinline__ void st_nt(T *p, T v) { __builtin_nontemporal_store(v, p); }

// ----------------------------------------------------------------- wave / block helpers
// XCD-aware block -> tile remap (cdna_hip_programming.md T1, the bijective form): blocks
// b and b+8 share an XCD (round-robin dispatch), so give each XCD a contiguous range of
// tiles.  Consecutive tiles write adjacent pieces of the same digit runs; on one XCD
// their partial lines merge in that XCD's L2.  Placement only changes speed.
__device__ __forceinline__ uint32_t xcd_swizzle(uint32_t b, uint32_t nblk) {
    const uint32_t xcd = b & 7u, q = nblk >> 3, r = nblk & 7u;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

__device__ __forceinline__ uint64_t lanemask_lt() {
    const int lane = threadIdx.x & 63;
    return (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
}

// Exclusive scan of one value per thread over a BLOCK-thread block; *total gets the
// sum.  `wsum` is BLOCK/64 words of LDS.  Every thread must call it (two barriers).
template <int BLOCK>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t *wsum, uint32_t *total) {
    constexpr int W = BLOCK / 64;
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
    for (int j = 0; j < W; ++j) {
        const uint32_t s = wsum[j];
        pre += (j < w) ? s : 0u;
        tot += s;
    }
    *total = tot;
    __syncthreads();
    return pre + v - x;
}

// Stable local ranking of a tile of BLOCK*ITEMS elements by an 8-bit digit.
// Element e = it*BLOCK + threadIdx.x (striped, so global loads coalesce); tile order is
// e order.
//   A. every wave ballot-matches the 8 digit bits of each of its ITEMS rounds: in-wave
//      rank, and the wave's count per digit, written to cnt[it][wave][digit] (u16);
//   B. the 256 digit columns of cnt (ITEMS*W entries each, in tile order) are scanned
//      in place to exclusive prefixes -- two threads per column when BLOCK = 512 --
//      and a block scan of the column totals gives lstart[digit];
//   C. lpos = lstart[d] + cnt[it][wave][d] + in-wave rank.
// `cnt` needs ITEMS*W*256*2 bytes of LDS; callers alias it with their staging buffer
// (it is dead after C).  Four barriers per tile.
template <int BLOCK>
struct RankLds {
    static constexpr int W = BLOCK / 64;
    static constexpr int PARTS = BLOCK / kDigits;   // threads per digit column
    uint32_t lstart[kDigits];
    uint32_t part[PARTS][kDigits];                  // per-segment column sums
    uint32_t wsum[W];
};

template <int BLOCK, int ITEMS>
__device__ __forceinline__ void rank_tile(const uint32_t (&key)[ITEMS], int shift, int nvalid,
                                          RankLds<BLOCK> &L, uint16_t *cnt,
                                          uint32_t (&lpos)[ITEMS]) {
#define TBE_DIG(it) ((key[it] >> shift) & (kDigits - 1))
    constexpr int W = BLOCK / 64;
    constexpr int COL = ITEMS * W;                      // entries per digit column
    static_assert(BLOCK % kDigits == 0, "whole digit columns per thread group");
    const int tid = threadIdx.x, w = tid >> 6;
    {
        uint4 *z = reinterpret_cast<uint4 *>(cnt);
        const uint4 zero = {0u, 0u, 0u, 0u};
        for (int i = tid; i < COL * kDigits * 2 / 16; i += BLOCK) z[i] = zero;
    }
    __syncthreads();
    const uint64_t lt = lanemask_lt();
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const int e = it * BLOCK + tid;
        const bool valid = e < nvalid;
        const uint32_t dg = TBE_DIG(it);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < kDigitBits; ++b) {
            const bool bit = (dg >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        lpos[it] = (uint32_t)__popcll(peers & lt);   // in-wave rank for now
        if (valid && lpos[it] == 0) cnt[(it * W + w) * kDigits + dg] = (uint16_t)__popcll(peers);
    }
    __syncthreads();
    // B: column scans.  Entry j of column d is cnt[j*256 + d], j = it*W + wave; PARTS
    // threads share a column, each scanning one contiguous segment.
    constexpr int PARTS = BLOCK / kDigits;
    static_assert(COL % PARTS == 0, "column splits evenly");
    constexpr int SEG = COL / PARTS;
    const int d = tid & (kDigits - 1);
    const int part = tid / kDigits;
    uint32_t s = 0;
#pragma unroll 8
    for (int j = part * SEG; j < (part + 1) * SEG; ++j) {
        const uint32_t c = cnt[j * kDigits + d];
        cnt[j * kDigits + d] = (uint16_t)s;
        s += c;
    }
    L.part[part][d] = s;
    __syncthreads();
    uint32_t off = 0, total = 0;
#pragma unroll
    for (int q = 0; q < PARTS; ++q) {
        const uint32_t v = L.part[q][d];
        off += (q < part) ? v : 0u;
        total += v;
    }
    if (part > 0) {
#pragma unroll 8
        for (int j = part * SEG; j < (part + 1) * SEG; ++j)
            cnt[j * kDigits + d] = (uint16_t)(cnt[j * kDigits + d] + off);
    }
    {
        // exclusive scan of the column totals, contributed by the part-0 thread of each
        // column (threads 0..255, in digit order; everyone else adds 0)
        uint32_t all;
        const uint32_t ex = block_excl_scan<BLOCK>(part == 0 ? total : 0u, L.wsum, &all);
        if (part == 0) L.lstart[d] = ex;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITEMS; ++it)
        lpos[it] += L.lstart[TBE_DIG(it)] + cnt[(it * W + w) * kDigits + TBE_DIG(it)];
#undef TBE_DIG
}

// Stable local ranking with WAVE-BLOCKED element order: element e of the tile lives in
// wave w = e / (64*ITEMS), item slot it = (e / 64) % ITEMS, lane e % 64, so tile order is
// (wave, slot, lane) order and each wave can rank its own 64*ITEMS elements with a
// running per-digit count of its own:
//   A. per slot, ballot-match the 8 digit bits; the lowest lane of each digit group adds
//      the group's size to its wave's counter (LDS atomic returning the old value), and
//      every lane's rank is that old value (read from the leader) plus its rank among its
//      peers -- no per-slot count matrix and no column scan over slots;
//   B. one thread per digit scans the W wave counts into per-wave offsets, and a block
//      scan of the digit totals gives lstart[digit];
//   C. lpos = lstart[d] + wave offset + in-wave rank.
// LDS: W*256 words (callers alias it with their staging buffer) plus RankLds.  Three
// barriers plus the block scan's two.
template <int BLOCK, int ITEMS>
__device__ __forceinline__ int wb_elem(int it) {
    return (int)((threadIdx.x >> 6) * (64 * ITEMS) + it * 64 + (threadIdx.x & 63));
}

template <int BLOCK, int ITEMS>
__device__ __forceinline__ void rank_tile_wb(const uint32_t (&key)[ITEMS], int shift, int nvalid,
                                             RankLds<BLOCK> &L, uint32_t *wcnt, uint32_t (&lpos)[ITEMS]) {
    constexpr int W = BLOCK / 64;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    uint32_t *mine = wcnt + w * kDigits;
#pragma unroll
    for (int i = lane; i < kDigits; i += 64) mine[i] = 0;   // this wave's row only
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const uint64_t lt = lanemask_lt();
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const int e = wb_elem<BLOCK, ITEMS>(it);
        const bool valid = e < nvalid;
        const uint32_t dg = (key[it] >> shift) & (kDigits - 1);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < kDigitBits; ++b) {
            const bool bit = (dg >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const int leader = peers ? __ffsll((long long)peers) - 1 : lane;
        uint32_t old = 0;
        if (valid && leader == lane) old = atomicAdd(&mine[dg], (uint32_t)__popcll(peers));
        old = __shfl(old, leader, 64);
        lpos[it] = old + (uint32_t)__popcll(peers & lt);
    }
    __syncthreads();
    // B: per digit, the waves' counts -> exclusive per-wave offsets; block scan of totals
    uint32_t tot = 0;
    if (tid < kDigits) {
#pragma unroll
        for (int v = 0; v < W; ++v) {
            const uint32_t c = wcnt[v * kDigits + tid];
            wcnt[v * kDigits + tid] = tot;
            tot += c;
        }
    }
    {
        uint32_t all;
        const uint32_t ex = block_excl_scan<BLOCK>(tid < kDigits ? tot : 0u, L.wsum, &all);
        if (tid < kDigits) L.lstart[tid] = ex;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const uint32_t dg = (key[it] >> shift) & (kDigits - 1);
        lpos[it] += L.lstart[dg] + mine[dg];
    }
}

}  // namespace tbe
