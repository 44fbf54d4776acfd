// tbe_hash.hpp -- key hashing shared by the device code and its host-side mirrors
// (distributedratelimiting.redis_amd/cluster.py, workloads.py): the splitmix64
// finaliser, key ownership across GPUs and a fixed bijection of
// [0, n) used to spread dense ids.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define TBE_HASH_HD __host__ __device__
#else
#define TBE_HASH_HD
#endif

namespace tbe {

TBE_HASH_HD inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Owner GPU of a key among n: ((mix64(key) >> 32) * n) >> 32, which for n = 2^g is
// mix64(key) >> (64 - g), SURVEY.md §8e's partition (n = 8: mix64(key) >> 61).
TBE_HASH_HD inline uint32_t key_owner(uint64_t key, uint32_t n) {
    return (uint32_t)(((mix64(key) >> 32) * (uint64_t)n) >> 32);
}

// Virtual node of a key for table-driven ownership (include/tbe_cluster.h owner maps):
// the top kOwnerMapBits bits of mix64(key).  An owner map assigns each of the 4096 virtual
// nodes to a GPU; the map v -> (v * n) >> 12 reproduces key_owner for n = 2^g <= 4096.
constexpr int kOwnerMapBits = 12;
constexpr uint32_t kOwnerMapSize = 1u << kOwnerMapBits;
TBE_HASH_HD inline uint32_t key_vnode(uint64_t key) { return (uint32_t)(mix64(key) >> (64 - kOwnerMapBits)); }

// A fixed bijection of [0, 2^bits): odd multiply-add then xorshift, three rounds
// (workloads.py _scramble); `mask` = 2^bits - 1, `sh` = max(1, bits / 2).
TBE_HASH_HD inline uint64_t scramble(uint64_t x, uint64_t mask, uint32_t sh) {
    x = (x * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull) & mask;
    x ^= x >> sh;
    x = (x * 0xD1B54A32D192ED03ull + 0x8CB92BA72F3D8DD7ull) & mask;
    x ^= x >> sh;
    x = (x * 0xAEF17502108EF2D9ull + 0x2545F4914F6CDD1Dull) & mask;
    x ^= x >> sh;
    return x;
}

// The same bijection restricted to [0, n) by cycle walking (n <= mask + 1).
TBE_HASH_HD inline uint64_t scramble_walk(uint64_t x, uint64_t n, uint64_t mask, uint32_t sh) {
    x = scramble(x, mask, sh);
    while (x >= n) x = scramble(x, mask, sh);
    return x;
}

// bits = max(1, bit_length(n - 1)) for the bijection of [0, n)
inline void scramble_params(uint64_t n, uint64_t &mask, uint32_t &sh) {
    int bits = 1;
    while (bits < 64 && ((n - 1) >> bits) != 0) ++bits;
    mask = (bits >= 64) ? ~0ull : ((1ull << bits) - 1);
    sh = (uint32_t)(bits / 2 > 1 ? bits / 2 : 1);
}

}  // namespace tbe
