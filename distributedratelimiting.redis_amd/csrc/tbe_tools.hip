// tbe_tools.hip -- device-side synthetic trace generation (include/tbe_tools.h).
//
// Not part of the reference interface: bench.py and the GPU tests use it to build
// request batches directly in HBM so PCIe never sits in a timed region.  The streams
// are bit-identical to oracle/trace.py and oracle/tb_ref.c (splitmix64 finaliser over
// a global request counter g = batch * n + i).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tbe_tools.h"

namespace {

constexpr uint64_t kGamma = 0x9E3779B97F4A7C15ull;
constexpr uint64_t kStreamPermits = 0xA5A5A5A5A5A5A5A5ull;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_gen_batch(uint64_t seed, uint64_t n_keys, uint64_t g0, uint64_t n, int32_t p_lo,
                            int32_t p_hi, int64_t ts0_us, int64_t interval_us,
                            uint64_t *__restrict__ keys, int32_t *__restrict__ permits,
                            int64_t *__restrict__ ts) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t span = (uint64_t)(p_hi - p_lo + 1);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t g = g0 + i;
        const uint64_t r = mix64(seed + g * kGamma);
        keys[i] = ((r >> 32) * n_keys) >> 32;
        if (p_lo == p_hi) {
            permits[i] = p_lo;
        } else {
            const uint64_t r2 = mix64((seed ^ kStreamPermits) + g * kGamma);
            permits[i] = p_lo + (int32_t)(((r2 >> 32) * span) >> 32);
        }
        ts[i] = ts0_us + (int64_t)(((unsigned __int128)i * (uint64_t)interval_us) / n);
    }
}

}  // namespace

extern "C" int tbe_gen_batch_device(uint64_t seed, uint64_t n_keys, uint64_t g0, uint64_t n,
                                    int32_t p_lo, int32_t p_hi, int64_t ts0_us, int64_t interval_us,
                                    uint64_t *d_keys, int32_t *d_permits, int64_t *d_ts,
                                    void *stream) {
    if (n == 0) return 0;
    if (n_keys == 0 || n_keys >= (1ull << 32) || p_hi < p_lo) return 1;
    const unsigned blocks = (unsigned)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
    k_gen_batch<<<blocks, 256, 0, (hipStream_t)stream>>>(seed, n_keys, g0, n, p_lo, p_hi, ts0_us,
                                                         interval_us, d_keys, d_permits, d_ts);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}
