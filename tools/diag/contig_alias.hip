// Diagnostic (round 6): do physically contiguous device allocations
// (hipExtMallocWithFlags(..., hipDeviceMallocContiguous)) ever share memory with another
// live allocation of the same process?
//
// Round 5 saw intermittent wrong replies from queue / approximate engines whose rings were
// allocated contiguous, only in engines created after another engine was freed.  This
// program takes the engine out of the picture: it replays engine-shaped allocation
// sequences (a table, queue headers, a ring -- contiguous or ordinary -- and workspace
// buffers), creating and freeing "engines" of several sizes in turn.  After every create it
// stamps each live buffer with its own pattern (buffer id << 40 | word index), then checks
// every live buffer.  A word that reads another buffer's pattern means two live
// allocations alias.  Nothing is timed; nothing runs on the engine.
//
// build: hipcc --offload-arch=gfx950 -O2 -o tools/diag/contig_alias tools/diag/contig_alias.hip
// usage: tools/diag/contig_alias [trials] [contig_mask]   (mask bit 0 table, 1 headers, 2 ring)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                      \
        }                                                                                      \
    } while (0)

__global__ void k_stamp(uint64_t *p, uint64_t n, uint64_t id) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = (id << 40) | i;
}

// counts words that do not hold this buffer's stamp; records the first foreign id seen.
// `rot` shifts the block -> word mapping against k_stamp's, so a word is read by a
// workgroup on another XCD than the one that wrote it (workgroups go round-robin over the
// 8 XCDs, each with its own L2 and address-translation caches)
__global__ void k_check(const uint64_t *p, uint64_t n, uint64_t id, unsigned long long *bad,
                        unsigned long long *foreign, uint32_t rot) {
    const uint64_t blk = (blockIdx.x + rot) % gridDim.x;
    for (uint64_t i = blk * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t v = p[i];
        if (v != ((id << 40) | i)) {
            atomicAdd(bad, 1ull);
            atomicCAS(foreign, 0ull, v | (1ull << 63));
        }
    }
}

struct Buf {
    uint64_t *p;
    uint64_t words;
    bool contig;
    const char *what;
};

static Buf alloc(uint64_t bytes, bool contig, const char *what) {
    Buf b{nullptr, bytes / 8, contig, what};
    if (contig) {
        if (hipExtMallocWithFlags(reinterpret_cast<void **>(&b.p), bytes, hipDeviceMallocContiguous) != hipSuccess) {
            (void)hipGetLastError();
            b.contig = false;
            CK(hipMalloc(&b.p, bytes));
        }
    } else {
        CK(hipMalloc(&b.p, bytes));
    }
    return b;
}

// one engine's resident buffers and a workspace of n requests (sizes as tbe_create /
// ensure_workspace make them for the queueing kind, QueueLimit 16)
static std::vector<Buf> make_engine(uint64_t n_keys, uint64_t n, unsigned mask) {
    std::vector<Buf> v;
    v.push_back(alloc(n_keys * 16, mask & 1, "table"));
    v.push_back(alloc(((n_keys + 1) & ~1ull) * 8, mask & 2, "qhdr"));
    v.push_back(alloc(n_keys * 16 * 8, mask & 4, "ring"));
    for (int pass = 0; pass < 2; ++pass) {
        v.push_back(alloc(n * 8, false, "rec"));
        v.push_back(alloc(n * 4, false, "perm"));
        v.push_back(alloc(n * 4, false, "idx"));
    }
    v.push_back(alloc(n * 4, false, "res0"));
    v.push_back(alloc(n * 4, false, "res1"));
    v.push_back(alloc(((n_keys >> 8) + 8) * 4, false, "bcount"));
    return v;
}

int main(int argc, char **argv) {
    const int trials = argc > 1 ? std::atoi(argv[1]) : 24;
    const unsigned mask = argc > 2 ? (unsigned)std::strtoul(argv[2], nullptr, 0) : 4u;
    unsigned long long *d_bad, *d_foreign;
    CK(hipMalloc(&d_bad, 8));
    CK(hipMalloc(&d_foreign, 8));
    // engine sizes in the order round 5's diagnostic created them (200k keys x 7, 5k, 1M,
    // 200k x 2), then a config-D engine (1e8 keys: a 12.8 GB ring) between small ones
    struct Shape { uint64_t keys, n; };
    const Shape seq[] = {{200000, 1 << 18}, {200000, 1 << 18}, {200000, 1 << 18}, {200000, 1 << 18},
                         {200000, 1 << 18}, {200000, 1 << 18}, {200000, 1 << 18}, {5000, 60000},
                         {1000000, 1 << 20}, {200000, 1 << 18}, {200000, 1 << 18},
                         {100000000, 1 << 22}, {200000, 1 << 18}, {1000000, 1 << 20}};
    const int nseq = sizeof(seq) / sizeof(seq[0]);
    std::vector<Buf> keep;   // an allocation that outlives every engine (as torch's cache does)
    keep.push_back(alloc(64ull << 20, false, "outside"));
    uint64_t total_bad = 0, engines = 0, contig_ok = 0;
    for (int t = 0; t < trials; ++t) {
        const Shape s = seq[t % nseq];
        std::vector<Buf> eng = make_engine(s.keys, s.n, mask);
        for (auto &b : eng) contig_ok += b.contig;
        std::vector<Buf> all = keep;
        all.insert(all.end(), eng.begin(), eng.end());
        for (size_t i = 0; i < all.size(); ++i)
            k_stamp<<<2048, 256>>>(all[i].p, all[i].words, i + 1);
        CK(hipDeviceSynchronize());
        uint64_t bad_here = 0;
        for (size_t i = 0; i < all.size(); ++i) {
            CK(hipMemset(d_bad, 0, 8));
            CK(hipMemset(d_foreign, 0, 8));
            unsigned long long bad = 0, foreign = 0;
            for (uint32_t rot = 0; rot < 8 && !bad; ++rot) {
                k_check<<<2048, 256>>>(all[i].p, all[i].words, i + 1, d_bad, d_foreign, rot);
                CK(hipMemcpy(&bad, d_bad, 8, hipMemcpyDeviceToHost));
                CK(hipMemcpy(&foreign, d_foreign, 8, hipMemcpyDeviceToHost));
            }
            // the copy engine's view of the first and last 8 MB (a path with its own translation)
            if (!bad) {
                const uint64_t w = std::min<uint64_t>(all[i].words, 1u << 20);
                std::vector<uint64_t> h(w);
                for (int end = 0; end < 2 && !bad; ++end) {
                    const uint64_t off = end ? all[i].words - w : 0;
                    CK(hipMemcpy(h.data(), all[i].p + off, w * 8, hipMemcpyDeviceToHost));
                    for (uint64_t j = 0; j < w; ++j)
                        if (h[j] != (((uint64_t)(i + 1) << 40) | (off + j))) {
                            if (!bad) foreign = h[j] | (1ull << 63);
                            ++bad;
                        }
                }
                if (bad) std::printf("  (seen by the copy engine)\n");
            }
            if (bad) {
                const uint64_t fid = (foreign & ~(1ull << 63)) >> 40;
                std::printf("trial %d (keys %llu): buffer %zu (%s%s, %llu words) has %llu foreign words, first from "
                            "buffer %llu (%s)\n",
                            t, (unsigned long long)s.keys, i, all[i].what, all[i].contig ? ", contiguous" : "",
                            (unsigned long long)all[i].words, bad, (unsigned long long)fid,
                            fid >= 1 && fid <= all.size() ? all[fid - 1].what : "?");
                bad_here += bad;
            }
        }
        total_bad += bad_here;
        ++engines;
        for (auto &b : eng) CK(hipFree(b.p));
        if (t % 4 == 3) std::printf("after %d engines: %llu foreign words\n", t + 1, (unsigned long long)total_bad);
        std::fflush(stdout);
    }
    for (auto &b : keep) CK(hipFree(b.p));
    std::printf("mask %u: %llu engines, %llu contiguous allocations granted, %llu foreign words in total\n", mask,
                (unsigned long long)engines, (unsigned long long)contig_ok, (unsigned long long)total_bad);
    return total_bad ? 1 : 0;
}
