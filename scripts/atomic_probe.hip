// Scattered-atomic throughput on MI355X (not part of the library): could a count-only grid
// be aggregated with per-XCD private copies small enough to stay in each XCD's 4 MB L2,
// instead of the tile path's partition exchange?  Each workgroup adds 1 to random words of
// the copy of its XCD (blockIdx % 8); copy sizes from 256 KB to 8 MB; returning and
// non-returning 32-bit atomics.
// build: hipcc --offload-arch=gfx950 -O3 -o scripts/atomic_probe scripts/atomic_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

__device__ inline uint32_t mix(uint64_t x) {
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return (uint32_t)(x ^ (x >> 31));
}

template <bool RET>
__global__ __launch_bounds__(256) void k_atom(uint32_t *grids, uint32_t words, uint64_t n, uint32_t *sink) {
    uint32_t *g = grids + (uint64_t)(blockIdx.x & 7) * words;
    uint32_t acc = 0;
    const uint64_t step = (uint64_t)gridDim.x * 256;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += step) {
        const uint32_t w = (uint32_t)(((uint64_t)mix(i) * words) >> 32);
        if (RET) acc += atomicAdd(&g[w], 1u);
        else atomicAdd(&g[w], 1u);
    }
    if (RET && acc == 0xdeadbeef) sink[0] = acc;
}

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? (uint64_t)atof(argv[1]) : 1000000000ull;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *grids, *sink;
    const uint32_t max_words = (16u << 20) / 4;
    CK(hipMalloc(&grids, (size_t)8 * max_words * 4));
    CK(hipMalloc(&sink, 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (uint32_t kb : {256u, 1024u, 2048u, 3072u, 4096u, 8192u}) {
        const uint32_t words = kb * 256;
        for (int ret = 0; ret < 2; ret++) {
            float best = 1e30f;
            for (int rep = 0; rep < 4; rep++) {
                CK(hipMemset(grids, 0, (size_t)8 * words * 4));
                CK(hipEventRecord(a));
                if (ret) hipLaunchKernelGGL(k_atom<true>, dim3(cus * 8), dim3(256), 0, 0, grids, words, n, sink);
                else hipLaunchKernelGGL(k_atom<false>, dim3(cus * 8), dim3(256), 0, 0, grids, words, n, sink);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                if (rep && ms < best) best = ms;
            }
            printf("copy %5u KB per XCD, %s: %8.3f ms  %6.2e atomics/s\n", kb, ret ? "returning   " : "no return   ", best,
                   n / (best * 1e-3));
        }
    }
    return 0;
}
