// HBM ceilings for pass A's traffic mix, second probe (not part of the library): does the
// read+write mix of the tile path's pass A (16 B read + 2 B written per row, count-only C2)
// really cap reads at ~58 % of peak, or was the first probe (one 16-B load per column in
// flight, 4-B stores per lane) the limit?  Variants:
//   U     16-B loads in flight per column per lane (1, 2, 4)
//   SW    bytes stored per lane per store (4: u16 pair, 16: eight u16 cells)
//   NT    nontemporal stores (__builtin_nontemporal_store)
//   REG   stores go to per-workgroup contiguous regions (pass A's layout) instead of row order
// build: hipcc --offload-arch=gfx950 -O3 -o scripts/bw_probe2 scripts/bw_probe2.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

// rows are processed in units of 8 (one lane: 4 x double2 of each column = 8 rows = 16 B of
// u16 cells); a workgroup walks units blockIdx.x, +gridDim.x, ... (grid stride)
template <int U, int SW, bool NT, bool WRITE>
__global__ __launch_bounds__(256) void k_mix8(const double2 *__restrict__ x, const double2 *__restrict__ y, uint64_t nunits,
                                              uint16_t *out, double *sink) {
    double acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (; u + (U - 1) * stride < nunits; u += U * stride) {
        double2 a[U][4], b[U][4];
#pragma unroll
        for (int q = 0; q < U; q++)
#pragma unroll
            for (int k = 0; k < 4; k++) {
                a[q][k] = x[(u + q * stride) * 4 + k];
                b[q][k] = y[(u + q * stride) * 4 + k];
            }
#pragma unroll
        for (int q = 0; q < U; q++) {
            uint16_t c[8];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                c[2 * k] = (uint16_t)((int)(a[q][k].x * 100.0) + (int)(b[q][k].x * 7.0));
                c[2 * k + 1] = (uint16_t)((int)(a[q][k].y * 100.0) + (int)(b[q][k].y * 7.0));
                acc += a[q][k].x + b[q][k].y;
            }
            if constexpr (WRITE) {
                const uint64_t row = (u + q * stride) * 8;
                if constexpr (SW == 16) {
                    u32x4 w;
                    w.x = c[0] | (uint32_t)c[1] << 16;
                    w.y = c[2] | (uint32_t)c[3] << 16;
                    w.z = c[4] | (uint32_t)c[5] << 16;
                    w.w = c[6] | (uint32_t)c[7] << 16;
                    u32x4 *dst = reinterpret_cast<u32x4 *>(out + row);
                    if constexpr (NT) __builtin_nontemporal_store(w, dst);
                    else *dst = w;
                } else {
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        uint32_t w = c[2 * k] | (uint32_t)c[2 * k + 1] << 16;
                        uint32_t *dst = reinterpret_cast<uint32_t *>(out + row) + k;
                        if constexpr (NT) __builtin_nontemporal_store(w, dst);
                        else *dst = w;
                    }
                }
            }
        }
    }
    if (acc == 12345.678) sink[0] = acc;
}

// region layout: workgroup w processes a contiguous range of units and writes its cells to
// its own contiguous region in 64 runs (like 64 tiles), each run a 16-B store per lane
template <bool NT>
__global__ __launch_bounds__(256) void k_regions(const double2 *__restrict__ x, const double2 *__restrict__ y, uint64_t nunits,
                                                 uint16_t *out, double *sink) {
    double acc = 0;
    const uint64_t per = (nunits + gridDim.x - 1) / gridDim.x;
    const uint64_t u0 = blockIdx.x * per, u1 = u0 + per < nunits ? u0 + per : nunits;
    // 64 sub-regions of per*8/64 cells each (+ slack): a run is appended to sub-region (u % 64)
    const uint64_t sub = (per + 7) / 8 + 64;
    uint16_t *reg = out + blockIdx.x * (sub * 64);
    uint64_t fill = 0;
    for (uint64_t u = u0 + threadIdx.x; u < u1 + 255; u += 256) {
        const bool ok = u < u1;
        double2 a[4], b[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            a[k] = ok ? x[u * 4 + k] : make_double2(0, 0);
            b[k] = ok ? y[u * 4 + k] : make_double2(0, 0);
        }
        u32x4 w;
        w.x = (uint32_t)(a[0].x * 10) | (uint32_t)(b[0].y * 10) << 16;
        w.y = (uint32_t)(a[1].x * 10) | (uint32_t)(b[1].y * 10) << 16;
        w.z = (uint32_t)(a[2].x * 10) | (uint32_t)(b[2].y * 10) << 16;
        w.w = (uint32_t)(a[3].x * 10) | (uint32_t)(b[3].y * 10) << 16;
        acc += a[0].x + b[3].y;
        // the batch of 256 lanes writes 4 KB: 64 runs of 64 B (4 lanes) into 64 sub-regions
        const int t = threadIdx.x >> 2;
        u32x4 *dst = reinterpret_cast<u32x4 *>(reg + (uint64_t)t * sub + fill) + (threadIdx.x & 3);
        if (ok && fill + 32 <= sub) {
            if constexpr (NT) __builtin_nontemporal_store(w, dst);
            else *dst = w;
        }
        fill += 32;
    }
    if (acc == 12345.678) sink[0] = acc;
}

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? (uint64_t)atof(argv[1]) : 1000000000ull;
    const uint64_t nunits = n / 8;
    double *x, *y, *sink;
    uint16_t *out;
    CK(hipMalloc(&x, n * 8));
    CK(hipMalloc(&y, n * 8));
    CK(hipMemset(x, 0, n * 8));
    CK(hipMemset(y, 0, n * 8));
    CK(hipMalloc(&out, n * 2 + (64ull << 20)));
    CK(hipMalloc(&sink, 8));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](const char *name, auto launch) {
        for (int bpc : {4, 8}) {
            const unsigned g = cus * bpc;
            float best = 1e30f;
            for (int rep = 0; rep < 6; rep++) {
                CK(hipEventRecord(a));
                launch(g);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                if (rep && ms < best) best = ms;
            }
            printf("%-44s blocks/CU %d: %7.3f ms  reads %5.2f TB/s (%4.1f %% of 8)\n", name, bpc, best,
                   16.0 * n / best / 1e9, 16.0 * n / best / 1e9 / 8.0 * 100);
        }
    };
    const double2 *X = reinterpret_cast<const double2 *>(x), *Y = reinterpret_cast<const double2 *>(y);
#define K(U, SW, NT, W) [&](unsigned g) { hipLaunchKernelGGL((k_mix8<U, SW, NT, W>), dim3(g), dim3(256), 0, 0, X, Y, nunits, out, sink); }
    run("read 16 B/row, U=1", K(1, 16, false, false));
    run("read 16 B/row, U=2", K(2, 16, false, false));
    run("read 16 + write 2, U=1, 4-B stores", K(1, 4, false, true));
    run("read 16 + write 2, U=1, 16-B stores", K(1, 16, false, true));
    run("read 16 + write 2, U=2, 16-B stores", K(2, 16, false, true));
    run("read 16 + write 2, U=1, 16-B NT stores", K(1, 16, true, true));
    run("read 16 + write 2, U=2, 16-B NT stores", K(2, 16, true, true));
    run("read 16 + write 2, U=1, 4-B NT stores", K(1, 4, true, true));
    run("regions: read 16 + write 2 (64 runs/WG)",
        [&](unsigned g) { hipLaunchKernelGGL((k_regions<false>), dim3(g), dim3(256), 0, 0, X, Y, nunits, out, sink); });
    run("regions: read 16 + write 2, NT",
        [&](unsigned g) { hipLaunchKernelGGL((k_regions<true>), dim3(g), dim3(256), 0, 0, X, Y, nunits, out, sink); });
    return 0;
}
