// Pass-A exchange layouts and allocation placement (not part of the library).
// the same C2 pass A takes 6.2-7.4 ms depending on how much was
// allocated before its region scratch.  This probe writes the two exchange layouts pass A
// can use, at several placements of the scratch, in one process:
//   regions:  private (workgroup, tile) regions, each commit's C entries appended as T runs
//             of C / T entries (what tiled.hip does today; bw_probe5 part 2)
//   wgstream: one contiguous stream per workgroup, each commit's C entries (sorted by tile)
//             appended whole; pass B then gathers a tile's run from every (workgroup, commit)
// and the matching pass-B reads (tile t's entries from every region / every commit segment).
// Wide 16-B non-temporal stores, 512 threads, one workgroup per CU, 1e9 rows, best of 5.
// usage: bw_probe6 [rows] [dummy GB list, e.g. 0,1,2.5,7]
// build: hipcc --offload-arch=gfx950 -O3 -o scripts/bw_probe6 scripts/bw_probe6.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef unsigned int u4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

template <typename T> __device__ __forceinline__ void stnt(T *p, T v) { __builtin_nontemporal_store(v, p); }

// STREAM = false: entry j of commit c_local goes to region (w, t = j / RUN) at c_local * RUN + j % RUN
// STREAM = true:  entry j goes to w * wg_cap + c_local * (T * RUN) + j
template <int TH, int C, int NV, bool WV, bool STREAM>
__global__ __launch_bounds__(TH) void k_write(const d2 *__restrict__ v0, const d2 *__restrict__ v1, const d2 *__restrict__ v2,
                                              uint64_t n, int T, int RUN, uint64_t cap, uint16_t *ecell, double *eval,
                                              unsigned *sink) {
    constexpr int RPT = C / TH;
    const unsigned W = gridDim.x, w = blockIdx.x;
    const uint64_t ncommits = n / C;
    const d2 *vc[3] = {v0, v1, v2};
    uint64_t c_local = 0;
    for (uint64_t c = w; c < ncommits; c += W, c_local++) {
        const uint64_t r0 = c * C;
        d2 v[3][RPT / 2];
#pragma unroll
        for (int k = 0; k < NV; k++)
#pragma unroll
            for (int q = 0; q < RPT / 2; q++) v[k][q] = vc[k][r0 / 2 + q * TH + threadIdx.x];
        unsigned x = threadIdx.x;
#pragma unroll
        for (int k = 0; k < NV; k++)
#pragma unroll
            for (int q = 0; q < RPT / 2; q++) x += (unsigned)__builtin_bit_cast(uint64_t, v[k][q].x);
        auto dest = [&](int j) -> uint64_t {
            if constexpr (STREAM) return (uint64_t)w * cap + c_local * (uint64_t)(T * RUN) + j;
            const int t = j / RUN;
            return ((uint64_t)w * T + t) * cap + c_local * RUN + (j - t * RUN);
        };
#pragma unroll
        for (int q = 0; q < RPT / 8; q++) {
            const int j = 8 * (q * TH + threadIdx.x);
            if (j >= T * RUN) continue;
            stnt<u4>(reinterpret_cast<u4 *>(ecell + dest(j)), u4{x, x + q, x ^ q, x});
        }
        if constexpr (WV) {
#pragma unroll
            for (int q = 0; q < RPT / 2; q++) {
                const int j = 2 * (q * TH + threadIdx.x);
                if (j >= T * RUN) continue;
                stnt<d2>(reinterpret_cast<d2 *>(eval + dest(j)), v[0][q]);
            }
        }
    }
}

// pass-B reads: workgroup u = tile t x a slice of the pass-A workgroups; a wave reads one
// (workgroup, commit) segment of RUN entries per 16 lanes (STREAM) or one region whole (!STREAM)
template <int TH, bool WV, bool STREAM>
__global__ __launch_bounds__(TH) void k_read(int W, int T, int RUN, uint64_t ncw, uint64_t cap, const uint16_t *ecell,
                                             const double *eval, int wslices, unsigned *sink) {
    const int t = blockIdx.x / wslices, sl = blockIdx.x % wslices;
    const int w0 = (int)((int64_t)W * sl / wslices), w1 = (int)((int64_t)W * (sl + 1) / wslices);
    double acc = 0;
    unsigned ac = 0;
    if constexpr (STREAM) {
        // segments (w, c): RUN entries at w * cap + c * T * RUN + t * RUN; a wave per segment,
        // lane l reads entries 8l .. 8l + 7 (cells, one 16-B load) and pairs of values
        const int grp = threadIdx.x / 16, lane = threadIdx.x % 16, ng = TH / 16;  // 16 lanes per segment
        const uint64_t nseg = (uint64_t)(w1 - w0) * ncw;
        for (uint64_t s = grp; s < nseg; s += ng) {
            const uint64_t w = w0 + s / ncw, c = s % ncw;
            const uint64_t base = w * cap + c * (uint64_t)(T * RUN) + (uint64_t)t * RUN;
            for (int j = 8 * lane; j < RUN; j += 128) {
                u4 cw = *reinterpret_cast<const u4 *>(ecell + base + j);
                ac += cw.x ^ cw.w;
                if constexpr (WV) {
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        d2 vv = *reinterpret_cast<const d2 *>(eval + base + j + 2 * q);
                        acc += vv.x + vv.y;
                    }
                }
            }
        }
    } else {
        const uint64_t len = ncw * RUN;
        for (int w = w0; w < w1; w++) {
            const uint64_t base = ((uint64_t)w * T + t) * cap;
            for (uint64_t j = 8 * threadIdx.x; j < len; j += 8 * TH) {
                u4 cw = *reinterpret_cast<const u4 *>(ecell + base + j);
                ac += cw.x ^ cw.w;
                if constexpr (WV) {
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        d2 vv = *reinterpret_cast<const d2 *>(eval + base + j + 2 * q);
                        acc += vv.x + vv.y;
                    }
                }
            }
        }
    }
    if (acc == 12345.678 || ac == 0xdeadbeefu) sink[0] = ac;
}

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? (uint64_t)atof(argv[1]) : 1000000000ull;
    std::vector<double> dummies = {0, 1, 2.5, 7};
    if (argc > 2) {
        dummies.clear();
        char *s = strdup(argv[2]);
        for (char *tok = strtok(s, ","); tok; tok = strtok(nullptr, ",")) dummies.push_back(atof(tok));
    }
    void *v[3];
    unsigned *sink;
    for (auto &p : v) {
        CK(hipMalloc(&p, n * 8));
        CK(hipMemset(p, 1, n * 8));
    }
    CK(hipMalloc(&sink, 8));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const unsigned W = cus;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto time = [&](auto launch) {
        float best = 1e30f;
        for (int rep = 0; rep < 6; rep++) {
            CK(hipEventRecord(a));
            launch();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (rep && ms < best) best = ms;
        }
        return best;
    };
    const d2 *V0 = (const d2 *)v[0], *V1 = (const d2 *)v[1], *V2 = (const d2 *)v[2];
    for (double gb : dummies) {
        void *dummy = nullptr, *cell, *wv;
        if (gb > 0) CK(hipMalloc(&dummy, (size_t)(gb * 1e9)));
        const uint64_t ecap = n + n / 4 + (64ull << 20);
        CK(hipMalloc(&cell, ecap * 2));
        CK(hipMalloc(&wv, ecap * 8));
        printf("dummy %.1f GB  cells %p  values %p\n", gb, cell, wv);
        uint16_t *C_ = (uint16_t *)cell;
        double *W_ = (double *)wv;
        auto one = [&](const char *name, int C, int T, double rd, double wr, auto kw_reg, auto kw_str, auto kr_reg, auto kr_str) {
            const uint64_t nn = n / C * C;
            const int RUN = (C / T) & ~7;
            const uint64_t ncw = (nn / C + W - 1) / W;  // commits per workgroup
            const uint64_t cap_reg = ncw * RUN + 64, cap_str = ncw * (uint64_t)T * RUN + 64;
            const double scale = (double)RUN * T / C;
            float ar = time([&] { hipLaunchKernelGGL(kw_reg, dim3(W), dim3(512), 0, 0, V0, V1, V2, nn, T, RUN, cap_reg, C_, W_, sink); });
            float br = time([&] { hipLaunchKernelGGL(kr_reg, dim3(T * 8), dim3(512), 0, 0, (int)W, T, RUN, ncw, cap_reg, C_, W_, 8, sink); });
            float as = time([&] { hipLaunchKernelGGL(kw_str, dim3(W), dim3(512), 0, 0, V0, V1, V2, nn, T, RUN, cap_str, C_, W_, sink); });
            float bs = time([&] { hipLaunchKernelGGL(kr_str, dim3(T * 8), dim3(512), 0, 0, (int)W, T, RUN, ncw, cap_str, C_, W_, 8, sink); });
            const double wb = wr * scale;
            printf("  %-18s T%3d run%4d  regions: A %6.3f ms (%4.2f of 8 TB/s reads) B %6.3f ms (%4.2f TB/s)   wgstream: A %6.3f ms (%4.2f) B %6.3f ms (%4.2f TB/s)\n",
                   name, T, RUN, ar, rd * n / ar / 1e9 / 8.0, br, wb * n / br / 1e9, as, rd * n / as / 1e9 / 8.0, bs, wb * n / bs / 1e9);
            fflush(stdout);
        };
        one("count 16+2", 8192, 65, 16, 2, k_write<512, 8192, 2, false, false>, k_write<512, 8192, 2, false, true>,
            k_read<512, false, false>, k_read<512, false, true>);
        one("c+s 24+10", 12288, 129, 24, 10, k_write<512, 12288, 3, true, false>, k_write<512, 12288, 3, true, true>,
            k_read<512, true, false>, k_read<512, true, true>);
        CK(hipFree(cell));
        CK(hipFree(wv));
        if (dummy) CK(hipFree(dummy));
    }
    return 0;
}
