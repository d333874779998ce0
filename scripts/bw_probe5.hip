// HBM ceilings of the pass mixes with LANE-CONTIGUOUS accesses (not part of the library).
// bw_probe3 let each lane load and store four consecutive 16-B words, so every wave
// instruction was 64-B lane-strided; its copy reached 4.23 TB/s against the 6.29 TB/s float4
// copy of MI355X_MICROARCH.md.  Here every wave instruction covers one contiguous span
// (lane l of the block touches word base + q * TH + l), so this probe must reproduce the
// guide's copy rate before its mix numbers mean anything.
//
// Part 1, contiguous streams, 8 rows per lane per step, grid-stride:
//   a row reads KEY (0 / 4 B int32) + NV x 8 B (float64 columns) and writes CELL (0 / 2 B)
//   + WV x 8 B; the stores are either "narrow" (one 2-B cell / one 8-B value per lane per
//   instruction, what pass A issues today) or "wide" (16 B per lane: 8 cells / 2 values),
//   plain or non-temporal.
// Part 2, private (workgroup, tile) regions as pass A writes them: one workgroup per CU
//   (512 threads), commits of C rows dealt round-robin, each commit's entries appended to T
//   per-(workgroup, tile) regions as T runs of C / T entries (run length rounded to 8 so the
//   wide form has no head / tail), narrow or wide, plain or nt.
// Best of 6 (first run dropped).  build: hipcc --offload-arch=gfx950 -O3 -o scripts/bw_probe5 scripts/bw_probe5.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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

template <typename T, bool NT> __device__ __forceinline__ void st(T *p, T v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// WIDE: 16-B stores; NT: non-temporal stores
template <int TH, bool KEY, int NV, bool CELL, bool WV, bool WIDE, bool NT>
__global__ __launch_bounds__(TH) void k_mix(const u4 *__restrict__ key, const d2 *__restrict__ v0, const d2 *__restrict__ v1,
                                            const d2 *__restrict__ v2, uint64_t nsteps, uint16_t *cell, double *wv,
                                            unsigned *sink) {
    unsigned acc = 0;
    const d2 *vc[3] = {v0, v1, v2};
    for (uint64_t s = blockIdx.x; s < nsteps; s += gridDim.x) {
        const uint64_t r0 = s * (uint64_t)TH * 8;  // 8 rows per lane
        u4 k[2];
        d2 v[3][4];
        if constexpr (KEY) {
#pragma unroll
            for (int q = 0; q < 2; q++) k[q] = key[r0 / 4 + q * TH + threadIdx.x];
        }
#pragma unroll
        for (int c = 0; c < NV; c++)
#pragma unroll
            for (int q = 0; q < 4; q++) v[c][q] = vc[c][r0 / 2 + q * TH + threadIdx.x];
        // fold the loads into a few words so nothing is dead
        unsigned x = threadIdx.x;
        if constexpr (KEY) x ^= k[0].x ^ k[1].w;
#pragma unroll
        for (int c = 0; c < NV; c++)
#pragma unroll
            for (int q = 0; q < 4; q++) x = (x ^ (unsigned)__builtin_bit_cast(uint64_t, v[c][q].x)) + (unsigned)__builtin_bit_cast(uint64_t, v[c][q].y);
        if constexpr (CELL) {
            if constexpr (WIDE) {
                u4 cw = {x, x + 1, x + 2, x + 3};
                st<u4, NT>(reinterpret_cast<u4 *>(cell) + r0 / 8 + threadIdx.x, cw);
            } else {
#pragma unroll
                for (int q = 0; q < 8; q++) st<uint16_t, NT>(cell + r0 + q * TH + threadIdx.x, (uint16_t)(x + q));
            }
        } else {
            asm volatile("" ::"v"(x));  // keep the loads live
        }
        if constexpr (WV) {
            if constexpr (WIDE) {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    d2 o = NV ? v[0][q] : d2{(double)x, (double)q};
                    st<d2, NT>(reinterpret_cast<d2 *>(wv) + r0 / 2 + q * TH + threadIdx.x, o);
                }
            } else {
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    double o = NV ? ((q & 1) ? v[0][q >> 1].y : v[0][q >> 1].x) : (double)(x + q);
                    st<double, NT>(wv + r0 + q * TH + threadIdx.x, o);
                }
            }
        }
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

// Part 2: private (workgroup, tile) regions.  The workgroup's C rows per commit are loaded
// coalesced (NV f64 columns; the cell is derived from the loaded bits), and each commit's
// entries go out as T runs of RUN entries: entry j of the commit belongs to tile j / RUN and
// lands at region (w, t) offset c_local * RUN + (j - t * RUN).  Narrow: one 2-B cell + one
// 8-B value per lane per entry; wide: a lane stores 8 consecutive cells (16 B) and, per
// value, 2 consecutive values (16 B).
template <int TH, int C, int NV, bool WV, bool WIDE, bool NT>
__global__ __launch_bounds__(TH) void k_regions(const d2 *__restrict__ v0, const d2 *__restrict__ v1, const d2 *__restrict__ v2,
                                                uint64_t n, int T, int RUN, uint64_t region_cap, uint16_t *ecell, double *eval,
                                                unsigned *sink) {
    constexpr int RPT = C / TH;
    const unsigned W = gridDim.x, w = blockIdx.x;
    const uint64_t ncommits = n / C;
    const d2 *vc[3] = {v0, v1, v2};
    uint64_t c_local = 0;
    unsigned acc = 0;
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
        const uint64_t reg0 = (uint64_t)w * T * region_cap + c_local * RUN;
        if constexpr (!WIDE) {
#pragma unroll
            for (int q = 0; q < RPT; q++) {
                const int j = q * TH + threadIdx.x;
                const int t = j / RUN;
                if (t >= T) continue;
                const uint64_t e = reg0 + (uint64_t)t * region_cap + (j - t * RUN);
                st<uint16_t, NT>(ecell + e, (uint16_t)(x + q));
                if constexpr (WV) {
                    const double o = NV ? ((q & 1) ? v[0][q >> 1].y : v[0][q >> 1].x) : (double)x;
                    st<double, NT>(eval + e, o);
                }
            }
        } else {
            // cells: 8 entries per lane-store
#pragma unroll
            for (int q = 0; q < RPT / 8; q++) {
                const int j = 8 * (q * TH + threadIdx.x);
                const int t = j / RUN;
                if (t >= T) continue;
                const uint64_t e = reg0 + (uint64_t)t * region_cap + (j - t * RUN);
                u4 cw = {x, x + q, x ^ q, x};
                st<u4, NT>(reinterpret_cast<u4 *>(ecell + e), cw);
            }
            if constexpr (WV) {
#pragma unroll
                for (int q = 0; q < RPT / 2; q++) {
                    const int j = 2 * (q * TH + threadIdx.x);
                    const int t = j / RUN;
                    if (t >= T) continue;
                    const uint64_t e = reg0 + (uint64_t)t * region_cap + (j - t * RUN);
                    st<d2, NT>(reinterpret_cast<d2 *>(eval + e), NV ? v[0][q] : d2{(double)x, 0.0});
                }
            }
        }
    }
    if (acc == 0xdeadbeefu) sink[0] = acc ^ 1;
}

template <bool K, int N, bool C, bool W> struct Tag {
    static constexpr bool KEY = K;
    static constexpr int NV = N;
    static constexpr bool CELL = C;
    static constexpr bool WV = W;
};

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? (uint64_t)atof(argv[1]) : 1000000000ull;
    void *key, *v[3], *cell, *wv;
    unsigned *sink;
    CK(hipMalloc(&key, n * 4));
    for (auto &p : v) {
        CK(hipMalloc(&p, n * 8));
        CK(hipMemset(p, 1, n * 8));
    }
    CK(hipMemset(key, 1, n * 4));
    const uint64_t ecap = n + n / 4 + (64ull << 20);
    CK(hipMalloc(&cell, ecap * 2));
    CK(hipMalloc(&wv, ecap * 8));
    CK(hipMalloc(&sink, 8));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
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
    auto report = [&](const char *name, const char *var, double rd, double wr, float ms) {
        const double r = rd * n / ms / 1e9, w = wr * n / ms / 1e9;
        printf("%-30s %-22s %7.3f ms  reads %5.2f  writes %5.2f  total %5.2f TB/s (%4.1f %% of 8)\n", name, var, ms, r, w, r + w,
               (r + w) / 8.0 * 100);
        fflush(stdout);
    };
    const u4 *K_ = (const u4 *)key;
    const d2 *V0 = (const d2 *)v[0], *V1 = (const d2 *)v[1], *V2 = (const d2 *)v[2];
    uint16_t *C_ = (uint16_t *)cell;
    double *W_ = (double *)wv;

    // Part 1
    auto mix = [&](const char *name, double rd, double wr, auto tag) {
        using Tag = decltype(tag);
        constexpr bool KEY = Tag::KEY, CELL = Tag::CELL, WV = Tag::WV;
        constexpr int NV = Tag::NV;
        auto one = [&](const char *var, auto kern, int TH, int bpc) {
            const uint64_t nsteps = n / ((uint64_t)TH * 8);
            float ms = time([&] { hipLaunchKernelGGL(kern, dim3(cus * bpc), dim3(TH), 0, 0, K_, V0, V1, V2, nsteps, C_, W_, sink); });
            char buf[64];
            snprintf(buf, sizeof buf, "%s TH%d x%d", var, TH, bpc);
            report(name, buf, rd, wr, ms);
        };
        for (int bpc : {2, 4, 8}) {
            one("narrow", k_mix<256, KEY, NV, CELL, WV, false, false>, 256, bpc);
            one("wide", k_mix<256, KEY, NV, CELL, WV, true, false>, 256, bpc);
            one("wide-nt", k_mix<256, KEY, NV, CELL, WV, true, true>, 256, bpc);
        }
        for (int bpc : {1, 2}) {
            one("narrow", k_mix<512, KEY, NV, CELL, WV, false, false>, 512, bpc);
            one("wide", k_mix<512, KEY, NV, CELL, WV, true, false>, 512, bpc);
            one("wide-nt", k_mix<512, KEY, NV, CELL, WV, true, true>, 512, bpc);
        }
    };
    mix("read 16", 16, 0, Tag<false, 2, false, false>{});
    mix("read 24", 24, 0, Tag<false, 3, false, false>{});
    mix("copy 8 + 8", 8, 8, Tag<false, 1, false, true>{});
    mix("C2 count: read 16 + write 2", 16, 2, Tag<false, 2, true, false>{});
    mix("C2 c+s: read 24 + write 10", 24, 10, Tag<false, 3, true, true>{});
    mix("C3 A: read 12 + write 10", 12, 10, Tag<true, 1, true, true>{});

    // Part 2: regions, 512 threads, one workgroup per CU (pass A's shape)
    auto regions = [&](const char *name, double rd, double wr, int T, auto k_narrow, auto k_wide, auto k_wide_nt, int C) {
        const unsigned W = cus;
        const uint64_t nn = n / C * C;
        int RUN = (C / T) & ~7;
        const uint64_t commits_per_wg = (nn / C + W - 1) / W;
        const uint64_t region_cap = commits_per_wg * RUN + 64;
        const double scale = (double)RUN * T / C;  // fraction of rows written
        auto one = [&](const char *var, auto kern) {
            float ms = time([&] { hipLaunchKernelGGL(kern, dim3(W), dim3(512), 0, 0, V0, V1, V2, nn, T, RUN, region_cap, C_, W_, sink); });
            char buf[64];
            snprintf(buf, sizeof buf, "%s T%d run%d", var, T, RUN);
            report(name, buf, rd, wr * scale, ms);
        };
        one("narrow", k_narrow);
        one("wide", k_wide);
        one("wide-nt", k_wide_nt);
    };
    for (int T : {65, 129, 256}) {
        regions("regions count: 16 + 2", 16, 2, T, k_regions<512, 8192, 2, false, false, false>,
                k_regions<512, 8192, 2, false, true, false>, k_regions<512, 8192, 2, false, true, true>, 8192);
        regions("regions c+s: 24 + 10", 24, 10, T, k_regions<512, 12288, 3, true, false, false>,
                k_regions<512, 12288, 3, true, true, false>, k_regions<512, 12288, 3, true, true, true>, 12288);
    }
    return 0;
}
