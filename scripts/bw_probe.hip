// HBM ceilings for the C2 pass-A traffic mix, measured on the box (not part of the library):
//   read-only streams, and reads mixed with contiguous writes in pass A's ratio
//   (count+sum: 24 B read + 10 B written per row; count-only: 16 B + 2 B).
// build: hipcc --offload-arch=gfx950 -O3 -o scripts/bw_probe scripts/bw_probe.hip
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

// NC read columns of doubles (16-B loads), per row `wb` bytes written contiguously
// (wb = 0, 2 or 10: a u16 array and optionally a double array)
template <int NC>
__global__ __launch_bounds__(256) void k_mix(const double *const *cols, uint64_t n, uint16_t *e16, double *e64, int wb,
                                             double *sink) {
    double acc = 0;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; 2 * i < n; i += step) {
        double2 v[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) v[c] = reinterpret_cast<const double2 *>(cols[c])[i];
        double s = 0;
#pragma unroll
        for (int c = 0; c < NC; c++) s += v[c].x + v[c].y;
        acc += s;
        if (wb >= 2) reinterpret_cast<uint32_t *>(e16)[i] = (uint32_t)(s > 0 ? 1 : 0);
        if (wb >= 10) reinterpret_cast<double2 *>(e64)[i] = v[NC - 1];
    }
    if (acc == 12345.678) sink[0] = acc;
}

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? (uint64_t)atof(argv[1]) : 1000000000ull;
    double *cols[3];
    for (int c = 0; c < 3; c++) {
        CK(hipMalloc(&cols[c], n * 8));
        CK(hipMemset(cols[c], 0, n * 8));
    }
    double **dcols;
    CK(hipMalloc(&dcols, sizeof(cols)));
    CK(hipMemcpy(dcols, cols, sizeof(cols), hipMemcpyHostToDevice));
    uint16_t *e16;
    double *e64, *sink;
    CK(hipMalloc(&e16, n * 2));
    CK(hipMalloc(&e64, n * 8));
    CK(hipMalloc(&sink, 8));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    struct Case {
        const char *name;
        int nc, wb;
    } cases[] = {{"read 16 B/row", 2, 0}, {"read 16 + write 2 B/row", 2, 2}, {"read 24 B/row", 3, 0},
                 {"read 24 + write 10 B/row", 3, 10}};
    for (auto &cs : cases) {
        for (int blocks_per_cu : {8, 16}) {
            const unsigned g = cus * blocks_per_cu;
            float best = 1e30f;
            for (int rep = 0; rep < 6; rep++) {
                CK(hipEventRecord(a));
                if (cs.nc == 2) hipLaunchKernelGGL(k_mix<2>, dim3(g), dim3(256), 0, 0, dcols, n, e16, e64, cs.wb, sink);
                else hipLaunchKernelGGL(k_mix<3>, dim3(g), dim3(256), 0, 0, dcols, n, e16, e64, cs.wb, sink);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                if (rep && ms < best) best = ms;
            }
            const double bytes = (double)n * (8.0 * cs.nc + cs.wb);
            printf("%-26s blocks/CU %2d: %8.3f ms  %6.2f TB/s moved (%6.2f TB/s of reads)\n", cs.name, blocks_per_cu, best,
                   bytes / best / 1e9, (double)n * 8.0 * cs.nc / best / 1e9);
        }
    }
    return 0;
}
