// Device -> pinned host read-back rates for grid-sized buffers (the C2 step reads two 8.4 MB
// grids back): hipMemcpyAsync (SDMA) vs a copy kernel writing the mapped host buffer directly.
// build: hipcc --offload-arch=gfx950 -O3 -o scripts/d2h_probe scripts/d2h_probe.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_copy(const uint4 *src, uint4 *dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) dst[i] = src[i];
}

int main() {
    const size_t sizes[] = {1u << 20, 8630000, 16u << 20, 64u << 20};
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    for (size_t bytes : sizes) {
        void *d, *h, *hd;
        CK(hipMalloc(&d, bytes));
        CK(hipMemset(d, 1, bytes));
        CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
        CK(hipHostGetDevicePointer(&hd, h, 0));
        const int reps = 20;
        for (int mode = 0; mode < 3; mode++) {
            std::vector<double> t;
            for (int r = 0; r < reps + 2; r++) {
                auto t0 = std::chrono::steady_clock::now();
                if (mode == 0) {
                    CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, st));
                } else if (mode == 1) {
                    const size_t n = bytes / 16;
                    hipLaunchKernelGGL(k_copy, dim3(1024), dim3(256), 0, st, (const uint4 *)d, (uint4 *)hd, n);
                } else {  // two halves on the copy engine back to back
                    CK(hipMemcpyAsync(h, d, bytes / 2, hipMemcpyDeviceToHost, st));
                    CK(hipMemcpyAsync((char *)h + bytes / 2, (char *)d + bytes / 2, bytes - bytes / 2, hipMemcpyDeviceToHost, st));
                }
                CK(hipStreamSynchronize(st));
                auto t1 = std::chrono::steady_clock::now();
                if (r >= 2) t.push_back(std::chrono::duration<double>(t1 - t0).count());
            }
            double best = 1e9, sum = 0;
            for (double x : t) { best = x < best ? x : best; sum += x; }
            printf("%-9s %10zu B: best %8.1f us (%6.1f GB/s)  mean %8.1f us\n", mode == 0 ? "memcpy" : mode == 1 ? "kernel" : "memcpy x2",
                   bytes, best * 1e6, bytes / best / 1e9, sum / t.size() * 1e6);
        }
        CK(hipFree(d));
        CK(hipHostFree(h));
    }
    return 0;
}
