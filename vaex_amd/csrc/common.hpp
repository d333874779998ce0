// Shared plumbing for libvaexhip.so: error state, dtype traits, the library
// stream, kernel timing, launch helpers.  gfx950 only (wave64, 256 CUs).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/vaexhip.h"

namespace vh {

// Ablation switches (VH_TILE_DEBUG / VH_HA_DEBUG / VH_SI_DEBUG: timing breakdowns whose
// results are wrong by design) exist only in the `make ablation` build
// (libvaexhip_ablation.so, -DVH_ABLATION) that scripts/ load; in the product library DBG(x)
// is 0, the environment is never read for them and every switch compiles away.
#ifdef VH_ABLATION
#define DBG(x) (x)
#else
#define DBG(x) 0u
#endif

// ---- errors --------------------------------------------------------------
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

void set_error(const char *fmt, ...);
void set_error_str(const std::string &s);

[[noreturn]] inline void fail(int code, const std::string &msg) { throw Error(code, msg); }

#define VH_HIP(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            ::vh::fail(VH_ERR_HIP, std::string("HIP error '") + hipGetErrorString(e_) +     \
                                       "' in " #expr " at " __FILE__ ":" +                  \
                                       std::to_string(__LINE__));                           \
    } while (0)

// every C entry point: translate exceptions into status codes + last error
#define VH_API_BEGIN try {
#define VH_API_END                                                                          \
    return VH_OK;                                                                           \
    }                                                                                       \
    catch (const ::vh::Error &e) {                                                          \
        ::vh::set_error_str(e.what());                                                      \
        return e.code;                                                                      \
    }                                                                                       \
    catch (const std::bad_alloc &) {                                                        \
        ::vh::set_error_str("out of host memory");                                          \
        return VH_ERR_NOMEM;                                                                \
    }                                                                                       \
    catch (const std::exception &e) {                                                       \
        ::vh::set_error_str(e.what());                                                      \
        return VH_ERR_RUNTIME;                                                              \
    }

// ---- dtypes ---------------------------------------------------------------
// numpy bool is one byte holding 0 or 1
struct vbool {
    uint8_t v;
};

inline int dtype_itemsize(int dtype) {
    switch (dtype) {
    case VH_F64: case VH_I64: case VH_U64: return 8;
    case VH_F32: case VH_I32: case VH_U32: return 4;
    case VH_I16: case VH_U16: return 2;
    case VH_I8: case VH_U8: case VH_BOOL: return 1;
    }
    fail(VH_ERR_ARG, "unknown dtype code " + std::to_string(dtype));
}

// upcast<T> (superagg.cpp:289-346) as dtype codes
inline int upcast_dtype(int dtype) {
    switch (dtype) {
    case VH_F64: case VH_F32: return VH_F64;
    case VH_I64: case VH_I32: case VH_I16: case VH_I8: case VH_BOOL: return VH_I64;
    default: return VH_U64;
    }
}

#define VH_DISPATCH_DTYPE(code, T, ...)                                                     \
    switch (code) {                                                                         \
    case VH_F64: { using T = double; __VA_ARGS__; break; }                                  \
    case VH_F32: { using T = float; __VA_ARGS__; break; }                                   \
    case VH_I64: { using T = int64_t; __VA_ARGS__; break; }                                 \
    case VH_I32: { using T = int32_t; __VA_ARGS__; break; }                                 \
    case VH_I16: { using T = int16_t; __VA_ARGS__; break; }                                 \
    case VH_I8: { using T = int8_t; __VA_ARGS__; break; }                                   \
    case VH_U64: { using T = uint64_t; __VA_ARGS__; break; }                                \
    case VH_U32: { using T = uint32_t; __VA_ARGS__; break; }                                \
    case VH_U16: { using T = uint16_t; __VA_ARGS__; break; }                                \
    case VH_U8: { using T = uint8_t; __VA_ARGS__; break; }                                  \
    case VH_BOOL: { using T = ::vh::vbool; __VA_ARGS__; break; }                            \
    default: ::vh::fail(VH_ERR_ARG, "unknown dtype code");                                  \
    }

// ---- device-side helpers ---------------------------------------------------
// rank of a row in an LDS histogram (partition / tile / bucket counts).  Every lane of the
// wave calls it (no exec divergence).  When all taking lanes share one bin (sorted or
// clustered rows) one atomic reserves the wave's ranks and each lane takes its position among
// them -- 64 same-address LDS atomics would serialise; otherwise one atomic per taking lane,
// and rows that do not take (past the range, folded) touch nothing.
__device__ __forceinline__ int32_t wave_rank(uint32_t *hist, uint32_t t, bool take) {
    const uint64_t act = __ballot(take);
    if (!act) return -1;
    // the bin of the first TAKING lane (lane 0 may be a folded row or past the range)
    const int lead = __builtin_ctzll(act);
    const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)t, lead);
    if (__ballot(take && t != t0) == 0) {
        const int lane = threadIdx.x & 63;
        uint32_t base = 0;
        if (lane == lead) base = atomicAdd(&hist[t0], (uint32_t)__builtin_popcountll(act));
        base = (uint32_t)__shfl((int)base, lead, 64);
        return take ? (int32_t)(base + (uint32_t)__builtin_popcountll(act & ((1ull << lane) - 1))) : -1;
    }
    return take ? (int32_t)atomicAdd(&hist[t], 1u) : -1;
}

// Block-level slot reservation for compaction: every thread emits `my` items; one atomic on
// the output counter per workgroup and call (a counter bumped by every wave is one
// same-address atomic per 64 items: ~9 ms per 1e8).  Returns this thread's first slot.
// Every thread of the block calls it (it holds three barriers).
template <int THREADS, typename C>
__device__ inline uint64_t block_reserve(uint32_t my, uint32_t *s_w, unsigned long long *s_base, C *counter) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc = my;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off, 64);
        if (lane >= off) inc += y;
    }
    if (lane == 63) s_w[wave] = inc;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int k = 0; k < THREADS / 64; k++) {
        before += k < wave ? s_w[k] : 0u;
        total += s_w[k];
    }
    if (threadIdx.x == 0) *s_base = total ? (unsigned long long)atomicAdd(counter, (C)total) : 0ull;
    __syncthreads();
    const uint64_t base = *s_base + before + inc - my;
    __syncthreads();  // s_w / s_base reused by the next call
    return base;
}


template <typename T> struct is_float_t { static constexpr bool value = false; };
template <> struct is_float_t<double> { static constexpr bool value = true; };
template <> struct is_float_t<float> { static constexpr bool value = true; };

template <typename T> struct is_signed_int_t { static constexpr bool value = false; };
template <> struct is_signed_int_t<int64_t> { static constexpr bool value = true; };
template <> struct is_signed_int_t<int32_t> { static constexpr bool value = true; };
template <> struct is_signed_int_t<int16_t> { static constexpr bool value = true; };
template <> struct is_signed_int_t<int8_t> { static constexpr bool value = true; };

// _to_native<T> (agg.hpp:13-21)
__host__ __device__ inline double bswap_v(double v) {
    uint64_t u;
    __builtin_memcpy(&u, &v, 8);
    u = __builtin_bswap64(u);
    __builtin_memcpy(&v, &u, 8);
    return v;
}
__host__ __device__ inline float bswap_v(float v) {
    uint32_t u;
    __builtin_memcpy(&u, &v, 4);
    u = __builtin_bswap32(u);
    __builtin_memcpy(&v, &u, 4);
    return v;
}
__host__ __device__ inline int64_t bswap_v(int64_t v) { return (int64_t)__builtin_bswap64((uint64_t)v); }
__host__ __device__ inline uint64_t bswap_v(uint64_t v) { return __builtin_bswap64(v); }
__host__ __device__ inline int32_t bswap_v(int32_t v) { return (int32_t)__builtin_bswap32((uint32_t)v); }
__host__ __device__ inline uint32_t bswap_v(uint32_t v) { return __builtin_bswap32(v); }
__host__ __device__ inline int16_t bswap_v(int16_t v) { return (int16_t)__builtin_bswap16((uint16_t)v); }
__host__ __device__ inline uint16_t bswap_v(uint16_t v) { return __builtin_bswap16(v); }
__host__ __device__ inline int8_t bswap_v(int8_t v) { return v; }
__host__ __device__ inline uint8_t bswap_v(uint8_t v) { return v; }
__host__ __device__ inline vbool bswap_v(vbool v) { return v; }

template <typename T> __device__ inline T load_v(const void *p, uint64_t i, int flip) {
    T v = reinterpret_cast<const T *>(p)[i];
    return flip ? bswap_v(v) : v;
}

template <typename T> __device__ inline double to_double(T v) { return (double)v; }
template <> __device__ inline double to_double<vbool>(vbool v) { return v.v ? 1.0 : 0.0; }

template <typename T> __device__ inline bool is_nan_v(T v) {
    if constexpr (is_float_t<T>::value) return v != v;
    else return false;
}

// AggFirst's order value as an order-preserving u64 (floats: -0.0 == 0.0, as `<` compares
// them; signed: offset binary) -- min over it = the reference's strict `<` minimum
template <typename T> __device__ inline uint64_t order_key(T v) {
    if constexpr (is_float_t<T>::value) {
        double d = (double)v;
        if (d == 0.0) d = 0.0;
        uint64_t u;
        __builtin_memcpy(&u, &d, 8);
        return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
    } else if constexpr (is_signed_int_t<T>::value) {
        return (uint64_t)(int64_t)v ^ 0x8000000000000000ULL;
    } else if constexpr (std::is_same<T, vbool>::value) {
        return v.v;
    } else {
        return (uint64_t)v;
    }
}


// ---- runtime ---------------------------------------------------------------
hipStream_t stream();
hipStream_t copy_stream();  // H2D staging copies (overlap the compute stream)
void parallel_memcpy(void *dst, const void *src, uint64_t bytes, int threads);
bool host_registered(const void *p, uint64_t bytes);  // inside a vh_host_register range
int current_device();
int cu_count();

// `dev` is this thread's current device for the scope (restored after)
struct DeviceScope {
    int prev, dev;
    explicit DeviceScope(int dev);
    ~DeviceScope();
    DeviceScope(const DeviceScope &) = delete;
    DeviceScope &operator=(const DeviceScope &) = delete;
};

// grid size for a grid-stride kernel over n items
inline unsigned blocks_for(uint64_t n, unsigned threads, unsigned per_cu = 8) {
    uint64_t b = (n + threads - 1) / threads;
    uint64_t cap = (uint64_t)cu_count() * per_cu;
    if (b > cap) b = cap;
    if (b == 0) b = 1;
    return (unsigned)b;
}

// upper bound on the rows one workgroup of a grid-stride kernel visits: launched with
// `blocks` workgroups of `threads` lanes, each lane taking `unroll` rows per step (bounds
// narrow per-workgroup partial sums; derive `blocks` from the launch's own dim3)
inline uint64_t rows_per_wg(uint64_t n, unsigned blocks, unsigned threads, unsigned unroll) {
    return (n + blocks - 1) / blocks + (uint64_t)threads * unroll;
}

// kernel timing (hipEvents around named launches on the library stream)
struct TimedScope {
    const char *name;
    hipEvent_t start = nullptr, stop = nullptr;
    bool on;
    explicit TimedScope(const char *n);
    ~TimedScope();
};

// Device block cache (runtime.hip): a freed block of <= 256 MiB is kept for reuse (sizes
// rounded up to 4 KiB / 1 MiB), up to 2 GiB per device, instead of hipFree -- hipFree
// costs ~0.4 ms per 17 MB grid, and a query creates and drops its grids every time.
// Reuse is ordered by the library stream, which every kernel touching these blocks uses.
void *dev_alloc(uint64_t &bytes);  // rounds bytes up
void dev_free(void *ptr, uint64_t bytes);

// device memory owned by the library (RAII)
struct DevBuf {
    void *ptr = nullptr;
    uint64_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (ptr) dev_free(ptr, bytes);
        ptr = nullptr;
        bytes = 0;
    }
    void ensure(uint64_t b) {
        if (b <= bytes) return;
        release();
        if (b == 0) return;
        ptr = dev_alloc(b);
        bytes = b;
    }
    template <typename T> T *as() const { return reinterpret_cast<T *>(ptr); }
};

void *host_block_alloc(uint64_t bytes);  // page-locked, from the library's block cache
void host_block_free(void *ptr, uint64_t bytes);
void host_cache_trim();  // free every cached page-locked block
void dense_rank_scratch_release();  // hashagg.hip: the dense rank's per-device sort scratch
// device -> host copy on `st` (asynchronous): a page-locked destination of >= 256 KiB is
// written by a copy kernel through its mapped address (the GPU's PCIe writes run at the
// link rate on every box; the copy engine measured 21-54 GB/s for the same 8.4 MB grid
// depending on the box), anything else by hipMemcpyAsync
void copy_to_host(void *dst, const void *src, uint64_t bytes, hipStream_t st);

// page-locked host buffer (DMA source of the H2D staging pipeline)
struct PinnedBuf {
    void *ptr = nullptr;
    uint64_t bytes = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf &) = delete;
    PinnedBuf &operator=(const PinnedBuf &) = delete;
    ~PinnedBuf() { release(); }
    void release() {
        if (ptr) host_block_free(ptr, bytes);
        ptr = nullptr;
        bytes = 0;
    }
    void ensure(uint64_t b) {
        if (b <= bytes) return;
        release();
        ptr = host_block_alloc(b);
        bytes = b;
    }
    template <typename T> T *as() const { return reinterpret_cast<T *>(ptr); }
};

// resolve VH_LOC_AUTO
int resolve_loc(const void *ptr, int loc);

}  // namespace vh
