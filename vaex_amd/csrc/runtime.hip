// Device/runtime plumbing of libvaexhip.so: last-error state, the per-device
// library stream, device memory entry points, synthetic data generation in
// HBM, kernel timing and the NaN-ignoring min/max limits pre-pass
// (the reference's vaexfast statisticNd<op_min_max>, vaexfast.cpp:1043-1055).
#include <map>
#include <mutex>
#include <thread>
#include <cstring>

#include "common.hpp"
#include "engine.hpp"

namespace vh {

static thread_local std::string g_last_error;

void set_error_str(const std::string &s) { g_last_error = s; }
void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

static std::mutex g_mu;
static std::map<int, hipStream_t> g_streams;
static std::map<int, int> g_cus;

// The process's GPU (one process per GPU): vh_set_device records it, and every other thread
// adopts it on its first library call -- HIP's current device is per thread, so a task run
// from a worker thread (the executor allows that) would otherwise land on device 0.
// A thread re-adopts after every vh_set_device (generation counter), so a thread that called
// the library before the device was chosen (a pool created before comm init) follows it too.
static int g_default_device = -1;
static int g_device_gen = 0;
static thread_local int t_device_gen = 0;

int current_device() {
    const int gen = __atomic_load_n(&g_device_gen, __ATOMIC_ACQUIRE);
    if (t_device_gen != gen) {
        t_device_gen = gen;
        const int want = __atomic_load_n(&g_default_device, __ATOMIC_ACQUIRE);
        if (want >= 0) VH_HIP(hipSetDevice(want));
    }
    int d = 0;
    VH_HIP(hipGetDevice(&d));
    return d;
}

DeviceScope::DeviceScope(int dev) : prev(current_device()), dev(dev) {
    if (prev != dev) VH_HIP(hipSetDevice(dev));
}
DeviceScope::~DeviceScope() {
    if (prev != dev) (void)hipSetDevice(prev);
}

// ---- device block cache (common.hpp) ---------------------------------------------------
namespace {
// Freed device blocks are kept for reuse (exact sizes, 1 MiB granularity): at most 1/4 of
// the device's memory (VAEX_AMD_DEVICE_CACHE_MB overrides it per process, 0 disables the
// cache), blocks of up to 1/16 of it.  Large blocks matter: a 1e9-row query
// allocates multi-GB temporaries (h2o q10's 8 GB combined key column), and a fresh hipMalloc
// of 8 GB stalled for 5.7 s every few queries on a device holding ~60 GB.  A freed block
// past the cap evicts the longest-cached blocks first (a full cache of an earlier query's
// block sizes made every q10 hipMalloc its temporaries: 1.1 s of 1.7 s, round 6).  A failed
// allocation drops the cache and retries.
struct BlockCache {
    std::multimap<uint64_t, std::pair<void *, uint64_t>> free;  // size -> (block, free sequence)
    uint64_t cached = 0, seq = 0;
    uint64_t max_bytes = 0, max_block = 0;
    bool limits_set = false;
};
void cache_limits(BlockCache &c) {
    if (c.limits_set) return;
    size_t fr = 0, total = 0;
    if (hipMemGetInfo(&fr, &total) != hipSuccess || total == 0) {
        (void)hipGetLastError();
        total = 32ull << 30;
    }
    c.max_bytes = total / 4;
    c.max_block = total / 16;
    if (const char *e = getenv("VAEX_AMD_DEVICE_CACHE_MB")) {
        c.max_bytes = (uint64_t)strtoull(e, nullptr, 10) << 20;
        c.max_block = std::min(c.max_block, c.max_bytes);
    }
    if (!c.max_bytes) c.max_block = 0;
    c.limits_set = true;
}
std::mutex g_cache_mu;
std::map<int, BlockCache> g_cache;
}  // namespace

void *dev_alloc(uint64_t &bytes) {
    const uint64_t gran = bytes >= (1ull << 20) ? (1ull << 20) : 4096;
    bytes = (bytes + gran - 1) / gran * gran;
    const int d = current_device();
    {
        std::lock_guard<std::mutex> lk(g_cache_mu);
        BlockCache &c = g_cache[d];
        auto it = c.free.find(bytes);
        if (it != c.free.end()) {
            void *p = it->second.first;
            c.free.erase(it);
            c.cached -= bytes;
            return p;
        }
    }
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        {  // drop the cache and retry once
            std::lock_guard<std::mutex> lk(g_cache_mu);
            BlockCache &c = g_cache[d];
            for (auto &kv : c.free) (void)hipFree(kv.second.first);
            c.free.clear();
            c.cached = 0;
        }
        e = hipMalloc(&p, bytes);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            fail(VH_ERR_NOMEM, "hipMalloc of " + std::to_string(bytes) + " bytes failed: " + hipGetErrorString(e));
        }
    }
    return p;
}

void dev_free(void *ptr, uint64_t bytes) {
    if (!ptr) return;
    {
        std::lock_guard<std::mutex> lk(g_cache_mu);
        BlockCache &c = g_cache[current_device()];
        cache_limits(c);
        if (bytes <= c.max_block && bytes <= c.max_bytes) {
            while (c.cached + bytes > c.max_bytes && !c.free.empty()) {  // evict the oldest
                auto old = c.free.begin();
                for (auto it = c.free.begin(); it != c.free.end(); ++it)
                    if (it->second.second < old->second.second) old = it;
                (void)hipFree(old->second.first);
                c.cached -= old->first;
                c.free.erase(old);
            }
            c.free.emplace(bytes, std::make_pair(ptr, ++c.seq));
            c.cached += bytes;
            return;
        }
    }
    (void)hipFree(ptr);
}

// ---- pinned host block cache (vh_host_alloc / vh_host_free) ---------------------------
// Result arrays (grids, groupby columns) are read back through page-locked blocks: a
// pageable D2H runs at ~5-10 GB/s, page-locked at PCIe/xGMI rate, and hipHostMalloc itself
// (and hipHostFree) are slow, so freed blocks are kept (sizes rounded to 64 KiB, <= 8 GiB
// cached: a 1e8-group result is three 800 MB columns); the host pipeline's bounce buffers come from the same cache.
// The cap is per process: VAEX_AMD_PINNED_CACHE_MB, else 8 GiB divided by the processes of
// this node (LOCAL_WORLD_SIZE, one per GPU), so eight ranks keep at most 8 GiB locked in all.
namespace {
std::mutex g_hcache_mu;
std::multimap<uint64_t, void *> g_hcache;
uint64_t g_hcached = 0;
uint64_t hcache_max_bytes() {
    static const uint64_t cap = []() -> uint64_t {
        if (const char *e = getenv("VAEX_AMD_PINNED_CACHE_MB")) return (uint64_t)strtoull(e, nullptr, 10) << 20;
        uint64_t ranks = 1;
        if (const char *e = getenv("LOCAL_WORLD_SIZE")) ranks = std::max<uint64_t>(1, strtoull(e, nullptr, 10));
        return (8ull << 30) / ranks;
    }();
    return cap;
}
}  // namespace

// device -> mapped page-locked host memory, 16 bytes per lane per step (the tail, < 16 B,
// by lane 0 of workgroup 0)
__global__ __launch_bounds__(256) void k_copy_to_host(const uint4 *src, uint4 *dst, uint64_t nvec, const uint8_t *tsrc,
                                                      uint8_t *tdst, uint32_t tail) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nvec; i += (uint64_t)gridDim.x * 256) dst[i] = src[i];
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (uint32_t k = 0; k < tail; k++) tdst[k] = tsrc[k];
}

void copy_to_host(void *dst, const void *src, uint64_t bytes, hipStream_t st) {
    if (!bytes) return;
    void *mapped = nullptr;
    if (bytes >= (256u << 10) && ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0) {
        hipPointerAttribute_t at{};
        if (hipPointerGetAttributes(&at, dst) == hipSuccess && at.type == hipMemoryTypeHost && at.devicePointer)
            mapped = at.devicePointer;
        else
            (void)hipGetLastError();  // pageable memory: not an error
    }
    if (!mapped) {
        VH_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
        return;
    }
    const uint64_t nvec = bytes / 16;
    const uint32_t tail = (uint32_t)(bytes - nvec * 16);
    const unsigned grid = (unsigned)std::min<uint64_t>((nvec + 255) / 256, 1024);
    hipLaunchKernelGGL(k_copy_to_host, dim3(grid), dim3(256), 0, st, static_cast<const uint4 *>(src),
                       static_cast<uint4 *>(mapped), nvec, static_cast<const uint8_t *>(src) + nvec * 16,
                       static_cast<uint8_t *>(mapped) + nvec * 16, tail);
    VH_HIP(hipGetLastError());
}

// return every cached page-locked block to the system (vh_host_cache_trim; vh_comm_destroy)
void host_cache_trim() {
    std::lock_guard<std::mutex> lk(g_hcache_mu);
    for (auto &kv : g_hcache) (void)hipHostFree(kv.second);
    g_hcache.clear();
    g_hcached = 0;
}

static uint64_t host_round(uint64_t bytes) { return (std::max<uint64_t>(bytes, 1) + 65535) & ~uint64_t(65535); }

void *host_block_alloc(uint64_t bytes) {
    const uint64_t b = host_round(bytes);
    {
        std::lock_guard<std::mutex> lk(g_hcache_mu);
        auto it = g_hcache.find(b);
        if (it != g_hcache.end()) {
            void *p = it->second;
            g_hcache.erase(it);
            g_hcached -= b;
            return p;
        }
    }
    void *p = nullptr;
    hipError_t e = hipHostMalloc(&p, b, hipHostMallocDefault);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        fail(VH_ERR_NOMEM, "hipHostMalloc of " + std::to_string(b) + " bytes failed: " + hipGetErrorString(e));
    }
    return p;
}

void host_block_free(void *ptr, uint64_t bytes) {
    if (!ptr) return;
    const uint64_t b = host_round(bytes);
    {
        std::lock_guard<std::mutex> lk(g_hcache_mu);
        if (g_hcached + b <= hcache_max_bytes()) {
            g_hcache.emplace(b, ptr);
            g_hcached += b;
            return;
        }
    }
    (void)hipHostFree(ptr);
}

hipStream_t stream() {
    int d = current_device();
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_streams.find(d);
    if (it != g_streams.end()) return it->second;
    hipStream_t s;
    VH_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    g_streams[d] = s;
    return s;
}

// ---- registered host ranges (vh_host_register): the host pipeline DMAs column chunks that
// lie inside one in place, with no bounce copy and no per-chunk registration
static std::mutex g_reg_mu;
static std::map<uintptr_t, uintptr_t> g_reg;  // start -> end

bool host_registered(const void *p, uint64_t bytes) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_reg.upper_bound(a);
    if (it == g_reg.begin()) return false;
    --it;
    return a >= it->first && a + bytes <= it->second;
}

static std::map<int, hipStream_t> g_copy_streams;

hipStream_t copy_stream() {
    int d = current_device();
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_copy_streams.find(d);
    if (it != g_copy_streams.end()) return it->second;
    hipStream_t s;
    VH_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    g_copy_streams[d] = s;
    return s;
}

// memcpy split over up to `threads` host threads (pageable -> pinned bounce copies)
void parallel_memcpy(void *dst, const void *src, uint64_t bytes, int threads) {
    const uint64_t min_part = 8ull << 20;
    int t = (int)std::min<uint64_t>((uint64_t)std::max(1, threads), std::max<uint64_t>(1, bytes / min_part));
    if (t <= 1) {
        memcpy(dst, src, bytes);
        return;
    }
    std::vector<std::thread> pool;
    const uint64_t part = (bytes / t + 63) & ~uint64_t(63);
    for (int i = 0; i < t; i++) {
        const uint64_t o = (uint64_t)i * part;
        if (o >= bytes) break;
        const uint64_t len = std::min(part, bytes - o);
        pool.emplace_back([=] { memcpy((char *)dst + o, (const char *)src + o, len); });
    }
    for (auto &th : pool) th.join();
}

int cu_count() {
    int d = current_device();
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_cus.find(d);
        if (it != g_cus.end()) return it->second;
    }
    int n = 0;
    VH_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d));
    if (n <= 0) n = 256;
    std::lock_guard<std::mutex> lk(g_mu);
    g_cus[d] = n;
    return n;
}

int resolve_loc(const void *ptr, int loc) {
    if (loc == VH_LOC_HOST || loc == VH_LOC_DEVICE) return loc;
    if (ptr == nullptr) return VH_LOC_HOST;
    hipPointerAttribute_t attr;
    hipError_t e = hipPointerGetAttributes(&attr, ptr);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return VH_LOC_HOST;
    }
    return attr.type == hipMemoryTypeDevice ? VH_LOC_DEVICE : VH_LOC_HOST;
}

// ---- kernel timing -----------------------------------------------------------
static bool g_timing = false;
struct TimingRec {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
};
static std::map<std::string, TimingRec> g_timing_recs;

TimedScope::TimedScope(const char *n) : name(n), on(g_timing) {
    if (!on) return;
    VH_HIP(hipEventCreate(&start));
    VH_HIP(hipEventCreate(&stop));
    VH_HIP(hipEventRecord(start, vh::stream()));
}

TimedScope::~TimedScope() {
    if (!on) return;
    if (hipEventRecord(stop, vh::stream()) != hipSuccess) return;
    std::lock_guard<std::mutex> lk(g_mu);
    g_timing_recs[name].ev.emplace_back(start, stop);
}

// ---- synthetic data (counter-based, reproducible for any row range) ------
__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}

__device__ inline double u01(uint64_t bits) { return (double)(bits >> 11) * 0x1.0p-53; }

__global__ void k_fill_random(void *dst, uint64_t n, int dtype, int dist, uint64_t seed, double a,
                              double b) {
    const uint64_t s = splitmix64(seed * 0x632be59bd9b4e019ULL + 0x1234567ULL);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t r1 = splitmix64(s ^ (2 * i));
        if (dist == 3) {  // sorted: a + b * the normal quantile of (i + 0.5) / n (ascending)
            reinterpret_cast<double *>(dst)[i] = a + b * normcdfinv(((double)i + 0.5) / (double)n);
            continue;
        }
        if (dist == 4) {  // sorted integers: [a, b) in equal consecutive runs
            const uint64_t span = (uint64_t)(int64_t)(b - a);
            const int64_t v = (int64_t)a + (int64_t)(span ? (uint64_t)(((unsigned __int128)i * span) / n) : 0);
            if (dtype == VH_I32) reinterpret_cast<int32_t *>(dst)[i] = (int32_t)v;
            else reinterpret_cast<int64_t *>(dst)[i] = v;
            continue;
        }
        if (dist == 0 || dist == 1) {
            double d;
            if (dist == 0) {
                d = a + (b - a) * u01(r1);
            } else {
                uint64_t r2 = splitmix64(s ^ (2 * i + 1));
                double u1 = 1.0 - u01(r1);  // (0, 1]
                double u2 = u01(r2);
                d = a + b * (sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
            }
            // float32: the float64 draw rounded (the h2o fixture's x4 = x.astype('float32'))
            if (dtype == VH_F32) reinterpret_cast<float *>(dst)[i] = (float)d;
            else reinterpret_cast<double *>(dst)[i] = d;
        } else {
            uint64_t span = (uint64_t)(int64_t)(b - a);
            int64_t v = (int64_t)a + (int64_t)(span ? r1 % span : 0);
            if (dtype == VH_I32) reinterpret_cast<int32_t *>(dst)[i] = (int32_t)v;
            else if (dtype == VH_I8) reinterpret_cast<int8_t *>(dst)[i] = (int8_t)v;
            else reinterpret_cast<int64_t *>(dst)[i] = v;
        }
    }
}

// ---- min/max limits pre-pass --------------------------------------------------
// order-preserving map double -> uint64 (non-NaN input)
__device__ inline uint64_t f64_key(double d) {
    if (d == 0.0) d = 0.0;  // -0 == +0
    uint64_t u;
    __builtin_memcpy(&u, &d, 8);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}
__host__ inline double f64_from_key(uint64_t k) {
    uint64_t u = (k >> 63) ? (k & 0x7fffffffffffffffULL) : ~k;
    double d;
    memcpy(&d, &u, 8);
    return d;
}

// (min key, max key) of a 256-lane workgroup -> out[0..1] (written by lane 0; no atomics:
// a few thousand same-address atomics at the end of a short launch cost more than the scan)
__device__ inline void block_minmax_keys(uint64_t lo, uint64_t hi, uint64_t *out) {
    __shared__ uint64_t s_lo[4], s_hi[4];
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t l2 = __shfl_down(lo, off, 64);
        const uint64_t h2 = __shfl_down(hi, off, 64);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
    }
    if ((threadIdx.x & 63) == 0) {
        s_lo[threadIdx.x >> 6] = lo;
        s_hi[threadIdx.x >> 6] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); w++) {
            lo = min(lo, s_lo[w]);
            hi = max(hi, s_hi[w]);
        }
        out[2 * blockIdx.x] = lo;
        out[2 * blockIdx.x + 1] = hi;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_minmax(const void *data, uint64_t n, int flip,
                                                const uint8_t *mask, uint64_t *part) {
    uint64_t lo = ~0ULL, hi = 0ULL;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        if (mask && mask[i]) continue;
        T v = load_v<T>(data, i, flip);
        double d = to_double(v);
        if (d != d) continue;
        uint64_t k = f64_key(d);
        lo = k < lo ? k : lo;
        hi = k > hi ? k : hi;
    }
    block_minmax_keys(lo, hi, part);
}

// Streaming form for native, unmasked, 16-B aligned columns of a numeric T: every lane
// keeps MM_UNROLL 16-byte loads in flight, min/max are kept in T (the T -> double map is
// monotone, so double(min T) == min of the doubles) and mapped to keys once per lane.
// NaN fails both compares and is skipped (nanmin/nanmax, tasks.py:173-185).
constexpr int MM_UNROLL = 4;
template <typename T>
__global__ __launch_bounds__(256) void k_minmax_vec(const T *data, uint64_t nvec, uint64_t *part) {
    constexpr int V = 16 / sizeof(T);
    struct alignas(16) Vec { T v[V]; };
    const Vec *src = reinterpret_cast<const Vec *>(data);
    T lo = data[0], hi = data[0];
    if constexpr (is_float_t<T>::value) {
        lo = __builtin_inf();
        hi = -__builtin_inf();
    }
    bool any = false;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (; i + (MM_UNROLL - 1) * stride < nvec; i += MM_UNROLL * stride) {
        Vec b[MM_UNROLL];
#pragma unroll
        for (int u = 0; u < MM_UNROLL; u++) b[u] = src[i + u * stride];
#pragma unroll
        for (int u = 0; u < MM_UNROLL; u++)
#pragma unroll
            for (int k = 0; k < V; k++) {
                const T v = b[u].v[k];
                lo = v < lo ? v : lo;
                hi = v > hi ? v : hi;
            }
        any = true;
    }
    for (; i < nvec; i += stride) {
        const Vec b = src[i];
#pragma unroll
        for (int k = 0; k < V; k++) {
            const T v = b.v[k];
            lo = v < lo ? v : lo;
            hi = v > hi ? v : hi;
        }
        any = true;
    }
    uint64_t klo = ~0ULL, khi = 0ULL;
    if (any && !(lo > hi)) {  // floats: an all-NaN lane leaves lo = inf > hi = -inf
        klo = f64_key((double)lo);
        khi = f64_key((double)hi);
    }
    block_minmax_keys(klo, khi, part);
}

// min / max of `ns` evenly spaced rows (row floor(j * n / ns)) of a native, unmasked column:
// the speculative key range of a dense groupby (vh_minmax_sample)
template <typename T>
__global__ __launch_bounds__(256) void k_minmax_sample(const T *data, uint64_t n, uint64_t ns, uint64_t *part) {
    uint64_t lo = ~0ULL, hi = 0ULL;
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < ns; j += (uint64_t)gridDim.x * blockDim.x) {
        const double d = to_double(data[(uint64_t)(((unsigned __int128)j * n) / ns)]);
        if (d != d) continue;
        const uint64_t k = f64_key(d);
        lo = k < lo ? k : lo;
        hi = k > hi ? k : hi;
    }
    block_minmax_keys(lo, hi, part);
}

// fold the `nb` workgroup partials into keys[0] (min) / keys[1] (max)
__global__ __launch_bounds__(256) void k_minmax_fin(const uint64_t *part, unsigned nb, uint64_t *keys) {
    uint64_t lo = ~0ULL, hi = 0ULL;
    for (unsigned b = threadIdx.x; b < nb; b += blockDim.x) {
        lo = min(lo, part[2 * b]);
        hi = max(hi, part[2 * b + 1]);
    }
    block_minmax_keys(lo, hi, keys);
}

}  // namespace vh

using namespace vh;

extern "C" {

const char *vh_last_error(void) { return g_last_error.c_str(); }
int vh_abi_version(void) { return VH_ABI_VERSION; }

int vh_device_count(int *count) {
    VH_API_BEGIN
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        n = 0;
    }
    *count = n;
    VH_API_END
}

int vh_set_device(int device) {
    VH_API_BEGIN
    VH_HIP(hipSetDevice(device));
    __atomic_store_n(&g_default_device, device, __ATOMIC_RELEASE);
    t_device_gen = __atomic_add_fetch(&g_device_gen, 1, __ATOMIC_ACQ_REL);
    VH_API_END
}

int vh_get_device(int *device) {
    VH_API_BEGIN
    *device = current_device();
    VH_API_END
}

int vh_synchronize(void) {
    VH_API_BEGIN
    VH_HIP(hipStreamSynchronize(stream()));
    VH_API_END
}

// user buffers (DeviceArray) come from the device block cache too; their rounded sizes are
// remembered for vh_free
namespace {
std::mutex g_user_mu;
std::map<void *, std::pair<uint64_t, int>> g_user_blocks;  // ptr -> (bytes, device)
}  // namespace

int vh_malloc(void **dptr, uint64_t bytes) {
    VH_API_BEGIN
    const int d = current_device();  // this thread on the process's GPU
    uint64_t b = bytes ? bytes : 1;
    void *p = dev_alloc(b);
    {
        std::lock_guard<std::mutex> lk(g_user_mu);
        g_user_blocks[p] = {b, d};
    }
    *dptr = p;
    VH_API_END
}

int vh_free(void *dptr) {
    VH_API_BEGIN
    if (!dptr) return VH_OK;
    VH_HIP(hipStreamSynchronize(stream()));
    std::pair<uint64_t, int> blk{0, -1};
    {
        std::lock_guard<std::mutex> lk(g_user_mu);
        auto it = g_user_blocks.find(dptr);
        if (it != g_user_blocks.end()) {
            blk = it->second;
            g_user_blocks.erase(it);
        }
    }
    if (blk.second < 0) {
        VH_HIP(hipFree(dptr));
    } else {
        DeviceScope ds(blk.second);
        dev_free(dptr, blk.first);
    }
    VH_API_END
}

int vh_host_alloc(void **ptr, uint64_t bytes) {
    VH_API_BEGIN
    *ptr = host_block_alloc(bytes);
    VH_API_END
}

int vh_host_free(void *ptr, uint64_t bytes) {
    VH_API_BEGIN
    host_block_free(ptr, bytes);
    VH_API_END
}

int vh_host_cache_trim(void) {
    VH_API_BEGIN
    host_cache_trim();
    VH_API_END
}

int vh_device_cache_trim(void) {
    VH_API_BEGIN
    VH_HIP(hipStreamSynchronize(stream()));
    dense_rank_scratch_release();
    // every device with cached blocks (a process may have run work on several)
    std::lock_guard<std::mutex> lk(g_cache_mu);
    for (auto &dc : g_cache) {
        BlockCache &c = dc.second;
        if (c.free.empty()) continue;
        DeviceScope ds(dc.first);
        VH_HIP(hipStreamSynchronize(stream()));
        for (auto &kv : c.free) (void)hipFree(kv.second.first);
        c.free.clear();
        c.cached = 0;
    }
    VH_API_END
}

/* dsts[c][i] = srcs[c][idx[i]] for ncols columns of itemsizes[c] (1/2/4/8) bytes, i < n, on up
 * to `threads` host threads, each thread one index range over every column (the permutation
 * of a groupby's result columns into first-appearance order; numpy's take holds the
 * interpreter lock and would re-read the index per column) */
int vh_host_take(int ncols, void *const *dsts, const void *const *srcs, const int *itemsizes, const int64_t *idx,
                 uint64_t n, int threads) {
    VH_API_BEGIN
    for (int c = 0; c < ncols; c++)
        if (itemsizes[c] != 1 && itemsizes[c] != 2 && itemsizes[c] != 4 && itemsizes[c] != 8)
            fail(VH_ERR_ARG, "vh_host_take: itemsize");
    std::vector<void *> d(dsts, dsts + ncols);
    std::vector<const void *> sr(srcs, srcs + ncols);
    std::vector<int> isz(itemsizes, itemsizes + ncols);
    auto part = [&](uint64_t i0, uint64_t i1) {
        for (uint64_t b = i0; b < i1; b += 4096) {  // blocks of the index: columns share its reads
            const uint64_t e = std::min(i1, b + 4096);
            for (int c = 0; c < ncols; c++) {
                switch (isz[c]) {
                case 8: for (uint64_t i = b; i < e; i++) static_cast<uint64_t *>(d[c])[i] = static_cast<const uint64_t *>(sr[c])[idx[i]]; break;
                case 4: for (uint64_t i = b; i < e; i++) static_cast<uint32_t *>(d[c])[i] = static_cast<const uint32_t *>(sr[c])[idx[i]]; break;
                case 2: for (uint64_t i = b; i < e; i++) static_cast<uint16_t *>(d[c])[i] = static_cast<const uint16_t *>(sr[c])[idx[i]]; break;
                default: for (uint64_t i = b; i < e; i++) static_cast<uint8_t *>(d[c])[i] = static_cast<const uint8_t *>(sr[c])[idx[i]];
                }
            }
        }
    };
    const int t = (int)std::min<uint64_t>((uint64_t)std::max(1, threads), std::max<uint64_t>(1, n / 32768));
    if (t <= 1) {
        part(0, n);
    } else {
        std::vector<std::thread> pool;
        for (int k = 1; k < t; k++) pool.emplace_back(part, n * k / t, n * (k + 1) / t);
        part(0, n / t);
        for (auto &th : pool) th.join();
    }
    VH_API_END
}

int vh_host_register(void *ptr, uint64_t bytes) {
    VH_API_BEGIN
    if (!ptr || !bytes) fail(VH_ERR_ARG, "vh_host_register: empty range");
    const uintptr_t page = 4096, a = reinterpret_cast<uintptr_t>(ptr);
    if (a % page) fail(VH_ERR_ARG, "vh_host_register: start must be page aligned");
    const uint64_t len = (bytes + page - 1) / page * page;
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_reg.upper_bound(a + len - 1);
    if (it != g_reg.begin() && std::prev(it)->second > a) fail(VH_ERR_ARG, "vh_host_register: range overlaps a registered one");
    hipError_t e = hipHostRegister(ptr, len, hipHostRegisterReadOnly);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        fail(VH_ERR_NOMEM, std::string("hipHostRegister failed: ") + hipGetErrorString(e));
    }
    g_reg[a] = a + len;
    VH_API_END
}

int vh_host_unregister(void *ptr) {
    VH_API_BEGIN
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_reg.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == g_reg.end()) fail(VH_ERR_ARG, "vh_host_unregister: not a registered range");
    // copies from the range were issued on the library's streams; drain them first
    VH_HIP(hipDeviceSynchronize());
    g_reg.erase(it);
    VH_HIP(hipHostUnregister(ptr));
    VH_API_END
}

int vh_memcpy_htod(void *dst, const void *src, uint64_t bytes) {
    VH_API_BEGIN
    VH_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream()));
    VH_HIP(hipStreamSynchronize(stream()));
    VH_API_END
}

int vh_memcpy_dtoh(void *dst, const void *src, uint64_t bytes) {
    VH_API_BEGIN
    copy_to_host(dst, src, bytes, stream());
    VH_HIP(hipStreamSynchronize(stream()));
    VH_API_END
}

int vh_memcpy_dtod(void *dst, const void *src, uint64_t bytes) {
    VH_API_BEGIN
    VH_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, stream()));
    VH_HIP(hipStreamSynchronize(stream()));
    VH_API_END
}

int vh_memset(void *dptr, int value, uint64_t bytes) {
    VH_API_BEGIN
    VH_HIP(hipMemsetAsync(dptr, value, bytes, stream()));
    VH_HIP(hipStreamSynchronize(stream()));
    VH_API_END
}

int vh_fill_random(void *dptr, uint64_t n, int dtype, int dist, uint64_t seed, double a, double b) {
    VH_API_BEGIN
    if (dist < 0 || dist > 4) fail(VH_ERR_ARG, "unknown distribution");
    if (dist < 2 && dtype != VH_F64 && dtype != VH_F32) fail(VH_ERR_ARG, "uniform/normal fill needs float64/float32");
    if (dist == 3 && dtype != VH_F64) fail(VH_ERR_ARG, "sorted normal fill needs float64");
    if (dist == 2 && dtype != VH_I32 && dtype != VH_I64 && dtype != VH_I8) fail(VH_ERR_ARG, "integer fill needs int8/int32/int64");
    if (dist == 4 && dtype != VH_I32 && dtype != VH_I64) fail(VH_ERR_ARG, "sorted integer fill needs int32/int64");
    if (n) {
        hipLaunchKernelGGL(k_fill_random, dim3(blocks_for(n, 256)), dim3(256), 0, stream(), dptr, n, dtype,
                           dist, seed, a, b);
        VH_HIP(hipGetLastError());
    }
    VH_HIP(hipStreamSynchronize(stream()));
    VH_API_END
}

int vh_timing_enable(int on) {
    VH_API_BEGIN
    g_timing = on != 0;
    VH_API_END
}

int vh_timing_reset(void) {
    VH_API_BEGIN
    VH_HIP(hipStreamSynchronize(stream()));
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto &kv : g_timing_recs)
        for (auto &p : kv.second.ev) {
            (void)hipEventDestroy(p.first);
            (void)hipEventDestroy(p.second);
        }
    g_timing_recs.clear();
    VH_API_END
}

int vh_timing_read(const char *kernel, uint64_t *launches, double *total_ms) {
    VH_API_BEGIN
    VH_HIP(hipStreamSynchronize(stream()));
    std::lock_guard<std::mutex> lk(g_mu);
    *launches = 0;
    *total_ms = 0;
    auto it = g_timing_recs.find(kernel);
    if (it == g_timing_recs.end()) return VH_OK;
    for (auto &p : it->second.ev) {
        float ms = 0;
        VH_HIP(hipEventElapsedTime(&ms, p.first, p.second));
        *total_ms += ms;
        *launches += 1;
    }
    VH_API_END
}

int vh_stat_read(const char *name, uint64_t *value, int reset) {
    VH_API_BEGIN
    const std::string n = name ? name : "";
    if (n == "tile_overflow_rows") *value = stat_tile_overflow(reset != 0);
    else if (n == "hashagg_overflow_rows") *value = stat_hashagg_overflow(reset != 0);
    else if (n == "set_overflow_rows") *value = stat_set_overflow(reset != 0);
    else if (n == "first_tiled_chunks") *value = stat_first_tiled(reset != 0);
    else fail(VH_ERR_ARG, "vh_stat_read: unknown statistic '" + n + "'");
    VH_API_END
}

int vh_stream(void **s) {
    VH_API_BEGIN
    *s = (void *)stream();
    VH_API_END
}

// the 16-B (min key, max key) result through a page-locked block (a pageable read-back
// costs more than the scan)
static void minmax_result(const DevBuf &keys, double *out_min, double *out_max) {
    thread_local PinnedBuf res_buf;
    res_buf.ensure(16);
    uint64_t *res = res_buf.as<uint64_t>();
    VH_HIP(hipMemcpyAsync(res, keys.ptr, 16, hipMemcpyDeviceToHost, stream()));
    VH_HIP(hipStreamSynchronize(stream()));
    if (res[0] == ~0ULL) {  // no non-NaN value (nanmin of all-NaN -> nan)
        *out_min = __builtin_nan("");
        *out_max = __builtin_nan("");
    } else {
        *out_min = f64_from_key(res[0]);
        *out_max = f64_from_key(res[1]);
    }
}

int vh_minmax_sample(const void *data, uint64_t n, int dtype, uint64_t nsample, double *out_min, double *out_max) {
    VH_API_BEGIN
    if (resolve_loc(data, VH_LOC_AUTO) != VH_LOC_DEVICE) throw std::runtime_error("vh_minmax_sample: column not in device memory");
    if (dtype == VH_BOOL) throw std::runtime_error("vh_minmax_sample: bool column");
    const uint64_t ns = std::min(n, nsample);
    DevBuf keys;
    const unsigned nb = ns ? (unsigned)std::min<uint64_t>((ns + 255) / 256, 256) : 0;
    keys.ensure(16 * ((uint64_t)nb + 1));
    uint64_t *part = keys.as<uint64_t>() + 2;
    if (nb) {
        VH_DISPATCH_DTYPE(dtype, T,
                          if constexpr (!std::is_same_v<T, vbool>)
                              hipLaunchKernelGGL(k_minmax_sample<T>, dim3(nb), dim3(256), 0, stream(),
                                                 static_cast<const T *>(data), n, ns, part));
        VH_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_minmax_fin, dim3(1), dim3(256), 0, stream(), part, nb, keys.as<uint64_t>());
    VH_HIP(hipGetLastError());
    minmax_result(keys, out_min, out_max);
    VH_API_END
}

int vh_minmax(const void *data, uint64_t n, int dtype, int flip, const uint8_t *mask, int loc,
              double *out_min, double *out_max) {
    VH_API_BEGIN
    loc = resolve_loc(data, loc);
    int isz = dtype_itemsize(dtype);
    DevBuf stage, mstage, keys;
    const void *d = data;
    const uint8_t *m = mask;
    if (loc == VH_LOC_HOST && n) {
        stage.ensure(n * isz);
        VH_HIP(hipMemcpyAsync(stage.ptr, data, n * isz, hipMemcpyHostToDevice, stream()));
        d = stage.ptr;
        if (mask) {
            mstage.ensure(n);
            VH_HIP(hipMemcpyAsync(mstage.ptr, mask, n, hipMemcpyHostToDevice, stream()));
            m = mstage.as<uint8_t>();
        }
    }
    // per-workgroup partials, folded by one workgroup (k_minmax_fin) into keys
    const bool vec_ok = !flip && !m && dtype != VH_BOOL && (reinterpret_cast<uintptr_t>(d) & 15) == 0;
    const uint64_t nvec = vec_ok && n * isz >= 16 ? n * isz / 16 : 0;
    const uint64_t done = nvec * (16 / isz);
    const unsigned nb1 = nvec ? blocks_for(nvec, 256, 8) : 0;
    const unsigned nb2 = done < n ? blocks_for(n - done, 256, 4) : 0;
    keys.ensure(16 * ((uint64_t)nb1 + nb2 + 1));
    uint64_t *part = keys.as<uint64_t>() + 2;
    {
        TimedScope ts("minmax");
        if (nb1) {
            VH_DISPATCH_DTYPE(dtype, T,
                              if constexpr (!std::is_same_v<T, vbool>)
                                  hipLaunchKernelGGL(k_minmax_vec<T>, dim3(nb1), dim3(256), 0,
                                                     stream(), static_cast<const T *>(d), nvec, part));
            VH_HIP(hipGetLastError());
        }
        if (nb2) {
            const void *rest = static_cast<const char *>(d) + done * isz;
            VH_DISPATCH_DTYPE(dtype, T,
                              hipLaunchKernelGGL(k_minmax<T>, dim3(nb2), dim3(256), 0,
                                                 stream(), rest, n - done, flip, m ? m + done : m, part + 2 * (uint64_t)nb1));
            VH_HIP(hipGetLastError());
        }
        hipLaunchKernelGGL(k_minmax_fin, dim3(1), dim3(256), 0, stream(), part, nb1 + nb2, keys.as<uint64_t>());
        VH_HIP(hipGetLastError());
    }
    minmax_result(keys, out_min, out_max);
    VH_API_END
}

}  // extern "C"
