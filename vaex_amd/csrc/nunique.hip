// AggNUnique on the GPU: the number of distinct values per grid cell
// (packages/vaex-core/src/agg_hash_primitive.cpp:6-102).
//
// The reference keeps one hash counter per cell.  Here every chunk appends the (cell,
// value) pairs of its rows to one list in HBM (missing / NaN rows only bump per-cell
// counters); when the grid is read the list is sorted by (cell, value) with two stable
// radix passes, equal neighbours collapse, and each cell counts its distinct values.  The
// deduplicated list is kept, so later chunks and reduce() keep appending to it.
//
// Per cell, as the reference computes it (agg_hash_primitive.cpp:24-38, hash.hpp:208-222):
//   distinct + (null rows > 0) + (nan rows > 0)
//            - (dropmissing ? null rows : 0) - (dropnan ? nan rows : 0)
// Rows outside a selection (a selection mask is set and the row's data mask is 0) are not
// seen at all; without a selection a data-mask 0 row is a missing value.  Values compare
// as the hash map's equal_to: -0.0 == 0.0; NaN never enters the list.
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>

#include "common.hpp"
#include "engine.hpp"

namespace vh {

constexpr uint64_t NU_COMPACT_AT = uint64_t(1) << 28;  // pairs before an eager dedup

template <typename T> __device__ inline T nu_load(const void *p, uint64_t i, int flip) {
    T v = static_cast<const T *>(p)[i];
    if constexpr (!std::is_same_v<T, vbool>) {
        if (flip) v = bswap_v(v);
    }
    return v;
}

// the value's key bits and whether it is NaN
template <typename T> __device__ inline uint64_t nu_bits(T v, bool *nan) {
    *nan = false;
    if constexpr (std::is_same_v<T, double> || std::is_same_v<T, float>) {
        const double d = (double)v;
        if (d != d) {
            *nan = true;
            return 0;
        }
        return __builtin_bit_cast(uint64_t, d == 0.0 ? 0.0 : d);
    } else if constexpr (std::is_same_v<T, vbool>) {
        return v.v ? 1 : 0;
    } else if constexpr (std::is_signed_v<T>) {
        return (uint64_t)(int64_t)v;
    } else {
        return (uint64_t)v;
    }
}

// Collect with a workgroup-private LDS dedup for values of <= 4 bytes (DEDUP): (cell,
// 32-bit value pattern) packs into one 64-bit LDS key and a pair is emitted only when its
// CAS claims an empty slot; the table is cleared between batches once half full, a pair that
// finds no slot in NU_PROBES probes is emitted anyway (the sort + unique at read time removes
// every duplicate).  It pays when a workgroup sees few distinct pairs (categorical values).
constexpr uint32_t NU_TAB = 8192;  // 64 KB of LDS
constexpr int NU_THREADS = 256, NU_RPT = 8, NU_PROBES = 16;
constexpr uint64_t NU_EMPTY = ~uint64_t(0);

template <typename T> __device__ inline uint32_t nu_pack32(T v) {
    if constexpr (std::is_same_v<T, float>) return __builtin_bit_cast(uint32_t, v == 0.0f ? 0.0f : v);
    else if constexpr (std::is_same_v<T, vbool>) return v.v ? 1u : 0u;
    else return (uint32_t)v;
}

template <typename T, bool DEDUP>
__global__ __launch_bounds__(NU_THREADS) void k_nu_collect_b(AggDev a, const uint64_t *idx, uint64_t n,
                                                             uint64_t rows_per_wg, uint64_t *null_cnt, uint64_t *nan_cnt,
                                                             uint64_t *out_cell, uint64_t *out_val,
                                                             unsigned long long *counter) {
    __shared__ uint64_t tab[DEDUP ? NU_TAB : 1];
    __shared__ uint32_t s_fill, s_w[NU_THREADS / 64];
    __shared__ unsigned long long s_base;
    if constexpr (DEDUP)
        for (uint32_t i = threadIdx.x; i < NU_TAB; i += NU_THREADS) tab[i] = NU_EMPTY;
    if (threadIdx.x == 0) s_fill = 0;
    __syncthreads();
    const uint64_t r0 = blockIdx.x * rows_per_wg, r1 = min(n, r0 + rows_per_wg);
    for (uint64_t b0 = r0; b0 < r1; b0 += (uint64_t)NU_THREADS * NU_RPT) {
        uint64_t cell[NU_RPT], bits[NU_RPT];
        uint32_t emit = 0;
#pragma unroll
        for (int r = 0; r < NU_RPT; r++) {
            const uint64_t i = b0 + (uint64_t)r * NU_THREADS + threadIdx.x;
            cell[r] = 0;
            bits[r] = 0;
            if (i >= r1) continue;
            const uint64_t c = idx[i];
            cell[r] = c;
            const bool masked = a.mask && a.mask[i] == 0;
            if (masked && a.has_selection) continue;  // outside the selection: not seen
            if (masked) {
                atomicAdd((unsigned long long *)&null_cnt[c], 1ULL);
                continue;
            }
            const T v = nu_load<T>(a.data, i, a.flip);
            bool nan;
            bits[r] = nu_bits<T>(v, &nan);
            if (nan) {
                atomicAdd((unsigned long long *)&nan_cnt[c], 1ULL);
                continue;
            }
            bool e = true;
            if constexpr (DEDUP) {
                const uint64_t key = (c << 32) | nu_pack32<T>(v);
                uint32_t h = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 51) & (NU_TAB - 1);
                for (int pr = 0; pr < NU_PROBES; pr++) {
                    const uint64_t old = atomicCAS((unsigned long long *)&tab[h], (unsigned long long)NU_EMPTY,
                                                   (unsigned long long)key);
                    if (old == NU_EMPTY) {
                        atomicAdd(&s_fill, 1u);
                        break;
                    }
                    if (old == key) {
                        e = false;
                        break;
                    }
                    h = (h + 1) & (NU_TAB - 1);
                }
            }
            if (e) emit |= 1u << r;
        }
        uint64_t pos = block_reserve<NU_THREADS>(__popc(emit), s_w, &s_base, counter);
#pragma unroll
        for (int r = 0; r < NU_RPT; r++) {
            if (!((emit >> r) & 1)) continue;
            out_cell[pos] = cell[r];
            out_val[pos] = bits[r];
            pos++;
        }
        if constexpr (DEDUP) {
            if (s_fill > NU_TAB / 2) {  // uniform: read after block_reserve's barriers
                __syncthreads();
                for (uint32_t k = threadIdx.x; k < NU_TAB; k += NU_THREADS) tab[k] = NU_EMPTY;
                __syncthreads();
                if (threadIdx.x == 0) s_fill = 0;
                __syncthreads();
            }
        }
    }
}

// after the (cell, value) sort: the first of each run of equal pairs counts for its cell and
// is written to the deduplicated list.  A thread takes NU_RPT consecutive pairs; counts of a
// wave whose pairs all lie in one cell (the common case of a cell-sorted list) are summed
// into one atomic, the list slots are reserved once per workgroup.
__global__ __launch_bounds__(NU_THREADS) void k_nu_unique(const uint64_t *cell, const uint64_t *val, uint64_t n,
                                                          uint64_t *distinct, uint64_t *out_cell, uint64_t *out_val,
                                                          unsigned long long *counter) {
    __shared__ uint32_t s_w[NU_THREADS / 64];
    __shared__ unsigned long long s_base;
    constexpr uint64_t TILE = (uint64_t)NU_THREADS * NU_RPT;
    const int lane = threadIdx.x & 63;
    for (uint64_t t0 = blockIdx.x * TILE; t0 < n; t0 += (uint64_t)gridDim.x * TILE) {
        const uint64_t i0 = t0 + (uint64_t)threadIdx.x * NU_RPT;
        uint32_t first = 0, cnt = 0;
        const uint64_t c0 = i0 < n ? cell[i0] : ~uint64_t(0);
        bool one_cell = true;
#pragma unroll
        for (int r = 0; r < NU_RPT; r++) {
            const uint64_t i = i0 + r;
            if (i >= n) break;
            const uint64_t c = cell[i];
            const bool f = i == 0 || c != cell[i - 1] || val[i] != val[i - 1];
            if (f) {
                first |= 1u << r;
                cnt++;
            }
            one_cell = one_cell && c == c0;
        }
        // distinct counts: one atomic per wave when every lane's pairs are in lane 0's cell
        const uint64_t wc = __shfl(c0, 0, 64);
        const bool wave_one = __all(i0 >= n || (one_cell && c0 == wc));
        if (wave_one) {
            uint32_t sum = cnt;
#pragma unroll
            for (int off = 32; off; off >>= 1) sum += __shfl_xor(sum, off, 64);
            if (lane == 0 && sum) atomicAdd((unsigned long long *)&distinct[wc], (unsigned long long)sum);
        } else {
#pragma unroll
            for (int r = 0; r < NU_RPT; r++)
                if ((first >> r) & 1) atomicAdd((unsigned long long *)&distinct[cell[i0 + r]], 1ULL);
        }
        uint64_t pos = block_reserve<NU_THREADS>(cnt, s_w, &s_base, counter);
#pragma unroll
        for (int r = 0; r < NU_RPT; r++) {
            if (!((first >> r) & 1)) continue;
            out_cell[pos] = cell[i0 + r];
            out_val[pos] = val[i0 + r];
            pos++;
        }
    }
}

__global__ __launch_bounds__(256) void k_nu_grid(const uint64_t *distinct, const uint64_t *null_cnt,
                                                 const uint64_t *nan_cnt, uint64_t L, uint32_t flags, int64_t *grid) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < L; i += (uint64_t)gridDim.x * blockDim.x) {
        int64_t v = (int64_t)distinct[i] + (null_cnt[i] ? 1 : 0) + (nan_cnt[i] ? 1 : 0);
        if (flags & 1) v -= (int64_t)null_cnt[i];
        if (flags & 2) v -= (int64_t)nan_cnt[i];
        grid[i] = v;
    }
}

__global__ void k_nu_add(uint64_t *a, const uint64_t *b, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        a[i] += b[i];
}

static unsigned bits_for(uint64_t v) {
    unsigned b = 1;
    while (b < 64 && (v >> b)) b++;
    return b;
}

static uint64_t read_counter(const DevBuf &b) {
    uint64_t v = 0;
    VH_HIP(hipMemcpyAsync(&v, b.ptr, 8, hipMemcpyDeviceToHost, stream()));
    VH_HIP(hipStreamSynchronize(stream()));
    return v;
}

// room for `extra` more pairs (the list is copied into a doubled buffer)
static void nu_reserve(vh_agg *a, uint64_t extra) {
    const uint64_t need = (a->nu_n + extra) * 8;
    if (need <= a->nu_cell.bytes) return;
    uint64_t cap = std::max<uint64_t>(need, a->nu_cell.bytes * 2);
    cap = std::max<uint64_t>(cap, 1 << 16);
    DevBuf nc, nv;
    nc.ensure(cap);
    nv.ensure(cap);
    if (a->nu_n) {
        VH_HIP(hipMemcpyAsync(nc.ptr, a->nu_cell.ptr, a->nu_n * 8, hipMemcpyDeviceToDevice, stream()));
        VH_HIP(hipMemcpyAsync(nv.ptr, a->nu_val.ptr, a->nu_n * 8, hipMemcpyDeviceToDevice, stream()));
    }
    VH_HIP(hipStreamSynchronize(stream()));
    std::swap(a->nu_cell.ptr, nc.ptr);
    std::swap(a->nu_cell.bytes, nc.bytes);
    std::swap(a->nu_val.ptr, nv.ptr);
    std::swap(a->nu_val.bytes, nv.bytes);
}

// sort the list by (cell, value), count distinct pairs per cell into `distinct` (L
// counters, or a scratch when null) and replace the list by its deduplicated form
static void nu_dedup(vh_agg *a, uint64_t *distinct) {
    const uint64_t n = a->nu_n, L = a->L;
    hipStream_t st = stream();
    if (distinct) VH_HIP(hipMemsetAsync(distinct, 0, L * 8, st));
    if (!n) return;
    TimedScope ts("nunique_dedup");
    DevBuf c1, v1, c2, v2, tmp, ctr, dscratch;
    c1.ensure(n * 8);
    v1.ensure(n * 8);
    c2.ensure(n * 8);
    v2.ensure(n * 8);
    ctr.ensure(8);
    const unsigned cbits = bits_for(L);
    size_t t1 = 0, t2 = 0;
    VH_HIP(rocprim::radix_sort_pairs(nullptr, t1, (uint64_t *)nullptr, (uint64_t *)nullptr, (uint64_t *)nullptr,
                                     (uint64_t *)nullptr, (size_t)n, 0, 64, st));
    VH_HIP(rocprim::radix_sort_pairs(nullptr, t2, (uint64_t *)nullptr, (uint64_t *)nullptr, (uint64_t *)nullptr,
                                     (uint64_t *)nullptr, (size_t)n, 0, cbits, st));
    tmp.ensure(std::max<size_t>(std::max(t1, t2), 16));
    // LSD: by value, then stably by cell
    size_t tb = tmp.bytes;
    VH_HIP(rocprim::radix_sort_pairs(tmp.ptr, tb, a->nu_val.as<uint64_t>(), v1.as<uint64_t>(),
                                     a->nu_cell.as<uint64_t>(), c1.as<uint64_t>(), (size_t)n, 0, 64, st));
    tb = tmp.bytes;
    VH_HIP(rocprim::radix_sort_pairs(tmp.ptr, tb, c1.as<uint64_t>(), c2.as<uint64_t>(), v1.as<uint64_t>(),
                                     v2.as<uint64_t>(), (size_t)n, 0, cbits, st));
    uint64_t *dist = distinct;
    if (!dist) {
        dscratch.ensure(L * 8);
        dist = dscratch.as<uint64_t>();
        VH_HIP(hipMemsetAsync(dist, 0, L * 8, st));
    }
    VH_HIP(hipMemsetAsync(ctr.ptr, 0, 8, st));
    hipLaunchKernelGGL(k_nu_unique, dim3(blocks_for((n + NU_RPT - 1) / NU_RPT, NU_THREADS)), dim3(NU_THREADS), 0, st,
                       c2.as<uint64_t>(), v2.as<uint64_t>(),
                       n, dist, a->nu_cell.as<uint64_t>(), a->nu_val.as<uint64_t>(),
                       reinterpret_cast<unsigned long long *>(ctr.ptr));
    VH_HIP(hipGetLastError());
    a->nu_n = read_counter(ctr);
}

void nunique_init(vh_agg *a) {
    const uint64_t L = a->L;
    a->g2.ensure(std::max<uint64_t>(L, 1) * 8);
    a->s_key.ensure(std::max<uint64_t>(L, 1) * 8);
    VH_HIP(hipMemsetAsync(a->g.ptr, 0, L * 8, stream()));
    VH_HIP(hipMemsetAsync(a->g2.ptr, 0, L * 8, stream()));
    VH_HIP(hipMemsetAsync(a->s_key.ptr, 0, L * 8, stream()));
    VH_HIP(hipStreamSynchronize(stream()));
    a->nu_n = 0;
    a->nu_dirty = false;
}

void nunique_collect(vh_agg *a, const AggDev &ad, const uint64_t *idx, uint64_t len) {
    if (!len) return;
    if (a->nu_n + len > NU_COMPACT_AT && a->nu_n) nu_dedup(a, nullptr);
    nu_reserve(a, len);
    DevBuf ctr;
    ctr.ensure(8);
    VH_HIP(hipMemsetAsync(ctr.ptr, 0, 8, stream()));
    {
        TimedScope ts("nunique_collect");
        // VH_NU_LDS=1: workgroup LDS dedup of <= 4-byte values (opt-in: at 1e8 rows with 3e4 or
        // more distinct pairs it was 0.2-0.35 ms slower than the plain collect)
        const char *e = getenv("VH_NU_LDS");
        const bool lds_on = e && atoi(e) != 0;
        const bool narrow = lds_on && dtype_itemsize(ad.dtype) <= 4 && a->L < (uint64_t(1) << 32);
        const unsigned nb = blocks_for((len + NU_RPT - 1) / NU_RPT, NU_THREADS, 4);
        const uint64_t per = ((len + nb - 1) / nb + NU_RPT - 1) / NU_RPT * NU_RPT;
        VH_DISPATCH_DTYPE(ad.dtype, T, {
            if (narrow)
                hipLaunchKernelGGL((k_nu_collect_b<T, true>), dim3(nb), dim3(NU_THREADS), 0, stream(), ad, idx, len, per,
                                   a->g2.as<uint64_t>(), a->s_key.as<uint64_t>(), a->nu_cell.as<uint64_t>() + a->nu_n,
                                   a->nu_val.as<uint64_t>() + a->nu_n, reinterpret_cast<unsigned long long *>(ctr.ptr));
            else
                hipLaunchKernelGGL((k_nu_collect_b<T, false>), dim3(nb), dim3(NU_THREADS), 0, stream(), ad, idx, len, per,
                                   a->g2.as<uint64_t>(), a->s_key.as<uint64_t>(), a->nu_cell.as<uint64_t>() + a->nu_n,
                                   a->nu_val.as<uint64_t>() + a->nu_n, reinterpret_cast<unsigned long long *>(ctr.ptr));
        })
        VH_HIP(hipGetLastError());
    }
    a->nu_n += read_counter(ctr);
    a->nu_dirty = true;
}

void nunique_merge(vh_agg *a, vh_agg *o) {
    nunique_finalize(o);  // deduplicated first: fewer pairs to copy
    const uint64_t L = a->L;
    nu_reserve(a, o->nu_n);
    if (o->nu_n) {
        VH_HIP(hipMemcpyAsync(a->nu_cell.as<uint64_t>() + a->nu_n, o->nu_cell.ptr, o->nu_n * 8,
                              hipMemcpyDeviceToDevice, stream()));
        VH_HIP(hipMemcpyAsync(a->nu_val.as<uint64_t>() + a->nu_n, o->nu_val.ptr, o->nu_n * 8,
                              hipMemcpyDeviceToDevice, stream()));
    }
    a->nu_n += o->nu_n;
    if (L) {
        hipLaunchKernelGGL(k_nu_add, dim3(blocks_for(L, 256)), dim3(256), 0, stream(), a->g2.as<uint64_t>(),
                           o->g2.as<uint64_t>(), L);
        hipLaunchKernelGGL(k_nu_add, dim3(blocks_for(L, 256)), dim3(256), 0, stream(), a->s_key.as<uint64_t>(),
                           o->s_key.as<uint64_t>(), L);
        VH_HIP(hipGetLastError());
    }
    a->nu_dirty = true;
}

void nunique_finalize(vh_agg *a) {
    if (a->kind != VH_AGG_NUNIQUE || !a->nu_dirty) return;
    const uint64_t L = a->L;
    DevBuf distinct;
    distinct.ensure(std::max<uint64_t>(L, 1) * 8);
    nu_dedup(a, distinct.as<uint64_t>());
    if (L) {
        hipLaunchKernelGGL(k_nu_grid, dim3(blocks_for(L, 256)), dim3(256), 0, stream(), distinct.as<uint64_t>(),
                           a->g2.as<uint64_t>(), a->s_key.as<uint64_t>(), L, a->moment, a->g.as<int64_t>());
        VH_HIP(hipGetLastError());
    }
    VH_HIP(hipStreamSynchronize(stream()));
    a->nu_dirty = false;
}

}  // namespace vh

using namespace vh;

// Pairs and per-cell missing / NaN counts of an AggNUnique, to host memory and back: the
// multi-GPU combine gathers them from every rank (distributed.py), like counter::merge
// merges the per-thread counters (hash_primitives.hpp:393-415).
extern "C" int vh_agg_nunique_export(vh_agg *a, uint64_t *n, uint64_t *cells, uint64_t *vals, uint64_t *nulls,
                                     uint64_t *nans) {
    VH_API_BEGIN
    if (a->kind != VH_AGG_NUNIQUE) fail(VH_ERR_ARG, "not an AggNUnique");
    nunique_finalize(a);  // deduplicated
    if (n) *n = a->nu_n;
    hipStream_t st = stream();
    if (cells && a->nu_n) VH_HIP(hipMemcpyAsync(cells, a->nu_cell.ptr, a->nu_n * 8, hipMemcpyDeviceToHost, st));
    if (vals && a->nu_n) VH_HIP(hipMemcpyAsync(vals, a->nu_val.ptr, a->nu_n * 8, hipMemcpyDeviceToHost, st));
    if (nulls) VH_HIP(hipMemcpyAsync(nulls, a->g2.ptr, a->L * 8, hipMemcpyDeviceToHost, st));
    if (nans) VH_HIP(hipMemcpyAsync(nans, a->s_key.ptr, a->L * 8, hipMemcpyDeviceToHost, st));
    VH_HIP(hipStreamSynchronize(st));
    VH_API_END
}

extern "C" int vh_agg_nunique_import(vh_agg *a, uint64_t n, const uint64_t *cells, const uint64_t *vals,
                                     const uint64_t *nulls, const uint64_t *nans) {
    VH_API_BEGIN
    if (a->kind != VH_AGG_NUNIQUE) fail(VH_ERR_ARG, "not an AggNUnique");
    hipStream_t st = stream();
    for (uint64_t i = 0; i < n; i++)
        if (cells[i] >= a->L) fail(VH_ERR_ARG, "nunique import: cell index out of range");
    nu_reserve(a, n);
    if (n) {
        VH_HIP(hipMemcpyAsync(a->nu_cell.as<uint64_t>() + a->nu_n, cells, n * 8, hipMemcpyHostToDevice, st));
        VH_HIP(hipMemcpyAsync(a->nu_val.as<uint64_t>() + a->nu_n, vals, n * 8, hipMemcpyHostToDevice, st));
    }
    a->nu_n += n;
    DevBuf tmp;
    tmp.ensure(a->L * 16);
    VH_HIP(hipMemcpyAsync(tmp.ptr, nulls, a->L * 8, hipMemcpyHostToDevice, st));
    VH_HIP(hipMemcpyAsync(tmp.as<uint64_t>() + a->L, nans, a->L * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_nu_add, dim3(blocks_for(a->L, 256)), dim3(256), 0, st, a->g2.as<uint64_t>(), tmp.as<uint64_t>(),
                       a->L);
    hipLaunchKernelGGL(k_nu_add, dim3(blocks_for(a->L, 256)), dim3(256), 0, st, a->s_key.as<uint64_t>(),
                       tmp.as<uint64_t>() + a->L, a->L);
    VH_HIP(hipGetLastError());
    VH_HIP(hipStreamSynchronize(st));
    a->nu_dirty = true;
    VH_API_END
}
