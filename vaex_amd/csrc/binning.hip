// Grid / Binner / Aggregator engine of libvaexhip.so -- the MI355X (gfx950)
// realisation of vaex-core's superagg module:
//   Grid<>::bin / bin_            packages/vaex-core/src/agg.hpp:76-136
//   BinnerScalar / BinnerOrdinal  packages/vaex-core/src/superagg_binners.cpp:5-184
//   AggCount/Sum/Min/Max/First/SumMoment  packages/vaex-core/src/superagg.cpp:155-511
//
// Execution:
//  * fused path -- binner index math in registers, no indices1d round trip;
//    count/sum aggregators accumulate into LDS-privatised per-workgroup grids
//    when the grid fits (small grids), otherwise into tile-partitioned LDS
//    sub-grids (tiled.hip) or global atomics;
//  * generic path -- any binner/aggregator/dtype mix: an index kernel writes
//    indices1d for a chunk of rows, then one kernel per aggregator.
// Host (numpy) columns are staged to HBM chunk by chunk; HBM columns are read
// in place.
#include <limits>
#include <map>
#include <memory>
#include <mutex>

#include "common.hpp"
#include "engine.hpp"
#include "binner_dev.hpp"
#include "hashset.hpp"

using namespace vh;

// ============================================================================
// host objects
// ============================================================================
struct vh_binner {
    int kind = 0;  // 0 scalar, 1 ordinal, 2 set-ordinal
    std::string expression;
    int dtype = VH_F64;
    int flip = 0;
    double vmin = 0, vmax = 0;
    uint64_t bins = 0;
    uint64_t ordinal_count = 0, min_value = 0;
    vh_set *set = nullptr;
    ColumnRef data, mask;
    uint64_t shape() const { return (kind == 0 ? bins : ordinal_count) + 3; }
};



namespace vh {

// ============================================================================
// device: binner index math
// ============================================================================
// ============================================================================
// device: generic path
// ============================================================================
__global__ __launch_bounds__(256) void k_indices(BinPlan p, uint64_t n, uint64_t *idx) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        idx[i] = plan_index(p, i);
}

template <typename T> __device__ inline void atomic_add_grid(T *addr, T v);
template <> __device__ inline void atomic_add_grid<double>(double *a, double v) { atomicAdd(a, v); }
template <> __device__ inline void atomic_add_grid<int64_t>(int64_t *a, int64_t v) {
    atomicAdd((unsigned long long *)a, (unsigned long long)v);
}
template <> __device__ inline void atomic_add_grid<uint64_t>(uint64_t *a, uint64_t v) {
    atomicAdd((unsigned long long *)a, (unsigned long long)v);
}


template <typename T> struct Upcast { using type = int64_t; };
template <> struct Upcast<double> { using type = double; };
template <> struct Upcast<float> { using type = double; };
template <> struct Upcast<uint64_t> { using type = uint64_t; };
template <> struct Upcast<uint32_t> { using type = uint64_t; };
template <> struct Upcast<uint16_t> { using type = uint64_t; };
template <> struct Upcast<uint8_t> { using type = uint64_t; };

template <typename T> __device__ inline typename Upcast<T>::type upcast_v(T v) {
    return (typename Upcast<T>::type)v;
}
template <> __device__ inline int64_t upcast_v<vbool>(vbool v) { return v.v ? 1 : 0; }

// AggCount (superagg.cpp:168-191), AggSum (:362-388), AggMin/AggMax (:213-286),
// AggSumMoment (:406-432) over one chunk of precomputed indices
template <int KIND, typename T>
__global__ __launch_bounds__(256) void k_agg(AggDev a, const uint64_t *idx, uint64_t n) {
    using G = typename Upcast<T>::type;
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n;
         j += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t c = idx[j];
        if constexpr (KIND == VH_AGG_COUNT) {
            if (a.mask && a.mask[j] != 1) continue;
            if (a.data) {
                T v = load_v<T>(a.data, j, a.flip);
                if (is_nan_v(v)) continue;
            }
            atomicAdd((unsigned long long *)a.grid + c, 1ULL);
        } else if constexpr (KIND == VH_AGG_SUM) {
            if (a.mask && a.mask[j] != 1) continue;
            T v = load_v<T>(a.data, j, a.flip);
            if (is_nan_v(v)) continue;
            atomic_add_grid<G>(reinterpret_cast<G *>(a.grid) + c, upcast_v(v));
        } else if constexpr (KIND == VH_AGG_MIN || KIND == VH_AGG_MAX) {
            if (a.mask && a.mask[j] != 1) continue;
            T v = load_v<T>(a.data, j, a.flip);
            if (is_nan_v(v)) continue;
            atomic_minmax<T>(reinterpret_cast<T *>(a.grid) + c, v, KIND == VH_AGG_MAX);
        } else if constexpr (KIND == VH_AGG_SUM_MOMENT) {
            if (a.mask && a.mask[j] != 1) continue;
            // the reference converts to the upcast type first, then byte swaps (superagg.cpp:415-417)
            G value = upcast_v(reinterpret_cast<const T *>(a.data)[j]);
            if (a.flip) value = bswap_v(value);
            if (is_nan_v(value)) continue;
            double p;
            if (a.moment == 0) p = 1.0;
            else if (a.moment == 1) p = (double)value;
            else if (a.moment == 2) p = (double)value * (double)value;
            else p = pow((double)value, (double)a.moment);
            atomic_add_grid<G>(reinterpret_cast<G *>(a.grid) + c, (G)p);
        }
    }
}

// Small grids (<= LDS_AGG_MAX_BYTES of cells): every workgroup aggregates into its own LDS
// copy of the grid in the same pass that bins the rows (no indices1d round trip, no global
// atomic per row -- a few hundred cells hit by every row would serialise on them), then
// flushes it with one global atomic per touched cell.  Per-row semantics exactly as k_agg.
constexpr uint64_t LDS_AGG_MAX_BYTES = 96 * 1024;

template <int KIND, typename T> struct LdsCell {
    using G = typename Upcast<T>::type;
    using type = std::conditional_t<KIND == VH_AGG_MIN || KIND == VH_AGG_MAX, T,
                                    std::conditional_t<KIND == VH_AGG_COUNT, unsigned long long, G>>;
};

template <int KIND, typename T>
__global__ __launch_bounds__(256) void k_agg_lds(BinPlan p, AggDev a, uint64_t n, uint64_t L, T fill) {
    using G = typename Upcast<T>::type;
    using C = typename LdsCell<KIND, T>::type;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    C *g = reinterpret_cast<C *>(lds_raw);
    for (uint64_t c = threadIdx.x; c < L; c += blockDim.x) {
        if constexpr (KIND == VH_AGG_MIN || KIND == VH_AGG_MAX) g[c] = fill;
        else g[c] = (C)0;
    }
    __syncthreads();
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
        if (a.mask && a.mask[j] != 1) continue;
        const uint64_t c = plan_index(p, j);
        if constexpr (KIND == VH_AGG_COUNT) {
            if (a.data) {
                T v = load_v<T>(a.data, j, a.flip);
                if (is_nan_v(v)) continue;
            }
            atomicAdd(g + c, 1ULL);
        } else if constexpr (KIND == VH_AGG_SUM) {
            T v = load_v<T>(a.data, j, a.flip);
            if (is_nan_v(v)) continue;
            atomic_add_grid<G>(g + c, upcast_v(v));
        } else if constexpr (KIND == VH_AGG_MIN || KIND == VH_AGG_MAX) {
            T v = load_v<T>(a.data, j, a.flip);
            if (is_nan_v(v)) continue;
            atomic_minmax<T>(g + c, v, KIND == VH_AGG_MAX);
        } else if constexpr (KIND == VH_AGG_SUM_MOMENT) {
            G value = upcast_v(reinterpret_cast<const T *>(a.data)[j]);
            if (a.flip) value = bswap_v(value);
            if (is_nan_v(value)) continue;
            double pw;
            if (a.moment == 0) pw = 1.0;
            else if (a.moment == 1) pw = (double)value;
            else if (a.moment == 2) pw = (double)value * (double)value;
            else pw = pow((double)value, (double)a.moment);
            atomic_add_grid<G>(g + c, (G)pw);
        }
    }
    __syncthreads();
    for (uint64_t c = threadIdx.x; c < L; c += blockDim.x) {
        const C v = g[c];
        if constexpr (KIND == VH_AGG_MIN || KIND == VH_AGG_MAX) {
            using W = std::conditional_t<sizeof(T) == 8, uint64_t,
                                         std::conditional_t<sizeof(T) == 4, uint32_t,
                                                            std::conditional_t<sizeof(T) == 2, uint16_t, uint8_t>>>;
            W vb, fb;
            __builtin_memcpy(&vb, &v, sizeof(T));
            __builtin_memcpy(&fb, &fill, sizeof(T));
            if (vb != fb)
                atomic_minmax<T>(reinterpret_cast<T *>(a.grid) + c, v, KIND == VH_AGG_MAX);
        } else if constexpr (KIND == VH_AGG_COUNT) {
            if (v) atomicAdd((unsigned long long *)a.grid + c, v);
        } else {
            if (v != (C)0) atomic_add_grid<G>(reinterpret_cast<G *>(a.grid) + c, v);
        }
    }
}

// Small grids, binner dispatch hoisted out of the row loop.  k_agg_lds evaluates the
// generic plan_index per row and aggregator: a switch over kind and dtype per binner per
// row, measured at ~75 scalar + branch instructions per wave iteration (SQ counters, h2o
// q1), so those passes ran at ~1e11 rows/s whatever the column width.  Here one launch per
// dimension (kind and dtype as template arguments) adds index * stride into a u16 cell
// column (cells < 2^16 by the LDS bound), and each aggregator's pass reads that column.
constexpr int CELL_U = 4;  // rows per thread per step, loads issued together

// 8 consecutive rows of a column into registers: one 8- to 64-byte load when the column is
// 8 * sizeof(T) aligned (one byte per lane per instruction made the small-grid passes
// instruction-bound), else per row; `cnt` < 8 rows (the tail) load per row
constexpr int RU = 8;
template <typename T> __device__ __forceinline__ void load_rows8(const T *p, uint64_t j, uint32_t cnt, bool al, T (&out)[RU]) {
    if (al && cnt == RU) {
        if constexpr (sizeof(T) == 1) {
            const uint2 v = *reinterpret_cast<const uint2 *>(p + j);
            __builtin_memcpy(out, &v, 8);
        } else {
            uint4 v[sizeof(T) / 2];
#pragma unroll
            for (int k = 0; k < (int)sizeof(T) / 2; k++) v[k] = reinterpret_cast<const uint4 *>(p + j)[k];
            __builtin_memcpy(out, v, sizeof(out));
        }
    } else {
#pragma unroll
        for (int u = 0; u < RU; u++) out[u] = (uint32_t)u < cnt ? p[j + u] : T{};
    }
}
__device__ __forceinline__ bool aligned_rows8(const void *p, int isz) {
    return (reinterpret_cast<uintptr_t>(p) % (uintptr_t)(8 * isz)) == 0;
}

template <int KIND_B, typename T>
__global__ __launch_bounds__(256) void k_cells_dim(BinnerDev b, uint64_t n, uint16_t *cells, int first) {
    // thread = 8 consecutive rows per step: wide loads of the key, mask and previous cells,
    // one 16-byte store of the cells
    const bool al = aligned_rows8(b.data, sizeof(T)) && (!b.mask || aligned_rows8(b.mask, 1)) &&
                    aligned_rows8(cells, 2);
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x * RU;
    for (uint64_t j = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * RU; j < n; j += step) {
        const uint32_t cnt = (uint32_t)min<uint64_t>(RU, n - j);
        T raw[RU];
        uint8_t m[RU];
        uint16_t prev[RU];
        load_rows8<T>(reinterpret_cast<const T *>(b.data), j, cnt, al, raw);
        if (b.mask) load_rows8<uint8_t>(b.mask, j, cnt, al, m);
        if (!first) load_rows8<uint16_t>(cells, j, cnt, al, prev);
        uint16_t out[RU];
#pragma unroll
        for (int u = 0; u < RU; u++) {
            const bool mu = b.mask ? m[u] == 1 : false;
            const uint64_t c = KIND_B == 0 ? scalar_cell<T>(b, raw[u], mu) : ordinal_cell<T>(b, raw[u], mu);
            out[u] = (uint16_t)((first ? 0 : prev[u]) + c * b.stride);
        }
        if (al && cnt == RU) {
            uint4 v;
            __builtin_memcpy(&v, out, 16);
            *reinterpret_cast<uint4 *>(cells + j) = v;
        } else {
#pragma unroll
            for (int u = 0; u < RU; u++)
                if ((uint32_t)u < cnt) cells[j + u] = out[u];
        }
    }
}

// NARROW: 32-bit LDS cells (counts; sums of 8/16-bit integers when a workgroup's rows
// cannot overflow them, checked on the host), half the LDS of a sub-grid, so grids of
// ~10^4 cells keep several workgroups per CU
template <int KIND, typename T, bool NARROW = false>
__global__ __launch_bounds__(256) void k_agg_lds_c(AggDev a, const uint16_t *cells, uint64_t n, uint64_t L, T fill) {
    using G = typename Upcast<T>::type;
    using C = std::conditional_t<NARROW,
                                 std::conditional_t<KIND == VH_AGG_COUNT || !is_signed_int_t<T>::value, uint32_t, int32_t>,
                                 typename LdsCell<KIND, T>::type>;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    C *g = reinterpret_cast<C *>(lds_raw);
    for (uint64_t c = threadIdx.x; c < L; c += blockDim.x) {
        if constexpr (KIND == VH_AGG_MIN || KIND == VH_AGG_MAX) g[c] = fill;
        else g[c] = (C)0;
    }
    __syncthreads();
    // a thread takes RU consecutive rows per step (wide loads; the host's narrow-cell bound is
    // rows_per_wg(n, grid, block, RU))
    const bool al = aligned_rows8(cells, 2) && (!a.data || aligned_rows8(a.data, sizeof(T))) &&
                    (!a.mask || aligned_rows8(a.mask, 1));
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x * RU;
    for (uint64_t j = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * RU; j < n; j += step) {
        const uint32_t cnt = (uint32_t)min<uint64_t>(RU, n - j);
        uint16_t cell[RU];
        uint8_t m[RU];
        T v[RU];
        load_rows8<uint16_t>(cells, j, cnt, al, cell);
        if (a.mask) load_rows8<uint8_t>(a.mask, j, cnt, al, m);
        if (a.data) load_rows8<T>(reinterpret_cast<const T *>(a.data), j, cnt, al, v);
        else
#pragma unroll
            for (int u = 0; u < RU; u++) v[u] = T{};
#pragma unroll
        for (int u = 0; u < RU; u++) {
            if ((uint32_t)u >= cnt || (a.mask && m[u] != 1)) continue;
            const uint32_t c = cell[u];
            if constexpr (KIND == VH_AGG_COUNT) {
                if (a.data && is_nan_v(a.flip ? bswap_v(v[u]) : v[u])) continue;
                atomicAdd(g + c, (C)1);
            } else if constexpr (KIND == VH_AGG_SUM) {
                const T x = a.flip ? bswap_v(v[u]) : v[u];
                if (is_nan_v(x)) continue;
                if constexpr (NARROW) atomicAdd(g + c, (C)x);
                else atomic_add_grid<G>(g + c, upcast_v(x));
            } else if constexpr (KIND == VH_AGG_MIN || KIND == VH_AGG_MAX) {
                const T x = a.flip ? bswap_v(v[u]) : v[u];
                if (is_nan_v(x)) continue;
                atomic_minmax<T>(g + c, x, KIND == VH_AGG_MAX);
            } else if constexpr (KIND == VH_AGG_SUM_MOMENT) {
                // the reference converts to the upcast type first, then byte swaps (superagg.cpp:415-417)
                G value = upcast_v(v[u]);
                if (a.flip) value = bswap_v(value);
                if (is_nan_v(value)) continue;
                double pw;
                if (a.moment == 0) pw = 1.0;
                else if (a.moment == 1) pw = (double)value;
                else if (a.moment == 2) pw = (double)value * (double)value;
                else pw = pow((double)value, (double)a.moment);
                atomic_add_grid<G>(g + c, (G)pw);
            }
        }
    }
    __syncthreads();
    for (uint64_t c = threadIdx.x; c < L; c += blockDim.x) {
        const C v = g[c];
        if constexpr (KIND == VH_AGG_MIN || KIND == VH_AGG_MAX) {
            using W = std::conditional_t<sizeof(T) == 8, uint64_t,
                                         std::conditional_t<sizeof(T) == 4, uint32_t,
                                                            std::conditional_t<sizeof(T) == 2, uint16_t, uint8_t>>>;
            W vb, fb;
            __builtin_memcpy(&vb, &v, sizeof(T));
            __builtin_memcpy(&fb, &fill, sizeof(T));
            if (vb != fb)
                atomic_minmax<T>(reinterpret_cast<T *>(a.grid) + c, v, KIND == VH_AGG_MAX);
        } else if constexpr (KIND == VH_AGG_COUNT) {
            if (v) atomicAdd((unsigned long long *)a.grid + c, (unsigned long long)v);
        } else {
            if (v != (C)0) atomic_add_grid<G>(reinterpret_cast<G *>(a.grid) + c, (G)v);
        }
    }
}

// indices1d of the generic path with the binner dispatch hoisted out of the row loop (one
// launch per dimension, kind and dtype as template arguments; k_indices keeps set-ordinal
// binners, whose per-row hash probe dominates anyway)
template <int KIND_B, typename T>
__global__ __launch_bounds__(256) void k_idx_dim(BinnerDev b, uint64_t n, uint64_t *idx, int first) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j0 < n; j0 += step * CELL_U) {
        T raw[CELL_U];
        bool m[CELL_U];
        uint64_t prev[CELL_U];
#pragma unroll
        for (int u = 0; u < CELL_U; u++) {
            const uint64_t j = j0 + (uint64_t)u * step;
            const bool in = j < n;
            raw[u] = in ? reinterpret_cast<const T *>(b.data)[j] : T{};
            m[u] = (in && b.mask) ? b.mask[j] == 1 : false;
            prev[u] = (in && !first) ? idx[j] : 0;
        }
#pragma unroll
        for (int u = 0; u < CELL_U; u++) {
            const uint64_t j = j0 + (uint64_t)u * step;
            if (j >= n) continue;
            const uint64_t c = KIND_B == 0 ? scalar_cell<T>(b, raw[u], m[u]) : ordinal_cell<T>(b, raw[u], m[u]);
            idx[j] = prev[u] + c * b.stride;
        }
    }
}

// Several count / sum aggregators of one small grid in ONE pass over the u16 cells (each
// aggregator of k_agg_lds_c re-reads the cells and pays its own loop).  Per step a thread
// takes SF_U rows; the aggregator's dtype is dispatched once per step (not per row), its
// values and mask loaded for all SF_U rows, then added into its LDS sub-grid.
constexpr int SF_MAX = 8;
constexpr int SF_U = 8;
// one fused launch's sub-grids: at most 48 KB, so three workgroups stay resident per CU
// (a 2 x 42 KB fused launch of h2o q2 ran at one per CU: 8.7 -> 10.8 ms)
constexpr uint64_t SF_LDS_BUDGET = 48 * 1024;
struct SmallAggs {
    int na, pad;
    uint32_t lds_off[SF_MAX];  // byte offset of each aggregator's sub-grid
    uint32_t shared;           // bit k: aggregator k is a row count equal to an earlier one
                               // (count(*) / count of an unmasked integer column): it adds
                               // nothing itself and flushes that one's sub-grid
    uint32_t narrow;           // bit k: 32-bit LDS cells (counts; 8/16-bit integer sums whose
                               // per-workgroup partials fit, checked on the host)
    AggDev a[SF_MAX];
};

template <typename T>
__device__ inline void sf_rows(const AggDev &a, unsigned char *lds, const uint16_t (&cell)[SF_U], uint64_t j, uint32_t cnt,
                               bool narrow) {
    using G = typename Upcast<T>::type;
    static_assert(SF_U == RU, "sf_rows takes one load_rows8 group");
    T v[SF_U];
    uint8_t m[SF_U];
    const bool al = (!a.data || aligned_rows8(a.data, sizeof(T))) && (!a.mask || aligned_rows8(a.mask, 1));
    if (a.data) load_rows8<T>(reinterpret_cast<const T *>(a.data), j, cnt, al, v);
    else
#pragma unroll
        for (int u = 0; u < SF_U; u++) v[u] = T{};
    if (a.mask) load_rows8<uint8_t>(a.mask, j, cnt, al, m);
#pragma unroll
    for (int u = 0; u < SF_U; u++) {
        if ((uint32_t)u >= cnt || (a.mask && m[u] != 1)) continue;
        const T x = a.flip ? bswap_v(v[u]) : v[u];
        if (a.kind == VH_AGG_COUNT) {
            if (a.data && is_nan_v(x)) continue;
            if (narrow) atomicAdd(reinterpret_cast<uint32_t *>(lds) + cell[u], 1u);
            else atomicAdd(reinterpret_cast<unsigned long long *>(lds) + cell[u], 1ULL);
        } else {
            if (is_nan_v(x)) continue;
            if constexpr (std::is_integral_v<T> && sizeof(T) <= 2) {
                if (narrow) {
                    atomicAdd(reinterpret_cast<int32_t *>(lds) + cell[u], (int32_t)x);
                    continue;
                }
            }
            atomic_add_grid<G>(reinterpret_cast<G *>(lds) + cell[u], upcast_v(x));
        }
    }
}

template <typename T>
__device__ inline void sf_flush(const AggDev &a, const unsigned char *lds, uint64_t L, bool narrow) {
    using G = typename Upcast<T>::type;
    for (uint64_t c = threadIdx.x; c < L; c += blockDim.x) {
        if (a.kind == VH_AGG_COUNT) {
            const unsigned long long v = narrow ? (unsigned long long)reinterpret_cast<const uint32_t *>(lds)[c]
                                                : reinterpret_cast<const unsigned long long *>(lds)[c];
            if (v) atomicAdd((unsigned long long *)a.grid + c, v);
        } else {
            // a narrow partial is an int32 (two's complement of the exact sum, which fits)
            const G v = narrow ? (G)(int64_t)reinterpret_cast<const int32_t *>(lds)[c] : reinterpret_cast<const G *>(lds)[c];
            if (v != (G)0) atomic_add_grid<G>(reinterpret_cast<G *>(a.grid) + c, v);
        }
    }
}

__global__ __launch_bounds__(256) void k_small_fused(SmallAggs sa, const uint16_t *cells, uint64_t n, uint64_t L,
                                                      uint32_t lds_words) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    uint32_t *w = reinterpret_cast<uint32_t *>(lds_raw);
    for (uint32_t i = threadIdx.x; i < lds_words; i += blockDim.x) w[i] = 0;
    __syncthreads();
    // a thread takes SF_U consecutive rows per step (wide loads; rows per workgroup stay
    // within rows_per_wg(n, grid, block, SF_U), the narrow-cell overflow bound)
    const bool cal = aligned_rows8(cells, 2);
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x * SF_U;
    for (uint64_t j = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * SF_U; j < n; j += step) {
        const uint32_t cnt = (uint32_t)min<uint64_t>(SF_U, n - j);
        uint16_t cell[SF_U];
        load_rows8<uint16_t>(cells, j, cnt, cal, cell);
        for (int k = 0; k < sa.na; k++) {
            if ((sa.shared >> k) & 1) continue;
            const AggDev &a = sa.a[k];
            unsigned char *lds = lds_raw + sa.lds_off[k];
            const bool nw = (sa.narrow >> k) & 1;
            VH_DEV_DISPATCH(a.dtype, T, sf_rows<T>(a, lds, cell, j, cnt, nw); break)
        }
    }
    __syncthreads();
    for (int k = 0; k < sa.na; k++) {
        const AggDev &a = sa.a[k];
        const unsigned char *lds = lds_raw + sa.lds_off[k];
        const bool nw = (sa.narrow >> k) & 1;
        VH_DEV_DISPATCH(a.dtype, T, sf_flush<T>(a, lds, L, nw); break)
    }
}

// AggFirst (superagg.cpp:481-505).  Per chunk: (A) min order key per cell,
// (B) lowest row holding that key, (C) per cell: take it if strictly smaller
// than the grid's order -- ties go to the earliest row, as a serial pass does.
// (order_key: common.hpp; the tile path, tiled.hip, fills the same (A)/(B) scratch.)
template <typename T>
__global__ __launch_bounds__(256) void k_first_a(AggDev a, const uint64_t *idx, uint64_t n) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n;
         j += (uint64_t)gridDim.x * blockDim.x) {
        T v = load_v<T>(a.data, j, a.flip), o = load_v<T>(a.data2, j, a.flip);
        if (is_nan_v(v) || is_nan_v(o)) continue;
        atomicMin((unsigned long long *)a.s_key + idx[j], (unsigned long long)order_key(o));
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_first_b(AggDev a, const uint64_t *idx, uint64_t n, uint64_t row0) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n;
         j += (uint64_t)gridDim.x * blockDim.x) {
        T v = load_v<T>(a.data, j, a.flip), o = load_v<T>(a.data2, j, a.flip);
        if (is_nan_v(v) || is_nan_v(o)) continue;
        const uint64_t c = idx[j];
        if (order_key(o) == reinterpret_cast<const uint64_t *>(a.s_key)[c])
            atomicMin((unsigned long long *)a.s_row + c, (unsigned long long)(row0 + j));
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_first_c(AggDev a, uint64_t cells, uint64_t row0) {
    uint64_t *sk = reinterpret_cast<uint64_t *>(a.s_key);
    uint64_t *sr = reinterpret_cast<uint64_t *>(a.s_row);
    for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < cells;
         c += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t r = sr[c];
        if (r == ~0ULL) continue;
        uint64_t j = r - row0;
        T o = load_v<T>(a.data2, j, a.flip);
        T v = load_v<T>(a.data, j, a.flip);
        T *g = reinterpret_cast<T *>(a.grid);
        T *g2 = reinterpret_cast<T *>(a.grid2);
        if (o < g2[c]) {
            g[c] = v;
            g2[c] = o;
        }
        sk[c] = ~0ULL;
        sr[c] = ~0ULL;
    }
}

// AggFirst on a small grid (L cells of 12 B of LDS each fit a workgroup): each workgroup
// keeps, per cell, the smallest order key of its rows and the lowest row holding it -- per
// 2048-row step, phase 1 lowers the key (a row that lowers it clears the cell's row), phase 2
// lowers the row among rows holding the key -- and writes its (key, row) cells as partials;
// k_first_small_fold folds the partials per cell into s_key / s_row (global rows) for
// k_first_c.  No per-row global atomics (the generic k_first_a/b contend on few cells).
constexpr int FS_THREADS = 256, FS_RPT = 8;
template <typename T>
__global__ __launch_bounds__(FS_THREADS) void k_first_small(AggDev a, const uint16_t *cells, uint64_t n, uint32_t L,
                                                            unsigned long long *pkey, uint32_t *prow) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    unsigned long long *lkey = reinterpret_cast<unsigned long long *>(lds_raw);
    uint32_t *lrow = reinterpret_cast<uint32_t *>(lkey + L);
    for (uint32_t c = threadIdx.x; c < L; c += FS_THREADS) {
        lkey[c] = ~0ull;
        lrow[c] = ~0u;
    }
    __syncthreads();
    // workgroup w takes steps w, w + W, ... of FS_THREADS * FS_RPT rows (uniform trip count)
    constexpr uint64_t STEP = (uint64_t)FS_THREADS * FS_RPT;
    for (uint64_t b0 = blockIdx.x * STEP; b0 < n; b0 += (uint64_t)gridDim.x * STEP) {
        uint32_t cl[FS_RPT];
        unsigned long long kk[FS_RPT];
        bool take[FS_RPT];
#pragma unroll
        for (int r = 0; r < FS_RPT; r++) {
            const uint64_t i = b0 + (uint64_t)r * FS_THREADS + threadIdx.x;
            take[r] = false;
            cl[r] = 0;
            kk[r] = ~0ull;
            if (i < n) {
                const T v = load_v<T>(a.data, i, a.flip), o = load_v<T>(a.data2, i, a.flip);
                take[r] = !is_nan_v(v) && !is_nan_v(o);
                cl[r] = cells[i];
                kk[r] = order_key(o);
            }
        }
#pragma unroll
        for (int r = 0; r < FS_RPT; r++)
            if (take[r] && atomicMin(&lkey[cl[r]], kk[r]) > kk[r]) lrow[cl[r]] = ~0u;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < FS_RPT; r++)
            if (take[r] && kk[r] == lkey[cl[r]]) atomicMin(&lrow[cl[r]], (uint32_t)(b0 + (uint64_t)r * FS_THREADS + threadIdx.x));
        __syncthreads();
    }
    for (uint32_t c = threadIdx.x; c < L; c += FS_THREADS) {
        pkey[(uint64_t)blockIdx.x * L + c] = lkey[c];
        prow[(uint64_t)blockIdx.x * L + c] = lrow[c];
    }
}

// one workgroup per cell: the lexicographic (key, row) minimum over the W partials
__global__ __launch_bounds__(256) void k_first_small_fold(const unsigned long long *pkey, const uint32_t *prow, uint32_t W,
                                                          uint32_t L, uint64_t row0, unsigned long long *s_key,
                                                          unsigned long long *s_row) {
    __shared__ unsigned long long sk[4];
    __shared__ uint32_t sr[4];
    const uint32_t c = blockIdx.x;
    unsigned long long bk = ~0ull;
    uint32_t br = ~0u;
    for (uint32_t w = threadIdx.x; w < W; w += 256) {
        const unsigned long long k = pkey[(uint64_t)w * L + c];
        const uint32_t r = prow[(uint64_t)w * L + c];
        if (k < bk || (k == bk && r < br)) {
            bk = k;
            br = r;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long k = __shfl_xor(bk, off, 64);
        const uint32_t r = (uint32_t)__shfl_xor((int)br, off, 64);
        if (k < bk || (k == bk && r < br)) {
            bk = k;
            br = r;
        }
    }
    if ((threadIdx.x & 63) == 0) {
        sk[threadIdx.x >> 6] = bk;
        sr[threadIdx.x >> 6] = br;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int q = 1; q < 4; q++)
            if (sk[q] < bk || (sk[q] == bk && sr[q] < br)) {
                bk = sk[q];
                br = sr[q];
            }
        if (bk != ~0ull) {
            s_key[c] = bk;
            s_row[c] = row0 + br;
        }
    }
}

// ============================================================================
// device: grid fill / reduce (Aggregator::reduce)
// ============================================================================
template <typename T> __global__ void k_fill(T *p, uint64_t n, T value) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = value;
}

template <typename G> __global__ void k_reduce_add(G *dst, const G *src, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = dst[i] + src[i];
}

// std::max(this, other) / std::min(this, other) (superagg.cpp:209,256)
template <typename T> __global__ void k_reduce_minmax(T *dst, const T *src, uint64_t n, int is_max) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        T a = dst[i], b = src[i];
        dst[i] = is_max ? ((a < b) ? b : a) : ((b < a) ? b : a);
    }
}

template <typename T>
__global__ void k_reduce_first(T *dst, T *dst2, const T *src, const T *src2, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        if (src2[i] < dst2[i]) {
            dst[i] = src[i];
            dst2[i] = src2[i];
        }
    }
}

// ============================================================================
// device: fused count/sum path (global atomics or LDS-privatised grid)
// ============================================================================
template <bool USE_LDS, int ND>
__global__ __launch_bounds__(256) void k_fused(BinPlan p, FusedAggs fa, uint64_t n, uint64_t cells) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    if constexpr (USE_LDS) {
        // zero the per-workgroup sub-grids
        uint32_t *w = reinterpret_cast<uint32_t *>(lds_raw);
        for (uint32_t i = threadIdx.x; i < fa.lds_words; i += blockDim.x) w[i] = 0;
        __syncthreads();
    }
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t c;
        if constexpr (ND == 0) {
            c = plan_index(p, i);
        } else {
            c = 0;
#pragma unroll
            for (int d = 0; d < ND; d++) c += scalar_index<double>(p.b[d], i) * p.b[d].stride;
        }
        #pragma unroll
        for (int k = 0; k < MAX_FUSED_AGGS; k++) {
            if (k >= fa.na) break;
            const FusedAgg &a = fa.a[k];
            if (a.mask && a.mask[i] != 1) continue;
            if (a.kind == VH_AGG_COUNT) {
                if (a.data && is_nan_v(a.data[i])) continue;
                if constexpr (USE_LDS)
                    atomicAdd(reinterpret_cast<uint32_t *>(lds_raw + a.lds_off) + c, 1u);
                else
                    atomicAdd((unsigned long long *)a.grid + c, 1ULL);
            } else {
                double v = a.data[i];
                if (v != v) continue;
                if constexpr (USE_LDS)
                    atomicAdd(reinterpret_cast<double *>(lds_raw + a.lds_off) + c, v);
                else
                    atomicAdd(reinterpret_cast<double *>(a.grid) + c, v);
            }
        }
    }
    if constexpr (USE_LDS) {
        __syncthreads();
        #pragma unroll
        for (int k = 0; k < MAX_FUSED_AGGS; k++) {
            if (k >= fa.na) break;
            const FusedAgg &a = fa.a[k];
            for (uint64_t c = threadIdx.x; c < cells; c += blockDim.x) {
                if (a.kind == VH_AGG_COUNT) {
                    uint32_t v = reinterpret_cast<const uint32_t *>(lds_raw + a.lds_off)[c];
                    if (v) atomicAdd((unsigned long long *)a.grid + c, (unsigned long long)v);
                } else {
                    double v = reinterpret_cast<const double *>(lds_raw + a.lds_off)[c];
                    if (v != 0.0) atomicAdd(reinterpret_cast<double *>(a.grid) + c, v);
                }
            }
        }
    }
}


// ============================================================================
// device: small grids of float64 scalar binners with count / float64-sum aggregators
// (C1: df.count(binby='x', shape=256), agg.hpp:106-136 over a grid that fits LDS).  Each
// lane takes two rows per 16-B load of every column (SG_U loads in flight), bins them with
// the reference's scalar math, adds into the workgroup's LDS sub-grids, and the workgroup
// writes its sub-grids out as partials (plain stores): with a few hundred cells every
// workgroup touches every hot cell, and one global atomic per (workgroup, cell) serialised
// on those cells cost more than the scan.  k_small_f64_fin folds the partials, CHUNK
// workgroups per lane, with one atomic per (chunk, cell).
// ============================================================================
constexpr int SG_U = 4;
constexpr unsigned SG_FIN_CHUNK = 64;
struct SmallF64 {
    int32_t na, ncol;
    uint32_t lds_words, pad;
    const double2 *col[MAX_FUSED_AGGS];  // distinct aggregator data columns (16-B aligned)
    int8_t acol[MAX_FUSED_AGGS], akind[MAX_FUSED_AGGS];
    uint32_t lds_off[MAX_FUSED_AGGS];    // byte offset of each aggregator's sub-grid
    void *grid[MAX_FUSED_AGGS];
};

template <int ND, int NC>
__device__ inline void sg_row(const BinPlan &p, const SmallF64 &s, unsigned char *lds, const double *bx,
                              const double *ax) {
    uint32_t c = 0;
#pragma unroll
    for (int d = 0; d < ND; d++) c += (uint32_t)scalar_cell<double>(p.b[d], bx[d], false) * (uint32_t)p.b[d].stride;
#pragma unroll
    for (int k = 0; k < MAX_FUSED_AGGS; k++) {
        if (k >= s.na) break;
        double v = 0.0;  // count(*) reads nothing (selected by compare: no indexed registers)
#pragma unroll
        for (int q = 0; q < NC; q++)
            if (q == s.acol[k]) v = ax[q];
        if (v != v) continue;  // count(expr) skips NaN, sum skips NaN
        if (s.akind[k] == VH_AGG_COUNT)
            atomicAdd(reinterpret_cast<uint32_t *>(lds + s.lds_off[k]) + c, 1u);
        else
            atomicAdd(reinterpret_cast<double *>(lds + s.lds_off[k]) + c, v);
    }
}

// BT = float: float32 binner columns (8-byte row pairs), each value widened to double before
// the scalar index math -- BinnerScalar<float>::to_bins scales the value as double
// (superagg_binners.cpp:14-56); aggregator columns stay float64 (the fusable kinds)
template <int ND, int NC, typename BT = double>
__global__ __launch_bounds__(256) void k_small_f64(BinPlan p, SmallF64 s, uint64_t n, uint32_t *part) {
    using B2 = std::conditional_t<std::is_same_v<BT, float>, float2, double2>;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    uint32_t *w = reinterpret_cast<uint32_t *>(lds_raw);
    for (uint32_t i = threadIdx.x; i < s.lds_words; i += blockDim.x) w[i] = 0;
    __syncthreads();
    const uint64_t nvec = n / 2, stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t v = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (; v + (SG_U - 1) * stride < nvec; v += SG_U * stride) {
        B2 b[ND][SG_U];
        double2 a[NC > 0 ? NC : 1][SG_U];
#pragma unroll
        for (int d = 0; d < ND; d++)
#pragma unroll
            for (int u = 0; u < SG_U; u++) b[d][u] = reinterpret_cast<const B2 *>(p.b[d].data)[v + u * stride];
#pragma unroll
        for (int q = 0; q < NC; q++)
#pragma unroll
            for (int u = 0; u < SG_U; u++) a[q][u] = s.col[q][v + u * stride];
#pragma unroll
        for (int u = 0; u < SG_U; u++) {
            double bx[ND], ax[NC > 0 ? NC : 1];
#pragma unroll
            for (int d = 0; d < ND; d++) bx[d] = (double)b[d][u].x;
#pragma unroll
            for (int q = 0; q < NC; q++) ax[q] = a[q][u].x;
            sg_row<ND, NC>(p, s, lds_raw, bx, ax);
#pragma unroll
            for (int d = 0; d < ND; d++) bx[d] = (double)b[d][u].y;
#pragma unroll
            for (int q = 0; q < NC; q++) ax[q] = a[q][u].y;
            sg_row<ND, NC>(p, s, lds_raw, bx, ax);
        }
    }
    // the rest of the pairs one at a time, then the odd last row (block 0, lane 0)
    for (; v < nvec; v += stride) {
        B2 b2[ND];
        double2 a2[NC > 0 ? NC : 1];
        double bx[ND], ax[NC > 0 ? NC : 1];
#pragma unroll
        for (int d = 0; d < ND; d++) b2[d] = reinterpret_cast<const B2 *>(p.b[d].data)[v];
#pragma unroll
        for (int q = 0; q < NC; q++) a2[q] = s.col[q][v];
#pragma unroll
        for (int d = 0; d < ND; d++) bx[d] = (double)b2[d].x;
#pragma unroll
        for (int q = 0; q < NC; q++) ax[q] = a2[q].x;
        sg_row<ND, NC>(p, s, lds_raw, bx, ax);
#pragma unroll
        for (int d = 0; d < ND; d++) bx[d] = (double)b2[d].y;
#pragma unroll
        for (int q = 0; q < NC; q++) ax[q] = a2[q].y;
        sg_row<ND, NC>(p, s, lds_raw, bx, ax);
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
        double bx[ND], ax[NC > 0 ? NC : 1];
#pragma unroll
        for (int d = 0; d < ND; d++) bx[d] = (double)reinterpret_cast<const BT *>(p.b[d].data)[n - 1];
#pragma unroll
        for (int q = 0; q < NC; q++) ax[q] = reinterpret_cast<const double *>(s.col[q])[n - 1];
        sg_row<ND, NC>(p, s, lds_raw, bx, ax);
    }
    __syncthreads();
    uint32_t *dst = part + (uint64_t)blockIdx.x * s.lds_words;
    for (uint32_t i = threadIdx.x; i < s.lds_words; i += blockDim.x) dst[i] = w[i];
}

// grid (cells / 256, chunks of SG_FIN_CHUNK workgroups, aggregators): fold partials in order
__global__ __launch_bounds__(256) void k_small_f64_fin(SmallF64 s, const uint32_t *part, unsigned nb, uint64_t L) {
    const uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const int k = blockIdx.z;
    if (c >= L) return;
    const unsigned b0 = blockIdx.y * SG_FIN_CHUNK, b1 = min(nb, b0 + SG_FIN_CHUNK);
    if (s.akind[k] == VH_AGG_COUNT) {
        uint64_t t = 0;
        for (unsigned b = b0; b < b1; b++) t += part[(uint64_t)b * s.lds_words + s.lds_off[k] / 4 + c];
        if (t) atomicAdd(reinterpret_cast<unsigned long long *>(s.grid[k]) + c, (unsigned long long)t);
    } else {
        double t = 0.0;
        for (unsigned b = b0; b < b1; b++)
            t += reinterpret_cast<const double *>(part + (uint64_t)b * s.lds_words + s.lds_off[k] / 4)[c];
        if (t != 0.0) atomicAdd(reinterpret_cast<double *>(s.grid[k]) + c, t);
    }
}

// ============================================================================
// device: 0-d aggregation -- no binners (df.count() / df.sum('w') / df.mean('w'); the
// reference's Grid::bin with a length and no binners, agg.hpp:76-105, puts every row in
// cell 0), so the grid is a reduction: 16-B loads of each distinct float64 column
// (R0_U in flight per lane), per-lane accumulators, a wave reduction with cross-lane
// shuffles, per-workgroup partials, and a one-workgroup finisher that folds the partials in
// a fixed order (run-to-run identical sums) into the grid cell.
// ============================================================================
constexpr int R0_U = 4;
struct Reduce0 {
    int32_t na, ncol, nmask, all_rows;  // all_rows: bit k = count(*) of every row (no read)
    const double2 *col[MAX_FUSED_AGGS];    // distinct float64 data columns (16-B aligned)
    const uint16_t *mask[MAX_FUSED_AGGS];  // distinct aggregator masks, 1 = keep (2-B aligned)
    int8_t acol[MAX_FUSED_AGGS], amask[MAX_FUSED_AGGS], akind[MAX_FUSED_AGGS], pad[4];
    void *grid[MAX_FUSED_AGGS];
};

__device__ inline double wave_sum_f64(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
__device__ inline uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// rows 2v, 2v+1 of every aggregator: x = its column's pair, m = its mask's pair
template <bool HAS_MASK>
__device__ inline void r0_rows(const Reduce0 &r, int k, double2 x, uint16_t m, double &s, uint64_t &c) {
    bool k0 = true, k1 = true;
    if constexpr (HAS_MASK) {
        k0 = (m & 0xff) == 1;
        k1 = (m >> 8) == 1;
    }
    if (r.acol[k] >= 0) {
        k0 = k0 && x.x == x.x;
        k1 = k1 && x.y == x.y;
    }
    c += (uint64_t)k0 + (uint64_t)k1;
    if (r.akind[k] == VH_AGG_SUM) s += (k0 ? x.x : 0.0) + (k1 ? x.y : 0.0);
}

template <bool HAS_MASK>
__global__ __launch_bounds__(256) void k_reduce0(Reduce0 r, uint64_t n, double *psum, uint64_t *pcnt) {
    double s[MAX_FUSED_AGGS];
    uint64_t c[MAX_FUSED_AGGS];
#pragma unroll
    for (int k = 0; k < MAX_FUSED_AGGS; k++) {
        s[k] = 0.0;
        c[k] = 0;
    }
    const uint64_t nvec = n / 2, stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t v = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (; v + (R0_U - 1) * stride < nvec; v += R0_U * stride) {
        double2 x[MAX_FUSED_AGGS][R0_U];
        uint16_t m[MAX_FUSED_AGGS][R0_U];
#pragma unroll
        for (int q = 0; q < MAX_FUSED_AGGS; q++) {
            if (q >= r.ncol) break;
#pragma unroll
            for (int u = 0; u < R0_U; u++) x[q][u] = r.col[q][v + u * stride];
        }
        if constexpr (HAS_MASK) {
#pragma unroll
            for (int q = 0; q < MAX_FUSED_AGGS; q++) {
                if (q >= r.nmask) break;
#pragma unroll
                for (int u = 0; u < R0_U; u++) m[q][u] = r.mask[q][v + u * stride];
            }
        }
#pragma unroll
        for (int k = 0; k < MAX_FUSED_AGGS; k++) {
            if (k >= r.na) break;
#pragma unroll
            for (int u = 0; u < R0_U; u++) {
                double2 xv = make_double2(0.0, 0.0);
                uint16_t mv = 0x0101;
#pragma unroll
                for (int q = 0; q < MAX_FUSED_AGGS; q++) {
                    if (q == r.acol[k]) xv = x[q][u];
                    if constexpr (HAS_MASK)
                        if (q == r.amask[k]) mv = m[q][u];
                }
                r0_rows<HAS_MASK>(r, k, xv, mv, s[k], c[k]);
            }
        }
    }
    for (; v < nvec; v += stride) {
#pragma unroll
        for (int k = 0; k < MAX_FUSED_AGGS; k++) {
            if (k >= r.na) break;
            const double2 xv = r.acol[k] >= 0 ? r.col[r.acol[k]][v] : make_double2(0.0, 0.0);
            const uint16_t mv = HAS_MASK && r.amask[k] >= 0 ? r.mask[r.amask[k]][v] : (uint16_t)0x0101;
            r0_rows<HAS_MASK>(r, k, xv, mv, s[k], c[k]);
        }
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {  // the odd last row
#pragma unroll
        for (int k = 0; k < MAX_FUSED_AGGS; k++) {
            if (k >= r.na) break;
            bool keep = true;
            double xv = 0.0;
            if (HAS_MASK && r.amask[k] >= 0) keep = reinterpret_cast<const uint8_t *>(r.mask[r.amask[k]])[n - 1] == 1;
            if (r.acol[k] >= 0) {
                xv = reinterpret_cast<const double *>(r.col[r.acol[k]])[n - 1];
                keep = keep && xv == xv;
            }
            c[k] += keep ? 1 : 0;
            if (r.akind[k] == VH_AGG_SUM && keep) s[k] += xv;
        }
    }
    __shared__ double ss[4][MAX_FUSED_AGGS];
    __shared__ uint64_t sc[4][MAX_FUSED_AGGS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < MAX_FUSED_AGGS; k++) {
        if (k >= r.na) break;
        const double ws = wave_sum_f64(s[k]);
        const uint64_t wc = wave_sum_u64(c[k]);
        if (lane == 0) {
            ss[wave][k] = ws;
            sc[wave][k] = wc;
        }
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)r.na) {
        const int k = threadIdx.x;
        psum[(uint64_t)blockIdx.x * MAX_FUSED_AGGS + k] = (ss[0][k] + ss[1][k]) + (ss[2][k] + ss[3][k]);
        pcnt[(uint64_t)blockIdx.x * MAX_FUSED_AGGS + k] = sc[0][k] + sc[1][k] + sc[2][k] + sc[3][k];
    }
}

// fold `nb` workgroup partials in a fixed order and add them to the grid cells
__global__ __launch_bounds__(256) void k_reduce0_fin(Reduce0 r, const double *psum, const uint64_t *pcnt, unsigned nb,
                                                      uint64_t n) {
    __shared__ double ss[4][MAX_FUSED_AGGS];
    __shared__ uint64_t sc[4][MAX_FUSED_AGGS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < MAX_FUSED_AGGS; k++) {
        if (k >= r.na) break;
        double s = 0.0;
        uint64_t c = 0;
        for (unsigned b = threadIdx.x; b < nb; b += blockDim.x) {
            s += psum[(uint64_t)b * MAX_FUSED_AGGS + k];
            c += pcnt[(uint64_t)b * MAX_FUSED_AGGS + k];
        }
        s = wave_sum_f64(s);
        c = wave_sum_u64(c);
        if (lane == 0) {
            ss[wave][k] = s;
            sc[wave][k] = c;
        }
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)r.na) {
        const int k = threadIdx.x;
        if (r.akind[k] == VH_AGG_COUNT) {
            const uint64_t c = ((r.all_rows >> k) & 1) ? n : sc[0][k] + sc[1][k] + sc[2][k] + sc[3][k];
            reinterpret_cast<int64_t *>(r.grid[k])[0] += (int64_t)c;
        } else {
            reinterpret_cast<double *>(r.grid[k])[0] += (ss[0][k] + ss[1][k]) + (ss[2][k] + ss[3][k]);
        }
    }
}
}  // namespace vh

// ============================================================================
// host helpers
// ============================================================================
namespace {

void check_column(const ColumnRef &c, uint64_t length, const char *what) {
    if (!c.set) fail(VH_ERR_RUNTIME, std::string(what) + " not set");
    if (c.size < length)
        fail(VH_ERR_RUNTIME, std::string(what) + " has " + std::to_string(c.size) + " rows, bin() asked for " +
                                 std::to_string(length));
}

ColumnRef make_col(const void *ptr, uint64_t length, int itemsize, int loc) {
    ColumnRef c;
    c.ptr = ptr;
    c.size = length;
    c.itemsize = itemsize;
    c.loc = resolve_loc(ptr, loc);
    c.set = true;
    return c;
}

template <typename T> void fill_grid(void *p, uint64_t n, T v) {
    if (!n) return;
    hipLaunchKernelGGL(k_fill<T>, dim3(blocks_for(n, 256)), dim3(256), 0, stream(), (T *)p, n, v);
    VH_HIP(hipGetLastError());
}

template <typename T> T minmax_fill(bool mx) {
    if constexpr (std::is_same<T, vbool>::value) {
        T v;
        v.v = mx ? 0 : 1;
        return v;
    } else if constexpr (is_float_t<T>::value) {
        return mx ? -std::numeric_limits<T>::infinity() : std::numeric_limits<T>::infinity();
    } else {
        return mx ? std::numeric_limits<T>::min() : std::numeric_limits<T>::max();
    }
}

template <typename T> T max_fill() {
    if constexpr (std::is_same<T, vbool>::value) {
        T v;
        v.v = 1;
        return v;
    } else {
        return std::numeric_limits<T>::max();
    }
}

void init_agg_grid(vh_agg *a) {
    const uint64_t L = a->grid->length1d;
    VH_HIP(hipMemsetAsync(a->g.ptr, 0, L * a->grid_isz, stream()));
    if (a->kind == VH_AGG_MIN || a->kind == VH_AGG_MAX) {
        // numeric_limits fill (superagg.cpp:199-204, 246-251)
        const bool mx = a->kind == VH_AGG_MAX;
        VH_DISPATCH_DTYPE(a->dtype, T, fill_grid<T>(a->g.ptr, L, minmax_fill<T>(mx)));
    } else if (a->kind == VH_AGG_FIRST) {
        // order grid = numeric_limits<T>::max() (superagg.cpp:441-445), data grid 0
        VH_DISPATCH_DTYPE(a->dtype, T, fill_grid<T>(a->g2.ptr, L, max_fill<T>()));
        VH_HIP(hipMemsetAsync(a->s_key.ptr, 0xff, L * 8, stream()));
        VH_HIP(hipMemsetAsync(a->s_row.ptr, 0xff, L * 8, stream()));
    }
    // no host wait: every later use of the grid is ordered after the fills on the library
    // stream, and every host read (download, device_ptr users) synchronises the stream
}

// chunk-relative device pointer of a column: HBM columns in place, host columns from the
// pipeline buffer the chunk was staged into
struct Stager {
    Workspace &ws;
    uint64_t row0 = 0, len = 0;
    int buf = 0;
    const void *get(const ColumnRef &c) {
        if (!c.set) return nullptr;
        const char *base = reinterpret_cast<const char *>(c.ptr) + row0 * c.itemsize;
        if (c.loc == VH_LOC_DEVICE) return base;
        const int i = ws.pipe.find(c.ptr);
        if (i < 0) fail(VH_ERR_RUNTIME, "internal: host column not staged");
        return ws.pipe.dev[buf].as<char>() + ws.pipe.off[i];
    }
};

}  // namespace

namespace vh {
Workspace::~Workspace() = default;

HostPipe::~HostPipe() {
    for (int b = 0; b < 2; b++) {
        if (copied[b]) {
            (void)hipEventSynchronize(copied[b]);
            release_registered(b);
            (void)hipEventDestroy(copied[b]);
        }
        if (consumed[b]) (void)hipEventDestroy(consumed[b]);
    }
}

void HostPipe::release_registered(int b) {
    for (void *p : registered[b]) (void)hipHostUnregister(p);
    registered[b].clear();
}

// How chunks of host columns outside a vh_host_register range reach the DMA engine
// (VH_HOST_PIPE, read per chunk so a caller may switch it):
//   0 (default) host threads copy the chunk into the pinned bounce buffer, DMA from there
//   1 page-aligned chunks >= 1 MiB are registered for the copy and DMA'd in place
//   2 the runtime's own pageable copy path
static int host_pipe_mode() {
    const char *e = getenv("VH_HOST_PIPE");
    return e ? atoi(e) : 0;
}

void HostPipe::add(const ColumnRef &c) {
    if (!c.set || c.loc != VH_LOC_HOST || find(c.ptr) >= 0) return;
    cols.push_back(c.ptr);
    isz.push_back(c.itemsize);
}

int HostPipe::find(const void *ptr) const {
    for (size_t i = 0; i < cols.size(); i++)
        if (cols[i] == ptr) return (int)i;
    return -1;
}

void HostPipe::plan(uint64_t chunk_rows) {
    chunk = chunk_rows;
    off.assign(cols.size(), 0);
    uint64_t o = 0;
    for (size_t i = 0; i < cols.size(); i++) {
        off[i] = o;
        o = (o + chunk_rows * isz[i] + 255) & ~uint64_t(255);
    }
    bytes = o;
    for (int b = 0; b < 2; b++) {
        // the previous bin() call's copies and kernels are done (run_bin syncs at its end)
        pending_copy[b] = pending_use[b] = false;
        release_registered(b);
        dev[b].ensure(bytes);  // the pinned bounce buffer is taken when a chunk needs it
        if (!copied[b]) VH_HIP(hipEventCreateWithFlags(&copied[b], hipEventDisableTiming));
        if (!consumed[b]) VH_HIP(hipEventCreateWithFlags(&consumed[b], hipEventDisableTiming));
    }
}

void HostPipe::issue(uint64_t ci, uint64_t row0, uint64_t len) {
    static const int threads = [] {
        const char *e = getenv("VH_COPY_THREADS");
        return e ? std::max(1, atoi(e)) : 16;
    }();
    const int b = (int)(ci & 1);
    hipStream_t cs = copy_stream();
    if (pending_copy[b]) {
        VH_HIP(hipEventSynchronize(copied[b]));  // bounce buffer b drained
        release_registered(b);
    }
    // the DMA source of each column: its registered pages, or the pinned bounce buffer
    std::vector<const char *> src(cols.size());
    const uint64_t page = 4096;
    for (size_t i = 0; i < cols.size(); i++) {
        const char *p = reinterpret_cast<const char *>(cols[i]) + row0 * isz[i];
        const uint64_t bytes = len * isz[i];
        src[i] = nullptr;
        const int mode = host_pipe_mode();
        if (host_registered(p, bytes) || mode == 2) {
            src[i] = p;
        } else if (mode == 1 && (reinterpret_cast<uintptr_t>(p) % page) == 0 && bytes >= (1u << 20)) {
            const uint64_t rb = (bytes + page - 1) / page * page;
            hipError_t e = hipHostRegister(const_cast<char *>(p), rb, hipHostRegisterReadOnly);
            if (e == hipSuccess) {
                registered[b].push_back(const_cast<char *>(p));
                src[i] = p;
            } else {
                (void)hipGetLastError();
            }
        }
        if (!src[i]) {
            pinned[b].ensure(this->bytes);
            parallel_memcpy(pinned[b].as<char>() + off[i], p, bytes, threads);
            src[i] = pinned[b].as<char>() + off[i];
        }
    }
    if (pending_use[b]) VH_HIP(hipStreamWaitEvent(cs, consumed[b], 0));  // chunk ci-2 binned
    for (size_t i = 0; i < cols.size(); i++)
        VH_HIP(hipMemcpyAsync(dev[b].as<char>() + off[i], src[i], len * isz[i], hipMemcpyHostToDevice, cs));
    VH_HIP(hipEventRecord(copied[b], cs));
    pending_copy[b] = true;
}

void HostPipe::wait_copied(int b) { VH_HIP(hipStreamWaitEvent(stream(), copied[b], 0)); }

void HostPipe::mark_consumed(int b) {
    VH_HIP(hipEventRecord(consumed[b], stream()));
    pending_use[b] = true;
}
}  // namespace vh

// ============================================================================
// C ABI
// ============================================================================
namespace {
// nonzero cells of grid words [begin, end): count, first and last index (+1) -- the occupied
// range of a dense groupby's count(*) grid (groupby.py:484-533 keeps the cells with count > 0)
template <typename W>
__global__ __launch_bounds__(256) void k_occupancy(const W *g, uint64_t begin, uint64_t end, unsigned long long *part) {
    unsigned long long nnz = 0, first = ~0ull, last = 0;
    for (uint64_t i = begin + blockIdx.x * 256ull + threadIdx.x; i < end; i += (uint64_t)gridDim.x * 256) {
        if (g[i] != 0) {
            nnz++;
            first = first < i - begin ? first : i - begin;
            last = i - begin + 1;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        nnz += __shfl_down(nnz, off, 64);
        const unsigned long long f = __shfl_down(first, off, 64), l = __shfl_down(last, off, 64);
        first = f < first ? f : first;
        last = l > last ? l : last;
    }
    // one partial per workgroup (no atomics: nothing to initialise, k_occupancy_fin reduces)
    __shared__ unsigned long long s_n[4], s_f[4], s_l[4];
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_n[wv] = nnz;
        s_f[wv] = first;
        s_l[wv] = last;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 4; k++) {
            nnz += s_n[k];
            first = s_f[k] < first ? s_f[k] : first;
            last = s_l[k] > last ? s_l[k] : last;
        }
        part[3 * blockIdx.x] = nnz;
        part[3 * blockIdx.x + 1] = first;
        part[3 * blockIdx.x + 2] = last;
    }
}

// the workgroup partials (at most 256) into the caller's page-locked result, written through
// its device mapping (read on the host after a stream sync: no copy calls)
__global__ __launch_bounds__(256) void k_occupancy_fin(const unsigned long long *part, uint32_t nb, unsigned long long *out) {
    unsigned long long nnz = 0, first = ~0ull, last = 0;
    if (threadIdx.x < nb) {
        nnz = part[3 * threadIdx.x];
        first = part[3 * threadIdx.x + 1];
        last = part[3 * threadIdx.x + 2];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        nnz += __shfl_down(nnz, off, 64);
        const unsigned long long f = __shfl_down(first, off, 64), l = __shfl_down(last, off, 64);
        first = f < first ? f : first;
        last = l > last ? l : last;
    }
    __shared__ unsigned long long s_n[4], s_f[4], s_l[4];
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_n[wv] = nnz;
        s_f[wv] = first;
        s_l[wv] = last;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 4; k++) {
            nnz += s_n[k];
            first = s_f[k] < first ? s_f[k] : first;
            last = s_l[k] > last ? s_l[k] : last;
        }
        out[0] = nnz;
        out[1] = first;
        out[2] = last;
    }
}

}  // namespace

extern "C" {

int vh_binner_scalar_create(const char *expression, int dtype, int flip, double vmin, double vmax,
                            uint64_t bins, vh_binner **out) {
    VH_API_BEGIN
    dtype_itemsize(dtype);
    auto *b = new vh_binner();
    b->kind = 0;
    b->expression = expression ? expression : "";
    b->dtype = dtype;
    b->flip = flip ? 1 : 0;
    b->vmin = vmin;
    b->vmax = vmax;
    b->bins = bins;
    *out = b;
    VH_API_END
}

int vh_binner_ordinal_create(const char *expression, int dtype, int flip, uint64_t ordinal_count,
                             uint64_t min_value, vh_binner **out) {
    VH_API_BEGIN
    dtype_itemsize(dtype);
    auto *b = new vh_binner();
    b->kind = 1;
    b->expression = expression ? expression : "";
    b->dtype = dtype;
    b->flip = flip ? 1 : 0;
    b->ordinal_count = ordinal_count;
    b->min_value = min_value;
    *out = b;
    VH_API_END
}

int vh_binner_set_ordinal_create(const char *expression, vh_set *set, uint64_t ordinal_count,
                                 vh_binner **out) {
    VH_API_BEGIN
    if (!set) fail(VH_ERR_ARG, "set is NULL");
    auto *b = new vh_binner();
    b->kind = 2;
    b->expression = expression ? expression : "";
    b->dtype = set_dtype(set);
    b->set = set;
    b->ordinal_count = ordinal_count;
    *out = b;
    VH_API_END
}

int vh_binner_copy(const vh_binner *binner, vh_binner **out) {
    VH_API_BEGIN
    *out = new vh_binner(*binner);
    VH_API_END
}

int vh_binner_destroy(vh_binner *binner) {
    VH_API_BEGIN
    delete binner;
    VH_API_END
}

int vh_binner_set_data(vh_binner *b, const void *ptr, uint64_t length, int itemsize, int ndim, int loc) {
    VH_API_BEGIN
    if (ndim != 1) fail(VH_ERR_RUNTIME, "Expected a 1d array");
    if (itemsize != dtype_itemsize(b->dtype)) fail(VH_ERR_RUNTIME, "Itemsize of data and binner are not equal");
    b->data = make_col(ptr, length, itemsize, loc);
    VH_API_END
}

int vh_binner_set_data_mask(vh_binner *b, const uint8_t *mask, uint64_t length, int ndim, int loc) {
    VH_API_BEGIN
    if (ndim != 1) fail(VH_ERR_RUNTIME, "Expected a 1d array");
    b->mask = make_col(mask, length, 1, loc);
    VH_API_END
}

int vh_binner_clear_data_mask(vh_binner *b) {
    VH_API_BEGIN
    b->mask = ColumnRef();
    VH_API_END
}

int vh_binner_shape(const vh_binner *b, uint64_t *shape) {
    VH_API_BEGIN
    *shape = b->shape();
    VH_API_END
}

int vh_binner_size(const vh_binner *b, uint64_t *size) {
    VH_API_BEGIN
    *size = b->data.set ? b->data.size : 0;
    VH_API_END
}

int vh_grid_create(vh_binner *const *binners, int nbinners, vh_grid **out) {
    VH_API_BEGIN
    if (nbinners < 0 || nbinners > MAX_DIM) fail(VH_ERR_ARG, "at most 16 binners (agg.hpp:25)");
    auto *g = new vh_grid();
    g->length1d = 1;
    for (int i = 0; i < nbinners; i++) {
        g->binners.push_back(binners[i]);
        g->shapes.push_back(binners[i]->shape());
        g->length1d *= binners[i]->shape();
    }
    g->strides.resize(nbinners);
    if (nbinners > 0) {
        g->strides[0] = 1;  // agg.hpp:64-69, first binner varies fastest
        for (int i = 1; i < nbinners; i++) g->strides[i] = g->strides[i - 1] * g->shapes[i - 1];
    }
    *out = g;
    VH_API_END
}

int vh_grid_destroy(vh_grid *g) {
    VH_API_BEGIN
    if (g) (void)hipStreamSynchronize(stream());
    delete g;
    VH_API_END
}

int vh_grid_info(const vh_grid *g, int *dims, uint64_t *shapes, uint64_t *strides, uint64_t *length1d) {
    VH_API_BEGIN
    if (dims) *dims = (int)g->binners.size();
    for (size_t i = 0; i < g->binners.size(); i++) {
        if (shapes) shapes[i] = g->shapes[i];
        if (strides) strides[i] = g->strides[i];
    }
    if (length1d) *length1d = g->length1d;
    VH_API_END
}

int vh_agg_create(vh_grid *grid, int kind, int dtype, int flip, uint32_t arg, vh_agg **out) {
    VH_API_BEGIN
    if (kind < VH_AGG_COUNT || kind > VH_AGG_NUNIQUE) fail(VH_ERR_ARG, "unknown aggregator kind");
    dtype_itemsize(dtype);
    std::unique_ptr<vh_agg> a(new vh_agg());
    a->grid = grid;
    a->L = grid->length1d;
    a->kind = kind;
    a->dtype = dtype;
    a->flip = flip ? 1 : 0;
    a->moment = arg;
    switch (kind) {
    case VH_AGG_COUNT: case VH_AGG_NUNIQUE: a->grid_dtype = VH_I64; break;
    case VH_AGG_SUM: case VH_AGG_SUM_MOMENT: a->grid_dtype = upcast_dtype(dtype); break;
    default: a->grid_dtype = dtype;
    }
    a->grid_isz = dtype_itemsize(a->grid_dtype);
    const uint64_t L = grid->length1d;
    a->g.ensure(L * a->grid_isz);
    if (kind == VH_AGG_FIRST) {
        a->g2.ensure(L * a->grid_isz);
        a->s_key.ensure(L * 8);
        a->s_row.ensure(L * 8);
    }
    if (kind == VH_AGG_NUNIQUE) nunique_init(a.get());
    else init_agg_grid(a.get());
    *out = a.release();
    VH_API_END
}

int vh_agg_destroy(vh_agg *a) {
    VH_API_BEGIN
    if (a) (void)hipStreamSynchronize(stream());
    delete a;
    VH_API_END
}

int vh_agg_set_data(vh_agg *a, const void *ptr, uint64_t length, int itemsize, int ndim, int index, int loc) {
    VH_API_BEGIN
    if (ndim != 1) fail(VH_ERR_RUNTIME, "Expected a 1d array");
    if (itemsize != dtype_itemsize(a->dtype))
        fail(VH_ERR_RUNTIME, "Itemsize of data and aggregator are not equal");
    if (a->kind == VH_AGG_FIRST && index == 1) a->data2 = make_col(ptr, length, itemsize, loc);
    else a->data = make_col(ptr, length, itemsize, loc);
    VH_API_END
}

int vh_agg_set_data_mask(vh_agg *a, const uint8_t *mask, uint64_t length, int ndim, int loc) {
    VH_API_BEGIN
    if (ndim != 1) fail(VH_ERR_RUNTIME, "Expected a 1d array");
    a->mask = make_col(mask, length, 1, loc);
    VH_API_END
}

int vh_agg_clear_data_mask(vh_agg *a) {
    VH_API_BEGIN
    a->mask = ColumnRef();
    VH_API_END
}

int vh_agg_set_selection_mask(vh_agg *a, const uint8_t *mask, uint64_t length, int ndim, int loc) {
    VH_API_BEGIN
    (void)length;
    (void)loc;
    if (ndim != 1) fail(VH_ERR_RUNTIME, "Expected a 1d array");
    // as agg_hash_primitive.cpp:46-47 only its presence matters: rows whose data mask is 0
    // are then outside the selection (not missing)
    a->has_selection = mask != nullptr;
    VH_API_END
}

int vh_agg_info(const vh_agg *a, uint64_t *bytes, int *grid_dtype, uint64_t *itemsize) {
    VH_API_BEGIN
    if (bytes) *bytes = a->grid->length1d * a->grid_isz;
    if (grid_dtype) *grid_dtype = a->grid_dtype;
    if (itemsize) *itemsize = a->grid_isz;
    VH_API_END
}

int vh_agg_download(vh_agg *a, void *host, uint64_t bytes) {
    VH_API_BEGIN
    std::lock_guard<std::mutex> lk(a->grid->mu);
    if (bytes != a->grid->length1d * a->grid_isz) fail(VH_ERR_ARG, "download size mismatch");
    nunique_finalize(a);
    if (bytes <= (1u << 20)) {
        // small grids through a page-locked block: a pageable read-back is a staged copy
        thread_local PinnedBuf small;
        small.ensure(1u << 20);
        VH_HIP(hipMemcpyAsync(small.ptr, a->g.ptr, bytes, hipMemcpyDeviceToHost, stream()));
        VH_HIP(hipStreamSynchronize(stream()));
        memcpy(host, small.ptr, bytes);
    } else {
        copy_to_host(host, a->g.ptr, bytes, stream());
        VH_HIP(hipStreamSynchronize(stream()));
    }
    VH_API_END
}

int vh_agg_occupancy(vh_agg *a, uint64_t begin, uint64_t end, int64_t *out3) {
    VH_API_BEGIN
    std::lock_guard<std::mutex> lk(a->grid->mu);
    if (begin > end || end > a->grid->length1d) fail(VH_ERR_ARG, "occupancy range outside the grid");
    nunique_finalize(a);
    // per-device workgroup partials (a grid lives for one query: a buffer of its own would be
    // allocated per query) and a per-thread page-locked result the final kernel writes
    static std::mutex occ_mu;
    static std::map<int, std::unique_ptr<DevBuf>> occ_bufs;
    std::lock_guard<std::mutex> olk(occ_mu);
    auto &slot = occ_bufs[current_device()];
    if (!slot) slot = std::make_unique<DevBuf>();
    DevBuf &dpart = *slot;
    thread_local PinnedBuf hres;
    thread_local unsigned long long *hres_dev = nullptr;
    constexpr uint32_t OCC_BLOCKS = 256;
    dpart.ensure((size_t)OCC_BLOCKS * 3 * 8);
    if (!hres.ptr) {
        hres.ensure(64);
        hipPointerAttribute_t at{};
        VH_HIP(hipPointerGetAttributes(&at, hres.ptr));
        if (!at.devicePointer) fail(VH_ERR_HIP, "page-locked result buffer without a device mapping");
        hres_dev = static_cast<unsigned long long *>(at.devicePointer);
    }
    auto *part = dpart.as<unsigned long long>();
    const uint64_t n = end - begin;
    const uint32_t nb = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(blocks_for(n, 256, 1), OCC_BLOCKS));
    const dim3 grd(nb), blk(256);
    switch (a->grid_isz) {
    case 1: hipLaunchKernelGGL(k_occupancy<uint8_t>, grd, blk, 0, stream(), static_cast<const uint8_t *>(a->g.ptr), begin, end, part); break;
    case 2: hipLaunchKernelGGL(k_occupancy<uint16_t>, grd, blk, 0, stream(), static_cast<const uint16_t *>(a->g.ptr), begin, end, part); break;
    case 4: hipLaunchKernelGGL(k_occupancy<uint32_t>, grd, blk, 0, stream(), static_cast<const uint32_t *>(a->g.ptr), begin, end, part); break;
    default: hipLaunchKernelGGL(k_occupancy<uint64_t>, grd, blk, 0, stream(), static_cast<const uint64_t *>(a->g.ptr), begin, end, part);
    }
    hipLaunchKernelGGL(k_occupancy_fin, dim3(1), dim3(256), 0, stream(), part, nb, hres_dev);
    VH_HIP(hipGetLastError());
    VH_HIP(hipStreamSynchronize(stream()));
    const auto *r = reinterpret_cast<const volatile unsigned long long *>(hres.ptr);
    out3[0] = (int64_t)r[0];
    out3[1] = r[0] ? (int64_t)r[1] : -1;
    out3[2] = r[0] ? (int64_t)r[2] - 1 : -1;
    VH_API_END
}

int vh_agg_download_order(vh_agg *a, void *host, uint64_t bytes) {
    VH_API_BEGIN
    std::lock_guard<std::mutex> lk(a->grid->mu);
    if (a->kind != VH_AGG_FIRST) fail(VH_ERR_ARG, "not an AggFirst");
    if (bytes != a->grid->length1d * a->grid_isz) fail(VH_ERR_ARG, "download size mismatch");
    copy_to_host(host, a->g2.ptr, bytes, stream());
    VH_HIP(hipStreamSynchronize(stream()));
    VH_API_END
}

int vh_agg_upload_order(vh_agg *a, const void *host, uint64_t bytes) {
    VH_API_BEGIN
    std::lock_guard<std::mutex> lk(a->grid->mu);
    if (a->kind != VH_AGG_FIRST) fail(VH_ERR_ARG, "not an AggFirst");
    if (bytes != a->grid->length1d * a->grid_isz) fail(VH_ERR_ARG, "upload size mismatch");
    VH_HIP(hipMemcpyAsync(a->g2.ptr, host, bytes, hipMemcpyHostToDevice, stream()));
    VH_HIP(hipStreamSynchronize(stream()));
    VH_API_END
}

int vh_agg_upload(vh_agg *a, const void *host, uint64_t bytes) {
    VH_API_BEGIN
    std::lock_guard<std::mutex> lk(a->grid->mu);
    if (bytes != a->grid->length1d * a->grid_isz) fail(VH_ERR_ARG, "upload size mismatch");
    if (a->kind == VH_AGG_NUNIQUE) return VH_OK;  // a derived grid (recomputed when read)
    VH_HIP(hipMemcpyAsync(a->g.ptr, host, bytes, hipMemcpyHostToDevice, stream()));
    VH_HIP(hipStreamSynchronize(stream()));
    VH_API_END
}

int vh_agg_device_ptr(vh_agg *a, void **grid_dptr, void **grid2_dptr) {
    VH_API_BEGIN
    std::lock_guard<std::mutex> lk(a->grid->mu);
    nunique_finalize(a);
    VH_HIP(hipStreamSynchronize(stream()));  // the grid's fills and bins are done for any stream
    if (grid_dptr) *grid_dptr = a->g.ptr;
    if (grid2_dptr) *grid2_dptr = a->g2.ptr;
    VH_API_END
}

int vh_agg_reduce(vh_agg *a, vh_agg *const *others, int nothers) {
    VH_API_BEGIN
    std::lock_guard<std::mutex> lk(a->grid->mu);
    const uint64_t L = a->grid->length1d;
    for (int k = 0; k < nothers; k++) {
        vh_agg *o = others[k];
        if (o->kind != a->kind || o->dtype != a->dtype || o->grid->length1d != L)
            fail(VH_ERR_RUNTIME, "cannot reduce aggregators of different type or grid");
        if (!L) continue;
        dim3 grd(blocks_for(L, 256)), blk(256);
        switch (a->kind) {
        case VH_AGG_COUNT:
            hipLaunchKernelGGL(k_reduce_add<int64_t>, grd, blk, 0, stream(), a->g.as<int64_t>(), o->g.as<int64_t>(), L);
            break;
        case VH_AGG_SUM: case VH_AGG_SUM_MOMENT:
            if (a->grid_dtype == VH_F64)
                hipLaunchKernelGGL(k_reduce_add<double>, grd, blk, 0, stream(), a->g.as<double>(), o->g.as<double>(), L);
            else if (a->grid_dtype == VH_I64)
                hipLaunchKernelGGL(k_reduce_add<int64_t>, grd, blk, 0, stream(), a->g.as<int64_t>(), o->g.as<int64_t>(), L);
            else
                hipLaunchKernelGGL(k_reduce_add<uint64_t>, grd, blk, 0, stream(), a->g.as<uint64_t>(), o->g.as<uint64_t>(), L);
            break;
        case VH_AGG_MIN: case VH_AGG_MAX:
            VH_DISPATCH_DTYPE(a->dtype, T,
                              hipLaunchKernelGGL(k_reduce_minmax<T>, grd, blk, 0, stream(), a->g.as<T>(),
                                                 o->g.as<T>(), L, (int)(a->kind == VH_AGG_MAX)));
            break;
        case VH_AGG_FIRST:
            VH_DISPATCH_DTYPE(a->dtype, T,
                              hipLaunchKernelGGL(k_reduce_first<T>, grd, blk, 0, stream(), a->g.as<T>(),
                                                 a->g2.as<T>(), o->g.as<T>(), o->g2.as<T>(), L));
            break;
        case VH_AGG_NUNIQUE:
            nunique_merge(a, o);  // counter::merge (hash_primitives.hpp:393-415)
            break;
        }
        VH_HIP(hipGetLastError());
    }
    VH_HIP(hipStreamSynchronize(stream()));
    VH_API_END
}

int vh_grid_bin(vh_grid *g, vh_agg *const *aggs, int naggs, uint64_t length, int has_length) {
    VH_API_BEGIN
    std::lock_guard<std::mutex> lk(g->mu);
    if (!has_length) {
        if (g->binners.empty()) fail(VH_ERR_RUNTIME, "no binners set and no length given");
        if (!g->binners[0]->data.set) fail(VH_ERR_RUNTIME, "data not set");
        length = g->binners[0]->data.size;
    }
    for (auto *b : g->binners) {
        check_column(b->data, length, "binner data");
        if (b->mask.set) check_column(b->mask, length, "binner mask");
    }
    for (int k = 0; k < naggs; k++) {
        vh_agg *a = aggs[k];
        if (a->grid != g) fail(VH_ERR_RUNTIME, "aggregator belongs to another grid");
        const bool needs_data = a->kind != VH_AGG_COUNT;
        if (needs_data && !a->data.set) fail(VH_ERR_RUNTIME, "data not set");
        if (a->kind == VH_AGG_FIRST && !a->data2.set) fail(VH_ERR_RUNTIME, "data2 not set");
        if (a->data.set) check_column(a->data, length, "aggregator data");
        if (a->data2.set) check_column(a->data2, length, "aggregator data2");
        if (a->mask.set) check_column(a->mask, length, "aggregator mask");
    }
    if (length == 0 || naggs == 0) return VH_OK;
    run_bin(g, aggs, naggs, length);
    VH_API_END
}

}  // extern "C"

// ============================================================================
// the bin driver
// ============================================================================
namespace vh {

static BinnerDev binner_dev(vh_binner *b, uint64_t stride, Stager &st) {
    BinnerDev d{};
    d.kind = b->kind;
    d.dtype = b->dtype;
    d.flip = b->flip;
    d.data = st.get(b->data);
    d.mask = reinterpret_cast<const uint8_t *>(st.get(b->mask));
    d.vmin = b->vmin;
    d.scale = 1. / (b->vmax - b->vmin);  // scale_v, superagg_binners.cpp:15
    d.bins = b->bins;
    d.ordinal_count = b->ordinal_count;
    d.min_value = b->min_value;
    d.stride = stride;
    if (b->kind == 2) d.set = set_device_view(b->set);
    return d;
}

static AggDev agg_dev(vh_agg *a, Stager &st) {
    AggDev d{};
    d.kind = a->kind;
    d.dtype = a->dtype;
    d.flip = a->flip;
    d.moment = a->moment;
    d.has_selection = a->has_selection ? 1 : 0;
    d.data = st.get(a->data);
    d.data2 = st.get(a->data2);
    d.mask = reinterpret_cast<const uint8_t *>(st.get(a->mask));
    d.grid = a->g.ptr;
    d.grid2 = a->g2.ptr;
    d.s_key = a->s_key.ptr;
    d.s_row = a->s_row.ptr;
    return d;
}

// count (any data dtype=f64 or none) / sum(float64), native byte order
static bool fusable(vh_agg *a) {
    if (a->kind == VH_AGG_COUNT) return !a->data.set || (a->dtype == VH_F64 && !a->flip);
    if (a->kind == VH_AGG_SUM) return a->dtype == VH_F64 && !a->flip;
    return false;
}

static int scalar_f64_dims(vh_grid *g) {
    for (auto *b : g->binners)
        if (!(b->kind == 0 && b->dtype == VH_F64 && !b->flip)) return 0;
    return (int)g->binners.size();
}

void run_bin(vh_grid *g, vh_agg *const *aggs, int naggs, uint64_t length) {
    bool all_fusable = naggs <= MAX_FUSED_AGGS;
    for (int k = 0; k < naggs && all_fusable; k++) all_fusable = fusable(aggs[k]);
    bool any_host = false;
    auto note = [&](const ColumnRef &c) { any_host |= c.set && c.loc == VH_LOC_HOST; };
    for (auto *b : g->binners) {
        note(b->data);
        note(b->mask);
    }
    for (int k = 0; k < naggs; k++) {
        note(aggs[k]->data);
        note(aggs[k]->data2);
        note(aggs[k]->mask);
    }
    const uint64_t L = g->length1d;
    // count / sum of other native dtypes without masks on grids beyond the LDS sub-grid size
    // (any number of them: run in groups of at most MAX_FUSED_AGGS with at most two sums, one
    // tile pass per group over the same staged chunk)
    bool tile_generic = !all_fusable && L * 8 > LDS_AGG_MAX_BYTES;
    // (min / max too: LDS min / max cells in pass B; not of bool data)
    // (and AggSumMoment of float data -- var / std: a moment cell beside the sum's in pass B)
    auto tile_kind = [](const vh_agg *a) {
        return (a->kind == VH_AGG_COUNT || (a->kind == VH_AGG_SUM && a->data.set) ||
                ((a->kind == VH_AGG_MIN || a->kind == VH_AGG_MAX) && a->data.set && a->dtype != VH_BOOL) ||
                (a->kind == VH_AGG_SUM_MOMENT && a->data.set && (a->dtype == VH_F64 || a->dtype == VH_F32))) &&
               !a->mask.set && !a->flip;
    };
    for (int k = 0; k < naggs && tile_generic; k++) tile_generic = tile_kind(aggs[k]);
    if (!all_fusable && !tile_generic && !any_host && naggs > 1 && L * 8 > LDS_AGG_MAX_BYTES) {
        // a mix on a large grid (e.g. groupby count(*) + min + max): the count / sum
        // aggregators take the tile path, only the rest pays the generic path's global
        // atomics (one scattered atomic per row each: ~2.4e10 rows/s chip-wide)
        std::vector<vh_agg *> tiled, rest;
        for (int k = 0; k < naggs; k++) {
            const vh_agg *a = aggs[k];
            const bool t = tile_kind(a);
            (t && tiled.size() < (size_t)MAX_FUSED_AGGS ? tiled : rest).push_back(aggs[k]);
        }
        if (!tiled.empty() && !rest.empty()) {
            run_bin(g, tiled.data(), (int)tiled.size(), length);
            run_bin(g, rest.data(), (int)rest.size(), length);
            return;
        }
    }
    // AggFirst alone needs no per-row index buffer (tiled engine on large grids, LDS kernels on
    // small ones): HBM columns in one chunk, like the tile path (< 2^32 rows per launch)
    bool first_only = naggs > 0;
    for (int k = 0; k < naggs; k++) first_only = first_only && aggs[k]->kind == VH_AGG_FIRST;
    const uint64_t chunk_max = any_host ? (uint64_t(1) << 24)
                               : (all_fusable || tile_generic) ? length
                               : first_only ? std::min<uint64_t>(length, (uint64_t(1) << 32) - 4096)
                                            : (uint64_t(1) << 26);
    HostPipe &pipe = g->ws.pipe;
    if (any_host) {
        pipe.cols.clear();
        pipe.isz.clear();
        for (auto *b : g->binners) {
            pipe.add(b->data);
            pipe.add(b->mask);
        }
        for (int k = 0; k < naggs; k++) {
            pipe.add(aggs[k]->data);
            pipe.add(aggs[k]->data2);
            pipe.add(aggs[k]->mask);
        }
        pipe.plan(std::min(chunk_max, std::max<uint64_t>(length, 1)));
        if (length) pipe.issue(0, 0, std::min(chunk_max, length));
    }
    for (uint64_t row0 = 0, ci = 0; row0 < length; row0 += chunk_max, ci++) {
        const uint64_t len = std::min(chunk_max, length - row0);
        const int buf = (int)(ci & 1);
        if (any_host) {
            // stage the next chunk while this one is binned
            if (row0 + len < length) pipe.issue(ci + 1, row0 + len, std::min(chunk_max, length - row0 - len));
            pipe.wait_copied(buf);
        }
        Stager st{g->ws, row0, len, buf};
        BinPlan plan{};
        plan.nb = (int)g->binners.size();
        for (int d = 0; d < plan.nb; d++) plan.b[d] = binner_dev(g->binners[d], g->strides[d], st);
        // aggregators a tile group already binned in this chunk (a later group the tile path
        // refuses -- more carried values or bytes per cell than the first -- falls back to
        // the generic path below for its own aggregators only)
        std::vector<char> tdone(naggs, 0);
        if (all_fusable) {
            FusedAggs fa{};
            fa.na = naggs;
            for (int k = 0; k < naggs; k++) {
                AggDev ad = agg_dev(aggs[k], st);
                fa.a[k].kind = ad.kind;
                fa.a[k].data = reinterpret_cast<const double *>(ad.data);
                fa.a[k].mask = ad.mask;
                fa.a[k].grid = ad.grid;
                fa.a[k].dtype = ad.dtype;
                fa.a[k].vint = 0;
            }
            launch_fused(plan, fa, len, L, scalar_f64_dims(g), g->ws);
        } else if (tile_generic && [&] {
                       // count / sum / min / max of any native dtype over a grid too large for
                       // LDS: the tile-partitioned path with per-dtype loads, in groups of at
                       // most two carried value columns; a group the path refuses leaves its
                       // aggregators (and the later groups') to the generic path
                       std::vector<FusedAgg> all(naggs);
                       for (int k = 0; k < naggs; k++) {
                           AggDev ad = agg_dev(aggs[k], st);
                           FusedAgg &f = all[k];
                           f = FusedAgg{};
                           f.kind = ad.kind;
                           f.data = reinterpret_cast<const double *>(ad.data);
                           f.mask = nullptr;
                           f.grid = ad.grid;
                           f.dtype = ad.dtype;
                           f.vint = ad.kind == VH_AGG_SUM && ad.dtype != VH_F64 && ad.dtype != VH_F32;
                           f.moment = ad.moment;
                       }
                       // at most two carried value columns per group (sums, min, max of one
                       // column share one: same_value_slot)
                       std::vector<std::vector<int>> groups(1);
                       std::vector<int> slots;
                       for (int k = 0; k < naggs; k++) {
                           bool fresh = all[k].kind != VH_AGG_COUNT;
                           for (int j : slots) fresh = fresh && !same_value_slot(all[j], all[k]);
                           if ((fresh && slots.size() == 2) || groups.back().size() == (size_t)MAX_FUSED_AGGS) {
                               groups.emplace_back();
                               slots.clear();
                               fresh = all[k].kind != VH_AGG_COUNT;
                           }
                           if (fresh) slots.push_back(k);
                           groups.back().push_back(k);
                       }
                       for (size_t gi = 0; gi < groups.size(); gi++) {
                           FusedAggs fa{};
                           fa.na = (int)groups[gi].size();
                           fa.generic_vals = 1;
                           for (int j = 0; j < fa.na; j++) fa.a[j] = all[groups[gi][j]];
                           if (!try_tiled(plan, fa, len, L, scalar_f64_dims(g), g->ws)) return false;
                           for (int k : groups[gi]) tdone[k] = 1;
                       }
                       return true;
                   }()) {
            // done by the tile path
        } else {
            std::vector<AggDev> ads;
            for (int k = 0; k < naggs; k++) ads.push_back(agg_dev(aggs[k], st));
            // small grids: LDS sub-grid per workgroup for every kind but AggFirst / AggNUnique
            const bool small = L * 8 <= LDS_AGG_MAX_BYTES;
            auto lds_ok = [&](int kind) { return small && kind != VH_AGG_FIRST && kind != VH_AGG_NUNIQUE; };
            // AggFirst over a large grid: the tile-partitioned engine (first.hip) fills its
            // s_key / s_row scratch without per-row global atomics; k_first_c merges as below
            for (int k = 0; k < naggs; k++) {
                if (tdone[k] || ads[k].kind != VH_AGG_FIRST || small) continue;
                if (!try_tiled_first(plan, ads[k], len, L, row0, scalar_f64_dims(g))) continue;
                VH_DISPATCH_DTYPE(ads[k].dtype, T, hipLaunchKernelGGL(k_first_c<T>, dim3(blocks_for(L, 256)), dim3(256), 0, stream(), ads[k], L, row0));
                VH_HIP(hipGetLastError());
                tdone[k] = 1;
            }
            // binners the cell kernels handle (scalar / ordinal); set-ordinal binners keep
            // the per-row plan_index of k_agg_lds
            bool cells_ok = small && L <= 65536;
            for (int d = 0; d < plan.nb; d++) cells_ok = cells_ok && (plan.b[d].kind == 0 || plan.b[d].kind == 1);
            uint16_t *cells = nullptr;
            uint64_t *idx = nullptr;
            // AggFirst on a small grid takes the LDS kernels below (no indices)
            const bool first_lds = cells_ok && len && len < (1ull << 32) && 12 * L <= 96 * 1024;
            // per-row grid indices of `n` rows of plan `p` into `out`
            auto compute_idx = [&](const BinPlan &p, uint64_t n, uint64_t *out) {
                TimedScope ts("bin_indices");
                bool hoist = p.nb > 0;
                for (int d = 0; d < p.nb; d++) hoist = hoist && (p.b[d].kind == 0 || p.b[d].kind == 1);
                if (hoist) {
                    const dim3 cg(blocks_for(n, 256, 8)), cb(256);
                    for (int d = 0; d < p.nb; d++) {
                        const BinnerDev &b = p.b[d];
                        const int first = d == 0 ? 1 : 0;
                        if (b.kind == 0) {
                            VH_DISPATCH_DTYPE(b.dtype, T, hipLaunchKernelGGL((k_idx_dim<0, T>), cg, cb, 0, stream(), b, n, out, first));
                        } else {
                            VH_DISPATCH_DTYPE(b.dtype, T, hipLaunchKernelGGL((k_idx_dim<1, T>), cg, cb, 0, stream(), b, n, out, first));
                        }
                        VH_HIP(hipGetLastError());
                    }
                } else {
                    hipLaunchKernelGGL(k_indices, dim3(blocks_for(n, 256)), dim3(256), 0, stream(), p, n, out);
                    VH_HIP(hipGetLastError());
                }
            };
            // AggFirst-only chunks of HBM columns run up to 2^32 rows (the engines above need no
            // index buffer); one the engines refused takes the index path in IDX_ROWS pieces, so
            // its index buffer stays 512 MB (rows numbered from each piece's first row)
            constexpr uint64_t IDX_ROWS = uint64_t(1) << 26;
            if (first_only && len > IDX_ROWS) {
                for (uint64_t s0 = 0; s0 < len; s0 += IDX_ROWS) {
                    const uint64_t sl = std::min(IDX_ROWS, len - s0);
                    Stager ss{g->ws, row0 + s0, sl, buf};
                    BinPlan sp{};
                    sp.nb = plan.nb;
                    for (int d = 0; d < sp.nb; d++) sp.b[d] = binner_dev(g->binners[d], g->strides[d], ss);
                    g->ws.idx.ensure(sl * 8);
                    uint64_t *sidx = g->ws.idx.as<uint64_t>();
                    bool any = false;
                    for (int k = 0; k < naggs; k++) {
                        if (tdone[k] || first_lds) continue;
                        if (!any) compute_idx(sp, sl, sidx);
                        any = true;
                        const AggDev sad = agg_dev(aggs[k], ss);
                        TimedScope ts("bin_aggregate");
                        const dim3 grd(blocks_for(sl, 256)), blk(256);
                        VH_DISPATCH_DTYPE(sad.dtype, T, {
                            hipLaunchKernelGGL(k_first_a<T>, grd, blk, 0, stream(), sad, sidx, sl);
                            hipLaunchKernelGGL(k_first_b<T>, grd, blk, 0, stream(), sad, sidx, sl, row0 + s0);
                            hipLaunchKernelGGL(k_first_c<T>, dim3(blocks_for(L, 256)), blk, 0, stream(), sad, L, row0 + s0);
                        });
                        VH_HIP(hipGetLastError());
                    }
                    if (!any) break;
                }
                if (!first_lds)
                    for (int k = 0; k < naggs; k++) tdone[k] = 1;
            }
            for (int k = 0; k < naggs && !idx; k++) {
                if (tdone[k] || lds_ok(ads[k].kind) || (first_lds && ads[k].kind == VH_AGG_FIRST)) continue;
                g->ws.idx.ensure(len * 8);
                idx = g->ws.idx.as<uint64_t>();
                compute_idx(plan, len, idx);
            }
            auto make_cells = [&]() {
                if (cells) return;
                TimedScope ts("bin_cells");
                g->ws.cells.ensure(std::max<uint64_t>(len, 1) * 2);
                cells = g->ws.cells.as<uint16_t>();
                // no binners (a 0-d grid, df.sum('x')): every row is cell 0
                if (plan.nb == 0) VH_HIP(hipMemsetAsync(cells, 0, std::max<uint64_t>(len, 1) * 2, stream()));
                const dim3 cg(blocks_for(len, 256, 8)), cb(256);
                for (int d = 0; d < plan.nb; d++) {
                    const BinnerDev &b = plan.b[d];
                    const int first = d == 0 ? 1 : 0;
                    if (b.kind == 0) {
                        VH_DISPATCH_DTYPE(b.dtype, T, hipLaunchKernelGGL((k_cells_dim<0, T>), cg, cb, 0, stream(), b, len, cells, first));
                    } else {
                        VH_DISPATCH_DTYPE(b.dtype, T, hipLaunchKernelGGL((k_cells_dim<1, T>), cg, cb, 0, stream(), b, len, cells, first));
                    }
                    VH_HIP(hipGetLastError());
                }
            };
            // count / sum aggregators share one pass over the cells, as many per launch as
            // their sub-grids fit the LDS budget
            std::vector<char> done(tdone);
            if (cells_ok && len) {
                std::vector<int> pend;
                for (int k = 0; k < naggs; k++)
                    if (!done[k] && (ads[k].kind == VH_AGG_COUNT || ads[k].kind == VH_AGG_SUM)) pend.push_back(k);
                size_t i = 0;
                while (i < pend.size()) {
                    SmallAggs sa{};
                    uint64_t off = 0;
                    size_t j = i;
                    // a count that sees every row (no mask; no data, or integer data that
                    // is never NaN) equals any other such count of the same chunk
                    auto plain_count = [](const AggDev &a) {
                        return a.kind == VH_AGG_COUNT && !a.mask && (!a.data || (a.dtype != VH_F64 && a.dtype != VH_F32));
                    };
                    int first_plain = -1;
                    // rows one workgroup adds into its sub-grids (bounds 32-bit partials)
                    const dim3 sf_grid(blocks_for(len, 256, 8)), sf_block(256);
                    const uint64_t rows_wg = rows_per_wg(len, sf_grid.x, sf_block.x, SF_U);
                    auto narrow_ok = [&](const AggDev &a) {
                        if (a.kind == VH_AGG_COUNT) return rows_wg < (1ull << 32);
                        if (a.flip) return false;
                        if (a.dtype == VH_I8 || a.dtype == VH_U8) return rows_wg < (1ull << 23);
                        if (a.dtype == VH_I16 || a.dtype == VH_U16) return rows_wg < (1ull << 15);
                        return false;
                    };
                    while (j < pend.size() && sa.na < SF_MAX) {
                        const AggDev &a = ads[pend[j]];
                        if (plain_count(a) && first_plain >= 0) {
                            sa.lds_off[sa.na] = sa.lds_off[first_plain];
                            sa.shared |= 1u << sa.na;
                            if ((sa.narrow >> first_plain) & 1) sa.narrow |= 1u << sa.na;
                            sa.a[sa.na++] = a;
                            j++;
                            continue;
                        }
                        const bool nw = narrow_ok(a);
                        const uint64_t bytes = L * (nw ? 4 : 8);
                        if (off + bytes > SF_LDS_BUDGET) break;
                        if (plain_count(a)) first_plain = sa.na;
                        if (nw) sa.narrow |= 1u << sa.na;
                        sa.lds_off[sa.na] = (uint32_t)off;
                        sa.a[sa.na++] = a;
                        off += (bytes + 15) & ~uint64_t(15);
                        j++;
                    }
                    if (j == i) {
                        // the first candidate alone exceeds the fused pass's budget: it takes
                        // the per-aggregator LDS path below
                        i++;
                        continue;
                    }
                    if (sa.na >= 2) {
                        make_cells();
                        TimedScope ts("bin_aggregate_lds");
                        hipLaunchKernelGGL(k_small_fused, sf_grid, sf_block, (size_t)off, stream(), sa,
                                           cells, len, L, (uint32_t)(off / 4));
                        VH_HIP(hipGetLastError());
                        for (size_t q = i; q < j; q++) done[pend[q]] = 1;
                    }
                    i = j;
                }
            }
            // AggFirst on a small grid: per-workgroup LDS (key, row) cells + a fold of the
            // partials (k_first_small / k_first_small_fold), then the usual merge
            const uint64_t fs_lds = 12 * L;
            if (first_lds) {
                for (int k = 0; k < naggs; k++) {
                    AggDev &ad = ads[k];
                    if (done[k] || ad.kind != VH_AGG_FIRST) continue;
                    make_cells();
                    TimedScope ts("bin_first_lds");
                    const unsigned W = std::max(1u, std::min<unsigned>(blocks_for(len, FS_THREADS * FS_RPT, 4),
                                                                       (unsigned)((64ull << 20) / (12 * L))));
                    g->ws.first_part.ensure((uint64_t)W * L * 12 + 256);
                    auto *pkey = g->ws.first_part.as<unsigned long long>();
                    auto *prow = reinterpret_cast<uint32_t *>(pkey + (uint64_t)W * L);
                    VH_DISPATCH_DTYPE(ad.dtype, T, {
                        hipLaunchKernelGGL(k_first_small<T>, dim3(W), dim3(FS_THREADS), (size_t)fs_lds, stream(), ad, cells, len,
                                           (uint32_t)L, pkey, prow);
                        hipLaunchKernelGGL(k_first_small_fold, dim3((unsigned)L), dim3(256), 0, stream(), pkey, prow, W,
                                           (uint32_t)L, row0, static_cast<unsigned long long *>(ad.s_key),
                                           static_cast<unsigned long long *>(ad.s_row));
                        hipLaunchKernelGGL(k_first_c<T>, dim3(blocks_for(L, 256)), dim3(256), 0, stream(), ad, L, row0);
                    });
                    VH_HIP(hipGetLastError());
                    done[k] = 1;
                }
            }
            for (int k = 0; k < naggs; k++) {
                AggDev &ad = ads[k];
                if (done[k]) continue;
                if (lds_ok(ad.kind) && cells_ok) {
                    make_cells();
                    TimedScope ts("bin_aggregate_lds");
                    dim3 grd(blocks_for(len, 256, 8)), blk(256);
                    const size_t shm = (size_t)((L * 8 + 15) & ~uint64_t(15));
                    const size_t shm32 = (size_t)((L * 4 + 15) & ~uint64_t(15));
                    const bool mx = ad.kind == VH_AGG_MAX;
                    // rows one workgroup adds into its sub-grid (bounds 32-bit partials)
                    const uint64_t rows_wg = rows_per_wg(len, grd.x, blk.x, RU);
                    const bool narrow_sum = !ad.flip && (((ad.dtype == VH_I8 || ad.dtype == VH_U8) && rows_wg < (1ull << 23)) ||
                                                         ((ad.dtype == VH_I16 || ad.dtype == VH_U16) && rows_wg < (1ull << 15)));
                    switch (ad.kind) {
                    case VH_AGG_COUNT:
                        if (rows_wg < (1ull << 32)) {
                            VH_DISPATCH_DTYPE(ad.dtype, T, hipLaunchKernelGGL((k_agg_lds_c<VH_AGG_COUNT, T, true>), grd, blk, shm32, stream(), ad, cells, len, L, T{}));
                        } else {
                            VH_DISPATCH_DTYPE(ad.dtype, T, hipLaunchKernelGGL((k_agg_lds_c<VH_AGG_COUNT, T>), grd, blk, shm, stream(), ad, cells, len, L, T{}));
                        }
                        break;
                    case VH_AGG_SUM:
                        if (narrow_sum) {
                            switch (ad.dtype) {
                            case VH_I8: hipLaunchKernelGGL((k_agg_lds_c<VH_AGG_SUM, int8_t, true>), grd, blk, shm32, stream(), ad, cells, len, L, (int8_t)0); break;
                            case VH_U8: hipLaunchKernelGGL((k_agg_lds_c<VH_AGG_SUM, uint8_t, true>), grd, blk, shm32, stream(), ad, cells, len, L, (uint8_t)0); break;
                            case VH_I16: hipLaunchKernelGGL((k_agg_lds_c<VH_AGG_SUM, int16_t, true>), grd, blk, shm32, stream(), ad, cells, len, L, (int16_t)0); break;
                            default: hipLaunchKernelGGL((k_agg_lds_c<VH_AGG_SUM, uint16_t, true>), grd, blk, shm32, stream(), ad, cells, len, L, (uint16_t)0);
                            }
                        } else {
                            VH_DISPATCH_DTYPE(ad.dtype, T, hipLaunchKernelGGL((k_agg_lds_c<VH_AGG_SUM, T>), grd, blk, shm, stream(), ad, cells, len, L, T{}));
                        }
                        break;
                    case VH_AGG_MIN:
                        VH_DISPATCH_DTYPE(ad.dtype, T, hipLaunchKernelGGL((k_agg_lds_c<VH_AGG_MIN, T>), grd, blk, shm, stream(), ad, cells, len, L, minmax_fill<T>(false)));
                        break;
                    case VH_AGG_MAX:
                        VH_DISPATCH_DTYPE(ad.dtype, T, hipLaunchKernelGGL((k_agg_lds_c<VH_AGG_MAX, T>), grd, blk, shm, stream(), ad, cells, len, L, minmax_fill<T>(mx)));
                        break;
                    case VH_AGG_SUM_MOMENT:
                        VH_DISPATCH_DTYPE(ad.dtype, T, hipLaunchKernelGGL((k_agg_lds_c<VH_AGG_SUM_MOMENT, T>), grd, blk, shm, stream(), ad, cells, len, L, T{}));
                        break;
                    }
                    VH_HIP(hipGetLastError());
                    continue;
                }
                if (lds_ok(ad.kind)) {
                    TimedScope ts("bin_aggregate_lds");
                    dim3 grd(blocks_for(len, 256, 4)), blk(256);
                    const size_t shm = (size_t)((L * 8 + 15) & ~uint64_t(15));
                    const bool mx = ad.kind == VH_AGG_MAX;
                    switch (ad.kind) {
                    case VH_AGG_COUNT:
                        VH_DISPATCH_DTYPE(ad.dtype, T, hipLaunchKernelGGL((k_agg_lds<VH_AGG_COUNT, T>), grd, blk, shm, stream(), plan, ad, len, L, T{}));
                        break;
                    case VH_AGG_SUM:
                        VH_DISPATCH_DTYPE(ad.dtype, T, hipLaunchKernelGGL((k_agg_lds<VH_AGG_SUM, T>), grd, blk, shm, stream(), plan, ad, len, L, T{}));
                        break;
                    case VH_AGG_MIN:
                        VH_DISPATCH_DTYPE(ad.dtype, T, hipLaunchKernelGGL((k_agg_lds<VH_AGG_MIN, T>), grd, blk, shm, stream(), plan, ad, len, L, minmax_fill<T>(false)));
                        break;
                    case VH_AGG_MAX:
                        VH_DISPATCH_DTYPE(ad.dtype, T, hipLaunchKernelGGL((k_agg_lds<VH_AGG_MAX, T>), grd, blk, shm, stream(), plan, ad, len, L, minmax_fill<T>(mx)));
                        break;
                    case VH_AGG_SUM_MOMENT:
                        VH_DISPATCH_DTYPE(ad.dtype, T, hipLaunchKernelGGL((k_agg_lds<VH_AGG_SUM_MOMENT, T>), grd, blk, shm, stream(), plan, ad, len, L, T{}));
                        break;
                    }
                    VH_HIP(hipGetLastError());
                    continue;
                }
                dim3 grd(blocks_for(len, 256)), blk(256);
                TimedScope ts("bin_aggregate");
                switch (ad.kind) {
                case VH_AGG_COUNT:
                    VH_DISPATCH_DTYPE(ad.dtype, T, hipLaunchKernelGGL((k_agg<VH_AGG_COUNT, T>), grd, blk, 0, stream(), ad, idx, len));
                    break;
                case VH_AGG_SUM:
                    VH_DISPATCH_DTYPE(ad.dtype, T, hipLaunchKernelGGL((k_agg<VH_AGG_SUM, T>), grd, blk, 0, stream(), ad, idx, len));
                    break;
                case VH_AGG_MIN:
                    VH_DISPATCH_DTYPE(ad.dtype, T, hipLaunchKernelGGL((k_agg<VH_AGG_MIN, T>), grd, blk, 0, stream(), ad, idx, len));
                    break;
                case VH_AGG_MAX:
                    VH_DISPATCH_DTYPE(ad.dtype, T, hipLaunchKernelGGL((k_agg<VH_AGG_MAX, T>), grd, blk, 0, stream(), ad, idx, len));
                    break;
                case VH_AGG_SUM_MOMENT:
                    VH_DISPATCH_DTYPE(ad.dtype, T, hipLaunchKernelGGL((k_agg<VH_AGG_SUM_MOMENT, T>), grd, blk, 0, stream(), ad, idx, len));
                    break;
                case VH_AGG_FIRST:
                    VH_DISPATCH_DTYPE(ad.dtype, T, {
                        hipLaunchKernelGGL(k_first_a<T>, grd, blk, 0, stream(), ad, idx, len);
                        hipLaunchKernelGGL(k_first_b<T>, grd, blk, 0, stream(), ad, idx, len, row0);
                        hipLaunchKernelGGL(k_first_c<T>, dim3(blocks_for(L, 256)), blk, 0, stream(), ad, L, row0);
                    });
                    break;
                case VH_AGG_NUNIQUE:
                    nunique_collect(aggs[k], ad, idx, len);
                    break;
                }
                VH_HIP(hipGetLastError());
            }
        }
        if (any_host) pipe.mark_consumed(buf);
    }
    VH_HIP(hipStreamSynchronize(stream()));
}

// 0-d grids (no binners) of count / float64-sum aggregators: a reduction (k_reduce0);
// false when a column is not aligned for the vector loads (k_fused takes it)
static bool launch_reduce0(const FusedAggs &fa, uint64_t n, Workspace &ws) {
    Reduce0 r{};
    r.na = fa.na;
    for (int k = 0; k < fa.na; k++) {
        const FusedAgg &a = fa.a[k];
        r.akind[k] = (int8_t)a.kind;
        r.grid[k] = a.grid;
        r.acol[k] = r.amask[k] = -1;
        if (a.data) {
            if (reinterpret_cast<uintptr_t>(a.data) & 15) return false;
            int q = 0;
            while (q < r.ncol && r.col[q] != reinterpret_cast<const double2 *>(a.data)) q++;
            if (q == r.ncol) r.col[r.ncol++] = reinterpret_cast<const double2 *>(a.data);
            r.acol[k] = (int8_t)q;
        }
        if (a.mask) {
            if (reinterpret_cast<uintptr_t>(a.mask) & 1) return false;
            int q = 0;
            while (q < r.nmask && r.mask[q] != reinterpret_cast<const uint16_t *>(a.mask)) q++;
            if (q == r.nmask) r.mask[r.nmask++] = reinterpret_cast<const uint16_t *>(a.mask);
            r.amask[k] = (int8_t)q;
        }
        if (a.kind == VH_AGG_COUNT && !a.data && !a.mask) r.all_rows |= 1 << k;
    }
    const bool reads = r.ncol > 0 || r.nmask > 0;
    const unsigned nb = reads ? blocks_for(std::max<uint64_t>(n / 2, 1), 256, 8) : 0;
    ws.idx.ensure(std::max<uint64_t>((uint64_t)nb * MAX_FUSED_AGGS * 16, 16));
    double *psum = ws.idx.as<double>();
    uint64_t *pcnt = reinterpret_cast<uint64_t *>(psum + (uint64_t)nb * MAX_FUSED_AGGS);
    TimedScope ts("bin_reduce0");
    if (nb) {
        if (r.nmask)
            hipLaunchKernelGGL(k_reduce0<true>, dim3(nb), dim3(256), 0, stream(), r, n, psum, pcnt);
        else
            hipLaunchKernelGGL(k_reduce0<false>, dim3(nb), dim3(256), 0, stream(), r, n, psum, pcnt);
        VH_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_reduce0_fin, dim3(1), dim3(256), 0, stream(), r, psum, pcnt, nb, n);
    VH_HIP(hipGetLastError());
    return true;
}

static bool getenv_off(const char *name) {  // NAME=0 turns a default-on path off (A/B runs)
    const char *e = getenv(name);
    return e && e[0] == '0' && e[1] == 0;
}

// small grids over float64 scalar binners (k_small_f64): false when a column is masked or
// not 16-B aligned (k_fused takes it).  Native float32 scalar binners (8-B aligned) take the
// same kernel with float32 row pairs (64^2 count(*) over 1e9 float32 rows: k_fused's per-row
// dispatch 8.5 ms, profiles/r06_f32_small.txt)
static bool launch_small_f64(const BinPlan &plan, const FusedAggs &fa, uint64_t n, uint64_t cells, int nd_f64,
                             Workspace &ws) {
    int nd32 = 0;
    if (nd_f64 == 0 && plan.nb >= 1 && plan.nb <= 3 && !getenv_off("VH_SMALL_F32")) {
        bool ok = true;
        for (int d = 0; d < plan.nb; d++) ok = ok && plan.b[d].kind == 0 && plan.b[d].dtype == VH_F32 && !plan.b[d].flip;
        if (ok) nd32 = plan.nb;
    }
    const int nd = nd_f64 ? nd_f64 : nd32;
    if (nd < 1 || nd > 3 || n < 2) return false;
    const uintptr_t amask = nd32 ? 7 : 15;
    for (int d = 0; d < plan.nb; d++)
        if (plan.b[d].mask || (reinterpret_cast<uintptr_t>(plan.b[d].data) & amask)) return false;
    SmallF64 s{};
    s.na = fa.na;
    s.lds_words = fa.lds_words;
    for (int k = 0; k < fa.na; k++) {
        const FusedAgg &a = fa.a[k];
        if (a.mask) return false;
        s.akind[k] = (int8_t)a.kind;
        s.lds_off[k] = a.lds_off;
        s.grid[k] = a.grid;
        s.acol[k] = -1;
        if (a.data) {
            if (reinterpret_cast<uintptr_t>(a.data) & 15) return false;
            int q = 0;
            while (q < s.ncol && s.col[q] != reinterpret_cast<const double2 *>(a.data)) q++;
            if (q == s.ncol) s.col[s.ncol++] = reinterpret_cast<const double2 *>(a.data);
            s.acol[k] = (int8_t)q;
        }
    }
    if (s.ncol > 2) return false;
    const uint64_t lds_bytes = 4ull * fa.lds_words;
    const unsigned per_cu = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(8, (64 * 1024) / std::max<uint64_t>(lds_bytes, 1)));
    // at least two unrolled steps per lane before a workgroup pays its sub-grid flush
    const unsigned nb = blocks_for((n / 2 + 2 * SG_U - 1) / (2 * SG_U), 256, per_cu);
    ws.idx.ensure((uint64_t)nb * lds_bytes);
    uint32_t *part = ws.idx.as<uint32_t>();
    TimedScope ts(nd32 ? "bin_small_f32" : "bin_small_f64");
    const dim3 grd(nb), blk(256);
#define VH_SG(ND, NC)                                                                                        \
    if (nd32) hipLaunchKernelGGL((k_small_f64<ND, NC, float>), grd, blk, lds_bytes, stream(), plan, s, n, part); \
    else hipLaunchKernelGGL((k_small_f64<ND, NC>), grd, blk, lds_bytes, stream(), plan, s, n, part)
#define VH_SG_NC(ND) \
    switch (s.ncol) { \
    case 0: VH_SG(ND, 0); break; \
    case 1: VH_SG(ND, 1); break; \
    default: VH_SG(ND, 2); \
    }
    switch (nd) {
    case 1: VH_SG_NC(1); break;
    case 2: VH_SG_NC(2); break;
    default: VH_SG_NC(3);
    }
#undef VH_SG_NC
#undef VH_SG
    VH_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_small_f64_fin, dim3((unsigned)((cells + 255) / 256), (nb + SG_FIN_CHUNK - 1) / SG_FIN_CHUNK, fa.na),
                       blk, 0, stream(), s, part, nb, cells);
    VH_HIP(hipGetLastError());
    return true;
}

void launch_fused(const BinPlan &plan, FusedAggs &fa, uint64_t n, uint64_t cells, int nd_f64, Workspace &ws) {
    if (plan.nb == 0 && cells == 1 && launch_reduce0(fa, n, ws)) return;
    // LDS-privatised sub-grids when every aggregator's grid fits (u32 counts, f64 sums)
    uint64_t off = 0;
    for (int k = 0; k < fa.na; k++) {
        off = (off + 7) & ~uint64_t(7);
        fa.a[k].lds_off = (uint32_t)off;
        off += cells * (fa.a[k].kind == VH_AGG_COUNT ? 4 : 8);
    }
    const uint64_t lds_bytes = (off + 15) & ~uint64_t(15);
    const bool use_lds = lds_bytes <= LDS_FUSED_MAX && cells > 0;
    fa.lds_words = (uint32_t)(lds_bytes / 4);
    if (!use_lds && hashagg_bin_set_ordinal(plan, fa, n)) return;
    if (!use_lds && try_tiled(plan, fa, n, cells, nd_f64, ws)) return;
    if (use_lds && launch_small_f64(plan, fa, n, cells, nd_f64, ws)) return;
    const int per_cu = use_lds ? (int)std::max<uint64_t>(1, std::min<uint64_t>(8, (64 * 1024) / std::max<uint64_t>(lds_bytes, 1))) : 8;
    dim3 grd(blocks_for(n, 256, per_cu)), blk(256);
    const size_t shm = use_lds ? lds_bytes : 0;
    TimedScope ts(use_lds ? "bin_fused_lds" : "bin_fused_global");
#define VH_LAUNCH_FUSED(LDS, ND) hipLaunchKernelGGL((k_fused<LDS, ND>), grd, blk, shm, stream(), plan, fa, n, cells)
    if (use_lds) {
        switch (nd_f64) {
        case 1: VH_LAUNCH_FUSED(true, 1); break;
        case 2: VH_LAUNCH_FUSED(true, 2); break;
        case 3: VH_LAUNCH_FUSED(true, 3); break;
        default: VH_LAUNCH_FUSED(true, 0);
        }
    } else {
        switch (nd_f64) {
        case 1: VH_LAUNCH_FUSED(false, 1); break;
        case 2: VH_LAUNCH_FUSED(false, 2); break;
        case 3: VH_LAUNCH_FUSED(false, 3); break;
        default: VH_LAUNCH_FUSED(false, 0);
        }
    }
#undef VH_LAUNCH_FUSED
    VH_HIP(hipGetLastError());
}

}  // namespace vh
