/*
 * superagg_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A plain-C restatement of the reference's CPU binned-statistics path, written
 * from the reference sources (read as text; the reference itself is never
 * compiled or run -- see DESIGN.md "Oracle status"):
 *
 *   BinnerScalar<T>::to_bins     packages/vaex-core/src/superagg_binners.cpp:14-56
 *   BinnerOrdinal<T>::to_bins    packages/vaex-core/src/superagg_binners.cpp:104-142
 *   Grid strides / bin_ loop     packages/vaex-core/src/agg.hpp:54-69, 106-136
 *   AggCount::aggregate          packages/vaex-core/src/superagg.cpp:168-191
 *   AggMax / AggMin              packages/vaex-core/src/superagg.cpp:194-287
 *   upcast<T> table + AggSum     packages/vaex-core/src/superagg.cpp:289-389
 *   AggSumMoment                 packages/vaex-core/src/superagg.cpp:391-434
 *   AggFirst                     packages/vaex-core/src/superagg.cpp:436-511
 *   _hash64 (splitmix64 finaliser) packages/vaex-core/src/hash.hpp:25-30
 *   hash<int32/...> key widening packages/vaex-core/src/hash.hpp:35-84
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * this library.  The CPU-baseline drivers at the bottom (or_bench_*) reproduce
 * the reference threading model of ExecutorLocal/TaskPartAggregation
 * (packages/vaex-core/vaex/execution.py:149-156,214-289; cpu.py:487-499):
 * 1 Mi-row chunks, `nparts` private grids, serial reduce.
 *
 * Parity pins: tests/golden/kats.json (transcribed from the reference's own
 * tests) -- tests/test_oracle_kats.py checks this file against
 * every one of them before anything else trusts it.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum {
    OR_F64 = 0, OR_F32 = 1, OR_I64 = 2, OR_I32 = 3, OR_I16 = 4, OR_I8 = 5,
    OR_U64 = 6, OR_U32 = 7, OR_U16 = 8, OR_U8 = 9, OR_BOOL = 10
};

typedef uint8_t orbool;  /* numpy bool: one byte, 0 or 1 */

/* _to_native<T> (agg.hpp:13-21): reverse the bytes of one value */
#define DEF_BSWAP(NAME, T)                                   \
    static inline T NAME(T v) {                              \
        T r; unsigned char *s = (unsigned char *)&v;          \
        unsigned char *d = (unsigned char *)&r;              \
        for (size_t i = 0; i < sizeof(T); i++)               \
            d[sizeof(T) - 1 - i] = s[i];                     \
        return r;                                            \
    }
DEF_BSWAP(bs_f64, double)
DEF_BSWAP(bs_f32, float)
DEF_BSWAP(bs_i64, int64_t)
DEF_BSWAP(bs_i32, int32_t)
DEF_BSWAP(bs_i16, int16_t)
DEF_BSWAP(bs_i8, int8_t)
DEF_BSWAP(bs_u64, uint64_t)
DEF_BSWAP(bs_u32, uint32_t)
DEF_BSWAP(bs_u16, uint16_t)
DEF_BSWAP(bs_u8, uint8_t)
DEF_BSWAP(bs_b, orbool)

/* ---------------------------------------------------------------------- */
/* BinnerScalar<T>::to_bins  (superagg_binners.cpp:14-56)                  */
/* ---------------------------------------------------------------------- */
#define DEF_SCALAR(SUF, T, BS)                                                         \
    static void scalar_##SUF(const T *ptr, const uint8_t *mask, uint64_t n, int flip,   \
                             double vmin, double vmax, uint64_t bins, uint64_t stride,  \
                             uint64_t *out) {                                           \
        const double scale_v = 1. / (vmax - vmin);                                      \
        for (uint64_t i = 0; i < n; i++) {                                              \
            T value = ptr[i];                                                           \
            if (flip) value = BS(value);                                                \
            double value_double = (double)value;                                        \
            double scaled = (value_double - vmin) * scale_v;                            \
            uint64_t index = 0;                                                         \
            int masked = mask ? (mask[i] == 1) : 0;                                     \
            if (scaled != scaled || masked) {                                           \
            } else if (scaled < 0) {                                                    \
                index = 1;                                                              \
            } else if (scaled >= 1) {                                                   \
                index = bins - 1 + 3;                                                   \
            } else {                                                                    \
                index = (uint64_t)(int64_t)((int)(scaled * (double)(bins)) + 2);         \
            }                                                                           \
            out[i] += index * stride;                                                   \
        }                                                                               \
    }
DEF_SCALAR(f64, double, bs_f64)
DEF_SCALAR(f32, float, bs_f32)
DEF_SCALAR(i64, int64_t, bs_i64)
DEF_SCALAR(i32, int32_t, bs_i32)
DEF_SCALAR(i16, int16_t, bs_i16)
DEF_SCALAR(i8, int8_t, bs_i8)
DEF_SCALAR(u64, uint64_t, bs_u64)
DEF_SCALAR(u32, uint32_t, bs_u32)
DEF_SCALAR(u16, uint16_t, bs_u16)
DEF_SCALAR(u8, uint8_t, bs_u8)

/* bool: value_double = (double)(bool)ptr[i] */
static void scalar_b(const orbool *ptr, const uint8_t *mask, uint64_t n, int flip, double vmin,
                     double vmax, uint64_t bins, uint64_t stride, uint64_t *out) {
    (void)flip;
    const double scale_v = 1. / (vmax - vmin);
    for (uint64_t i = 0; i < n; i++) {
        double value_double = ptr[i] ? 1.0 : 0.0;
        double scaled = (value_double - vmin) * scale_v;
        uint64_t index = 0;
        int masked = mask ? (mask[i] == 1) : 0;
        if (scaled != scaled || masked) {
        } else if (scaled < 0) {
            index = 1;
        } else if (scaled >= 1) {
            index = bins - 1 + 3;
        } else {
            index = (uint64_t)(int64_t)((int)(scaled * (double)(bins)) + 2);
        }
        out[i] += index * stride;
    }
}

int or_binner_scalar(int dtype, int flip, const void *data, const uint8_t *mask, uint64_t n,
                     double vmin, double vmax, uint64_t bins, uint64_t stride, uint64_t *out) {
    switch (dtype) {
    case OR_F64: scalar_f64(data, mask, n, flip, vmin, vmax, bins, stride, out); break;
    case OR_F32: scalar_f32(data, mask, n, flip, vmin, vmax, bins, stride, out); break;
    case OR_I64: scalar_i64(data, mask, n, flip, vmin, vmax, bins, stride, out); break;
    case OR_I32: scalar_i32(data, mask, n, flip, vmin, vmax, bins, stride, out); break;
    case OR_I16: scalar_i16(data, mask, n, flip, vmin, vmax, bins, stride, out); break;
    case OR_I8: scalar_i8(data, mask, n, flip, vmin, vmax, bins, stride, out); break;
    case OR_U64: scalar_u64(data, mask, n, flip, vmin, vmax, bins, stride, out); break;
    case OR_U32: scalar_u32(data, mask, n, flip, vmin, vmax, bins, stride, out); break;
    case OR_U16: scalar_u16(data, mask, n, flip, vmin, vmax, bins, stride, out); break;
    case OR_U8: scalar_u8(data, mask, n, flip, vmin, vmax, bins, stride, out); break;
    case OR_BOOL: scalar_b(data, mask, n, flip, vmin, vmax, bins, stride, out); break;
    default: return -1;
    }
    return 0;
}

/* ---------------------------------------------------------------------- */
/* BinnerOrdinal<T>::to_bins  (superagg_binners.cpp:104-142)               */
/* `T value = ptr[i] - min_value` with min_value stored as uint64_t: the  */
/* subtraction happens in uint64 for integer T (then narrows to T), in T  */
/* for floating T (min_value converted to T); the byte swap is applied    */
/* AFTER the subtraction, exactly as the reference does.                  */
/* ---------------------------------------------------------------------- */
#define DEF_ORD_INT(SUF, T, BS, SIGNED)                                                      \
    static void ordinal_##SUF(const T *ptr, const uint8_t *mask, uint64_t n, int flip,        \
                              uint64_t ordinal_count, uint64_t min_value, uint64_t stride,     \
                              uint64_t *out) {                                                \
        for (uint64_t i = 0; i < n; i++) {                                                    \
            T value = (T)((uint64_t)(int64_t)ptr[i] - min_value);                             \
            if (!SIGNED) value = (T)((uint64_t)ptr[i] - min_value);                           \
            if (flip) value = BS(value);                                                      \
            uint64_t index = 0;                                                               \
            int masked = mask ? (mask[i] == 1) : 0;                                           \
            if (masked) {                                                                     \
            } else if (SIGNED && (int64_t)value < 0) {                                        \
                index = 1;                                                                    \
            } else if ((uint64_t)(int64_t)value >= ordinal_count) {                           \
                index = ordinal_count - 1 + 3;                                                \
            } else {                                                                          \
                index = (uint64_t)((int64_t)value + 2);                                       \
            }                                                                                 \
            out[i] += index * stride;                                                         \
        }                                                                                     \
    }
DEF_ORD_INT(i64, int64_t, bs_i64, 1)
DEF_ORD_INT(i32, int32_t, bs_i32, 1)
DEF_ORD_INT(i16, int16_t, bs_i16, 1)
DEF_ORD_INT(i8, int8_t, bs_i8, 1)
DEF_ORD_INT(u64, uint64_t, bs_u64, 0)
DEF_ORD_INT(u32, uint32_t, bs_u32, 0)
DEF_ORD_INT(u16, uint16_t, bs_u16, 0)
DEF_ORD_INT(u8, uint8_t, bs_u8, 0)

#define DEF_ORD_FLT(SUF, T, BS)                                                               \
    static void ordinal_##SUF(const T *ptr, const uint8_t *mask, uint64_t n, int flip,        \
                              uint64_t ordinal_count, uint64_t min_value, uint64_t stride,     \
                              uint64_t *out) {                                                \
        for (uint64_t i = 0; i < n; i++) {                                                    \
            T value = ptr[i] - (T)min_value;                                                  \
            if (flip) value = BS(value);                                                      \
            uint64_t index = 0;                                                               \
            int masked = mask ? (mask[i] == 1) : 0;                                           \
            if (value != value || masked) {                                                   \
            } else if (value < 0) {                                                           \
                index = 1;                                                                    \
            } else if (value >= (T)ordinal_count) {                                           \
                index = ordinal_count - 1 + 3;                                                \
            } else {                                                                          \
                index = (uint64_t)(value + 2);                                                \
            }                                                                                 \
            out[i] += index * stride;                                                         \
        }                                                                                     \
    }
DEF_ORD_FLT(f64, double, bs_f64)
DEF_ORD_FLT(f32, float, bs_f32)

static void ordinal_b(const orbool *ptr, const uint8_t *mask, uint64_t n, int flip,
                      uint64_t ordinal_count, uint64_t min_value, uint64_t stride, uint64_t *out) {
    (void)flip;
    for (uint64_t i = 0; i < n; i++) {
        /* bool promotes to int, minus uint64, converted back to bool: != 0 */
        int value = ((uint64_t)(ptr[i] ? 1 : 0) - min_value) != 0;
        uint64_t index = 0;
        int masked = mask ? (mask[i] == 1) : 0;
        if (masked) {
        } else if ((uint64_t)value >= ordinal_count) {
            index = ordinal_count - 1 + 3;
        } else {
            index = (uint64_t)(value + 2);
        }
        out[i] += index * stride;
    }
}

int or_binner_ordinal(int dtype, int flip, const void *data, const uint8_t *mask, uint64_t n,
                      uint64_t ordinal_count, uint64_t min_value, uint64_t stride, uint64_t *out) {
    switch (dtype) {
    case OR_F64: ordinal_f64(data, mask, n, flip, ordinal_count, min_value, stride, out); break;
    case OR_F32: ordinal_f32(data, mask, n, flip, ordinal_count, min_value, stride, out); break;
    case OR_I64: ordinal_i64(data, mask, n, flip, ordinal_count, min_value, stride, out); break;
    case OR_I32: ordinal_i32(data, mask, n, flip, ordinal_count, min_value, stride, out); break;
    case OR_I16: ordinal_i16(data, mask, n, flip, ordinal_count, min_value, stride, out); break;
    case OR_I8: ordinal_i8(data, mask, n, flip, ordinal_count, min_value, stride, out); break;
    case OR_U64: ordinal_u64(data, mask, n, flip, ordinal_count, min_value, stride, out); break;
    case OR_U32: ordinal_u32(data, mask, n, flip, ordinal_count, min_value, stride, out); break;
    case OR_U16: ordinal_u16(data, mask, n, flip, ordinal_count, min_value, stride, out); break;
    case OR_U8: ordinal_u8(data, mask, n, flip, ordinal_count, min_value, stride, out); break;
    case OR_BOOL: ordinal_b(data, mask, n, flip, ordinal_count, min_value, stride, out); break;
    default: return -1;
    }
    return 0;
}

/* ---------------------------------------------------------------------- */
/* Aggregators                                                             */
/* ---------------------------------------------------------------------- */
/* value read as "double-like" for NaN checks on the StorageType: for     */
/* integer types NaN never happens.                                        */

/* AggCount<T> (superagg.cpp:168-191).  grid is int64. */
#define DEF_COUNT(SUF, T, BS, ISFLT)                                                         \
    static void count_##SUF(const T *data, const uint8_t *mask, const uint64_t *idx,          \
                            uint64_t n, int flip, int64_t *grid) {                            \
        if (mask || data) {                                                                   \
            for (uint64_t j = 0; j < n; j++) {                                                \
                if (mask == NULL || mask[j] == 1) {                                           \
                    if (data) {                                                               \
                        T value = data[j];                                                    \
                        if (flip) value = BS(value);                                          \
                        if (ISFLT && value != value) continue;                                \
                    }                                                                         \
                    grid[idx[j]] += 1;                                                        \
                }                                                                             \
            }                                                                                 \
        } else {                                                                              \
            for (uint64_t j = 0; j < n; j++) grid[idx[j]] += 1;                               \
        }                                                                                     \
    }
DEF_COUNT(f64, double, bs_f64, 1)
DEF_COUNT(f32, float, bs_f32, 1)
DEF_COUNT(i64, int64_t, bs_i64, 0)
DEF_COUNT(i32, int32_t, bs_i32, 0)
DEF_COUNT(i16, int16_t, bs_i16, 0)
DEF_COUNT(i8, int8_t, bs_i8, 0)
DEF_COUNT(u64, uint64_t, bs_u64, 0)
DEF_COUNT(u32, uint32_t, bs_u32, 0)
DEF_COUNT(u16, uint16_t, bs_u16, 0)
DEF_COUNT(u8, uint8_t, bs_u8, 0)
DEF_COUNT(b, orbool, bs_b, 0)

int or_agg_count(int dtype, int flip, const void *data, const uint8_t *mask, const uint64_t *idx,
                 uint64_t n, int64_t *grid) {
    switch (dtype) {
    case OR_F64: count_f64(data, mask, idx, n, flip, grid); break;
    case OR_F32: count_f32(data, mask, idx, n, flip, grid); break;
    case OR_I64: count_i64(data, mask, idx, n, flip, grid); break;
    case OR_I32: count_i32(data, mask, idx, n, flip, grid); break;
    case OR_I16: count_i16(data, mask, idx, n, flip, grid); break;
    case OR_I8: count_i8(data, mask, idx, n, flip, grid); break;
    case OR_U64: count_u64(data, mask, idx, n, flip, grid); break;
    case OR_U32: count_u32(data, mask, idx, n, flip, grid); break;
    case OR_U16: count_u16(data, mask, idx, n, flip, grid); break;
    case OR_U8: count_u8(data, mask, idx, n, flip, grid); break;
    case OR_BOOL: count_b(data, mask, idx, n, flip, grid); break;
    default: return -1;
    }
    return 0;
}

/* AggSum<T> (superagg.cpp:362-388) with upcast<T> (:289-346):
 * float/double -> double, signed/bool -> int64, unsigned -> uint64. */
#define DEF_SUM(SUF, T, BS, G, ISFLT)                                                        \
    static void sum_##SUF(const T *data, const uint8_t *mask, const uint64_t *idx, uint64_t n, \
                          int flip, G *grid) {                                                \
        for (uint64_t j = 0; j < n; j++) {                                                    \
            if (mask && mask[j] != 1) continue;                                               \
            T value = data[j];                                                                \
            if (flip) value = BS(value);                                                      \
            if (ISFLT && value != value) continue;                                            \
            grid[idx[j]] += (G)value;                                                         \
        }                                                                                     \
    }
DEF_SUM(f64, double, bs_f64, double, 1)
DEF_SUM(f32, float, bs_f32, double, 1)
DEF_SUM(i64, int64_t, bs_i64, int64_t, 0)
DEF_SUM(i32, int32_t, bs_i32, int64_t, 0)
DEF_SUM(i16, int16_t, bs_i16, int64_t, 0)
DEF_SUM(i8, int8_t, bs_i8, int64_t, 0)
DEF_SUM(u64, uint64_t, bs_u64, uint64_t, 0)
DEF_SUM(u32, uint32_t, bs_u32, uint64_t, 0)
DEF_SUM(u16, uint16_t, bs_u16, uint64_t, 0)
DEF_SUM(u8, uint8_t, bs_u8, uint64_t, 0)

static void sum_b(const orbool *data, const uint8_t *mask, const uint64_t *idx, uint64_t n,
                  int flip, int64_t *grid) {
    (void)flip;
    for (uint64_t j = 0; j < n; j++) {
        if (mask && mask[j] != 1) continue;
        grid[idx[j]] += data[j] ? 1 : 0;
    }
}

int or_agg_sum(int dtype, int flip, const void *data, const uint8_t *mask, const uint64_t *idx,
               uint64_t n, void *grid) {
    switch (dtype) {
    case OR_F64: sum_f64(data, mask, idx, n, flip, grid); break;
    case OR_F32: sum_f32(data, mask, idx, n, flip, grid); break;
    case OR_I64: sum_i64(data, mask, idx, n, flip, grid); break;
    case OR_I32: sum_i32(data, mask, idx, n, flip, grid); break;
    case OR_I16: sum_i16(data, mask, idx, n, flip, grid); break;
    case OR_I8: sum_i8(data, mask, idx, n, flip, grid); break;
    case OR_U64: sum_u64(data, mask, idx, n, flip, grid); break;
    case OR_U32: sum_u32(data, mask, idx, n, flip, grid); break;
    case OR_U16: sum_u16(data, mask, idx, n, flip, grid); break;
    case OR_U8: sum_u8(data, mask, idx, n, flip, grid); break;
    case OR_BOOL: sum_b(data, mask, idx, n, flip, grid); break;
    default: return -1;
    }
    return 0;
}

/* AggMax / AggMin (superagg.cpp:194-287).  grid has the storage type T.
 * std::max(a, b) == (a < b) ? b : a ; std::min(a, b) == (b < a) ? b : a,
 * called as std::max(value, grid[i]) / std::min(value, grid[i]). */
#define DEF_MINMAX(SUF, T, BS, ISFLT)                                                        \
    static void minmax_##SUF(int is_max, const T *data, const uint8_t *mask,                  \
                             const uint64_t *idx, uint64_t n, int flip, T *grid) {            \
        for (uint64_t j = 0; j < n; j++) {                                                    \
            if (mask && mask[j] != 1) continue;                                               \
            T value = data[j];                                                                \
            if (flip) value = BS(value);                                                      \
            if (ISFLT && value != value) continue;                                            \
            T g = grid[idx[j]];                                                               \
            if (is_max) grid[idx[j]] = (value < g) ? g : value;                               \
            else grid[idx[j]] = (g < value) ? g : value;                                      \
        }                                                                                     \
    }
DEF_MINMAX(f64, double, bs_f64, 1)
DEF_MINMAX(f32, float, bs_f32, 1)
DEF_MINMAX(i64, int64_t, bs_i64, 0)
DEF_MINMAX(i32, int32_t, bs_i32, 0)
DEF_MINMAX(i16, int16_t, bs_i16, 0)
DEF_MINMAX(i8, int8_t, bs_i8, 0)
DEF_MINMAX(u64, uint64_t, bs_u64, 0)
DEF_MINMAX(u32, uint32_t, bs_u32, 0)
DEF_MINMAX(u16, uint16_t, bs_u16, 0)
DEF_MINMAX(u8, uint8_t, bs_u8, 0)
DEF_MINMAX(b, orbool, bs_b, 0)

int or_agg_minmax(int is_max, int dtype, int flip, const void *data, const uint8_t *mask,
                  const uint64_t *idx, uint64_t n, void *grid) {
    switch (dtype) {
    case OR_F64: minmax_f64(is_max, data, mask, idx, n, flip, grid); break;
    case OR_F32: minmax_f32(is_max, data, mask, idx, n, flip, grid); break;
    case OR_I64: minmax_i64(is_max, data, mask, idx, n, flip, grid); break;
    case OR_I32: minmax_i32(is_max, data, mask, idx, n, flip, grid); break;
    case OR_I16: minmax_i16(is_max, data, mask, idx, n, flip, grid); break;
    case OR_I8: minmax_i8(is_max, data, mask, idx, n, flip, grid); break;
    case OR_U64: minmax_u64(is_max, data, mask, idx, n, flip, grid); break;
    case OR_U32: minmax_u32(is_max, data, mask, idx, n, flip, grid); break;
    case OR_U16: minmax_u16(is_max, data, mask, idx, n, flip, grid); break;
    case OR_U8: minmax_u8(is_max, data, mask, idx, n, flip, grid); break;
    case OR_BOOL: minmax_b(is_max, data, mask, idx, n, flip, grid); break;
    default: return -1;
    }
    return 0;
}

/* AggFirst<T> (superagg.cpp:481-505).  Masks are ignored by the reference
 * ("TODO: masked support").  Update iff value and order are not NaN and
 * order < grid_order[i] (strict). */
#define DEF_FIRST(SUF, T, BS, ISFLT)                                                         \
    static void first_##SUF(const T *data, const T *order, const uint64_t *idx, uint64_t n,   \
                            int flip, T *grid, T *grid_order) {                               \
        for (uint64_t j = 0; j < n; j++) {                                                    \
            T value = data[j];                                                                \
            T value_order = order[j];                                                         \
            if (flip) { value = BS(value); value_order = BS(value_order); }                   \
            if (ISFLT && (value != value || value_order != value_order)) continue;            \
            uint64_t i = idx[j];                                                              \
            if (value_order < grid_order[i]) {                                                \
                grid[i] = value;                                                              \
                grid_order[i] = value_order;                                                  \
            }                                                                                 \
        }                                                                                     \
    }
DEF_FIRST(f64, double, bs_f64, 1)
DEF_FIRST(f32, float, bs_f32, 1)
DEF_FIRST(i64, int64_t, bs_i64, 0)
DEF_FIRST(i32, int32_t, bs_i32, 0)
DEF_FIRST(i16, int16_t, bs_i16, 0)
DEF_FIRST(i8, int8_t, bs_i8, 0)
DEF_FIRST(u64, uint64_t, bs_u64, 0)
DEF_FIRST(u32, uint32_t, bs_u32, 0)
DEF_FIRST(u16, uint16_t, bs_u16, 0)
DEF_FIRST(u8, uint8_t, bs_u8, 0)
DEF_FIRST(b, orbool, bs_b, 0)

int or_agg_first(int dtype, int flip, const void *data, const void *order, const uint64_t *idx,
                 uint64_t n, void *grid, void *grid_order) {
    switch (dtype) {
    case OR_F64: first_f64(data, order, idx, n, flip, grid, grid_order); break;
    case OR_F32: first_f32(data, order, idx, n, flip, grid, grid_order); break;
    case OR_I64: first_i64(data, order, idx, n, flip, grid, grid_order); break;
    case OR_I32: first_i32(data, order, idx, n, flip, grid, grid_order); break;
    case OR_I16: first_i16(data, order, idx, n, flip, grid, grid_order); break;
    case OR_I8: first_i8(data, order, idx, n, flip, grid, grid_order); break;
    case OR_U64: first_u64(data, order, idx, n, flip, grid, grid_order); break;
    case OR_U32: first_u32(data, order, idx, n, flip, grid, grid_order); break;
    case OR_U16: first_u16(data, order, idx, n, flip, grid, grid_order); break;
    case OR_U8: first_u8(data, order, idx, n, flip, grid, grid_order); break;
    case OR_BOOL: first_b(data, order, idx, n, flip, grid, grid_order); break;
    default: return -1;
    }
    return 0;
}

/* AggSumMoment<T> (superagg.cpp:406-432): the value is converted to the
 * upcast grid type BEFORE the (reference's) byte swap, then pow(value, m)
 * is added (int64 grids: grid = (int64)((double)grid + pow)). */
#define DEF_MOMENT(SUF, T, G, BSG, ISFLT)                                                    \
    static void moment_##SUF(const T *data, const uint8_t *mask, const uint64_t *idx,         \
                             uint64_t n, int flip, uint32_t moment, G *grid) {                \
        for (uint64_t j = 0; j < n; j++) {                                                    \
            if (mask && mask[j] != 1) continue;                                               \
            G value = (G)data[j];                                                             \
            if (flip) value = BSG(value);                                                     \
            if (ISFLT && value != value) continue;                                            \
            grid[idx[j]] = (G)((double)grid[idx[j]] + pow((double)value, (double)moment));     \
        }                                                                                     \
    }
DEF_MOMENT(f64, double, double, bs_f64, 1)
DEF_MOMENT(f32, float, double, bs_f64, 1)
DEF_MOMENT(i64, int64_t, int64_t, bs_i64, 0)
DEF_MOMENT(i32, int32_t, int64_t, bs_i64, 0)
DEF_MOMENT(i16, int16_t, int64_t, bs_i64, 0)
DEF_MOMENT(i8, int8_t, int64_t, bs_i64, 0)
DEF_MOMENT(u64, uint64_t, uint64_t, bs_u64, 0)
DEF_MOMENT(u32, uint32_t, uint64_t, bs_u64, 0)
DEF_MOMENT(u16, uint16_t, uint64_t, bs_u64, 0)
DEF_MOMENT(u8, uint8_t, uint64_t, bs_u64, 0)
DEF_MOMENT(b, orbool, int64_t, bs_i64, 0)

int or_agg_sum_moment(int dtype, int flip, const void *data, const uint8_t *mask,
                      const uint64_t *idx, uint64_t n, uint32_t moment, void *grid) {
    switch (dtype) {
    case OR_F64: moment_f64(data, mask, idx, n, flip, moment, grid); break;
    case OR_F32: moment_f32(data, mask, idx, n, flip, moment, grid); break;
    case OR_I64: moment_i64(data, mask, idx, n, flip, moment, grid); break;
    case OR_I32: moment_i32(data, mask, idx, n, flip, moment, grid); break;
    case OR_I16: moment_i16(data, mask, idx, n, flip, moment, grid); break;
    case OR_I8: moment_i8(data, mask, idx, n, flip, moment, grid); break;
    case OR_U64: moment_u64(data, mask, idx, n, flip, moment, grid); break;
    case OR_U32: moment_u32(data, mask, idx, n, flip, moment, grid); break;
    case OR_U16: moment_u16(data, mask, idx, n, flip, moment, grid); break;
    case OR_U8: moment_u8(data, mask, idx, n, flip, moment, grid); break;
    case OR_BOOL: moment_b(data, mask, idx, n, flip, moment, grid); break;
    default: return -1;
    }
    return 0;
}

/* ---------------------------------------------------------------------- */
/* Hash (hash.hpp:25-30): splitmix64 finaliser                             */
/* ---------------------------------------------------------------------- */
uint64_t or_hash64(uint64_t x) {
    x = (x ^ (x >> 30)) * (uint64_t)0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * (uint64_t)0x94d049bb133111ebULL;
    x = x ^ (x >> 31);
    return x;
}

/* ---------------------------------------------------------------------- */
/* ordered_set<int32/int64> restatement (hash_primitives.hpp:96-281,       */
/* 417-583; hash.hpp:124-257) for non-null, non-NaN integer keys,          */
/* processed in row order (one thread):                                   */
/*   map_index = hash(key) % nmaps; a new key gets ordinal = map.size();   */
/*   key_array[ordinal + offsets[map]] = key; offsets = prefix sums.       */
/* Open addressing with linear probing inside each map (the reference uses */
/* tsl::hopscotch_map; ordinals do not depend on the map internals,        */
/* SURVEY.md §8c).  or_set_* operate on int64-widened keys.                */
/* ---------------------------------------------------------------------- */
typedef struct {
    int64_t *keys;
    int64_t *vals;   /* ordinal within the map, -1 = empty */
    uint64_t cap;    /* power of two */
    uint64_t size;
} or_map;

typedef struct {
    int nmaps;
    or_map *maps;
} or_set;

static void map_init(or_map *m, uint64_t cap) {
    m->cap = cap;
    m->size = 0;
    m->keys = (int64_t *)malloc(sizeof(int64_t) * cap);
    m->vals = (int64_t *)malloc(sizeof(int64_t) * cap);
    for (uint64_t i = 0; i < cap; i++) m->vals[i] = -1;
}

static int64_t map_find(const or_map *m, int64_t key, uint64_t h) {
    uint64_t pos = h & (m->cap - 1);
    for (;;) {
        if (m->vals[pos] < 0) return -1;
        if (m->keys[pos] == key) return m->vals[pos];
        pos = (pos + 1) & (m->cap - 1);
    }
}

static void map_grow(or_map *m);

static int64_t map_insert(or_map *m, int64_t key, uint64_t h) {
    if ((m->size + 1) * 2 > m->cap) map_grow(m);
    uint64_t pos = h & (m->cap - 1);
    for (;;) {
        if (m->vals[pos] < 0) {
            m->keys[pos] = key;
            m->vals[pos] = (int64_t)m->size;
            m->size++;
            return m->vals[pos];
        }
        if (m->keys[pos] == key) return m->vals[pos];
        pos = (pos + 1) & (m->cap - 1);
    }
}

static void map_grow(or_map *m) {
    or_map n;
    map_init(&n, m->cap * 2);
    for (uint64_t i = 0; i < m->cap; i++) {
        if (m->vals[i] >= 0) {
            uint64_t h = or_hash64((uint64_t)m->keys[i]);
            uint64_t pos = h & (n.cap - 1);
            while (n.vals[pos] >= 0) pos = (pos + 1) & (n.cap - 1);
            n.keys[pos] = m->keys[i];
            n.vals[pos] = m->vals[i];
        }
    }
    n.size = m->size;
    free(m->keys);
    free(m->vals);
    *m = n;
}

void *or_set_create(int nmaps) {
    or_set *s = (or_set *)malloc(sizeof(or_set));
    s->nmaps = nmaps;
    s->maps = (or_map *)malloc(sizeof(or_map) * nmaps);
    for (int i = 0; i < nmaps; i++) map_init(&s->maps[i], 16);
    return s;
}

void or_set_destroy(void *p) {
    or_set *s = (or_set *)p;
    for (int i = 0; i < s->nmaps; i++) {
        free(s->maps[i].keys);
        free(s->maps[i].vals);
    }
    free(s->maps);
    free(s);
}

/* keys are widened to int64 by the caller (hash<int32> sign-extends:
 * hash.hpp:53-59); the hash sees the uint64 bit pattern. */
void or_set_update(void *p, const int64_t *keys, uint64_t n) {
    or_set *s = (or_set *)p;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t h = or_hash64((uint64_t)keys[i]);
        or_map *m = &s->maps[h % (uint64_t)s->nmaps];
        map_insert(m, keys[i], h);
    }
}

uint64_t or_set_length(void *p) {
    or_set *s = (or_set *)p;
    uint64_t c = 0;
    for (int i = 0; i < s->nmaps; i++) c += s->maps[i].size;
    return c;
}

void or_set_key_array(void *p, int64_t *out) {
    or_set *s = (or_set *)p;
    uint64_t offset = 0;
    for (int mi = 0; mi < s->nmaps; mi++) {
        or_map *m = &s->maps[mi];
        for (uint64_t i = 0; i < m->cap; i++)
            if (m->vals[i] >= 0) out[offset + (uint64_t)m->vals[i]] = m->keys[i];
        offset += m->size;
    }
}

/* _map_ordinal (hash_primitives.hpp:556-583): -1 for unknown keys */
void or_set_map_ordinal(void *p, const int64_t *keys, uint64_t n, int64_t *out) {
    or_set *s = (or_set *)p;
    int64_t *offsets = (int64_t *)malloc(sizeof(int64_t) * s->nmaps);
    int64_t off = 0;
    for (int i = 0; i < s->nmaps; i++) {
        offsets[i] = off;
        off += (int64_t)s->maps[i].size;
    }
    for (uint64_t i = 0; i < n; i++) {
        uint64_t h = or_hash64((uint64_t)keys[i]);
        uint64_t mi = h % (uint64_t)s->nmaps;
        int64_t v = map_find(&s->maps[mi], keys[i], h);
        out[i] = v < 0 ? -1 : v + offsets[mi];
    }
    free(offsets);
}

/* ---------------------------------------------------------------------- */
/* NaN-ignoring min/max (vaexfast.cpp:1043-1055 op_min_max; the limits     */
/* pre-pass of DataFrame.minmax, dataframe.py:1276-1333).                  */
/* ---------------------------------------------------------------------- */
void or_minmax_f64(const double *x, uint64_t n, double *out_min, double *out_max) {
    double lo = INFINITY, hi = -INFINITY;
    for (uint64_t i = 0; i < n; i++) {
        double v = x[i];
        if (v < lo) lo = v;
        if (v > hi) hi = v;
    }
    *out_min = lo;
    *out_max = hi;
}

/* ---------------------------------------------------------------------- */
/* CPU baseline drivers (bench.py cpu_baseline leg only).                  */
/* Reference threading model: ExecutorLocal splits rows into chunks of     */
/* chunk_size (execution.py:149-156), ThreadPoolIndex runs them on T       */
/* threads, each chunk aggregates into one of `nparts` private grids       */
/* (cpu.py:487-499 ideal_splits), then parts[0].reduce(parts[1:])          */
/* serially (execution.py:285, superagg.cpp:160-167,354-361).              */
/* ---------------------------------------------------------------------- */
int or_bench_grid2d(const double *x, const double *y, const double *w, uint64_t n,
                    double xmin, double xmax, double ymin, double ymax, uint64_t bins,
                    int nparts, int nthreads, uint64_t chunk, int64_t *count_out,
                    double *sum_out) {
    const uint64_t shape = bins + 3;
    const uint64_t cells = shape * shape;
    int64_t **counts = (int64_t **)malloc(sizeof(int64_t *) * nparts);
    double **sums = (double **)malloc(sizeof(double *) * nparts);
    for (int p = 0; p < nparts; p++) {
        counts[p] = (int64_t *)calloc(cells, sizeof(int64_t));
        sums[p] = w ? (double *)calloc(cells, sizeof(double)) : NULL;
    }
    const uint64_t nchunks = (n + chunk - 1) / chunk;
    const double sx = 1. / (xmax - xmin), sy = 1. / (ymax - ymin);
    int used = nthreads < nparts ? nthreads : nparts;
#pragma omp parallel for schedule(dynamic, 1) num_threads(used)
    for (uint64_t c = 0; c < nchunks; c++) {
#ifdef _OPENMP
        int part = omp_get_thread_num();
#else
        int part = 0;
#endif
        int64_t *cg = counts[part];
        double *sg = sums[part];
        uint64_t i1 = c * chunk, i2 = i1 + chunk < n ? i1 + chunk : n;
        uint64_t idx[1024];
        for (uint64_t b = i1; b < i2; b += 1024) {
            uint64_t len = i2 - b < 1024 ? i2 - b : 1024;
            for (uint64_t i = 0; i < len; i++) {
                double s = (x[b + i] - xmin) * sx;
                uint64_t ix = 0;
                if (s != s) ix = 0;
                else if (s < 0) ix = 1;
                else if (s >= 1) ix = bins + 2;
                else ix = (uint64_t)((int)(s * (double)bins) + 2);
                double t = (y[b + i] - ymin) * sy;
                uint64_t iy = 0;
                if (t != t) iy = 0;
                else if (t < 0) iy = 1;
                else if (t >= 1) iy = bins + 2;
                else iy = (uint64_t)((int)(t * (double)bins) + 2);
                idx[i] = ix + iy * shape;
            }
            for (uint64_t i = 0; i < len; i++) cg[idx[i]] += 1;
            if (sg)
                for (uint64_t i = 0; i < len; i++) {
                    double v = w[b + i];
                    if (v == v) sg[idx[i]] += v;
                }
        }
    }
    for (uint64_t i = 0; i < cells; i++) {
        int64_t c = 0;
        double s = 0;
        for (int p = 0; p < nparts; p++) {
            c += counts[p][i];
            if (w) s = s + sums[p][i];
        }
        count_out[i] = c;
        if (w && sum_out) sum_out[i] = s;
    }
    for (int p = 0; p < nparts; p++) {
        free(counts[p]);
        free(sums[p]);
    }
    free(counts);
    free(sums);
    return used;
}

/* C1 (BASELINE configs[0]): df.count(binby='x', shape=bins) on float64 rows with
 * limits=None, as ExecutorLocal runs it: the limits pre-pass (DataFrame.minmax ->
 * TaskStatistic OP_MIN_MAX, per-chunk vaexfast statisticNd<op_min_max> on T threads,
 * nanmin/nanmax reduce; dataframe.py:1276-1333, vaexfast.cpp:1043-1055, tasks.py:173-185),
 * then the count pass into one private 1-d grid per thread (a 259-cell part is < 1e5
 * bytes, so ideal_splits = T, cpu.py:487-499), chunk = min(1 Mi, max(1024, ceil(n/T)))
 * (execution.py:149-156), serial reduce.  do_minmax = 0 takes lim[] as given. */
int or_bench_count1d(const double *x, uint64_t n, int nthreads, uint64_t bins, int do_minmax, double *lim,
                     int64_t *count_out) {
    uint64_t chunk = (n + nthreads - 1) / nthreads;
    if (chunk < 1024) chunk = 1024;
    if (chunk > (1u << 20)) chunk = 1u << 20;
    const uint64_t nchunks = (n + chunk - 1) / chunk;
    if (do_minmax) {
        double *los = (double *)malloc(sizeof(double) * nthreads), *his = (double *)malloc(sizeof(double) * nthreads);
        for (int t = 0; t < nthreads; t++) {
            los[t] = INFINITY;
            his[t] = -INFINITY;
        }
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
        for (uint64_t c = 0; c < nchunks; c++) {
#ifdef _OPENMP
            int t = omp_get_thread_num();
#else
            int t = 0;
#endif
            uint64_t i1 = c * chunk, i2 = i1 + chunk < n ? i1 + chunk : n;
            double lo = los[t], hi = his[t];
            for (uint64_t i = i1; i < i2; i++) {
                double v = x[i];
                if (v < lo) lo = v;  /* NaN fails both compares */
                if (v > hi) hi = v;
            }
            los[t] = lo;
            his[t] = hi;
        }
        double lo = INFINITY, hi = -INFINITY;
        for (int t = 0; t < nthreads; t++) {
            if (los[t] < lo) lo = los[t];
            if (his[t] > hi) hi = his[t];
        }
        lim[0] = lo;
        lim[1] = hi;
        free(los);
        free(his);
    }
    const uint64_t shape = bins + 3;
    int64_t *grids = (int64_t *)calloc(shape * (uint64_t)nthreads, sizeof(int64_t));
    const double vmin = lim[0], scale = 1. / (lim[1] - lim[0]);
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
    for (uint64_t c = 0; c < nchunks; c++) {
#ifdef _OPENMP
        int t = omp_get_thread_num();
#else
        int t = 0;
#endif
        int64_t *g = grids + shape * (uint64_t)t;
        uint64_t i1 = c * chunk, i2 = i1 + chunk < n ? i1 + chunk : n;
        uint64_t idx[1024];
        for (uint64_t b = i1; b < i2; b += 1024) {
            uint64_t len = i2 - b < 1024 ? i2 - b : 1024;
            for (uint64_t i = 0; i < len; i++) {
                double s = (x[b + i] - vmin) * scale;
                uint64_t ix;
                if (s != s) ix = 0;
                else if (s < 0) ix = 1;
                else if (s >= 1) ix = bins + 2;
                else ix = (uint64_t)((int)(s * (double)bins) + 2);
                idx[i] = ix;
            }
            for (uint64_t i = 0; i < len; i++) g[idx[i]] += 1;
        }
    }
    for (uint64_t i = 0; i < shape; i++) {
        int64_t c = 0;
        for (int t = 0; t < nthreads; t++) c += grids[shape * (uint64_t)t + i];
        count_out[i] = c;
    }
    free(grids);
    return nthreads;
}

/* groupby(int32 key).agg({v: [sum, count]}) as the reference runs it
 * (groupby.py:97-168, cpu.py:147-195): pass 1 builds ordered_set with
 * nmaps = 7*T maps under per-map locks (hash_primitives.hpp:96-247), pass 2
 * map_ordinal + BinnerOrdinal + AggSum/AggCount into private grids.
 * Returns number of groups; keys_out/sum_out/count_out (capacity cap) are
 * in the set's key_array order. */
int64_t or_bench_groupby_i32(const int32_t *keys, const double *v, uint64_t n, int nthreads,
                             int nparts, uint64_t chunk, int64_t cap, int64_t *keys_out,
                             double *sum_out, int64_t *count_out) {
    const int nmaps = 7 * nthreads;
    or_set *s = (or_set *)or_set_create(nmaps);
#ifdef _OPENMP
    omp_lock_t *locks = (omp_lock_t *)malloc(sizeof(omp_lock_t) * nmaps);
    for (int i = 0; i < nmaps; i++) omp_init_lock(&locks[i]);
#endif
    const uint64_t nchunks = (n + chunk - 1) / chunk;
#pragma omp parallel num_threads(nthreads)
    {
        int64_t **buckets = (int64_t **)malloc(sizeof(int64_t *) * nmaps);
        uint64_t *bsz = (uint64_t *)calloc(nmaps, sizeof(uint64_t));
        for (int m = 0; m < nmaps; m++) buckets[m] = (int64_t *)malloc(sizeof(int64_t) * chunk);
#pragma omp for schedule(dynamic, 1)
        for (uint64_t c = 0; c < nchunks; c++) {
            uint64_t i1 = c * chunk, i2 = i1 + chunk < n ? i1 + chunk : n;
            for (int m = 0; m < nmaps; m++) bsz[m] = 0;
            for (uint64_t i = i1; i < i2; i++) {
                int64_t k = keys[i];
                uint64_t m = or_hash64((uint64_t)k) % (uint64_t)nmaps;
                buckets[m][bsz[m]++] = k;
            }
            for (int m = 0; m < nmaps; m++) {
                if (!bsz[m]) continue;
#ifdef _OPENMP
                omp_set_lock(&locks[m]);
#endif
                for (uint64_t j = 0; j < bsz[m]; j++)
                    map_insert(&s->maps[m], buckets[m][j], or_hash64((uint64_t)buckets[m][j]));
#ifdef _OPENMP
                omp_unset_lock(&locks[m]);
#endif
            }
        }
        for (int m = 0; m < nmaps; m++) free(buckets[m]);
        free(buckets);
        free(bsz);
    }
    int64_t ngroups = (int64_t)or_set_length(s);
    int64_t *offsets = (int64_t *)malloc(sizeof(int64_t) * nmaps);
    {
        int64_t off = 0;
        for (int i = 0; i < nmaps; i++) {
            offsets[i] = off;
            off += (int64_t)s->maps[i].size;
        }
    }
    const uint64_t shape = (uint64_t)ngroups + 3;
    int64_t **counts = (int64_t **)malloc(sizeof(int64_t *) * nparts);
    double **sums = (double **)malloc(sizeof(double *) * nparts);
    for (int p = 0; p < nparts; p++) {
        counts[p] = (int64_t *)calloc(shape, sizeof(int64_t));
        sums[p] = (double *)calloc(shape, sizeof(double));
    }
    int used = nthreads < nparts ? nthreads : nparts;
#pragma omp parallel for schedule(dynamic, 1) num_threads(used)
    for (uint64_t c = 0; c < nchunks; c++) {
#ifdef _OPENMP
        int part = omp_get_thread_num();
#else
        int part = 0;
#endif
        uint64_t i1 = c * chunk, i2 = i1 + chunk < n ? i1 + chunk : n;
        for (uint64_t i = i1; i < i2; i++) {
            int64_t k = keys[i];
            uint64_t h = or_hash64((uint64_t)k);
            uint64_t mi = h % (uint64_t)nmaps;
            int64_t o = map_find(&s->maps[mi], k, h);
            o = o < 0 ? -1 : o + offsets[mi];
            uint64_t index = o < 0 ? 1 : (uint64_t)o + 2;
            counts[part][index] += 1;
            double val = v[i];
            if (val == val) sums[part][index] += val;
        }
    }
    if (ngroups <= cap) {
        or_set_key_array(s, keys_out);
        for (int64_t g = 0; g < ngroups; g++) {
            int64_t c = 0;
            double sm = 0;
            for (int p = 0; p < nparts; p++) {
                c += counts[p][g + 2];
                sm = sm + sums[p][g + 2];
            }
            count_out[g] = c;
            sum_out[g] = sm;
        }
    }
    for (int p = 0; p < nparts; p++) {
        free(counts[p]);
        free(sums[p]);
    }
    free(counts);
    free(sums);
    free(offsets);
#ifdef _OPENMP
    for (int i = 0; i < nmaps; i++) omp_destroy_lock(&locks[i]);
    free(locks);
#endif
    or_set_destroy(s);
    return ngroups;
}
