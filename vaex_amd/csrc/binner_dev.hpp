// Device-side binner index math shared by binning.hip and tiled.hip.
//   BinnerScalar<T>::to_bins   packages/vaex-core/src/superagg_binners.cpp:14-56
//   BinnerOrdinal<T>::to_bins  packages/vaex-core/src/superagg_binners.cpp:104-142
//   Grid strides / sum of index*stride  packages/vaex-core/src/agg.hpp:60-69,113-123
#pragma once
#include "engine.hpp"

namespace vh {

#define VH_DEV_DISPATCH(code, T, ...)                                                       \
    switch (code) {                                                                         \
    case VH_F64: { using T = double; __VA_ARGS__; }                                         \
    case VH_F32: { using T = float; __VA_ARGS__; }                                          \
    case VH_I64: { using T = int64_t; __VA_ARGS__; }                                        \
    case VH_I32: { using T = int32_t; __VA_ARGS__; }                                        \
    case VH_I16: { using T = int16_t; __VA_ARGS__; }                                        \
    case VH_I8: { using T = int8_t; __VA_ARGS__; }                                          \
    case VH_U64: { using T = uint64_t; __VA_ARGS__; }                                       \
    case VH_U32: { using T = uint32_t; __VA_ARGS__; }                                       \
    case VH_U16: { using T = uint16_t; __VA_ARGS__; }                                       \
    case VH_U8: { using T = uint8_t; __VA_ARGS__; }                                         \
    default: { using T = vbool; __VA_ARGS__; }                                              \
    }

__device__ inline bool operator<(vbool a, vbool b) { return a.v < b.v; }

// BinnerScalar<T>::to_bins (superagg_binners.cpp:14-56), on an already loaded raw value
template <typename T> __device__ inline uint64_t scalar_cell(const BinnerDev &b, T raw, bool masked) {
    T value = b.flip ? bswap_v(raw) : raw;
    double value_double = to_double(value);
    double scaled = (value_double - b.vmin) * b.scale;
    if (scaled != scaled || masked) return 0;  // nan -> 0
    if (scaled < 0) return 1;                  // underflow -> 1
    if (scaled >= 1) return b.bins + 2;        // overflow (incl. vmax) -> bins+2
    return (uint64_t)(int64_t)((int)(scaled * (double)b.bins) + 2);
}

template <typename T> __device__ inline uint64_t scalar_index(const BinnerDev &b, uint64_t i) {
    return scalar_cell<T>(b, reinterpret_cast<const T *>(b.data)[i], b.mask ? (b.mask[i] == 1) : false);
}

// BinnerOrdinal<T>::to_bins (superagg_binners.cpp:104-142): the subtraction of
// the uint64 min_value happens before the byte swap, as in the reference.
template <typename T> __device__ inline uint64_t ordinal_cell(const BinnerDev &b, T raw, bool masked) {
    if constexpr (is_float_t<T>::value) {
        T value = raw - (T)b.min_value;
        if (b.flip) value = bswap_v(value);
        if (value != value || masked) return 0;
        if (value < 0) return 1;
        if (value >= (T)b.ordinal_count) return b.ordinal_count + 2;
        return (uint64_t)(value + 2);
    } else if constexpr (sizeof(T) == 1 && !is_signed_int_t<T>::value && !std::is_same<T, uint8_t>::value) {
        // bool: (int)b - min_value converted back to bool
        uint64_t value = (((uint64_t)raw.v) - b.min_value) != 0;
        if (masked) return 0;
        if (value >= b.ordinal_count) return b.ordinal_count + 2;
        return value + 2;
    } else {
        T value = (T)((uint64_t)(int64_t)raw - b.min_value);
        if (b.flip) value = bswap_v(value);
        if (masked) return 0;
        if constexpr (is_signed_int_t<T>::value) {
            if (value < 0) return 1;
        }
        if ((uint64_t)(int64_t)value >= b.ordinal_count) return b.ordinal_count + 2;
        return (uint64_t)((int64_t)value + 2);
    }
}

template <typename T> __device__ inline uint64_t ordinal_index(const BinnerDev &b, uint64_t i) {
    return ordinal_cell<T>(b, reinterpret_cast<const T *>(b.data)[i], b.mask ? (b.mask[i] == 1) : false);
}

// BinnerOrdinal over _ordinal_values(key, set): map_ordinal (hash_primitives.hpp:556-583)
// fused with the ordinal binner.  Masked keys go to the null ordinal when the set has
// one (the null group), else to cell 0.
template <typename T> __device__ inline uint64_t set_index(const BinnerDev &b, uint64_t i) {
    int64_t o;
    if (b.mask && b.mask[i] == 1) {
        if (b.set.null_ord < 0) return 0;
        o = b.set.null_ord;
    } else {
        o = set_lookup<T>(b.set, reinterpret_cast<const T *>(b.data)[i]);
    }
    if (o < 0) return 1;
    if ((uint64_t)o >= b.ordinal_count) return b.ordinal_count + 2;
    return (uint64_t)o + 2;
}

__device__ inline uint64_t binner_index(const BinnerDev &b, uint64_t i) {
    if (b.kind == 0) {
        VH_DEV_DISPATCH(b.dtype, T, return scalar_index<T>(b, i));
    } else if (b.kind == 1) {
        VH_DEV_DISPATCH(b.dtype, T, return ordinal_index<T>(b, i));
    } else {
        VH_DEV_DISPATCH(b.dtype, T, return set_index<T>(b, i));
    }
}

__device__ inline uint64_t plan_index(const BinPlan &p, uint64_t i) {
    uint64_t s = 0;
    for (int d = 0; d < p.nb; d++) s += binner_index(p.b[d], i) * p.b[d].stride;
    return s;
}

}  // namespace vh
