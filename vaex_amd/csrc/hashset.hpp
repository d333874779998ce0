// GPU open-address hash set shared by hashset.hip (ordered_set) and the
// fused set-ordinal binner in binning.hip.
//
// Layout in HBM: `tab[cap]` of 16-byte slots {key bits zero-extended (EMPTY = ~0),
// first row the key was seen at (the ordinal order)}, so an insert probe and its
// first-row update touch one cache line; after sealing, a lookup table (below).
// Linear probing from _hash64(bits) (the reference's splitmix64 finaliser,
// hash.hpp:25-30).
// 64-bit integer keys whose bits equal EMPTY (int64 -1, uint64 max) live in a
// side slot ("special").  NaN and null keys get their own ordinals like the
// reference's nan_value/null_value (hash_primitives.hpp:436-450).
#pragma once
#include "common.hpp"

namespace vh {

constexpr uint64_t SET_EMPTY = ~0ULL;
constexpr int SET_MAX_PROBE = 256;

__host__ __device__ inline uint64_t hash64(uint64_t x) {
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}

template <typename T> __device__ inline uint64_t key_bits(T v) {
    if constexpr (sizeof(T) == 8) {
        uint64_t u;
        __builtin_memcpy(&u, &v, 8);
        return u;
    } else if constexpr (sizeof(T) == 4) {
        uint32_t u;
        __builtin_memcpy(&u, &v, 4);
        return u;
    } else if constexpr (sizeof(T) == 2) {
        uint16_t u;
        __builtin_memcpy(&u, &v, 2);
        return u;
    } else {
        uint8_t u;
        __builtin_memcpy(&u, &v, 1);
        return u;
    }
}

// Lookup table built when the set is sealed: one 8-byte slot (ordinal << 32 | key bits)
// for keys of <= 4 bytes, one 16-byte slot {key bits, ordinal} for 8-byte keys, so a
// probe touches one cache line; EMPTY slots are all ones.
struct SetDev {
    const uint64_t *lut;
    int wide;             // 0: packed 8-byte slots, 1: {key, ord} 16-byte slots
    uint64_t cap_mask;
    int64_t nan_ord;      // ordinal of NaN (0x7fffffff when absent, as the reference)
    int64_t null_ord;     // ordinal of null / masked keys (-1 when absent)
    int64_t special_ord;  // ordinal of the EMPTY-bits key, -1 when absent
};

// ordinal of a key, -1 if unknown (hash_primitives.hpp:567-580)
__device__ inline int64_t set_lookup_bits(const SetDev &s, uint64_t kb) {
    if (kb == SET_EMPTY) return s.special_ord;
    uint64_t pos = hash64(kb) & s.cap_mask;
    if (!s.wide) {
        for (int p = 0; p <= SET_MAX_PROBE; p++) {
            const uint64_t e = s.lut[pos];
            if (e == SET_EMPTY) return -1;
            if ((uint32_t)e == (uint32_t)kb) return (int64_t)(e >> 32);
            pos = (pos + 1) & s.cap_mask;
        }
    } else {
        for (int p = 0; p <= SET_MAX_PROBE; p++) {
            const ulonglong2 e = reinterpret_cast<const ulonglong2 *>(s.lut)[pos];
            if (e.x == kb) return (int64_t)e.y;
            if (e.x == SET_EMPTY) return -1;
            pos = (pos + 1) & s.cap_mask;
        }
    }
    return -1;
}

template <typename T> __device__ inline int64_t set_lookup(const SetDev &s, T v) {
    if (is_nan_v(v)) return s.nan_ord;
    return set_lookup_bits(s, key_bits(v));
}

}  // namespace vh

// host-side view used by binning.hip to build a SetDev for a binner
struct vh_set;
namespace vh {
SetDev set_device_view(vh_set *set);  // seals the set if needed
int set_dtype(const vh_set *set);
}  // namespace vh
