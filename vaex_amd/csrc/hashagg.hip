// Fused hash groupby: df.groupby(key).agg({count, sum, mean}) for one integer key column
// (1-, 2-, 4- or 8-byte keys; a multi-key groupby first combines its keys into one int64,
// groupby.py:248-288) and up to two value columns, in one pass over the data.
//
// The reference runs the groupby as two passes: pass 1 builds the ordered_set of the key
// (hash_primitives.hpp:96-281, via Grouper, groupby.py:97-168), pass 2 maps every row to
// its ordinal (_ordinal_values -> map_ordinal, hash_primitives.hpp:543-583) and scatters
// into the AggCount/AggSum grids through BinnerOrdinal (superagg_binners.cpp:104-142,
// superagg.cpp:155-192, 349-389).  Here both passes collapse into a hash-partitioned
// aggregation whose per-key results equal those grids (groupby.py:484-533 output):
//
//   sample -- ~1 M evenly spaced rows: per fine bucket (top 12 bits of the key hash) row
//             counts, and the sample's distinct keys in a small HBM table -> Chao1
//             estimate of the key count -> P = 2^p buckets of <= ~2300 keys each.
//   pass A -- workgroup w owns a row range; per 4096-row batch it hashes the keys
//             (murmur3 fmix32 / splitmix64 finaliser), ranks rows per bucket in LDS,
//             counting-sorts (key, value bits) by bucket through LDS and streams the runs
//             to per-(w, bucket) regions (the tile-partition scheme of tiled.hip with
//             buckets for tiles).
//   pass B -- work unit = (bucket, range of pass-A workgroups): the unit's entries are
//             aggregated in an LDS table (two-choice 4-slot groups, CAS insert,
//             ds_add_u64 / ds_add_f64), then merged into one HBM open-address table with
//             global atomics (one merge per distinct key per unit, not per row).
//   finish -- occupied HBM slots are compacted, radix-sorted by key (rocPRIM) and
//             gathered: groups come out sorted by key (a valid sort=False order -- the
//             reference's is hash/thread dependent -- and exactly the sort=True order).
//
// With P == 1 (few keys) pass A is skipped: every workgroup aggregates its row range of
// the raw columns straight into its LDS table ("direct").
//
// Key bits KB: uint32_t for keys of <= 4 bytes (the value as int32 / uint32), uint64_t for
// 8-byte keys.  The all-ones pattern of KB marks an EMPTY LDS slot; keys with the top two
// patterns (e.g. -1, -2) live in two side records.  The HBM table stores keys as uint64
// (EMPTY = all ones); an 8-byte key with that pattern lives in a side slot after the table.
//
// Overflow, never wrong results: a row whose key finds both of its LDS groups full is
// aggregated straight into the HBM table (a key may so be split between an LDS record and
// the HBM table, or between two LDS records: every record merges into the key's one HBM
// slot with atomics).  A pass-A region that is full
// (a sampling miss) also adds its rows to the HBM table directly.  An HBM table that grows
// past 3/4 full is rehashed x4 after the update; one that fills up fails the update
// (VH_ERR_RUNTIME) and the caller falls back to the ordered_set path.
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cmath>
#include <map>
#include <memory>
#include <mutex>
#include <type_traits>

#include "comm.hpp"
#include "engine.hpp"
#include "common.hpp"
#include "hashset.hpp"

namespace vh {

constexpr int HA_MAX_V = 2;
// one value column with 8-byte keys: packed 16-byte {key, value} entries (one store / load);
// with <= 4-byte keys the key and value arrays are separate, 12 bytes per entry instead of 16
// (pass A and pass B run at the HBM read/write ceiling, so bytes are time)
#ifndef VH_HA_PACK4
#define VH_HA_PACK4 0
#endif
template <typename KB, int NV> __host__ __device__ constexpr bool ha_packed() {
    return NV == 1 && (sizeof(KB) == 8 || VH_HA_PACK4);
}
constexpr int HA_THREADS = 512;            // pass A
constexpr int HA_RPT = 8;
constexpr int HA_BATCH = HA_THREADS * HA_RPT;
constexpr int HB_THREADS = 1024;           // pass B / direct
constexpr int HB_M = 8;                    // entries per lane per pass-B step
constexpr uint32_t HA_FINE_LOG2 = 12;      // sample histogram: top 12 hash bits
constexpr uint32_t HA_MAX_P_LOG2 = 11;
constexpr int HA_SAMPLE_BLOCKS = 256;
constexpr uint32_t HA_DEST_OVERFLOW = 0x80000000u;
constexpr int HA_MAX_PROBE = 1 << 14;

__host__ __device__ inline uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

// 32-bit hash of the key bits: its top bits pick the bucket, its low bits the LDS group
__device__ inline uint32_t ha_h(uint32_t kb) { return fmix32(kb); }
__device__ inline uint32_t ha_h(uint64_t kb) { return (uint32_t)(hash64(kb) >> 32); }

template <typename K> using kb_t = std::conditional_t<sizeof(K) == 8, uint64_t, uint32_t>;

// key bits: <= 4-byte keys as int32 (signed, sign-extended) / uint32; 8-byte keys verbatim
template <typename K> __device__ inline kb_t<K> ha_kb(K v) {
    if constexpr (sizeof(K) == 8) return __builtin_bit_cast(uint64_t, v);
    else if constexpr (std::is_signed_v<K>) return (uint32_t)(int32_t)v;
    else return (uint32_t)v;
}

template <typename KB> __host__ __device__ constexpr KB kb_empty() { return ~KB(0); }
template <typename KB> __host__ __device__ constexpr KB kb_closed() { return ~KB(0) - 1; }

// a value as the 8 bytes pass A carries: float -> double bits, signed -> int64,
// unsigned / bool -> uint64 (the AggSum upcast, superagg.cpp:289-346)
__device__ inline uint64_t ha_load_val(const void *p, int dtype, uint64_t i) {
    switch (dtype) {
    case VH_F64: return __builtin_bit_cast(uint64_t, static_cast<const double *>(p)[i]);
    case VH_F32: return __builtin_bit_cast(uint64_t, (double)static_cast<const float *>(p)[i]);
    case VH_I64: return (uint64_t) static_cast<const int64_t *>(p)[i];
    case VH_I32: return (uint64_t)(int64_t) static_cast<const int32_t *>(p)[i];
    case VH_I16: return (uint64_t)(int64_t) static_cast<const int16_t *>(p)[i];
    case VH_I8: return (uint64_t)(int64_t) static_cast<const int8_t *>(p)[i];
    case VH_U64: return static_cast<const uint64_t *>(p)[i];
    case VH_U32: return static_cast<const uint32_t *>(p)[i];
    case VH_U16: return static_cast<const uint16_t *>(p)[i];
    case VH_U8: return static_cast<const uint8_t *>(p)[i];
    default: return static_cast<const uint8_t *>(p)[i] != 0;  // bool
    }
}

// HBM open-address table (linear probing from hash64 of the key bits); slot `mask + 1` is
// the side slot of the 8-byte key whose bits equal EMPTY
struct HaTable {
    uint64_t *keys;  // SET_EMPTY = free
    unsigned long long *cnt;
    unsigned long long *sum[HA_MAX_V];  // double bits (float columns) or int64/uint64
    unsigned long long *nn[HA_MAX_V];   // non-NaN counts (float columns)
    uint64_t mask;
    uint32_t *used, *err;               // err bit 0: past max_used (grow), bit 1: key lost
    uint32_t max_used;
    uint32_t vfloat;                    // bit s: value column s is floating point
    uint32_t nnmask;                    // bit s: count the non-NaN values of column s
    int nv;
};

// new_keys: a workgroup-local (LDS) count of the keys this call inserted, added to g.used
// once per workgroup by the caller; nullptr = count in g.used directly (one same-address
// atomic per new key: ~1e8 of them for h2o q10's groups)
__device__ inline uint64_t ha_slot(const HaTable &g, uint64_t key, uint32_t *new_keys = nullptr) {
    if (key == SET_EMPTY) return g.mask + 1;
    uint64_t pos = hash64(key) & g.mask;
    for (int p = 0; p < HA_MAX_PROBE; p++) {
        uint64_t cur = __hip_atomic_load(&g.keys[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == key) return pos;
        if (cur == SET_EMPTY) {
            cur = atomicCAS((unsigned long long *)&g.keys[pos], (unsigned long long)SET_EMPTY,
                            (unsigned long long)key);
            if (cur == SET_EMPTY) {
                if (new_keys) atomicAdd(new_keys, 1u);
                else if (atomicAdd(g.used, 1u) >= g.max_used) atomicOr(g.err, 1u);
                return pos;
            }
            if (cur == key) return pos;
        }
        pos = (pos + 1) & g.mask;
    }
    atomicOr(g.err, 2u);
    return ~0ULL;
}

// one row straight into the HBM table (LDS table closed, or pass-A region full)
template <int NV> __device__ inline void ha_global_row(const HaTable &g, uint64_t key, const uint64_t *vb) {
    const uint64_t s = ha_slot(g, key);
    if (s == ~0ULL) return;
    atomicAdd(&g.cnt[s], 1ULL);
#pragma unroll
    for (int v = 0; v < NV; v++) {
        if ((g.vfloat >> v) & 1) {
            const double d = __builtin_bit_cast(double, vb[v]);
            if (d == d) {
                atomicAdd(reinterpret_cast<double *>(g.sum[v]) + s, d);
                atomicAdd(&g.nn[v][s], 1ULL);
            }
        } else {
            atomicAdd(&g.sum[v][s], (unsigned long long)vb[v]);
        }
    }
}

// ---- LDS table --------------------------------------------------------------------------
// Per slot: key bits; a counter word; the value sums; the non-NaN count of value 1.  Wide
// table (4096 slots): the counter is count(*) << 32 | non-NaN count of value 0 (one
// ds_add_u64 updates both: a unit holds < 2^32 rows).  Narrow table (8192 slots; 4-byte
// keys, at most one value, no count(v)): a 32-bit count(*), 16 B per slot -- twice the keys
// per bucket, so pass A needs half the buckets and its region runs are twice as long.
// Records S and S + 1 (S = slots) hold the keys whose bits are the two top patterns
// (kb_closed, kb_empty).
#ifndef VH_LT_NARROW_SLOTS
#define VH_LT_NARROW_SLOTS 8192
#endif
template <bool N> __host__ __device__ constexpr uint32_t lt_slots() { return N ? VH_LT_NARROW_SLOTS : 4096u; }
template <bool N> __host__ __device__ constexpr uint32_t lt_target_keys() { return N ? VH_LT_NARROW_SLOTS * 9 / 16 : 2300u; }

template <typename KB> struct LdsTable {
    KB *keys;                           // [S]
    unsigned long long *cn;             // [S + 2] (wide)
    uint32_t *cn32;                     // [S + 2] (narrow)
    unsigned long long *sum[HA_MAX_V];  // [S + 2]
    uint32_t *nn1;                      // [S + 2]
    uint32_t *used;
};

// every array starts 16-byte aligned: the key groups are read with ds_read_b128, which a
// misaligned base splits (an 8-byte misalignment doubled pass B's time)
__host__ __device__ constexpr size_t lt_a16(size_t b) { return (b + 15) & ~(size_t)15; }
__host__ __device__ constexpr size_t lt_bytes(int nv, int kbsize, bool narrow) {
    const size_t S = narrow ? VH_LT_NARROW_SLOTS : 4096;
    return lt_a16((size_t)(narrow ? 4 : 8) * (S + 2)) + lt_a16((size_t)8 * (S + 2)) * nv + (size_t)kbsize * S +
           (nv > 1 ? (size_t)4 * (S + 2) : 0) + 64;
}

template <typename KB, int NV, bool N> __device__ inline LdsTable<KB> lt_layout(unsigned char *raw) {
    constexpr uint32_t S = lt_slots<N>();
    LdsTable<KB> t{};
    unsigned char *p = raw;
    if constexpr (N) {
        t.cn32 = reinterpret_cast<uint32_t *>(p);
        p += lt_a16(4 * (S + 2));
    } else {
        t.cn = reinterpret_cast<unsigned long long *>(p);
        p += lt_a16(8 * (S + 2));
    }
    for (int v = 0; v < NV; v++) {
        t.sum[v] = reinterpret_cast<unsigned long long *>(p);
        p += lt_a16(8 * (S + 2));
    }
    t.keys = reinterpret_cast<KB *>(p);
    p += sizeof(KB) * S;
    t.nn1 = reinterpret_cast<uint32_t *>(p);
    if (NV > 1) p += 4 * (S + 2);
    t.used = reinterpret_cast<uint32_t *>(p);
    return t;
}

template <typename KB, int NV, bool N> __device__ inline void lt_init(const LdsTable<KB> &t, int nthreads) {
    constexpr uint32_t S = lt_slots<N>();
    for (uint32_t i = threadIdx.x; i < S + 2; i += nthreads) {
        if (i < S) t.keys[i] = kb_empty<KB>();
        if constexpr (N) t.cn32[i] = 0;
        else t.cn[i] = 0;
#pragma unroll
        for (int v = 0; v < NV; v++) t.sum[v][i] = 0;
        if constexpr (NV > 1) t.nn1[i] = 0;
    }
    if (threadIdx.x == 0) *t.used = 0;
}

template <typename KB, int NV, bool N>
__device__ inline void lt_bump(const LdsTable<KB> &t, const HaTable &g, uint32_t slot, const uint64_t *vb) {
    unsigned long long c = 1ULL << 32;
#pragma unroll
    for (int v = 0; v < NV; v++) {
        if ((g.vfloat >> v) & 1) {
            const double d = __builtin_bit_cast(double, vb[v]);
            if (d == d) {
                atomicAdd(reinterpret_cast<double *>(t.sum[v]) + slot, d);
                if (!N && ((g.nnmask >> v) & 1)) {
                    if (v == 0) c |= 1;
                    else atomicAdd(&t.nn1[slot], 1u);
                }
            }
        } else {
            atomicAdd(&t.sum[v][slot], (unsigned long long)vb[v]);
        }
    }
    if constexpr (N) atomicAdd(&t.cn32[slot], 1u);
    else atomicAdd(&t.cn[slot], c);
}

// four consecutive key slots: one ds_read_b128 (4-byte keys) or two (8-byte keys)
template <typename KB> struct alignas(16) KB4 {
    KB v[4];
};

__device__ inline uint32_t lt_cas(uint32_t *p, uint32_t cmp, uint32_t val) { return atomicCAS(p, cmp, val); }
__device__ inline uint64_t lt_cas(uint64_t *p, uint64_t cmp, uint64_t val) {
    return atomicCAS(reinterpret_cast<unsigned long long *>(p), (unsigned long long)cmp, (unsigned long long)val);
}

// Two-choice LDS table: a key lives in one of two 4-slot groups (g1 from its hash, g2 from a
// second mix of it), so a lookup reads both groups at once and almost never needs more:
// with ~2300 keys in 1024 groups the less loaded of two groups is rarely full (one-group
// linear probing displaced ~5 % of keys, and the lanes holding them serialised every wave:
// 4.6 of pass B's 7.3 ms, VH_HA_DEBUG ablation).  Insertion CASes the first EMPTY slot of
// the group with more room; two lanes inserting one new key at once may place it in both
// groups -- harmless, both records merge into the same HBM slot.  A key whose two groups are
// full aggregates straight into the HBM table.  Keys whose bits are EMPTY / CLOSED live in
// the two side records.
template <typename KB, bool N> __device__ inline void lt2_groups(KB kb, uint32_t &g1, uint32_t &g2) {
    constexpr uint32_t S = lt_slots<N>();
    const uint32_t h = ha_h(kb);
    g1 = (h & (S - 1)) >> 2;
    g2 = (fmix32(h ^ 0x9e3779b9u) & (S - 1)) >> 2;
}

template <typename KB> __device__ inline uint32_t lt2_find(const KB4<KB> &q1, const KB4<KB> &q2, uint32_t g1, uint32_t g2,
                                                         KB kb) {
    uint32_t slot = ~0u;
#pragma unroll
    for (int j = 3; j >= 0; j--) {
        if (q2.v[j] == kb) slot = 4 * g2 + j;
        if (q1.v[j] == kb) slot = 4 * g1 + j;
    }
    return slot;
}

// a key not found in either group: insert it (or find it, if another lane just did)
template <typename KB, int NV, bool N>
__device__ inline void lt2_insert(const LdsTable<KB> &t, const HaTable &g, KB kb, const uint64_t *vb) {
    constexpr KB EMPTY = kb_empty<KB>();
    uint32_t g1, g2;
    lt2_groups<KB, N>(kb, g1, g2);
    for (int it = 0; it < 64; it++) {
        const KB4<KB> q1 = *reinterpret_cast<const KB4<KB> *>(t.keys + 4 * g1);
        const KB4<KB> q2 = *reinterpret_cast<const KB4<KB> *>(t.keys + 4 * g2);
        const uint32_t hit = lt2_find(q1, q2, g1, g2, kb);
        if (hit != ~0u) {
            lt_bump<KB, NV, N>(t, g, hit, vb);
            return;
        }
        int e1 = 0, e2 = 0, f1 = -1, f2 = -1;
#pragma unroll
        for (int j = 3; j >= 0; j--) {
            if (q1.v[j] == EMPTY) {
                e1++;
                f1 = j;
            }
            if (q2.v[j] == EMPTY) {
                e2++;
                f2 = j;
            }
        }
        if (e1 == 0 && e2 == 0) break;
        const uint32_t pos = e1 >= e2 ? 4 * g1 + f1 : 4 * g2 + f2;
        const KB cur = lt_cas(&t.keys[pos], EMPTY, kb);
        if (cur == EMPTY || cur == kb) {
            lt_bump<KB, NV, N>(t, g, pos, vb);
            return;
        }
        // another key took the slot: read the groups again
    }
    ha_global_row<NV>(g, (uint64_t)kb, vb);
}

// M entries at once: both group reads of every entry are issued together and the hits
// aggregated with fire-and-forget LDS atomics; only keys new to the table take lt2_insert.
template <typename KB, int NV, int M, bool N>
__device__ inline void lt2_add_many(const LdsTable<KB> &t, const HaTable &g, const KB *kb,
                                    const uint64_t (*vb)[NV > 0 ? NV : 1], const bool *valid) {
    constexpr uint32_t S = lt_slots<N>();
    KB4<KB> q1[M], q2[M];
    uint32_t g1[M], g2[M];
#pragma unroll
    for (int i = 0; i < M; i++) {
        lt2_groups<KB, N>(kb[i], g1[i], g2[i]);
        q1[i] = *reinterpret_cast<const KB4<KB> *>(t.keys + 4 * g1[i]);
        q2[i] = *reinterpret_cast<const KB4<KB> *>(t.keys + 4 * g2[i]);
    }
    bool slow[M];
#pragma unroll
    for (int i = 0; i < M; i++) {
        uint32_t slot = lt2_find(q1[i], q2[i], g1[i], g2[i], kb[i]);
        if (kb[i] >= kb_closed<KB>()) slot = S + (uint32_t)(kb[i] - kb_closed<KB>());
        slow[i] = valid[i] && slot == ~0u;
        if (valid[i] && slot != ~0u) lt_bump<KB, NV, N>(t, g, slot, vb[i]);
    }
#pragma unroll
    for (int i = 0; i < M; i++)
        if (slow[i]) lt2_insert<KB, NV, N>(t, g, kb[i], vb[i]);
}

// merge the LDS table into the HBM table (after a workgroup barrier, every thread); the
// workgroup's new keys are added to g.used once
template <typename KB, int NV, bool N> __device__ inline void lt_merge(const LdsTable<KB> &t, const HaTable &g, int nthreads) {
    constexpr uint32_t S = lt_slots<N>();
    __shared__ uint32_t s_new;
    if (threadIdx.x == 0) s_new = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < S + 2; i += nthreads) {
        const unsigned long long cn = N ? (unsigned long long)t.cn32[i] << 32 : t.cn[i];
        if (!cn) continue;
        const KB kb = i < S ? t.keys[i] : (KB)(kb_closed<KB>() + (i - S));
        const uint64_t s = ha_slot(g, (uint64_t)kb, &s_new);
        if (s == ~0ULL) continue;
        atomicAdd(&g.cnt[s], cn >> 32);
#pragma unroll
        for (int v = 0; v < NV; v++) {
            if ((g.vfloat >> v) & 1) {
                const double d = reinterpret_cast<const double *>(t.sum[v])[i];
                if (d != 0.0) atomicAdd(reinterpret_cast<double *>(g.sum[v]) + s, d);
                const uint32_t k = v == 0 ? (uint32_t)cn : t.nn1[i];
                if (k) atomicAdd(&g.nn[v][s], (unsigned long long)k);
            } else {
                atomicAdd(&g.sum[v][s], t.sum[v][i]);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && s_new && atomicAdd(g.used, s_new) + s_new > g.max_used) atomicOr(g.err, 1u);
}

// pass-A rows that missed their region since the last reset (vh_stat_read)
__device__ unsigned long long d_ha_overflow_rows;

// ---- partition parameters -----------------------------------------------------------------
struct HaParams {
    const void *keys;
    const void *vals[HA_MAX_V];
    int32_t vdtype[HA_MAX_V];
    uint32_t p_log2, P, W, debug;  // debug: VH_HA_DEBUG experiment switches, 0 in production
    uint64_t n, rows_per_wg, wg_stride;
    const uint32_t *cap;   // [P]
    const uint64_t *toff;  // [P]
    uint32_t *fills;       // [P][W]
    // regions: NV == 1 packed 16-byte entries {key bits (8 B), value bits (8 B)}; otherwise
    // a key-bits array and NV value-bits arrays.  W * HA_THREADS dummy slots follow.
    void *ent;
    uint64_t *vbits[HA_MAX_V];
    uint64_t dummy0;       // first dummy slot (idle lanes of the stream-out write there)
};

struct HaUnit {
    uint32_t bucket, w_begin, w_end, pad;
};

__device__ inline void ha_lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// ---- sample -------------------------------------------------------------------------------
template <typename K>
__global__ __launch_bounds__(HA_THREADS) void k_ha_sample(const K *keys, uint64_t n, uint64_t block_stride,
                                                          unsigned long long *fine_hist, uint64_t *skeys,
                                                          uint32_t *scnt, uint64_t smask) {
    __shared__ uint32_t h[1u << HA_FINE_LOG2];
    for (uint32_t t = threadIdx.x; t < (1u << HA_FINE_LOG2); t += HA_THREADS) h[t] = 0;
    __syncthreads();
    // rows at pseudo-random positions (block_stride: the block's seed): the distinct-key
    // estimate and the bucket histogram hold for any row order (evenly spaced blocks of a
    // sorted column saw a few keys each); each sampled row is also compared with the next
    // row -- the fraction of equal neighbours tells clustered keys (runs) apart
    uint32_t adj = 0;
    for (uint64_t r = threadIdx.x; r < HA_BATCH; r += HA_THREADS) {
        // a sample as large as the rows covers each row once (exact estimate)
        const uint64_t lin = blockIdx.x * (uint64_t)HA_BATCH + r;
        if ((uint64_t)gridDim.x * HA_BATCH >= n && lin >= n) break;
        const uint64_t i = (uint64_t)gridDim.x * HA_BATCH >= n ? lin : hash64(block_stride * 0x9E3779B97F4A7C15ULL + lin) % n;
        const auto kb = ha_kb(keys[i]);
        if (i + 1 < n && ha_kb(keys[i + 1]) == kb) adj++;
        atomicAdd(&h[ha_h(kb) >> (32 - HA_FINE_LOG2)], 1u);
        const uint64_t key = (uint64_t)kb;
        if (key == SET_EMPTY) continue;  // the estimate can miss one key
        uint64_t pos = hash64(key) & smask;
        for (int p = 0; p < HA_MAX_PROBE; p++) {
            uint64_t cur = __hip_atomic_load(&skeys[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur == SET_EMPTY)
                cur = atomicCAS((unsigned long long *)&skeys[pos], (unsigned long long)SET_EMPTY, (unsigned long long)key);
            if (cur == SET_EMPTY || cur == key) {
                atomicAdd(&scnt[pos], 1u);
                break;
            }
            pos = (pos + 1) & smask;
        }
    }
    for (int off = 32; off > 0; off >>= 1) adj += __shfl_down(adj, off, 64);
    if ((threadIdx.x & 63) == 0 && adj) atomicAdd(&fine_hist[(1u << HA_FINE_LOG2) + 3], (unsigned long long)adj);
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < (1u << HA_FINE_LOG2); t += HA_THREADS)
        if (h[t]) atomicAdd(&fine_hist[t], (unsigned long long)h[t]);
}

// distinct keys of the sample, and how many were seen once / twice (Chao1 inputs)
__global__ __launch_bounds__(256) void k_ha_sample_stats(const uint32_t *scnt, uint64_t slots,
                                                         unsigned long long *stats) {
    __shared__ uint32_t part[3][4];
    uint32_t d = 0, f1 = 0, f2 = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < slots; i += (uint64_t)gridDim.x * 256) {
        const uint32_t c = scnt[i];
        d += c != 0;
        f1 += c == 1;
        f2 += c == 2;
    }
    for (int off = 32; off > 0; off >>= 1) {
        d += __shfl_down(d, off, 64);
        f1 += __shfl_down(f1, off, 64);
        f2 += __shfl_down(f2, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {  // one atomic per block and counter, not per wave
        part[0][threadIdx.x >> 6] = d;
        part[1][threadIdx.x >> 6] = f1;
        part[2][threadIdx.x >> 6] = f2;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const uint32_t v = part[threadIdx.x][0] + part[threadIdx.x][1] + part[threadIdx.x][2] + part[threadIdx.x][3];
        if (v) atomicAdd(&stats[threadIdx.x], (unsigned long long)v);
    }
}

// ---- pass A -------------------------------------------------------------------------------
__host__ __device__ constexpr size_t ha_scatter_lds_bytes(int nv, int kbsize, uint32_t P) {
    return ((size_t)8 * nv + kbsize + 4) * (HA_BATCH + 1) + 16 * ((size_t)P + 1) + 64;
}

// LDS of pass A: staged value bits | staged key bits | staged destinations | per-bucket
// hist | batch offsets | region write base | region limit | wave sums
template <typename KB> struct HaScatterLds {
    uint64_t *sv;
    KB *sk;
    uint32_t *sd;
    uint32_t *hist, *boff, *base, *lim, *wave_sums;
};

template <typename KB, int NV> __device__ inline HaScatterLds<KB> ha_scatter_lds(unsigned char *raw, const HaParams &hp) {
    HaScatterLds<KB> l;
    l.sv = reinterpret_cast<uint64_t *>(raw);
    l.sk = reinterpret_cast<KB *>(l.sv + (size_t)NV * (HA_BATCH + 1));
    l.sd = reinterpret_cast<uint32_t *>(l.sk + HA_BATCH + 1);
    l.hist = l.sd + HA_BATCH + 1;
    l.boff = l.hist + hp.P + 1;  // hist[P]: the rank sink of rows past the range
    l.base = l.boff + hp.P;
    l.lim = l.base + hp.P;
    l.wave_sums = l.lim + hp.P;
    for (uint32_t t = threadIdx.x; t <= hp.P; t += HA_THREADS) l.hist[t] = 0;
    for (uint32_t t = threadIdx.x; t < hp.P; t += HA_THREADS) {
        l.base[t] = (uint32_t)hp.toff[t];
        l.lim[t] = (uint32_t)hp.toff[t] + hp.cap[t];
    }
    return l;
}

// A batch after every row has its bucket, key bits, rank (-1 = no row) and value bits:
// exclusive scan of the bucket histogram, counting sort of (destination, key) + values
// into LDS, the sorted runs streamed to the regions (consecutive lanes -> consecutive
// addresses), region bases advanced.  Rows past a region's capacity go to the HBM table.
// The stream-out issues a fixed number of stores per lane (idle lanes write a private
// dummy slot), so the compiler waits for the prefetched next batch with vmcnt(#stores)
// instead of draining every store of this batch; the rare overflow rows are applied after
// that loop.
template <typename KB, int NV>
__device__ inline void ha_commit(const HaScatterLds<KB> &l, const HaParams &hp, const HaTable &g, uint64_t region0,
                                 const uint32_t *bkt, const KB *kb, const int32_t *rank,
                                 const uint64_t (*vb)[NV > 0 ? NV : 1]) {
    __shared__ uint32_t s_total, s_over;
    const uint32_t P = hp.P;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    ha_lds_barrier();
    {
        const uint32_t per = (P + HA_THREADS - 1) / HA_THREADS;
        const uint32_t t0 = threadIdx.x * per;
        uint32_t s = 0;
        for (uint32_t t = t0; t < t0 + per && t < P; t++) s += l.hist[t];
        uint32_t inc = s;
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(inc, off, 64);
            if (lane >= off) inc += y;
        }
        if (lane == 63) l.wave_sums[wave] = inc;
        ha_lds_barrier();
        uint32_t wave_base = 0, total = 0;
        for (int k = 0; k < HA_THREADS / 64; k++) {
            if (k < wave) wave_base += l.wave_sums[k];
            total += l.wave_sums[k];
        }
        uint32_t acc = wave_base + inc - s;
        for (uint32_t t = t0; t < t0 + per && t < P; t++) {
            l.boff[t] = acc;
            acc += l.hist[t];
        }
        if (threadIdx.x == 0) {
            s_total = total;
            s_over = 0;
        }
    }
    ha_lds_barrier();
    bool over = false;
#pragma unroll
    for (int r = 0; r < HA_RPT; r++) {
        const bool valid = rank[r] >= 0;
        const uint32_t t = valid ? bkt[r] : 0u;
        const uint32_t pos = valid ? l.boff[t] + (uint32_t)rank[r] : (uint32_t)HA_BATCH;  // slot HA_BATCH: scratch
        const uint32_t d = l.base[t] + (uint32_t)rank[r];
        const bool fits = d < l.lim[t];
        over |= valid && !fits;
        l.sd[pos] = fits ? d : (HA_DEST_OVERFLOW | t);
        l.sk[pos] = kb[r];
#pragma unroll
        for (int v = 0; v < NV; v++) l.sv[v * (HA_BATCH + 1) + pos] = vb[r][v];
    }
    if (over) s_over = 1;
    ha_lds_barrier();
    const uint32_t tot = s_total;
    const uint64_t dummy = hp.dummy0 + (uint64_t)blockIdx.x * HA_THREADS + threadIdx.x;
#pragma unroll
    for (int r = 0; r < HA_RPT; r++) {
        const uint32_t k = r * HA_THREADS + threadIdx.x;
        const uint32_t dest = l.sd[k];
        const uint64_t key = (uint64_t)l.sk[k];
        const bool ok = k < tot && !(dest & HA_DEST_OVERFLOW);
        const uint64_t e = ok ? region0 + dest : dummy;
        if constexpr (ha_packed<KB, NV>()) {  // packed {key, value}: one 16-byte store per row
            const uint64_t vbits = l.sv[k];
            reinterpret_cast<uint4 *>(hp.ent)[e] =
                make_uint4((uint32_t)key, (uint32_t)(key >> 32), (uint32_t)vbits, (uint32_t)(vbits >> 32));
        } else {
            reinterpret_cast<KB *>(hp.ent)[e] = (KB)key;
#pragma unroll
            for (int v = 0; v < NV; v++) hp.vbits[v][e] = l.sv[v * (HA_BATCH + 1) + k];
        }
    }
    if (s_over) {
        uint32_t novf = 0;
        for (uint32_t k = threadIdx.x; k < tot; k += HA_THREADS) {
            if (!(l.sd[k] & HA_DEST_OVERFLOW)) continue;
            uint64_t vv[NV > 0 ? NV : 1];
#pragma unroll
            for (int v = 0; v < NV; v++) vv[v] = l.sv[v * (HA_BATCH + 1) + k];
            ha_global_row<NV>(g, (uint64_t)l.sk[k], vv);
            novf++;
        }
        if (novf) atomicAdd(&d_ha_overflow_rows, (unsigned long long)novf);
    }
    ha_lds_barrier();
    for (uint32_t t = threadIdx.x; t < P; t += HA_THREADS) {
        l.base[t] += l.hist[t];
        l.hist[t] = 0;
    }
    ha_lds_barrier();
}

// top p_log2 bits of the key hash (branch-free: p_log2 = 0 gives bucket 0)
template <typename KB> __device__ inline uint32_t ha_bucket(const HaParams &hp, KB kb) {
    return (uint32_t)(((uint64_t)ha_h(kb) << hp.p_log2) >> 32);
}

// generic pass A: any key type and value dtypes, scalar loads
template <typename K, int NV>
__global__ __launch_bounds__(HA_THREADS) void k_ha_scatter(HaParams hp, HaTable g) {
    using KB = kb_t<K>;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const HaScatterLds<KB> l = ha_scatter_lds<KB, NV>(lds_raw, hp);
    __syncthreads();
    // batches w, w + W, w + 2W, ...: every workgroup's rows spread over the whole range
    const uint32_t w = blockIdx.x;
    const uint64_t row_end = hp.n;
    const uint64_t region0 = (uint64_t)w * hp.wg_stride;
    const K *keys = static_cast<const K *>(hp.keys);
    for (uint64_t b0 = (uint64_t)w * HA_BATCH; b0 < row_end; b0 += (uint64_t)hp.W * HA_BATCH) {
        uint32_t bkt[HA_RPT];
        KB kb[HA_RPT];
        int32_t rank[HA_RPT];
        uint64_t vb[HA_RPT][NV > 0 ? NV : 1];
#pragma unroll
        for (int r = 0; r < HA_RPT; r++) {
            const uint64_t i = b0 + (uint64_t)r * HA_THREADS + threadIdx.x;
            rank[r] = -1;
            kb[r] = 0;
            if (i < row_end) {
                kb[r] = ha_kb(keys[i]);
#pragma unroll
                for (int v = 0; v < NV; v++) vb[r][v] = ha_load_val(hp.vals[v], hp.vdtype[v], i);
            }
        }
#pragma unroll
        for (int r = 0; r < HA_RPT; r++) {
            const uint64_t i = b0 + (uint64_t)r * HA_THREADS + threadIdx.x;
            if (i < row_end) {
                bkt[r] = ha_bucket(hp, kb[r]);
                rank[r] = (int32_t)atomicAdd(&l.hist[bkt[r]], 1u);
            }
        }
        ha_commit<KB, NV>(l, hp, g, region0, bkt, kb, rank, vb);
    }
    for (uint32_t t = threadIdx.x; t < hp.P; t += HA_THREADS)
        hp.fills[(uint64_t)t * hp.W + w] = l.base[t] - (uint32_t)hp.toff[t];
}

// fast pass A: 4- or 8-byte keys and float64 values, 16-byte aligned, n a multiple of 8.
// A lane owns 8 rows per batch in groups of KPL consecutive rows (one 16-byte key load
// each: KPL = 4 for 4-byte keys, 2 for 8-byte keys) and each value column as KPL / 2
// 16-byte loads; the next batch is prefetched into registers while this one is ranked and
// sorted.  Batches start at multiples of HA_BATCH, so a group is wholly inside or wholly
// past the rows; past-the-end groups load a clamped in-range address and drop.
template <typename K, int NV>
__global__ __launch_bounds__(HA_THREADS) void k_ha_scatter_f64(HaParams hp, HaTable g) {
    static_assert(sizeof(K) == 4 || sizeof(K) == 8, "fast pass A takes 4- or 8-byte keys");
    using KB = kb_t<K>;
    constexpr int KPL = 16 / sizeof(K), GROUPS = HA_RPT / KPL;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const HaScatterLds<KB> l = ha_scatter_lds<KB, NV>(lds_raw, hp);
    __syncthreads();
    const uint32_t w = blockIdx.x;
    const uint64_t row_end = hp.n, bstep = (uint64_t)hp.W * HA_BATCH;  // batches w, w + W, ...
    const uint64_t region0 = (uint64_t)w * hp.wg_stride;
    const K *keys = static_cast<const K *>(hp.keys);
    const double *vcol[NV > 0 ? NV : 1];
#pragma unroll
    for (int v = 0; v < NV; v++) vcol[v] = static_cast<const double *>(hp.vals[v]);
    struct Regs {
        uint4 k[GROUPS];
        double2 v[GROUPS][NV > 0 ? NV : 1][KPL / 2];
    };
    auto load = [&](uint64_t b0, Regs &R) {
#pragma unroll
        for (int q = 0; q < GROUPS; q++) {
            const uint64_t i = b0 + KPL * ((uint64_t)q * HA_THREADS + threadIdx.x);
            const uint64_t is = i < hp.n ? i : hp.n - KPL;
            R.k[q] = *reinterpret_cast<const uint4 *>(keys + is);
#pragma unroll
            for (int v = 0; v < NV; v++)
#pragma unroll
                for (int h = 0; h < KPL / 2; h++) R.v[q][v][h] = *reinterpret_cast<const double2 *>(vcol[v] + is + 2 * h);
        }
    };
    Regs cur, nxt;
    load((uint64_t)w * HA_BATCH, cur);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): cur is not pending at the loop header
    for (uint64_t b0 = (uint64_t)w * HA_BATCH; b0 < row_end; b0 += bstep) {
        load(b0 + bstep, nxt);
        uint32_t bkt[HA_RPT];
        KB kb[HA_RPT];
        int32_t rank[HA_RPT];
        uint64_t vb[HA_RPT][NV > 0 ? NV : 1];
#pragma unroll
        for (int q = 0; q < GROUPS; q++) {
            const uint64_t i = b0 + KPL * ((uint64_t)q * HA_THREADS + threadIdx.x);
            const bool valid = i < row_end;  // uniform but for a range's last batch
            KB words[KPL];
            __builtin_memcpy(words, &cur.k[q], 16);
#pragma unroll
            for (int j = 0; j < KPL; j++) {
                const int r = q * KPL + j;
                kb[r] = ha_kb(__builtin_bit_cast(K, words[j]));
#pragma unroll
                for (int v = 0; v < NV; v++)
                    vb[r][v] = __builtin_bit_cast(uint64_t, (j & 1) ? cur.v[q][v][j >> 1].y : cur.v[q][v][j >> 1].x);
                bkt[r] = ha_bucket(hp, kb[r]);
                const uint32_t rk = atomicAdd(&l.hist[valid ? bkt[r] : hp.P], 1u);
                rank[r] = valid ? (int32_t)rk : -1;
            }
        }
        ha_commit<KB, NV>(l, hp, g, region0, bkt, kb, rank, vb);
        cur = nxt;
    }
    for (uint32_t t = threadIdx.x; t < hp.P; t += HA_THREADS)
        hp.fills[(uint64_t)t * hp.W + w] = l.base[t] - (uint32_t)hp.toff[t];
}

// Pass A for 4-byte keys and NV <= 1 float64 values (the C3 shape), after the tile path's
// fast scatter (tiled.hip k_tile_scatter_ord): SB batches of 4096 rows are ranked before
// one commit, so a bucket's run per commit is SB times longer -- with P = 512 buckets a
// 4096-row commit leaves ~8 rows per bucket, and such short runs are partial cache lines
// that HBM receives twice (PMC: 18.7 GB written for 12 GB of entries).  LDS holds only the
// staged key bits and values (12 B per row); a staged row's bucket is recomputed from its
// key at stream-out, and one wave's scan turns the histogram into sorted offsets, the
// destination bases and the advanced region bases (three LDS barriers per commit).
__host__ __device__ constexpr size_t ha_fast_lds_bytes(int nv, int sb, uint32_t P) {
    return (size_t)(8 * nv + 4) * sb * HA_BATCH + 20 * ((size_t)P + 1) + 64;
}

// A run of rows with one key (count(*), non-NaN values: their sum and count)
struct HaRun {
    uint32_t cnt, nn;
    double sum;
};
__device__ inline HaRun ha_run_of(double v) { return HaRun{1u, v == v ? 1u : 0u, v == v ? v : 0.0}; }
__device__ inline HaRun ha_run_add(HaRun a, HaRun b) { return HaRun{a.cnt + b.cnt, a.nn + b.nn, a.sum + b.sum}; }
__device__ inline HaRun ha_run_shfl_up(HaRun a, int off) {
    return HaRun{(uint32_t)__shfl_up((int)a.cnt, off, 64), (uint32_t)__shfl_up((int)a.nn, off, 64), __shfl_up(a.sum, off, 64)};
}

// a whole run into the HBM table (new keys counted in the workgroup's LDS counter)
template <int NV> __device__ inline void ha_global_run(const HaTable &g, uint64_t key, const HaRun &r, uint32_t *s_new) {
    const uint64_t s = ha_slot(g, key, s_new);
    if (s == ~0ULL) return;
    atomicAdd(&g.cnt[s], (unsigned long long)r.cnt);
    if constexpr (NV > 0) {
        if (r.nn) {
            atomicAdd(reinterpret_cast<double *>(g.sum[0]) + s, r.sum);
            atomicAdd(&g.nn[0][s], (unsigned long long)r.nn);
        }
    }
}

// RUNS (clustered keys -- the sample saw most rows equal to their neighbour, e.g. a sorted
// key column): a wave's 128 consecutive rows of one pair group that hold at most 16 runs of
// equal keys are folded per run (segmented scan over the lanes) and each run goes to the HBM
// table as ONE update at its last row; those rows skip the partition.  Other groups (and
// every group of shuffled keys, which never take this variant) are partitioned row by row.
template <typename K, int NV, int SB, bool RUNS>
__global__ __launch_bounds__(HA_THREADS) void k_ha_scatter_k4(HaParams hp, HaTable g) {
    static_assert(sizeof(K) == 4 && NV <= 1, "4-byte keys, at most one float64 value");
    constexpr int PAIRS = HA_RPT / 2;
    constexpr uint32_t CAP = SB * HA_BATCH;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    __shared__ uint32_t s_new;
    const uint32_t P = hp.P;
    double *sv = reinterpret_cast<double *>(lds_raw);
    uint32_t *sk = reinterpret_cast<uint32_t *>(lds_raw + (size_t)8 * NV * CAP);
    uint32_t *hist = sk + CAP;  // [P + 1]: hist[P] takes the ranks of rows past the range
    uint32_t *boff = hist + P + 1, *dbase = boff + P, *base = dbase + P, *lim = base + P;
    uint32_t *wave_sums = lim + P;
    for (uint32_t t = threadIdx.x; t <= P; t += HA_THREADS) hist[t] = 0;
    for (uint32_t t = threadIdx.x; t < P; t += HA_THREADS) {
        base[t] = (uint32_t)hp.toff[t];
        lim[t] = (uint32_t)hp.toff[t] + hp.cap[t];
    }
    if (threadIdx.x == 0) s_new = 0;
    __syncthreads();
    // batches w, w + W, w + 2W, ... of HA_BATCH rows: every workgroup's rows spread over
    // the whole range, so its bucket distribution is the global one whatever the row order
    const uint32_t w = blockIdx.x;
    const uint64_t n = hp.n, bstep = (uint64_t)hp.W * HA_BATCH;
    const uint64_t row_end = n;
    const uint64_t region0 = (uint64_t)w * hp.wg_stride;
    const K *keys = static_cast<const K *>(hp.keys);
    const double *vcol = static_cast<const double *>(hp.vals[0]);
    uint32_t *ekeys = static_cast<uint32_t *>(hp.ent);
    uint64_t *evals = hp.vbits[0];
    const int lane = threadIdx.x & 63;
    struct Regs {
        uint2 k[PAIRS];
        double2 v[PAIRS][NV > 0 ? NV : 1];
    };
    // branch-free pair loads: n is a multiple of 8 here and batches start at multiples of
    // HA_BATCH, so a pair is wholly inside the rows or past them (clamped, then dropped)
    auto load = [&](uint64_t b0, Regs &R) {
#pragma unroll
        for (int q = 0; q < PAIRS; q++) {
            const uint64_t i = b0 + 2 * ((uint64_t)q * HA_THREADS + threadIdx.x);
            const uint64_t is = i < n - 2 ? i : n - 2;
            R.k[q] = *reinterpret_cast<const uint2 *>(keys + is);
            if constexpr (NV > 0) R.v[q][0] = *reinterpret_cast<const double2 *>(vcol + is);
        }
    };
    auto rows = [&](uint64_t b0, const Regs &cur, uint32_t *kb, int32_t *rank, double *vals) {
        bool folded[PAIRS];
#pragma unroll
        for (int q = 0; q < PAIRS; q++) folded[q] = false;
        if constexpr (RUNS) {
            // a run of uniform groups not yet in the HBM table: its key, row and non-NaN counts
            // (wave-uniform) and each lane's partial sum -- reduced over the wave once per run
            bool pend = false;
            uint32_t pkey = 0, pcnt = 0, pnn = 0;
            double psum = 0.0;
            auto flush = [&]() __attribute__((always_inline)) {
                double t = psum;
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
                if (lane == 63) ha_global_run<NV>(g, (uint64_t)pkey, HaRun{pcnt, pnn, t}, &s_new);
            };
#pragma unroll
            for (int q = 0; q < PAIRS; q++) {
                const uint64_t i0 = b0 + 2 * ((uint64_t)q * HA_THREADS + threadIdx.x);
                const uint32_t k0 = ha_kb(__builtin_bit_cast(K, cur.k[q].x)), k1 = ha_kb(__builtin_bit_cast(K, cur.k[q].y));
                const double v0 = NV > 0 ? cur.v[q][0].x : 0.0, v1 = NV > 0 ? cur.v[q][0].y : 0.0;
                const uint32_t kp = (uint32_t)__shfl_up((int)k1, 1, 64);
                const bool cin = lane > 0 && kp == k0;  // row 2l continues the previous lane's run
                const bool same = k1 == k0;
                const uint64_t heads = __builtin_popcountll(__ballot(!cin)) + __builtin_popcountll(__ballot(!same));
                const bool all_in = __ballot(i0 >= row_end) == 0;
                if (!all_in || heads > 16) continue;  // wave-uniform
                if (__ballot(!same || (lane > 0 && !cin)) == 0) {
                    // the wave's 128 rows hold one key (a long run of a sorted column): no
                    // segmented scan; consecutive such groups of one key add up (counts in
                    // wave-uniform registers, sums per lane), one HBM-table update per key
                    double sl = 0.0;
                    uint32_t nn = 0;
                    if constexpr (NV > 0) {
                        sl = (v0 == v0 ? v0 : 0.0) + (v1 == v1 ? v1 : 0.0);
                        nn = (uint32_t)(__builtin_popcountll(__ballot(v0 == v0)) + __builtin_popcountll(__ballot(v1 == v1)));
                    }
                    const uint32_t ku = (uint32_t)__builtin_amdgcn_readfirstlane((int)k1);
                    if (pend && pkey == ku) {
                        pcnt += 128u;
                        pnn += nn;
                        psum += sl;
                    } else {
                        if (pend) flush();
                        pend = true;
                        pkey = ku;
                        pcnt = 128u;
                        pnn = nn;
                        psum = sl;
                    }
                    folded[q] = true;
                    continue;
                }
                // segmented inclusive scan of the run through row 2l+1 (flag: starts in this lane)
                HaRun a = same ? ha_run_add(ha_run_of(v0), ha_run_of(v1)) : ha_run_of(v1);
                bool f = !(same && cin);
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const HaRun up = ha_run_shfl_up(a, off);
                    const bool uf = __shfl_up((int)f, off, 64) != 0;
                    if (lane >= off && !f) {
                        a = ha_run_add(up, a);
                        f = uf;
                    }
                }
                const HaRun prev = ha_run_shfl_up(a, 1);  // the run through row 2l-1
                const bool cin_next = __shfl_down((int)cin, 1, 64) != 0 && lane < 63;
                if (!same) {  // row 2l ends its run (row 2l+1 starts a new one)
                    const HaRun r0 = cin ? ha_run_add(prev, ha_run_of(v0)) : ha_run_of(v0);
                    ha_global_run<NV>(g, (uint64_t)k0, r0, &s_new);
                }
                if (!cin_next) ha_global_run<NV>(g, (uint64_t)k1, a, &s_new);
                folded[q] = true;
            }
            if (pend) flush();
        }
#pragma unroll
        for (int r = 0; r < HA_RPT; r++) {
            const int q = r >> 1, h = r & 1;
            const uint64_t i = b0 + 2 * ((uint64_t)q * HA_THREADS + threadIdx.x) + h;
            kb[r] = ha_kb(__builtin_bit_cast(K, h ? cur.k[q].y : cur.k[q].x));
            if constexpr (NV > 0) vals[r] = h ? cur.v[q][0].y : cur.v[q][0].x;
            const uint32_t t = ha_bucket(hp, kb[r]);
            const bool take = i < row_end && !folded[q];
            if constexpr (RUNS) {
                // folded rows and rows past the range touch no histogram word; a wave whose
                // rows share a bucket (a run of one key) reserves its ranks with one atomic
                rank[r] = wave_rank(hist, t, take);
            } else {
                const uint32_t rk = atomicAdd(&hist[take ? t : P], 1u);
                rank[r] = take ? (int32_t)rk : -1;
            }
        }
    };
    uint32_t novf = 0;
    Regs cur, nxt;
    load((uint64_t)w * HA_BATCH, cur);
    for (uint64_t b0 = (uint64_t)w * HA_BATCH; b0 < row_end; b0 += SB * bstep) {
        uint32_t kb[SB * HA_RPT];
        int32_t rank[SB * HA_RPT];
        double vals[SB * HA_RPT];
#pragma unroll
        for (int sb = 0; sb < SB; sb++) {
            load(b0 + (uint64_t)(sb + 1) * bstep, nxt);
            rows(b0 + (uint64_t)sb * bstep, cur, kb + sb * HA_RPT, rank + sb * HA_RPT, vals + sb * HA_RPT);
            cur = nxt;
        }
        // B1: every rank taken -> wave 0 scans the histogram.  A commit whose rows were all
        // folded into runs (sorted keys) has nothing to partition: the scan, staging and
        // stream-out are skipped
        bool took = false;
        if constexpr (RUNS) {
#pragma unroll
            for (int r = 0; r < SB * HA_RPT; r++) took = took || rank[r] >= 0;
            if (!__syncthreads_or(took)) continue;
        } else {
            ha_lds_barrier();
        }
        if (threadIdx.x < 64) {
            const uint32_t per = (P + 63) / 64;
            const uint32_t t0 = lane * per;
            uint32_t s = 0;
            for (uint32_t t = t0; t < t0 + per && t < P; t++) s += hist[t];
            uint32_t inc = s;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(inc, off, 64);
                if (lane >= off) inc += y;
            }
            uint32_t acc = inc - s;
            for (uint32_t t = t0; t < t0 + per && t < P; t++) {
                const uint32_t hh = hist[t], b = base[t];
                boff[t] = acc;
                dbase[t] = b - acc;
                base[t] = b + hh;
                hist[t] = 0;
                acc += hh;
            }
            if (lane == 0) hist[P] = 0;
            if (lane == 63) wave_sums[0] = inc;
        }
        // B2: rows stage their key bits and values at their sorted positions
        ha_lds_barrier();
        const uint32_t tot = wave_sums[0];
#pragma unroll
        for (int r = 0; r < SB * HA_RPT; r++) {
            if (rank[r] < 0) continue;
            const uint32_t pos = boff[ha_bucket(hp, kb[r])] + (uint32_t)rank[r];
            sk[pos] = kb[r];
            if constexpr (NV > 0) sv[pos] = vals[r];
        }
        // B3: the sorted runs stream to the regions; a full region (sampling miss) sends
        // its rows to the HBM table
        ha_lds_barrier();
        for (uint32_t k = threadIdx.x; k < tot; k += HA_THREADS) {
            const uint32_t key = sk[k];
            const uint32_t t = ha_bucket(hp, key);
            const uint32_t dest = dbase[t] + k;
            if (dest < lim[t]) {
                const uint64_t e = region0 + dest;
                ekeys[e] = key;
                if constexpr (NV > 0) evals[e] = __builtin_bit_cast(uint64_t, sv[k]);
            } else {
                uint64_t vb[NV > 0 ? NV : 1];
                if constexpr (NV > 0) vb[0] = __builtin_bit_cast(uint64_t, sv[k]);
                ha_global_row<NV>(g, (uint64_t)key, vb);
                novf++;
            }
        }
    }
    if (novf) atomicAdd(&d_ha_overflow_rows, (unsigned long long)novf);
    ha_lds_barrier();
    for (uint32_t t = threadIdx.x; t < P; t += HA_THREADS) hp.fills[(uint64_t)t * hp.W + w] = base[t] - (uint32_t)hp.toff[t];
    if (RUNS && threadIdx.x == 0 && s_new && atomicAdd(g.used, s_new) + s_new > g.max_used) atomicOr(g.err, 1u);
}

// rows [row0, n) straight into the HBM table (the < 8-row tail of the fast pass A)
template <typename K, int NV>
__global__ __launch_bounds__(64) void k_ha_tail(HaParams hp, HaTable g, uint64_t row0) {
    const uint64_t i = row0 + threadIdx.x;
    if (i >= hp.n) return;
    uint64_t vb[NV > 0 ? NV : 1];
#pragma unroll
    for (int v = 0; v < NV; v++) vb[v] = ha_load_val(hp.vals[v], hp.vdtype[v], i);
    ha_global_row<NV>(g, (uint64_t)ha_kb(static_cast<const K *>(hp.keys)[i]), vb);
}

// ---- pass B -------------------------------------------------------------------------------
// One work unit = one bucket x a range of pass-A workgroups.  The unit's regions are read
// as one flat stream of entries (prefix sums of the region fills in LDS), one entry per
// lane per load: consecutive lanes read consecutive entries (a wave's load is contiguous
// unless it crosses a region end); a lane finds the region of its entry by a forward scan.
template <typename KB, int NV, bool N>
__global__ __launch_bounds__(HB_THREADS) void k_ha_reduce(HaParams hp, HaTable g, const HaUnit *units) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    __shared__ uint32_t s_fill[1024];
    __shared__ uint32_t s_pre[1025];
    const HaUnit u = units[blockIdx.x];
    const uint32_t b = u.bucket;
    const uint32_t cap = hp.cap[b];
    const uint32_t nw = u.w_end - u.w_begin;  // <= 1024 (host checks)
    bool any = false;
    for (uint32_t k = threadIdx.x; k < nw; k += HB_THREADS) {
        const uint32_t f = min(hp.fills[(uint64_t)b * hp.W + u.w_begin + k], cap);
        s_fill[k] = f;
        any |= f != 0;
    }
    if (!__syncthreads_or(any)) return;
    const LdsTable<KB> t = lt_layout<KB, NV, N>(lds_raw);
    lt_init<KB, NV, N>(t, HB_THREADS);
    if (threadIdx.x < 64) {
        // exclusive scan of the region fills by the first wave (16 regions per lane)
        const uint32_t lane = threadIdx.x, k0 = lane * 16;
        uint32_t sum = 0;
        for (uint32_t k = k0; k < k0 + 16 && k < nw; k++) sum += s_fill[k];
        uint32_t inc = sum;
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(inc, off, 64);
            if ((int)lane >= off) inc += y;
        }
        uint32_t acc = inc - sum;
        for (uint32_t k = k0; k < k0 + 16 && k < nw; k++) {
            s_pre[k] = acc;
            acc += s_fill[k];
        }
        if (lane == 63) s_pre[nw] = inc;
    }
    __syncthreads();
    const uint32_t E = s_pre[nw];
    if (E == 0) return;  // uniform: the fetch below clamps to entry E - 1
    const uint64_t toff_b = hp.toff[b];
    uint32_t kr = 0;  // region of this lane's current entry (entry indices of a lane only grow)
    struct Batch {
        KB kb[HB_M];
        uint64_t vb[HB_M][NV > 0 ? NV : 1];
        bool valid[HB_M];
    };
    auto fetch = [&](uint32_t c0, Batch &B) {
#pragma unroll
        for (int j = 0; j < HB_M; j++) {
            const uint32_t c = c0 + j * HB_THREADS + threadIdx.x;
            const uint32_t cc = c < E ? c : E - 1;
            while (s_pre[kr + 1] <= cc) kr++;
            const uint64_t e = (uint64_t)(u.w_begin + kr) * hp.wg_stride + toff_b + (cc - s_pre[kr]);
            B.valid[j] = c < E;
            if constexpr (ha_packed<KB, NV>()) {
                const uint4 q = reinterpret_cast<const uint4 *>(hp.ent)[e];
                B.kb[j] = (KB)(((uint64_t)q.y << 32) | q.x);
                B.vb[j][0] = ((uint64_t)q.w << 32) | q.z;
            } else {
                B.kb[j] = reinterpret_cast<const KB *>(hp.ent)[e];
#pragma unroll
                for (int v = 0; v < NV; v++) B.vb[j][v] = hp.vbits[v][e];
            }
        }
    };
    auto process = [&](const Batch &B) {
        if (DBG(hp.debug) & 1) {  // experiment: entry stream only (wrong results)
#pragma unroll
            for (int j = 0; j < HB_M; j++) asm volatile("" ::"v"(B.kb[j]), "v"(B.vb[j][0]));
        } else {
            constexpr int MM = sizeof(KB) == 4 ? HB_M / 2 : HB_M / 4;  // 128 VGPRs at 1024 threads
#pragma unroll
            for (int h0 = 0; h0 < HB_M; h0 += MM) lt2_add_many<KB, NV, MM, N>(t, g, B.kb + h0, B.vb + h0, B.valid + h0);
        }
    };
    constexpr uint32_t STEP = HB_THREADS * HB_M;
    if constexpr (sizeof(KB) == 4 && NV <= 1) {
        // 4-byte keys: the next batch's entries load while this one is aggregated
        Batch cur, nxt;
        fetch(0, cur);
        for (uint32_t c0 = 0; c0 < E; c0 += STEP) {
            fetch(c0 + STEP, nxt);
            process(cur);
            cur = nxt;
        }
    } else {
        for (uint32_t c0 = 0; c0 < E; c0 += STEP) {
            Batch cur;
            fetch(c0, cur);
            process(cur);
        }
    }
    __syncthreads();
    if (DBG(hp.debug) & 1) return;
    lt_merge<KB, NV, N>(t, g, HB_THREADS);
}

// ---- repartition (high-cardinality keys) ------------------------------------------------
// P is capped at 2^HA_MAX_P_LOG2 buckets by pass A's LDS; with more keys than that many LDS
// tables hold (h2o q10: ~1e8 groups, ~5e4 keys per bucket for 2300-key tables) almost every
// pass-B entry missed its LDS table and went to the HBM table with global atomics (q10 at
// 1e9 rows: k_ha_reduce 229 ms).  Here every pass-B unit's entries are first split by the
// next hash bits into S sub-buckets (sub = ((h << p) * S) >> 32, independent of the bits the
// LDS groups use), one read and one write of each entry, into per-(unit, sub) regions; pass B
// then runs unchanged over those regions (one region per unit) with ~1/S of the keys.
constexpr int HR_M = 4;                      // entries per lane per step
constexpr uint32_t HR_CH = HB_THREADS * HR_M;
constexpr uint32_t HR_MAX_S = 64;

struct RepartParams {
    uint32_t S, p_log2;
    const uint64_t *base;  // [units] first entry of the unit's S regions
    const uint32_t *rcap;  // [units] entries per sub-bucket region of the unit
    uint32_t *fills;       // [units * S] entries produced (may exceed rcap)
    void *ent;             // output entries, same format as pass A's
    uint64_t *vbits[HA_MAX_V];
};

template <typename KB> __device__ inline uint32_t ha_sub(KB kb, uint32_t p_log2, uint32_t S) {
    const uint32_t rest = p_log2 ? (uint32_t)(ha_h(kb) << p_log2) : ha_h(kb);
    return (uint32_t)(((uint64_t)rest * S) >> 32);
}

template <typename KB, int NV>
__global__ __launch_bounds__(HB_THREADS) void k_ha_repart(HaParams hp, HaTable g, const HaUnit *units, RepartParams rq) {
    __shared__ uint32_t s_fill[1024];
    __shared__ uint32_t s_pre[1025];
    __shared__ uint32_t hist[HR_MAX_S], boff[HR_MAX_S], dbase[HR_MAX_S], cursor[HR_MAX_S], s_tot;
    __shared__ KB skb[HR_CH];
    __shared__ uint64_t svb[NV > 0 ? NV : 1][HR_CH];
    __shared__ uint8_t ssub[HR_CH];
    const uint32_t ui = blockIdx.x;
    const HaUnit u = units[ui];
    const uint32_t b = u.bucket, S = rq.S;
    const uint32_t cap = hp.cap[b];
    const uint32_t nw = u.w_end - u.w_begin;
    for (uint32_t k = threadIdx.x; k < nw; k += HB_THREADS) s_fill[k] = min(hp.fills[(uint64_t)b * hp.W + u.w_begin + k], cap);
    if (threadIdx.x < HR_MAX_S) {
        hist[threadIdx.x] = 0;
        cursor[threadIdx.x] = 0;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t lane = threadIdx.x, k0 = lane * 16;
        uint32_t sum = 0;
        for (uint32_t k = k0; k < k0 + 16 && k < nw; k++) sum += s_fill[k];
        uint32_t inc = sum;
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(inc, off, 64);
            if ((int)lane >= off) inc += y;
        }
        uint32_t acc = inc - sum;
        for (uint32_t k = k0; k < k0 + 16 && k < nw; k++) {
            s_pre[k] = acc;
            acc += s_fill[k];
        }
        if (lane == 63) s_pre[nw] = inc;
    }
    __syncthreads();
    const uint32_t E = s_pre[nw];
    const uint64_t toff_b = hp.toff[b];
    const uint64_t base = rq.base[ui];
    const uint32_t rcap = rq.rcap[ui];
    uint32_t kr = 0;
    for (uint32_t c0 = 0; c0 < E; c0 += HR_CH) {
        KB kb[HR_M];
        uint64_t vb[HR_M][NV > 0 ? NV : 1];
        int32_t rank[HR_M];
        uint32_t sub[HR_M];
#pragma unroll
        for (int j = 0; j < HR_M; j++) {
            const uint32_t c = c0 + j * HB_THREADS + threadIdx.x;
            const uint32_t cc = c < E ? c : E - 1;
            while (s_pre[kr + 1] <= cc) kr++;
            const uint64_t e = (uint64_t)(u.w_begin + kr) * hp.wg_stride + toff_b + (cc - s_pre[kr]);
            if constexpr (ha_packed<KB, NV>()) {
                const uint4 q = reinterpret_cast<const uint4 *>(hp.ent)[e];
                kb[j] = (KB)(((uint64_t)q.y << 32) | q.x);
                vb[j][0] = ((uint64_t)q.w << 32) | q.z;
            } else {
                kb[j] = reinterpret_cast<const KB *>(hp.ent)[e];
#pragma unroll
                for (int v = 0; v < NV; v++) vb[j][v] = hp.vbits[v][e];
            }
            sub[j] = ha_sub(kb[j], rq.p_log2, S);
            rank[j] = c < E ? (int32_t)atomicAdd(&hist[sub[j]], 1u) : -1;
        }
        __syncthreads();
        if (threadIdx.x < 64) {  // exclusive scan of the sub-bucket counts (S <= 64: one per lane)
            const uint32_t s = threadIdx.x;
            const uint32_t h = s < S ? hist[s] : 0u;
            uint32_t inc = h;
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(inc, off, 64);
                if ((int)s >= off) inc += y;
            }
            if (s < S) {
                boff[s] = inc - h;
                dbase[s] = cursor[s] - (inc - h);
                cursor[s] += h;
                hist[s] = 0;
            }
            if (s == 63) s_tot = inc;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < HR_M; j++) {
            if (rank[j] < 0) continue;
            const uint32_t pos = boff[sub[j]] + (uint32_t)rank[j];
            skb[pos] = kb[j];
            ssub[pos] = (uint8_t)sub[j];
#pragma unroll
            for (int v = 0; v < NV; v++) svb[v][pos] = vb[j][v];
        }
        __syncthreads();
        const uint32_t tot = s_tot;
        for (uint32_t k = threadIdx.x; k < tot; k += HB_THREADS) {
            const uint32_t s = ssub[k];
            const uint32_t d = dbase[s] + k;
            if (d < rcap) {
                const uint64_t e = base + (uint64_t)s * rcap + d;
                if constexpr (ha_packed<KB, NV>()) {
                    const uint64_t kk = (uint64_t)skb[k], vv = svb[0][k];
                    reinterpret_cast<uint4 *>(rq.ent)[e] = make_uint4((uint32_t)kk, (uint32_t)(kk >> 32), (uint32_t)vv,
                                                                      (uint32_t)(vv >> 32));
                } else {
                    reinterpret_cast<KB *>(rq.ent)[e] = skb[k];
#pragma unroll
                    for (int v = 0; v < NV; v++) rq.vbits[v][e] = svb[v][k];
                }
            } else {  // sub-bucket region full (an unlucky split): straight into the HBM table
                uint64_t vv[NV > 0 ? NV : 1];
#pragma unroll
                for (int v = 0; v < NV; v++) vv[v] = svb[v][k];
                ha_global_row<NV>(g, (uint64_t)skb[k], vv);
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < S) rq.fills[(uint64_t)ui * S + threadIdx.x] = cursor[threadIdx.x];
}

// ---- direct (P == 1): each workgroup aggregates a row range of the raw columns ------------
template <typename K, int NV, bool N>
__global__ __launch_bounds__(HB_THREADS) void k_ha_direct(HaParams hp, HaTable g) {
    using KB = kb_t<K>;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const LdsTable<KB> t = lt_layout<KB, NV, N>(lds_raw);
    lt_init<KB, NV, N>(t, HB_THREADS);
    __syncthreads();
    const uint64_t row_begin = (uint64_t)blockIdx.x * hp.rows_per_wg;
    const uint64_t row_end = min(hp.n, row_begin + hp.rows_per_wg);
    const K *keys = static_cast<const K *>(hp.keys);
    constexpr int U = 4;
    for (uint64_t b0 = row_begin; b0 < row_end; b0 += (uint64_t)U * HB_THREADS) {
        KB kb[U];
        uint64_t vb[U][NV > 0 ? NV : 1];
        bool valid[U];
#pragma unroll
        for (int r = 0; r < U; r++) {
            const uint64_t i = b0 + (uint64_t)r * HB_THREADS + threadIdx.x;
            valid[r] = i < row_end;
            kb[r] = 0;
            if (valid[r]) {
                kb[r] = ha_kb(keys[i]);
#pragma unroll
                for (int v = 0; v < NV; v++) vb[r][v] = ha_load_val(hp.vals[v], hp.vdtype[v], i);
            }
        }
        lt2_add_many<KB, NV, U, N>(t, g, kb, vb, valid);
    }
    __syncthreads();
    lt_merge<KB, NV, N>(t, g, HB_THREADS);
}

// ---- table maintenance / finish -----------------------------------------------------------
template <int NV> __global__ __launch_bounds__(256) void k_ha_rehash(HaTable src, uint64_t src_slots, HaTable dst) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i <= src_slots; i += (uint64_t)gridDim.x * 256) {
        uint64_t s;
        if (i == src_slots) {  // the side slot keeps its place
            if (!src.cnt[i]) continue;
            s = dst.mask + 1;
        } else {
            const uint64_t k = src.keys[i];
            if (k == SET_EMPTY) continue;
            s = ha_slot(dst, k);
            if (s == ~0ULL) continue;
        }
        dst.cnt[s] = src.cnt[i];
#pragma unroll
        for (int v = 0; v < NV; v++) {
            dst.sum[v][s] = src.sum[v][i];
            dst.nn[v][s] = src.nn[v][i];
        }
    }
}

// sortable key bits: signed keys with the sign bit flipped (radix order = value order)
template <typename KB> __device__ inline KB ha_sortable(uint64_t key, int is_signed) {
    const KB k = (KB)key;
    return is_signed ? (KB)(k ^ ((KB)1 << (8 * sizeof(KB) - 1))) : k;
}

template <typename KB>
__global__ __launch_bounds__(256) void k_ha_compact(const uint64_t *keys, const unsigned long long *cnt, uint64_t slots,
                                                    int is_signed, KB *skey, uint32_t *sslot, uint32_t *counter) {
    // 8 consecutive slots per thread, output slots reserved once per workgroup and tile (a
    // counter add per wave was 4e6 same-address atomics for a 2^28-slot table: 47 ms);
    // i == slots is the side slot (occupied when it counted rows)
    __shared__ uint32_t s_w[4];
    __shared__ unsigned long long s_base;
    constexpr int R = 8;
    const uint64_t tile = 256ull * R, step = (uint64_t)gridDim.x * tile;
    for (uint64_t t0 = blockIdx.x * tile; t0 <= slots; t0 += step) {
        const uint64_t i0 = t0 + (uint64_t)threadIdx.x * R;
        uint64_t k[R];
        uint32_t occ = 0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const uint64_t i = i0 + r;
            k[r] = SET_EMPTY;
            if (i < slots) {
                k[r] = keys[i];
                if (k[r] != SET_EMPTY) occ |= 1u << r;
            } else if (i == slots && cnt[i] != 0) {
                occ |= 1u << r;
            }
        }
        uint64_t j = block_reserve<256>((uint32_t)__popc(occ), s_w, &s_base, counter);
#pragma unroll
        for (int r = 0; r < R; r++) {
            if (!((occ >> r) & 1)) continue;
            skey[j] = ha_sortable<KB>(k[r], is_signed);
            sslot[j] = (uint32_t)(i0 + r);
            j++;
        }
    }
}

template <typename KB, int NV>
__global__ __launch_bounds__(256) void k_ha_gather(HaTable g, const KB *skey, const uint32_t *sslot, uint64_t m,
                                                   int is_signed, int64_t *okey, int64_t *ocnt, uint64_t *osum,
                                                   int64_t *onn) {
    for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
        const uint32_t s = sslot[j];
        const KB kb = ha_sortable<KB>((uint64_t)skey[j], is_signed);  // the flip is its own inverse
        if constexpr (sizeof(KB) == 4) okey[j] = is_signed ? (int64_t)(int32_t)kb : (int64_t)kb;
        else okey[j] = (int64_t)kb;
        const uint64_t c = g.cnt[s];
        ocnt[j] = (int64_t)c;
#pragma unroll
        for (int v = 0; v < NV; v++) {
            osum[(uint64_t)v * m + j] = g.sum[v][s];
            onn[(uint64_t)v * m + j] = ((g.vfloat >> v) & 1) ? (int64_t)g.nn[v][s] : (int64_t)c;
        }
    }
}

// ---- first-appearance order of the groups (groupby(key, assume_sparse=True) with sort=False:
// the ordered_set's ordinal order, hash_primitives.hpp:96-281, without building the set) ----
// gidx[slot] = the group's index in the key-sorted result
__global__ __launch_bounds__(256) void k_ha_gidx(const uint32_t *sslot, uint64_t m, uint32_t *gidx) {
    for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) gidx[sslot[j]] = (uint32_t)j;
}

// Rows [r0, r1): a row whose key differs from the row before it (a run head; every other row
// cannot be its key's first) probes the HBM table read-only and lowers its group's first row.
// stats[0] += groups seen for the first time, stats[1] += run heads, stats[2] |= 1 if a key is
// missing from the table (the caller passed another column).
// one row of the scan: a run head probes the table read-only and lowers its group's first row
template <typename K>
__device__ inline void ha_first_row(K k, uint64_t row, const HaTable &g, const uint32_t *gidx,
                                    unsigned long long *first, uint32_t &newly, uint32_t &lost) {
    const uint64_t kb = (uint64_t)ha_kb<K>(k);
    uint64_t s = g.mask + 1;
    if (kb != SET_EMPTY) {
        s = hash64(kb) & g.mask;
        int p = 0;
        for (; p < HA_MAX_PROBE; p++) {
            const uint64_t cur = g.keys[s];
            if (cur == kb) break;
            if (cur == SET_EMPTY) {
                p = HA_MAX_PROBE;
                break;
            }
            s = (s + 1) & g.mask;
        }
        if (p == HA_MAX_PROBE) {
            lost = 1;
            return;
        }
    }
    unsigned long long *f = first + gidx[s];
    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= row) return;
    newly += atomicMin(f, (unsigned long long)row) == ~0ull;
}

// Rows [0, nrow) of a chunk starting at global row `base` (keys 16-B aligned; keys[-1] is
// readable when base > 0): a lane takes 16 B of consecutive keys per step, two steps in
// flight; a row whose key differs from the row before it (a run head -- every other row
// cannot be its key's first) probes the HBM table.  stats[0] += groups seen for the first
// time, stats[1] += run heads, stats[2] |= 1 if a key is missing from the table (the caller
// passed another column).
template <typename K>
__global__ __launch_bounds__(256) void k_ha_first(const K *keys, uint64_t nrow, uint64_t base, HaTable g,
                                                  const uint32_t *gidx, unsigned long long *first,
                                                  unsigned long long *stats) {
    constexpr int V = 16 / sizeof(K);
    struct alignas(16) Vec { K k[V]; };
    const Vec *src = reinterpret_cast<const Vec *>(keys);
    uint32_t newly = 0, heads = 0, lost = 0;
    const uint64_t nvec = nrow / V, stride = (uint64_t)gridDim.x * 256;
    const int lane = threadIdx.x & 63;
    // every wave runs both loops with a wave-uniform trip count (lanes past nvec are guarded,
    // not retired): the neighbour shuffle below needs lane - 1 to hold vector v - 1 in the
    // same call
    auto vec = [&](uint64_t v, const Vec &x) {
        // the row before this lane's first is the previous lane's last (lane 0: a load)
        K prev = __shfl_up(x.k[V - 1], 1, 64);
        if (v >= nvec) return;
        const bool has_prev = base + v * V > 0;
        if (lane == 0 && has_prev) prev = keys[v * V - 1];
#pragma unroll
        for (int j = 0; j < V; j++) {
            const bool head = j ? x.k[j] != x.k[j - 1] : (!has_prev || x.k[0] != prev);
            if (head) {
                heads++;
                ha_first_row<K>(x.k[j], base + v * V + j, g, gidx, first, newly, lost);
            }
        }
    };
    const Vec none{};
    uint64_t w = blockIdx.x * 256ull + (threadIdx.x & ~63u);  // the wave's first vector
    for (; w + stride < nvec; w += 2 * stride) {
        const uint64_t va = w + lane, vb = va + stride;
        const Vec a = va < nvec ? src[va] : none, b = vb < nvec ? src[vb] : none;
        vec(va, a);
        vec(vb, b);
    }
    for (; w < nvec; w += stride) {
        const uint64_t va = w + lane;
        vec(va, va < nvec ? src[va] : none);
    }
    // the last nrow % V rows
    for (uint64_t i = nvec * V + blockIdx.x * 256ull + threadIdx.x; i < nrow; i += stride) {
        const K k = keys[i];
        if (base + i > 0 && keys[i - 1] == k) continue;
        heads++;
        ha_first_row<K>(k, base + i, g, gidx, first, newly, lost);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        newly += __shfl_xor(newly, off, 64);
        heads += __shfl_xor(heads, off, 64);
        lost |= __shfl_xor(lost, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (newly) atomicAdd(&stats[0], (unsigned long long)newly);
        if (heads) atomicAdd(&stats[1], (unsigned long long)heads);
        if (lost) atomicOr(&stats[2], 1ull);
    }
}

// fallback ranks: the ordinal of each group's key in an ordered_set built over all rows
__global__ __launch_bounds__(256) void k_ha_set_rank(const int64_t *okey, uint64_t m, int kisz, SetDev set,
                                                     unsigned long long *rank) {
    for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
        uint64_t kb = (uint64_t)okey[j];
        if (kisz < 8) kb &= (1ull << (8 * kisz)) - 1;  // the set holds the native bits zero-extended
        const int64_t o = set_lookup_bits(set, kb);
        rank[j] = o < 0 ? ~0ull : (unsigned long long)o;
    }
}

__global__ __launch_bounds__(256) void k_ha_iota(uint32_t *idx, uint64_t m) {
    for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) idx[j] = (uint32_t)j;
}

// result columns (key | count | sum[nv] | nonnull[nv], m each) permuted by order
__global__ __launch_bounds__(256) void k_ha_permute(const int64_t *src, int64_t *dst, uint64_t m, int ncols,
                                                    const uint32_t *order) {
    for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
        const uint64_t o = order[j];
        for (int c = 0; c < ncols; c++) dst[(uint64_t)c * m + j] = src[(uint64_t)c * m + o];
    }
}

// First row of every key of a dense key range [vmin, vmin + span): the run heads of rows
// [0, nrow) of a chunk starting at global row `base` (16-B aligned keys, keys[-1] readable when
// base > 0) lower first[key - vmin]; stats[0] += keys seen for the first time, stats[1] += run
// heads.  Same wave-uniform loop as k_ha_first, with a direct index instead of a table probe.
template <typename K>
__global__ __launch_bounds__(256) void k_dense_first(const K *keys, uint64_t nrow, uint64_t base, int64_t vmin, uint64_t span,
                                                     unsigned long long *first, unsigned long long *stats) {
    constexpr int V = 16 / sizeof(K);
    struct alignas(16) Vec { K k[V]; };
    const Vec *src = reinterpret_cast<const Vec *>(keys);
    uint32_t newly = 0, heads = 0;
    const uint64_t nvec = nrow / V, stride = (uint64_t)gridDim.x * 256;
    const int lane = threadIdx.x & 63;
    auto row_head = [&](K k, uint64_t row) {
        heads++;
        const uint64_t off = (uint64_t)((int64_t)k - vmin);
        if (off >= span) return;
        unsigned long long *f = first + off;
        if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= row) return;
        newly += atomicMin(f, (unsigned long long)row) == ~0ull;
    };
    auto vec = [&](uint64_t v, const Vec &x) {
        K prev = __shfl_up(x.k[V - 1], 1, 64);
        if (v >= nvec) return;
        const bool has_prev = base + v * V > 0;
        if (lane == 0 && has_prev) prev = keys[v * V - 1];
#pragma unroll
        for (int j = 0; j < V; j++)
            if (j ? x.k[j] != x.k[j - 1] : (!has_prev || x.k[0] != prev)) row_head(x.k[j], base + v * V + j);
    };
    const Vec none{};
    uint64_t w = blockIdx.x * 256ull + (threadIdx.x & ~63u);
    for (; w + stride < nvec; w += 2 * stride) {
        const uint64_t va = w + lane, vb = va + stride;
        const Vec a = va < nvec ? src[va] : none, b = vb < nvec ? src[vb] : none;
        vec(va, a);
        vec(vb, b);
    }
    for (; w < nvec; w += stride) {
        const uint64_t va = w + lane;
        vec(va, va < nvec ? src[va] : none);
    }
    for (uint64_t i = nvec * V + blockIdx.x * 256ull + threadIdx.x; i < nrow; i += stride) {
        const K k = keys[i];
        if (base + i > 0 && keys[i - 1] == k) continue;
        row_head(k, base + i);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        newly += __shfl_xor(newly, off, 64);
        heads += __shfl_xor(heads, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (newly) atomicAdd(&stats[0], (unsigned long long)newly);
        if (heads) atomicAdd(&stats[1], (unsigned long long)heads);
    }
}

// fr[j] = first row of labels[j] (sort key), idx[j] = j
__global__ __launch_bounds__(256) void k_dense_first_gather(const int64_t *labels, uint64_t m, int64_t vmin,
                                                            const unsigned long long *first, unsigned long long *fr, uint32_t *idx) {
    for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
        fr[j] = first[(uint64_t)(labels[j] - vmin)];
        idx[j] = (uint32_t)j;
    }
}

__global__ __launch_bounds__(256) void k_widen_u32(const uint32_t *src, uint64_t m, int64_t *dst) {
    for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) dst[j] = src[j];
}

// occupied cells of a count grid slice (any integer item size): flag[j] = count[j] != 0
__global__ __launch_bounds__(256) void k_nz_flags(const void *counts, int isz, uint64_t range, uint32_t *flag) {
    for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j < range; j += (uint64_t)gridDim.x * 256) {
        uint64_t c;
        switch (isz) {
        case 1: c = static_cast<const uint8_t *>(counts)[j]; break;
        case 2: c = static_cast<const uint16_t *>(counts)[j]; break;
        case 4: c = static_cast<const uint32_t *>(counts)[j]; break;
        default: c = static_cast<const uint64_t *>(counts)[j];
        }
        flag[j] = c != 0;
    }
}
// gidx[pos[j]] = j for the flagged cells; the group's first row and its index for the sort
__global__ __launch_bounds__(256) void k_nz_compact(const uint32_t *flag, const uint32_t *pos, uint64_t range,
                                                    const unsigned long long *first, uint32_t *gidx,
                                                    unsigned long long *fr, uint32_t *idx) {
    for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j < range; j += (uint64_t)gridDim.x * 256) {
        if (!flag[j]) continue;
        const uint32_t g = pos[j];
        gidx[g] = (uint32_t)j;
        fr[g] = first[j];
        idx[g] = g;
    }
}
// out[i] = src[gidx[perm[i]]] (items of isz bytes); labels: out[i] = vmin + gidx[perm[i]] as isz bytes
__global__ __launch_bounds__(256) void k_take_items(const void *src, int isz, const uint32_t *gidx, const uint32_t *perm,
                                                    uint64_t m, void *out, int labels, int64_t vmin) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
        const uint32_t j = gidx[perm[i]];
        const uint64_t v = labels ? (uint64_t)(vmin + (int64_t)j)
                         : isz == 8 ? static_cast<const uint64_t *>(src)[j]
                         : isz == 4 ? static_cast<const uint32_t *>(src)[j]
                         : isz == 2 ? static_cast<const uint16_t *>(src)[j]
                                    : static_cast<const uint8_t *>(src)[j];
        switch (isz) {
        case 1: static_cast<uint8_t *>(out)[i] = (uint8_t)v; break;
        case 2: static_cast<uint16_t *>(out)[i] = (uint16_t)v; break;
        case 4: static_cast<uint32_t *>(out)[i] = (uint32_t)v; break;
        default: static_cast<uint64_t *>(out)[i] = v;
        }
    }
}

// combined key of a multi-key groupby: sum_j (key_j - min_j) * mult_j as int64
// (groupby.py:248-288 _combine: the cartesian ordinal, first key most significant)
constexpr int HC_MAX_KEYS = 8;
struct HcParams {
    const void *col[HC_MAX_KEYS];
    int32_t dtype[HC_MAX_KEYS];
    int64_t min[HC_MAX_KEYS];
    int64_t mult[HC_MAX_KEYS];
    int nkeys;
};

__device__ inline int64_t hc_load(const void *p, int dtype, uint64_t i) {
    switch (dtype) {
    case VH_I64: return static_cast<const int64_t *>(p)[i];
    case VH_I32: return static_cast<const int32_t *>(p)[i];
    case VH_I16: return static_cast<const int16_t *>(p)[i];
    case VH_I8: return static_cast<const int8_t *>(p)[i];
    case VH_U64: return (int64_t) static_cast<const uint64_t *>(p)[i];
    case VH_U32: return static_cast<const uint32_t *>(p)[i];
    case VH_U16: return static_cast<const uint16_t *>(p)[i];
    default: return static_cast<const uint8_t *>(p)[i];
    }
}

__global__ __launch_bounds__(256) void k_combine_keys(HcParams p, uint64_t n, int64_t *out) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        int64_t c = 0;
        for (int j = 0; j < p.nkeys; j++) c += (hc_load(p.col[j], p.dtype[j], i) - p.min[j]) * p.mult[j];
        out[i] = c;
    }
}

}  // namespace vh

using namespace vh;

struct vh_hashagg {
    int key_dtype = VH_I32;
    int nv = 0;
    int vdtype[HA_MAX_V] = {VH_F64, VH_F64};
    uint32_t vfloat = 0;
    uint32_t nnmask = 0;  // value columns whose non-NaN count is read (count(v), mean)
    uint64_t slots = 0;  // HBM table slots (power of two), 0 = not allocated
    DevBuf tab;          // keys | cnt | sum[nv] | nn[nv] (slots + 1 each) | used, err
    DevBuf out;
    DevBuf xres;            // groups after a cross-rank exchange (vh_hashagg_exchange)
    const char *res = nullptr;  // result columns: key | count | sum[nv] | nonnull[nv], ngroups each
    uint64_t ngroups = 0;
    bool finished = false;
    uint64_t rows = 0;
};

namespace vh {

// Partition scratch shared by every hashagg of a device (the regions of a 1e9-row update
// are ~16 GB: allocating them per query would cost more than the query).  Updates hold
// the device's lock; they are stream-ordered on the library stream anyway.
struct HaScratch {
    std::mutex mu;
    DevBuf sample, meta, entries, vbits, stage, entries2, vbits2, meta2;
};
static HaScratch &scratch() {
    static std::mutex g;
    static std::map<int, std::unique_ptr<HaScratch>> m;
    std::lock_guard<std::mutex> lk(g);
    auto &p = m[current_device()];
    if (!p) p = std::make_unique<HaScratch>();
    return *p;
}

static bool key_dtype_ok(int d) { return d != VH_F64 && d != VH_F32 && d != VH_BOOL; }
static bool key_signed(int d) { return d == VH_I64 || d == VH_I32 || d == VH_I16 || d == VH_I8; }
static int key_bits_size(int d) { return dtype_itemsize(d) == 8 ? 8 : 4; }

// table arrays hold slots + 1 entries (the side slot); 8 spare words for used / err
static uint64_t tab_bytes(uint64_t slots, int nv) { return (slots + 1) * 8 * (2 + 2 * (uint64_t)nv) + 256; }

static HaTable table_view(void *base, uint64_t slots, int nv, uint32_t vfloat, uint32_t nnmask = 0) {
    HaTable g{};
    unsigned char *p = static_cast<unsigned char *>(base);
    const uint64_t a = 8 * (slots + 1);
    g.keys = reinterpret_cast<uint64_t *>(p);
    p += a;
    g.cnt = reinterpret_cast<unsigned long long *>(p);
    p += a;
    for (int v = 0; v < nv; v++) {
        g.sum[v] = reinterpret_cast<unsigned long long *>(p);
        p += a;
        g.nn[v] = reinterpret_cast<unsigned long long *>(p);
        p += a;
    }
    g.used = reinterpret_cast<uint32_t *>(p);
    g.err = g.used + 1;
    g.mask = slots - 1;
    g.max_used = (uint32_t)std::min<uint64_t>(slots / 4 * 3, 0xffffffffu);
    g.vfloat = vfloat;
    g.nnmask = nnmask;
    g.nv = nv;
    return g;
}

static void table_alloc(DevBuf &buf, uint64_t slots, int nv) {
    buf.ensure(tab_bytes(slots, nv));
    hipStream_t st = stream();
    const uint64_t a = 8 * (slots + 1);
    VH_HIP(hipMemsetAsync(buf.ptr, 0xff, a, st));  // keys = EMPTY
    VH_HIP(hipMemsetAsync(static_cast<char *>(buf.ptr) + a, 0, tab_bytes(slots, nv) - a, st));
}

template <typename F> static void dispatch_nv(int nv, F &&f) {
    switch (nv) {
    case 0: f(std::integral_constant<int, 0>()); break;
    case 1: f(std::integral_constant<int, 1>()); break;
    default: f(std::integral_constant<int, 2>());
    }
}

#define VH_DISPATCH_KEY(code, K, ...)                                   \
    switch (code) {                                                     \
    case VH_I64: { using K = int64_t; __VA_ARGS__; break; }             \
    case VH_I32: { using K = int32_t; __VA_ARGS__; break; }             \
    case VH_I16: { using K = int16_t; __VA_ARGS__; break; }             \
    case VH_I8: { using K = int8_t; __VA_ARGS__; break; }               \
    case VH_U64: { using K = uint64_t; __VA_ARGS__; break; }            \
    case VH_U32: { using K = uint32_t; __VA_ARGS__; break; }            \
    case VH_U16: { using K = uint16_t; __VA_ARGS__; break; }            \
    case VH_U8: { using K = uint8_t; __VA_ARGS__; break; }              \
    default: fail(VH_ERR_ARG, "hashagg: unsupported key dtype");       \
    }

template <typename F> static void dispatch_kb(int key_dtype, F &&f) {
    if (key_bits_size(key_dtype) == 8) f(uint64_t());
    else f(uint32_t());
}

static uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// grow (rehash) the HBM table to hold `need` keys at <= 1/2 load
static void ensure_table(vh_hashagg *h, uint64_t need) {
    const uint64_t want = std::max<uint64_t>(1u << 16, next_pow2(2 * need));
    if (h->slots >= want) return;
    if (want > (1ull << 31)) fail(VH_ERR_RUNTIME, "hashagg: too many groups for the fused hash path");
    if (!h->slots) {
        table_alloc(h->tab, want, h->nv);
        h->slots = want;
        return;
    }
    DevBuf nt;
    table_alloc(nt, want, h->nv);
    const HaTable src = table_view(h->tab.ptr, h->slots, h->nv, h->vfloat);
    HaTable dst = table_view(nt.ptr, want, h->nv, h->vfloat);
    dispatch_nv(h->nv, [&](auto nvc) {
        constexpr int NV = decltype(nvc)::value;
        hipLaunchKernelGGL(k_ha_rehash<NV>, dim3(blocks_for(h->slots + 1, 256, 8)), dim3(256), 0, stream(), src,
                           h->slots, dst);
    });
    VH_HIP(hipGetLastError());
    std::swap(h->tab.ptr, nt.ptr);
    std::swap(h->tab.bytes, nt.bytes);
    h->slots = want;
}

// used slots (not counting the side slot) and the error word
static uint32_t read_used(vh_hashagg *h, uint32_t *err) {
    const HaTable g = table_view(h->tab.ptr, h->slots, h->nv, h->vfloat);
    thread_local PinnedBuf pb;  // a page-locked target: no staged pageable copy
    pb.ensure(64);
    uint32_t *ue = pb.as<uint32_t>();
    VH_HIP(hipMemcpyAsync(ue, g.used, 8, hipMemcpyDeviceToHost, stream()));
    VH_HIP(hipStreamSynchronize(stream()));
    if (err) *err = ue[1];
    return ue[0];
}

static bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

static int blocks_per_cu(const void *kernel, int threads, size_t lds) {
    int nb = 0;
    VH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, threads, lds));
    return std::max(1, nb);
}

// one update over n <= 2^30 device-resident rows
static void update_device(vh_hashagg *h, HaScratch &S, const void *keys, const void *const *vals, uint64_t n) {
    hipStream_t st = stream();
    const int nv = h->nv;
    const int kbs = key_bits_size(h->key_dtype);
    // ---- sample: fine bucket histogram + distinct estimate
    const uint64_t sslots = 1ull << 21;
    const uint64_t nbatch = (n + HA_BATCH - 1) / HA_BATCH;
    const uint64_t sblocks = std::min<uint64_t>(nbatch, HA_SAMPLE_BLOCKS);
    const uint64_t bstride = std::max<uint64_t>(HA_BATCH, n / sblocks);
    const uint32_t FINE = 1u << HA_FINE_LOG2;
    S.sample.ensure(sslots * 12 + 8 * FINE + 64);
    uint64_t *skeys = S.sample.as<uint64_t>();
    uint32_t *scnt = reinterpret_cast<uint32_t *>(skeys + sslots);
    unsigned long long *fine = reinterpret_cast<unsigned long long *>(scnt + sslots);
    unsigned long long *stats = fine + FINE;
    VH_HIP(hipMemsetAsync(skeys, 0xff, 8 * sslots, st));
    VH_HIP(hipMemsetAsync(scnt, 0, 4 * sslots + 8 * FINE + 64, st));
    {
        TimedScope ts("ha_sample");
        VH_DISPATCH_KEY(h->key_dtype, K,
                        hipLaunchKernelGGL(k_ha_sample<K>, dim3(sblocks), dim3(HA_THREADS), 0, st,
                                           static_cast<const K *>(keys), n, bstride, fine, skeys, scnt, sslots - 1));
        hipLaunchKernelGGL(k_ha_sample_stats, dim3(blocks_for(sslots, 256, 4)), dim3(256), 0, st, scnt, sslots, stats);
        VH_HIP(hipGetLastError());
    }
    thread_local PinnedBuf fb;  // page-locked sample read-back
    fb.ensure(8 * (FINE + 4));
    const uint64_t *fh = fb.as<uint64_t>();
    VH_HIP(hipMemcpyAsync(fb.ptr, fine, 8 * (FINE + 4), hipMemcpyDeviceToHost, st));
    VH_HIP(hipStreamSynchronize(st));
    uint64_t sampled = 0;
    for (uint32_t i = 0; i < FINE; i++) sampled += fh[i];
    const double ds = (double)fh[FINE], f1 = (double)fh[FINE + 1], f2 = (double)fh[FINE + 2];
    // clustered keys: most sampled rows equal their next row (a sorted key column)
    bool runs = sampled > 0 && (double)fh[FINE + 3] > 0.5 * (double)sampled;
    if (const char *e = getenv("VH_HA_RUNS")) runs = atoi(e) != 0;  // A/B: same results either way
    double dest;
    if (sampled >= n) dest = ds;  // every row sampled: exact
    else dest = f2 > 0 ? ds + f1 * f1 / (2 * f2) : ds + f1 * (f1 - 1) / 2;  // Chao1
    dest = std::min<double>(dest, (double)n);
    uint32_t used_before = h->slots ? read_used(h, nullptr) : 0;
    ensure_table(h, (uint64_t)dest + used_before);
    HaTable g = table_view(h->tab.ptr, h->slots, nv, h->vfloat, h->nnmask);

    // the narrow LDS table (twice the slots) when no count(v) is read and keys are 4 bytes
#ifndef VH_HA_NARROW_DEFAULT
#define VH_HA_NARROW_DEFAULT 1
#endif
    static const bool narrow_on = [] {
        const char *e = getenv("VH_HA_NARROW");
        return e ? atoi(e) != 0 : VH_HA_NARROW_DEFAULT != 0;
    }();
    const bool narrow = narrow_on && kbs == 4 && nv <= 1 && h->nnmask == 0;
    const double target_keys = narrow ? lt_target_keys<true>() : lt_target_keys<false>();
    uint32_t p_log2 = 0;
    while (p_log2 < HA_MAX_P_LOG2 && dest / (double)(1u << p_log2) > target_keys) p_log2++;

    HaParams hp{};
    hp.keys = keys;
    for (int v = 0; v < nv; v++) {
        hp.vals[v] = vals[v];
        hp.vdtype[v] = h->vdtype[v];
    }
    hp.n = n;
#ifdef VH_ABLATION
    if (const char *dbg = getenv("VH_HA_DEBUG")) hp.debug = (uint32_t)atoi(dbg);
#endif
    hp.p_log2 = p_log2;
    hp.P = 1u << p_log2;
    const size_t lt_lds = lt_bytes(nv, kbs, narrow);
    if (p_log2 == 0) {
        // ---- direct: one LDS table per workgroup over a contiguous row range
        int bpc = 1;
        // f(kernel) for this key type / NV / table width
        auto with_direct = [&](auto &&f) {
            VH_DISPATCH_KEY(h->key_dtype, K, dispatch_nv(nv, [&](auto nvc) {
                constexpr int NV = decltype(nvc)::value;
                if constexpr (sizeof(kb_t<K>) == 4 && NV <= 1) {
                    if (narrow) f(k_ha_direct<K, NV, true>);
                    else f(k_ha_direct<K, NV, false>);
                } else {
                    f(k_ha_direct<K, NV, false>);
                }
            }));
        };
        with_direct([&](auto kernel) { bpc = blocks_per_cu(reinterpret_cast<const void *>(kernel), HB_THREADS, lt_lds); });
        const uint64_t W = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)cu_count() * bpc,
                                                                     (n + 4 * HB_THREADS - 1) / (4 * HB_THREADS)));
        hp.rows_per_wg = (n + W - 1) / W;
        TimedScope ts("ha_direct");
        with_direct([&](auto kernel) { hipLaunchKernelGGL(kernel, dim3((unsigned)W), dim3(HB_THREADS), lt_lds, st, hp, g); });
        VH_HIP(hipGetLastError());
        return;
    }
    const uint32_t P = hp.P;
    std::vector<uint64_t> bh(P, 0);
    for (uint32_t i = 0; i < FINE; i++) bh[i >> (HA_FINE_LOG2 - p_log2)] += fh[i];

    // ---- pass A geometry
    // the fast pass A: 4- or 8-byte keys, float64 values, 16-byte aligned columns; rows past
    // the last multiple of 8 go straight to the HBM table.  4-byte keys with at most one
    // value take the multi-batch commit (k_ha_scatter_k4) with as many batches per commit
    // as the LDS holds (VH_HA_K4=0: the one-batch kernel, for A/B runs).
    const int kisz = dtype_itemsize(h->key_dtype);
    bool fast = (kisz == 4 || kisz == 8) && aligned16(keys) && n >= 8;
    for (int v = 0; v < nv; v++) fast = fast && h->vdtype[v] == VH_F64 && aligned16(vals[v]);
#ifndef VH_HA_RUNS_SB_DEFAULT
#define VH_HA_RUNS_SB_DEFAULT 1
#endif
#ifndef VH_HA_K4_DEFAULT
#define VH_HA_K4_DEFAULT 1
#endif
    static const bool k4_on = [] {
        const char *e = getenv("VH_HA_K4");
        return e ? atoi(e) != 0 : VH_HA_K4_DEFAULT != 0;
    }();
    const bool k4 = fast && k4_on && kisz == 4 && nv <= 1;
    int sb = 0;
    if (k4) {
        // clustered keys (RUNS) fold most groups before the partition: fewer batches per commit
        // keep the registers of one commit's rows low (VH_HA_RUNS_SB: A/B)
        int sb_max = 3;
        if (runs) {
            sb_max = VH_HA_RUNS_SB_DEFAULT;
            if (const char *e = getenv("VH_HA_RUNS_SB")) sb_max = std::max(1, std::min(3, atoi(e)));
        }
        for (sb = sb_max; sb > 1 && ha_fast_lds_bytes(nv, sb, P) > 160 * 1024; sb--) {
        }
    }
    const size_t lds_a = k4 ? ha_fast_lds_bytes(nv, sb, P) : ha_scatter_lds_bytes(nv, kbs, P);
    int bpc = 1;
    auto k4_kernel = [&](auto kc, auto nvc, auto sbc) {
        using K = decltype(kc);
        constexpr int NV = decltype(nvc)::value, SB = decltype(sbc)::value;
        return runs ? reinterpret_cast<const void *>(k_ha_scatter_k4<K, NV, SB, true>)
                    : reinterpret_cast<const void *>(k_ha_scatter_k4<K, NV, SB, false>);
    };
    auto with_k4 = [&](auto &&f) {  // f(kernel instance) for this key type / NV / SB
        auto by_sb = [&](auto kc, auto nvc) {
            if (sb == 3) f(kc, nvc, std::integral_constant<int, 3>());
            else if (sb == 2) f(kc, nvc, std::integral_constant<int, 2>());
            else f(kc, nvc, std::integral_constant<int, 1>());
        };
        auto by_nv = [&](auto kc) {
            if (nv == 1) by_sb(kc, std::integral_constant<int, 1>());
            else by_sb(kc, std::integral_constant<int, 0>());
        };
        if (h->key_dtype == VH_I32) by_nv(int32_t());
        else by_nv(uint32_t());
    };
    if (k4) {
        with_k4([&](auto kc, auto nvc, auto sbc) { bpc = blocks_per_cu(k4_kernel(kc, nvc, sbc), HA_THREADS, lds_a); });
    } else {
        VH_DISPATCH_KEY(h->key_dtype, K, dispatch_nv(nv, [&](auto nvc) {
            constexpr int NV = decltype(nvc)::value;
            bpc = blocks_per_cu(reinterpret_cast<const void *>(k_ha_scatter<K, NV>), HA_THREADS, lds_a);
        }));
    }
    bpc = std::min(bpc, 4);
    const uint32_t W = std::min<uint32_t>(1024, (uint32_t)cu_count() * bpc);
    // pass-A workgroup w takes batches w, w + W, ...: at most ceil(batches / W) of them
    const uint64_t rows_per_wg = (nbatch + W - 1) / W * HA_BATCH;
    std::vector<uint32_t> cap(P);
    std::vector<uint64_t> toff(P);
    uint64_t stride = 0;
    for (uint32_t t = 0; t < P; t++) {
        const double e = (double)rows_per_wg * (double)bh[t] / (double)std::max<uint64_t>(sampled, 1);
        uint64_t c = (uint64_t)(e * 1.04 + 6.0 * std::sqrt(e + 1.0)) + 32;
        c = std::min<uint64_t>((c + 7) & ~uint64_t(7), rows_per_wg + 8);
        cap[t] = (uint32_t)c;
        toff[t] = stride;
        stride += c;
    }
    if (stride + rows_per_wg >= (uint64_t)HA_DEST_OVERFLOW) fail(VH_ERR_RUNTIME, "hashagg: region table too large");
    const uint64_t total = stride * W + (uint64_t)W * HA_THREADS;  // regions + dummy slots
    if (nv == 1 && (kbs == 8 || VH_HA_PACK4)) {
        S.entries.ensure(16 * total + 64);  // packed {key, value} entries
    } else {
        S.entries.ensure((uint64_t)kbs * total + 16);
        if (nv) S.vbits.ensure(8 * total * nv + 32);
    }
    // pass-B work units: buckets split over ranges of pass-A workgroups by expected size
    std::vector<HaUnit> units;
    const double target = std::max(1.0, (double)n / ((double)cu_count() * 2));
    for (uint32_t t = 0; t < P; t++) {
        const double e = (double)n * (double)bh[t] / (double)std::max<uint64_t>(sampled, 1);
        const uint32_t gq = (uint32_t)std::min<double>(W, std::max(1.0, std::ceil(e / target)));
        for (uint32_t k = 0; k < gq; k++)
            units.push_back({t, (uint32_t)((uint64_t)W * k / gq), (uint32_t)((uint64_t)W * (k + 1) / gq), 0});
    }
    const uint64_t meta_bytes = 4 * (uint64_t)P + 8 * (uint64_t)P + 4 * (uint64_t)P * W + sizeof(HaUnit) * units.size() + 256;
    S.meta.ensure(meta_bytes);
    unsigned char *mb = S.meta.as<unsigned char>();
    uint64_t *d_toff = reinterpret_cast<uint64_t *>(mb);
    HaUnit *d_units = reinterpret_cast<HaUnit *>(d_toff + P);
    uint32_t *d_cap = reinterpret_cast<uint32_t *>(d_units + units.size());
    uint32_t *d_fills = d_cap + P;
    VH_HIP(hipMemcpyAsync(d_toff, toff.data(), 8 * (uint64_t)P, hipMemcpyHostToDevice, st));
    VH_HIP(hipMemcpyAsync(d_units, units.data(), sizeof(HaUnit) * units.size(), hipMemcpyHostToDevice, st));
    VH_HIP(hipMemcpyAsync(d_cap, cap.data(), 4 * (uint64_t)P, hipMemcpyHostToDevice, st));
    hp.W = W;
    hp.rows_per_wg = rows_per_wg;
    hp.wg_stride = stride;
    hp.cap = d_cap;
    hp.toff = d_toff;
    hp.fills = d_fills;
    hp.ent = S.entries.ptr;
    hp.dummy0 = stride * W;
    if (!(nv == 1 && (kbs == 8 || VH_HA_PACK4)))
        for (int v = 0; v < nv; v++) hp.vbits[v] = S.vbits.as<uint64_t>() + (uint64_t)v * total;
    {
        TimedScope ts(fast ? "ha_scatter_f64" : "ha_scatter");
        if (fast) {
            const uint64_t n8 = n & ~uint64_t(7);
            hp.n = n8;
            if (k4) {
                with_k4([&](auto kc, auto nvc, auto sbc) {
                    using K = decltype(kc);
                    constexpr int NV = decltype(nvc)::value, SB = decltype(sbc)::value;
                    if (runs) hipLaunchKernelGGL((k_ha_scatter_k4<K, NV, SB, true>), dim3(W), dim3(HA_THREADS), lds_a, st, hp, g);
                    else hipLaunchKernelGGL((k_ha_scatter_k4<K, NV, SB, false>), dim3(W), dim3(HA_THREADS), lds_a, st, hp, g);
                    if (n8 < n) {
                        HaParams ht = hp;
                        ht.n = n;
                        hipLaunchKernelGGL((k_ha_tail<K, NV>), dim3(1), dim3(64), 0, st, ht, g, n8);
                    }
                });
            }
            auto launch = [&](auto kc) {
                using K = decltype(kc);
                dispatch_nv(nv, [&](auto nvc) {
                    constexpr int NV = decltype(nvc)::value;
                    hipLaunchKernelGGL((k_ha_scatter_f64<K, NV>), dim3(W), dim3(HA_THREADS), lds_a, st, hp, g);
                    if (n8 < n) {
                        HaParams ht = hp;
                        ht.n = n;
                        hipLaunchKernelGGL((k_ha_tail<K, NV>), dim3(1), dim3(64), 0, st, ht, g, n8);
                    }
                });
            };
            if (!k4) switch (h->key_dtype) {
            case VH_I32: launch(int32_t()); break;
            case VH_U32: launch(uint32_t()); break;
            case VH_I64: launch(int64_t()); break;
            default: launch(uint64_t());
            }
            hp.n = n;
        } else {
            VH_DISPATCH_KEY(h->key_dtype, K, dispatch_nv(nv, [&](auto nvc) {
                constexpr int NV = decltype(nvc)::value;
                hipLaunchKernelGGL((k_ha_scatter<K, NV>), dim3(W), dim3(HA_THREADS), lds_a, st, hp, g);
            }));
        }
        VH_HIP(hipGetLastError());
    }
    // ---- repartition: more keys per bucket than an LDS table holds (P at its cap)
    static const bool repart_on = [] {  // VH_HA_REPART=0: A/B runs without it
        const char *e = getenv("VH_HA_REPART");
        return !e || atoi(e) != 0;
    }();
    const double kpb = dest / (double)P;
    uint32_t S_sub = 1;
    if (repart_on && p_log2 == HA_MAX_P_LOG2 && kpb > target_keys * 1.25)
        S_sub = std::min<uint32_t>(HR_MAX_S, (uint32_t)std::ceil(kpb / target_keys));
    HaParams hpb = hp;
    std::vector<HaUnit> units_b;
    HaUnit *d_units_b = d_units;
    if (S_sub > 1) {
        const uint32_t U = (uint32_t)units.size();
        std::vector<uint64_t> rbase(U);
        std::vector<uint32_t> rcap(U);
        uint64_t total2 = 0;
        for (uint32_t ui = 0; ui < U; ui++) {
            const HaUnit &un = units[ui];
            // the unit's entries: at most its regions' capacities; expected ~ n p_b * share
            const double e = (double)n * (double)bh[un.bucket] / (double)std::max<uint64_t>(sampled, 1) *
                             (double)(un.w_end - un.w_begin) / (double)W;
            const double es = e / S_sub;
            uint64_t c = (uint64_t)(es * 1.05 + 8.0 * std::sqrt(es + 1.0)) + 64;
            c = (c + 7) & ~uint64_t(7);
            rcap[ui] = (uint32_t)c;
            rbase[ui] = total2;
            total2 += c * S_sub;
        }
        if (nv == 1 && (kbs == 8 || VH_HA_PACK4)) {
            S.entries2.ensure(16 * total2 + 64);
        } else {
            S.entries2.ensure((uint64_t)kbs * total2 + 16);
            if (nv) S.vbits2.ensure(8 * total2 * nv + 32);
        }
        const uint64_t P2 = (uint64_t)U * S_sub;
        units_b.resize(P2);
        std::vector<uint64_t> toff2(P2);
        std::vector<uint32_t> cap2(P2);
        for (uint32_t ui = 0; ui < U; ui++)
            for (uint32_t q = 0; q < S_sub; q++) {
                const uint64_t gi = (uint64_t)ui * S_sub + q;
                units_b[gi] = {(uint32_t)gi, 0, 1, 0};
                toff2[gi] = rbase[ui] + (uint64_t)q * rcap[ui];
                cap2[gi] = rcap[ui];
            }
        S.meta2.ensure(8 * (uint64_t)U + 4 * (uint64_t)U + 8 * P2 + 4 * P2 + 4 * P2 + sizeof(HaUnit) * P2 + 256);
        unsigned char *m2 = S.meta2.as<unsigned char>();
        uint64_t *d_rbase = reinterpret_cast<uint64_t *>(m2);
        uint64_t *d_toff2 = d_rbase + U;
        HaUnit *d_u2 = reinterpret_cast<HaUnit *>(d_toff2 + P2);
        uint32_t *d_rcap = reinterpret_cast<uint32_t *>(d_u2 + P2);
        uint32_t *d_cap2 = d_rcap + U;
        uint32_t *d_fills2 = d_cap2 + P2;
        VH_HIP(hipMemcpyAsync(d_rbase, rbase.data(), 8 * (uint64_t)U, hipMemcpyHostToDevice, st));
        VH_HIP(hipMemcpyAsync(d_rcap, rcap.data(), 4 * (uint64_t)U, hipMemcpyHostToDevice, st));
        VH_HIP(hipMemcpyAsync(d_toff2, toff2.data(), 8 * P2, hipMemcpyHostToDevice, st));
        VH_HIP(hipMemcpyAsync(d_cap2, cap2.data(), 4 * P2, hipMemcpyHostToDevice, st));
        VH_HIP(hipMemcpyAsync(d_u2, units_b.data(), sizeof(HaUnit) * P2, hipMemcpyHostToDevice, st));
        RepartParams rq{};
        rq.S = S_sub;
        rq.p_log2 = p_log2;
        rq.base = d_rbase;
        rq.rcap = d_rcap;
        rq.fills = d_fills2;
        rq.ent = S.entries2.ptr;
        if (!(nv == 1 && (kbs == 8 || VH_HA_PACK4)))
            for (int v = 0; v < nv; v++) rq.vbits[v] = S.vbits2.as<uint64_t>() + (uint64_t)v * total2;
        {
            TimedScope ts("ha_repart");
            dispatch_kb(h->key_dtype, [&](auto kbc) {
                using KB = decltype(kbc);
                dispatch_nv(nv, [&](auto nvc) {
                    constexpr int NV = decltype(nvc)::value;
                    hipLaunchKernelGGL((k_ha_repart<KB, NV>), dim3(U), dim3(HB_THREADS), 0, st, hp, g, d_units, rq);
                });
            });
            VH_HIP(hipGetLastError());
        }
        // pass B over the sub-bucket regions: one "workgroup" per region, units = regions
        hpb.W = 1;
        hpb.wg_stride = 0;
        hpb.cap = d_cap2;
        hpb.toff = d_toff2;
        hpb.fills = d_fills2;
        hpb.ent = S.entries2.ptr;
        for (int v = 0; v < HA_MAX_V; v++) hpb.vbits[v] = rq.vbits[v];
        d_units_b = d_u2;
    } else {
        units_b = units;
    }
    {
        TimedScope ts("ha_reduce");
        const HaParams &hp = hpb;
        const HaUnit *d_units = d_units_b;
        const std::vector<HaUnit> &units = units_b;
        dispatch_kb(h->key_dtype, [&](auto kbc) {
            using KB = decltype(kbc);
            dispatch_nv(nv, [&](auto nvc) {
                constexpr int NV = decltype(nvc)::value;
                const dim3 grid((unsigned)units.size()), block(HB_THREADS);
                if constexpr (sizeof(KB) == 4 && NV <= 1) {
                    if (narrow) hipLaunchKernelGGL((k_ha_reduce<KB, NV, true>), grid, block, lt_lds, st, hp, g, d_units);
                    else hipLaunchKernelGGL((k_ha_reduce<KB, NV, false>), grid, block, lt_lds, st, hp, g, d_units);
                } else {
                    hipLaunchKernelGGL((k_ha_reduce<KB, NV, false>), grid, block, lt_lds, st, hp, g, d_units);
                }
            });
        });
        VH_HIP(hipGetLastError());
    }
}

// ---- set-ordinal grids through the hash aggregation ------------------------------------------
// The Grouper route (groupby.py:97-168,484-533) bins BinnerOrdinal over map_ordinal(key):
// per row a random probe of the set's lookup table, ~100 B of random lines per row from a
// 16 MB table at 1e6 keys (C3: 26 ms).  For count / float64 sum aggregators the same grid
// comes out of the fused hash aggregation: rows aggregate per key (sample, pass A, pass B as
// above), then every key's totals add into the grid cell of its ordinal -- one lookup per
// distinct key instead of one per row.

// aggregator of the grid: what it takes from a key's totals
struct OgAgg {
    int what;  // 0 count(*), 1 non-NaN count of value `slot`, 2 sum of value `slot`
    int slot;
    void *grid;
};
struct OgParams {
    OgAgg a[MAX_FUSED_AGGS];
    int na, kisz;
    uint64_t count, stride;
};

template <int NV> __global__ __launch_bounds__(256) void k_ha_ordgrid(HaTable g, uint64_t slots, SetDev set, OgParams op) {
    for (uint64_t s = blockIdx.x * 256ull + threadIdx.x; s <= slots; s += (uint64_t)gridDim.x * 256) {
        const unsigned long long c = g.cnt[s];
        if (!c) continue;  // empty slot (the side slot holds the all-ones 8-byte key)
        uint64_t kb = s < slots ? g.keys[s] : SET_EMPTY;
        // hashagg sign-extends 1- and 2-byte keys; the set holds their bits zero-extended
        if (op.kisz < 8 && s < slots) kb &= (1ull << (8 * op.kisz)) - 1;
        const int64_t o = set_lookup_bits(set, kb);
        const uint64_t cell = (o < 0 ? 1 : (uint64_t)o >= op.count ? op.count + 2 : (uint64_t)o + 2) * op.stride;
        for (int k = 0; k < op.na; k++) {
            const OgAgg &a = op.a[k];
            if (a.what == 2) {
                const double v = __builtin_bit_cast(double, (uint64_t)g.sum[a.slot][s]);
                if (v != 0.0) atomicAdd(static_cast<double *>(a.grid) + cell, v);
            } else {
                const unsigned long long v = a.what == 0 ? c : g.nn[a.slot][s];
                if (v) atomicAdd(static_cast<unsigned long long *>(a.grid) + cell, v);
            }
        }
    }
}

bool hashagg_bin_set_ordinal(const BinPlan &plan, const FusedAggs &fa, uint64_t n) {
    static const bool on = [] {
        const char *e = getenv("VH_SET_HASHAGG");
        return !e || atoi(e) != 0;
    }();
    if (!on || n < (1u << 22) || plan.nb != 1) return false;
    const BinnerDev &b = plan.b[0];
    if (b.kind != 2 || b.mask || b.flip || !key_dtype_ok(b.dtype)) return false;
    const int kisz = dtype_itemsize(b.dtype);
    const void *vals[HA_MAX_V] = {nullptr, nullptr};
    int nv = 0;
    OgParams op{};
    op.na = fa.na;
    op.kisz = kisz;
    op.count = b.ordinal_count;
    op.stride = b.stride;
    uint32_t nnmask = 0;
    auto slot_of = [&](const void *d) {
        for (int v = 0; v < nv; v++)
            if (vals[v] == d) return v;
        if (nv == HA_MAX_V) return -1;
        vals[nv] = d;
        return nv++;
    };
    for (int k = 0; k < fa.na; k++) {
        const FusedAgg &a = fa.a[k];
        if (a.mask || a.vint) return false;
        op.a[k].grid = a.grid;
        if (a.kind == VH_AGG_COUNT && !a.data) {
            op.a[k].what = 0;
        } else if (a.data && a.dtype == VH_F64 && (a.kind == VH_AGG_COUNT || a.kind == VH_AGG_SUM)) {
            const int sl = slot_of(a.data);
            if (sl < 0) return false;
            op.a[k].slot = sl;
            op.a[k].what = a.kind == VH_AGG_SUM ? 2 : 1;
            if (a.kind == VH_AGG_COUNT) nnmask |= 1u << sl;
        } else {
            return false;
        }
    }
    vh_hashagg h;
    h.key_dtype = b.dtype;
    h.nv = nv;
    h.nnmask = nnmask;
    for (int v = 0; v < nv; v++) {
        h.vdtype[v] = VH_F64;
        h.vfloat |= 1u << v;
    }
    {
        HaScratch &S = scratch();
        std::lock_guard<std::mutex> lk(S.mu);
        constexpr uint64_t CHUNK = 1ull << 30;
        for (uint64_t r0 = 0; r0 < n; r0 += CHUNK) {
            const uint64_t m = std::min(CHUNK, n - r0);
            const void *vp[HA_MAX_V] = {nullptr, nullptr};
            for (int v = 0; v < nv; v++) vp[v] = static_cast<const double *>(vals[v]) + r0;
            update_device(&h, S, static_cast<const char *>(b.data) + r0 * kisz, vp, m);
            uint32_t err = 0;
            const uint32_t used = read_used(&h, &err);
            if (err & 2) return false;  // table overflow: the caller bins the chunk its own way
            if (err & 1) ensure_table(&h, 2 * (uint64_t)used);
        }
    }
    TimedScope ts("ha_ordgrid");
    const HaTable g = table_view(h.tab.ptr, h.slots, nv, h.vfloat, h.nnmask);
    dispatch_nv(nv, [&](auto nvc) {
        constexpr int NV = decltype(nvc)::value;
        hipLaunchKernelGGL(k_ha_ordgrid<NV>, dim3(blocks_for(h.slots + 1, 256, 8)), dim3(256), 0, stream(), g, h.slots,
                           b.set, op);
    });
    VH_HIP(hipGetLastError());
    return true;
}

static size_t sort_tmp_bytes(int kbs, uint64_t m) {
    size_t tmp = 0;
    if (kbs == 8)
        VH_HIP(rocprim::radix_sort_pairs(nullptr, tmp, (uint64_t *)nullptr, (uint64_t *)nullptr, (uint32_t *)nullptr,
                                         (uint32_t *)nullptr, (size_t)m, 0, 64, stream()));
    else
        VH_HIP(rocprim::radix_sort_pairs(nullptr, tmp, (uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                         (uint32_t *)nullptr, (size_t)m, 0, 32, stream()));
    return tmp;
}

// out buffer: skey | skey2 | sslot | sslot2 | counter | sort tmp | okey ocnt osum onn
static char *out_results(vh_hashagg *h, uint64_t m, size_t tmp_bytes) {
    const int kbs = key_bits_size(h->key_dtype);
    const uint64_t ak = (kbs * m + 255) & ~255ull, as = (4 * m + 255) & ~255ull;
    return h->out.as<char>() + 2 * ak + 2 * as + 256 + ((tmp_bytes + 255) & ~255ull);
}

}  // namespace vh

extern "C" {

int vh_hashagg_create(int key_dtype, int nvals, const int *val_dtypes, uint32_t nonnull_mask, vh_hashagg **out) {
    VH_API_BEGIN
    dtype_itemsize(key_dtype);
    if (!key_dtype_ok(key_dtype)) fail(VH_ERR_ARG, "hashagg: the key must be an integer column");
    if (nvals < 0 || nvals > HA_MAX_V) fail(VH_ERR_ARG, "hashagg: at most 2 value columns");
    auto h = std::make_unique<vh_hashagg>();
    h->key_dtype = key_dtype;
    h->nv = nvals;
    h->nnmask = nonnull_mask & ((1u << nvals) - 1);
    for (int v = 0; v < nvals; v++) {
        const int d = val_dtypes[v];
        dtype_itemsize(d);
        h->vdtype[v] = d;
        if (d == VH_F64 || d == VH_F32) h->vfloat |= 1u << v;
    }
    *out = h.release();
    VH_API_END
}

int vh_hashagg_destroy(vh_hashagg *h) {
    VH_API_BEGIN
    delete h;
    VH_API_END
}

int vh_hashagg_update(vh_hashagg *h, const void *keys, const void *const *vals, uint64_t n, int loc) {
    VH_API_BEGIN
    if (h->finished) fail(VH_ERR_RUNTIME, "hashagg: update after finish");
    if (!n) return VH_OK;
    loc = resolve_loc(keys, loc);
    const int kisz = dtype_itemsize(h->key_dtype);
    constexpr uint64_t CHUNK = 1ull << 30;
    HaScratch &S = scratch();
    std::lock_guard<std::mutex> lk(S.mu);
    for (uint64_t r0 = 0; r0 < n; r0 += CHUNK) {
        const uint64_t m = std::min(CHUNK, n - r0);
        const void *kp = static_cast<const char *>(keys) + r0 * kisz;
        const void *vp[HA_MAX_V] = {nullptr, nullptr};
        for (int v = 0; v < h->nv; v++) vp[v] = static_cast<const char *>(vals[v]) + r0 * dtype_itemsize(h->vdtype[v]);
        if (loc == VH_LOC_HOST) {
            uint64_t bytes = (m * kisz + 255) & ~255ull;
            for (int v = 0; v < h->nv; v++) bytes += ((m * dtype_itemsize(h->vdtype[v]) + 255) & ~255ull);
            S.stage.ensure(bytes + 512);
            char *d = S.stage.as<char>();
            VH_HIP(hipMemcpyAsync(d, kp, m * kisz, hipMemcpyHostToDevice, stream()));
            uint64_t off = (m * kisz + 255) & ~255ull;
            for (int v = 0; v < h->nv; v++) {
                const uint64_t b = m * dtype_itemsize(h->vdtype[v]);
                VH_HIP(hipMemcpyAsync(d + off, vp[v], b, hipMemcpyHostToDevice, stream()));
                vp[v] = d + off;
                off += (b + 255) & ~255ull;
            }
            kp = d;
        }
        update_device(h, S, kp, vp, m);
        uint32_t err = 0;
        const uint32_t used = read_used(h, &err);
        if (err & 2) fail(VH_ERR_RUNTIME, "hashagg: hash table overflow");
        if (err & 1) ensure_table(h, 2 * (uint64_t)used);  // past 3/4: grow before the next update
        h->rows += m;
    }
    VH_API_END
}

int vh_hashagg_finish(vh_hashagg *h, uint64_t *ngroups) {
    VH_API_BEGIN
    if (!h->finished) {
        hipStream_t st = stream();
        h->finished = true;
        h->ngroups = 0;
        if (h->slots) {
            const HaTable g = table_view(h->tab.ptr, h->slots, h->nv, h->vfloat);
            uint64_t side = 0;
            VH_HIP(hipMemcpyAsync(&side, g.cnt + h->slots, 8, hipMemcpyDeviceToHost, st));
            const uint64_t m = read_used(h, nullptr) + (side ? 1 : 0);
            h->ngroups = m;
            if (m) {
                const int kbs = key_bits_size(h->key_dtype);
                const size_t tmp_bytes = sort_tmp_bytes(kbs, m);
                const uint64_t ak = (kbs * m + 255) & ~255ull, as = (4 * m + 255) & ~255ull;
                const uint64_t out_bytes = 8 * m * (2 + 2 * (uint64_t)h->nv);
                h->out.ensure(2 * ak + 2 * as + 256 + ((tmp_bytes + 255) & ~255ull) + out_bytes + 256);
                char *base = h->out.as<char>();
                char *skey = base, *skey2 = base + ak;
                uint32_t *sslot = reinterpret_cast<uint32_t *>(base + 2 * ak);
                uint32_t *sslot2 = reinterpret_cast<uint32_t *>(base + 2 * ak + as);
                uint32_t *counter = reinterpret_cast<uint32_t *>(base + 2 * ak + 2 * as);
                void *tmp = base + 2 * ak + 2 * as + 256;
                char *outp = out_results(h, m, tmp_bytes);
                VH_HIP(hipMemsetAsync(counter, 0, 4, st));
                TimedScope ts("ha_finish");
                const int sg = key_signed(h->key_dtype);
                int64_t *okey = reinterpret_cast<int64_t *>(outp);
                int64_t *ocnt = okey + m;
                uint64_t *osum = reinterpret_cast<uint64_t *>(ocnt + m);
                int64_t *onn = reinterpret_cast<int64_t *>(osum + m * h->nv);
                dispatch_kb(h->key_dtype, [&](auto kbc) {
                    using KB = decltype(kbc);
                    hipLaunchKernelGGL(k_ha_compact<KB>, dim3(blocks_for((h->slots + 8) / 8, 256, 8)), dim3(256), 0, st, g.keys,
                                       g.cnt, h->slots, sg, reinterpret_cast<KB *>(skey), sslot, counter);
                    VH_HIP(hipGetLastError());
                    size_t tb = tmp_bytes;
                    VH_HIP(rocprim::radix_sort_pairs(tmp, tb, reinterpret_cast<KB *>(skey), reinterpret_cast<KB *>(skey2),
                                                     sslot, sslot2, (size_t)m, 0, 8 * (int)sizeof(KB), st));
                    dispatch_nv(h->nv, [&](auto nvc) {
                        constexpr int NV = decltype(nvc)::value;
                        hipLaunchKernelGGL((k_ha_gather<KB, NV>), dim3(blocks_for(m, 256, 8)), dim3(256), 0, st, g,
                                           reinterpret_cast<const KB *>(skey2), sslot2, m, sg, okey, ocnt, osum, onn);
                    });
                });
                VH_HIP(hipGetLastError());
                h->res = outp;
            }
        }
    }
    *ngroups = h->ngroups;
    VH_API_END
}

/* outputs (host, ngroups items each): keys as int64 (uint64 keys: their bits), count(*)
   int64, per value column its sum (double / int64 / uint64 bits, 8 bytes) and non-NaN count */
int vh_hashagg_read(vh_hashagg *h, int64_t *keys, int64_t *counts, void *const *sums, int64_t *const *nonnull) {
    VH_API_BEGIN
    if (!h->finished) fail(VH_ERR_RUNTIME, "hashagg: read before finish");
    const uint64_t m = h->ngroups;
    if (!m) return VH_OK;
    const int64_t *okey = reinterpret_cast<const int64_t *>(h->res);
    const int64_t *ocnt = okey + m;
    const uint64_t *osum = reinterpret_cast<const uint64_t *>(ocnt + m);
    const int64_t *onn = reinterpret_cast<const int64_t *>(osum + m * h->nv);
    hipStream_t st = stream();
    // destinations may be host or HBM (hipMemcpyDefault: unified addressing), so a caller
    // that decodes the keys on the device keeps them there
    auto out = [&](void *dst, const void *src) {
        if (resolve_loc(dst, VH_LOC_AUTO) == VH_LOC_DEVICE) VH_HIP(hipMemcpyAsync(dst, src, 8 * m, hipMemcpyDeviceToDevice, st));
        else copy_to_host(dst, src, 8 * m, st);
    };
    if (keys) out(keys, okey);
    if (counts) out(counts, ocnt);
    for (int v = 0; v < h->nv; v++) {
        if (sums && sums[v]) out(sums[v], osum + (uint64_t)v * m);
        if (nonnull && nonnull[v]) out(nonnull[v], onn + (uint64_t)v * m);
    }
    VH_HIP(hipStreamSynchronize(st));
    VH_API_END
}

/* groups in first-appearance order (vh_hashagg_order_first; see vaexhip.h) */
int vh_hashagg_order_first(vh_hashagg *h, const void *keys, uint64_t n, int loc) {
    VH_API_BEGIN
    if (!h->finished) fail(VH_ERR_RUNTIME, "hashagg: order_first before finish");
    if (n != h->rows) fail(VH_ERR_ARG, "hashagg: order_first needs the key column of every update");
    const uint64_t m = h->ngroups;
    if (m < 2) return VH_OK;
    loc = resolve_loc(keys, loc);
    hipStream_t st = stream();
    const int kisz = dtype_itemsize(h->key_dtype);
    const int kbs = key_bits_size(h->key_dtype);
    const uint64_t ak = (kbs * m + 255) & ~255ull, as = (4 * m + 255) & ~255ull;
    const uint32_t *sslot2 = reinterpret_cast<const uint32_t *>(h->out.as<char>() + 2 * ak + as);
    const int ncols = 2 + 2 * h->nv;
    // scratch: first/rank u64 [m] | rank2 u64 [m] | idx u32 [m] | idx2 u32 [m] | gidx u32 [slots + 2] | stats | sort tmp
    size_t tmp_bytes = 0;
    VH_HIP(rocprim::radix_sort_pairs(nullptr, tmp_bytes, (unsigned long long *)nullptr, (unsigned long long *)nullptr,
                                     (uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)m, 0, 64, st));
    const uint64_t a8 = (8 * m + 255) & ~255ull, a4 = (4 * m + 255) & ~255ull, ag = (4 * (h->slots + 2) + 255) & ~255ull;
    DevBuf work;
    work.ensure(2 * a8 + 2 * a4 + ag + 256 + tmp_bytes + 256);
    char *wb = work.as<char>();
    auto *first = reinterpret_cast<unsigned long long *>(wb);
    auto *rank2 = reinterpret_cast<unsigned long long *>(wb + a8);
    auto *idx = reinterpret_cast<uint32_t *>(wb + 2 * a8);
    auto *idx2 = reinterpret_cast<uint32_t *>(wb + 2 * a8 + a4);
    auto *gidx = reinterpret_cast<uint32_t *>(wb + 2 * a8 + 2 * a4);
    auto *stats = reinterpret_cast<unsigned long long *>(wb + 2 * a8 + 2 * a4 + ag);
    void *tmp = wb + 2 * a8 + 2 * a4 + ag + 256;
    thread_local PinnedBuf res_buf;
    res_buf.ensure(64);
    auto *hstats = res_buf.as<unsigned long long>();
    const int64_t *okey = reinterpret_cast<const int64_t *>(h->res);
    bool complete = false;
    {
        TimedScope ts("ha_first");
        VH_HIP(hipMemsetAsync(first, 0xff, 8 * m, st));
        VH_HIP(hipMemsetAsync(stats, 0, 24, st));
        hipLaunchKernelGGL(k_ha_gidx, dim3(blocks_for(m, 256, 8)), dim3(256), 0, st, sslot2, m, gidx);
        VH_HIP(hipGetLastError());
        const HaTable g = table_view(h->tab.ptr, h->slots, h->nv, h->vfloat, h->nnmask);
        // the prefix scan: chunks from 4 rows per group, growing by half each step, until every
        // group has its first row; input with long key runs (sorted / clustered) probes only
        // its run heads and scans to the end, otherwise past n / 8 rows the set build below
        // takes over (its cost does not depend on where keys first appear)
        HaScratch &S = scratch();
        std::lock_guard<std::mutex> lk(S.mu);
        uint64_t r0 = 0, chunk = std::max<uint64_t>(1u << 20, 4 * m);
        uint64_t heads = 0;
        const bool aligned = (reinterpret_cast<uintptr_t>(keys) & 15) == 0;
        while (r0 < n) {
            const uint64_t r1 = std::min(n, r0 + (chunk & ~uint64_t(1023)));
            const void *kp = static_cast<const char *>(keys) + r0 * kisz;
            if (loc == VH_LOC_HOST || !aligned) {
                // staged 16-B aligned, with the rows before the chunk in the 16 bytes ahead of
                // it (the run-head test reads row r0 - 1)
                const uint64_t lead = std::min<uint64_t>(r0, 16 / kisz);
                S.stage.ensure((r1 - r0) * kisz + 64);
                char *d = S.stage.as<char>() + 16;
                VH_HIP(hipMemcpyAsync(d - lead * kisz, static_cast<const char *>(keys) + (r0 - lead) * kisz,
                                      (r1 - r0 + lead) * kisz, hipMemcpyDefault, st));
                kp = d;
            }
            VH_DISPATCH_DTYPE(h->key_dtype, K, {
                if constexpr (std::is_integral_v<K>) {
                    if constexpr (sizeof(K) >= 1) {
                        hipLaunchKernelGGL(k_ha_first<K>, dim3(blocks_for((r1 - r0) / (16 / sizeof(K)) + 1, 256, 8)), dim3(256),
                                           0, st, static_cast<const K *>(kp), r1 - r0, r0, g, gidx, first, stats);
                    }
                }
            });
            VH_HIP(hipGetLastError());
            VH_HIP(hipMemcpyAsync(hstats, stats, 24, hipMemcpyDeviceToHost, st));
            VH_HIP(hipStreamSynchronize(st));
            if (hstats[2]) fail(VH_ERR_ARG, "hashagg: order_first got a key the aggregation never saw");
            heads = hstats[1];
            r0 = r1;
            if (hstats[0] >= m) {
                complete = true;
                break;
            }
            if (r0 >= n / 8 && heads * 16 > r0) break;  // no long runs: the set build is cheaper
            chunk = heads * 16 > r0 ? chunk + chunk / 2 : chunk * 4;  // runs: a full scan, few syncs
        }
    }
    if (!complete) {
        // ordinals of an ordered_set over every row (the reference's structure; first rows of
        // keys that appear late cost a probe per row in the scan above)
        vh_set *set = nullptr;
        if (vh_set_create(h->key_dtype, &set) != VH_OK) fail(VH_ERR_RUNTIME, vh_last_error());
        std::unique_ptr<vh_set, int (*)(vh_set *)> guard(set, vh_set_destroy);
        if (vh_set_update(set, keys, nullptr, n, loc) != VH_OK) fail(VH_ERR_RUNTIME, vh_last_error());
        const SetDev sd = set_device_view(set);
        hipLaunchKernelGGL(k_ha_set_rank, dim3(blocks_for(m, 256, 8)), dim3(256), 0, st, okey, m, kisz, sd, first);
        VH_HIP(hipGetLastError());
    }
    // order the groups by first row (or ordinal), then permute every result column
    hipLaunchKernelGGL(k_ha_iota, dim3(blocks_for(m, 256, 8)), dim3(256), 0, st, idx, m);
    VH_HIP(hipGetLastError());
    size_t tb = tmp_bytes;
    VH_HIP(rocprim::radix_sort_pairs(tmp, tb, first, rank2, idx, idx2, (size_t)m, 0, 64, st));
    h->xres.ensure(8 * m * (uint64_t)ncols);
    int64_t *dst = h->xres.as<int64_t>();
    if (reinterpret_cast<const char *>(dst) == h->res) fail(VH_ERR_RUNTIME, "hashagg: result buffer aliasing");
    hipLaunchKernelGGL(k_ha_permute, dim3(blocks_for(m, 256, 8)), dim3(256), 0, st, okey, dst, m, ncols, idx2);
    VH_HIP(hipGetLastError());
    VH_HIP(hipStreamSynchronize(st));
    h->res = reinterpret_cast<const char *>(dst);
    VH_API_END
}

/* first-appearance order of the groups of a dense key range (vh_dense_first_order; see
 * vaexhip.h) */
int vh_dense_first_order(const void *keys, uint64_t n, int loc, int key_dtype, int64_t vmin, uint64_t span,
                         const int64_t *labels, uint64_t m, int64_t *perm) {
    VH_API_BEGIN
    if (!key_dtype_ok(key_dtype)) fail(VH_ERR_ARG, "dense_first_order: integer keys only");
    if (m == 0) return VH_OK;
    if (span == 0 || m > span || m >= (1ull << 32)) fail(VH_ERR_ARG, "dense_first_order: bad key range");
    loc = resolve_loc(keys, loc);
    hipStream_t st = stream();
    const int kisz = dtype_itemsize(key_dtype);
    size_t tmp_bytes = 0;
    VH_HIP(rocprim::radix_sort_pairs(nullptr, tmp_bytes, (unsigned long long *)nullptr, (unsigned long long *)nullptr,
                                     (uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)m, 0, 64, st));
    const uint64_t af = (8 * span + 255) & ~255ull, a8 = (8 * m + 255) & ~255ull, a4 = (4 * m + 255) & ~255ull;
    DevBuf work;
    work.ensure(af + 3 * a8 + 2 * a4 + 256 + tmp_bytes + 256);
    char *wb = work.as<char>();
    auto *first = reinterpret_cast<unsigned long long *>(wb);
    auto *fr = reinterpret_cast<unsigned long long *>(wb + af);
    auto *fr2 = reinterpret_cast<unsigned long long *>(wb + af + a8);
    auto *dlab = reinterpret_cast<int64_t *>(wb + af + 2 * a8);
    auto *idx = reinterpret_cast<uint32_t *>(wb + af + 3 * a8);
    auto *idx2 = reinterpret_cast<uint32_t *>(wb + af + 3 * a8 + a4);
    auto *stats = reinterpret_cast<unsigned long long *>(wb + af + 3 * a8 + 2 * a4);
    void *tmp = wb + af + 3 * a8 + 2 * a4 + 256;
    VH_HIP(hipMemsetAsync(first, 0xff, 8 * span, st));
    VH_HIP(hipMemsetAsync(stats, 0, 16, st));
    VH_HIP(hipMemcpyAsync(dlab, labels, 8 * m, hipMemcpyDefault, st));
    thread_local PinnedBuf res_buf;
    res_buf.ensure(64);
    auto *hstats = res_buf.as<unsigned long long>();
    {
        TimedScope ts("dense_first");
        HaScratch &S = scratch();
        std::lock_guard<std::mutex> lk(S.mu);
        // prefix scan of run heads in growing chunks until every group has its first row
        uint64_t r0 = 0, chunk = std::max<uint64_t>(1u << 20, 4 * m);
        const bool aligned = (reinterpret_cast<uintptr_t>(keys) & 15) == 0;
        while (r0 < n) {
            const uint64_t r1 = std::min(n, r0 + (chunk & ~uint64_t(1023)));
            const void *kp = static_cast<const char *>(keys) + r0 * kisz;
            if (loc == VH_LOC_HOST || !aligned) {
                const uint64_t lead = std::min<uint64_t>(r0, 16 / kisz);
                S.stage.ensure((r1 - r0) * kisz + 64);
                char *d = S.stage.as<char>() + 16;
                VH_HIP(hipMemcpyAsync(d - lead * kisz, static_cast<const char *>(keys) + (r0 - lead) * kisz,
                                      (r1 - r0 + lead) * kisz, hipMemcpyDefault, st));
                kp = d;
            }
            VH_DISPATCH_DTYPE(key_dtype, K, {
                if constexpr (std::is_integral_v<K>) {
                    hipLaunchKernelGGL(k_dense_first<K>, dim3(blocks_for((r1 - r0) / (16 / sizeof(K)) + 1, 256, 8)), dim3(256),
                                       0, st, static_cast<const K *>(kp), r1 - r0, r0, vmin, span, first, stats);
                }
            });
            VH_HIP(hipGetLastError());
            VH_HIP(hipMemcpyAsync(hstats, stats, 16, hipMemcpyDeviceToHost, st));
            VH_HIP(hipStreamSynchronize(st));
            r0 = r1;
            if (hstats[0] >= m) break;
            chunk = hstats[1] * 16 > r0 ? chunk + chunk / 2 : chunk * 4;
        }
        if (hstats[0] < m) fail(VH_ERR_ARG, "dense_first_order: a label's key does not occur in the column");
    }
    hipLaunchKernelGGL(k_dense_first_gather, dim3(blocks_for(m, 256, 8)), dim3(256), 0, st, dlab, m, vmin, first, fr, idx);
    VH_HIP(hipGetLastError());
    size_t tb = tmp_bytes;
    VH_HIP(rocprim::radix_sort_pairs(tmp, tb, fr, fr2, idx, idx2, (size_t)m, 0, 64, st));
    // perm as int64 (into the first-row scratch, then one copy to the caller's buffer)
    auto *p64 = reinterpret_cast<int64_t *>(first);
    hipLaunchKernelGGL(k_widen_u32, dim3(blocks_for(m, 256, 8)), dim3(256), 0, st, idx2, m, p64);
    VH_HIP(hipGetLastError());
    copy_to_host(perm, p64, 8 * m, st);
    VH_HIP(hipStreamSynchronize(st));
    VH_API_END
}

int vh_dense_first_take(const void *keys, uint64_t n, int loc, int key_dtype, int64_t vmin, uint64_t range,
                        const void *counts, int count_isz, uint64_t m, int ncols, const void *const *src, const int *isz,
                        void *const *dst, int label_isz, void *labels) {
    VH_API_BEGIN
    if (!key_dtype_ok(key_dtype)) fail(VH_ERR_ARG, "dense_first_take: integer keys only");
    if (m == 0) return VH_OK;
    if (range == 0 || m > range || range >= (1ull << 32)) fail(VH_ERR_ARG, "dense_first_take: bad key range");
    if (resolve_loc(counts, VH_LOC_AUTO) != VH_LOC_DEVICE) fail(VH_ERR_ARG, "dense_first_take: device count grid only");
    for (int c = 0; c < ncols; c++) {
        if (resolve_loc(src[c], VH_LOC_AUTO) != VH_LOC_DEVICE) fail(VH_ERR_ARG, "dense_first_take: device columns only");
        if (isz[c] != 1 && isz[c] != 2 && isz[c] != 4 && isz[c] != 8) fail(VH_ERR_ARG, "dense_first_take: item size");
    }
    if (label_isz != 1 && label_isz != 2 && label_isz != 4 && label_isz != 8) fail(VH_ERR_ARG, "dense_first_take: label size");
    loc = resolve_loc(keys, loc);
    hipStream_t st = stream();
    const int kisz = dtype_itemsize(key_dtype);
    size_t sort_bytes = 0, scan_bytes = 0;
    VH_HIP(rocprim::radix_sort_pairs(nullptr, sort_bytes, (unsigned long long *)nullptr, (unsigned long long *)nullptr,
                                     (uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)m, 0, 64, st));
    VH_HIP(rocprim::exclusive_scan(nullptr, scan_bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr, 0u, (size_t)range,
                                   rocprim::plus<uint32_t>(), st));
    const uint64_t af = (8 * range + 255) & ~255ull, a4r = (4 * range + 255) & ~255ull, a8 = (8 * m + 255) & ~255ull,
                   a4 = (4 * m + 255) & ~255ull, tb = std::max(sort_bytes, scan_bytes);
    DevBuf work;
    work.ensure(af + 2 * a4r + 3 * a8 + 3 * a4 + 256 + tb + 256);
    char *wb = work.as<char>();
    auto *first = reinterpret_cast<unsigned long long *>(wb);
    auto *flag = reinterpret_cast<uint32_t *>(wb + af);
    auto *pos = reinterpret_cast<uint32_t *>(wb + af + a4r);
    auto *fr = reinterpret_cast<unsigned long long *>(wb + af + 2 * a4r);
    auto *fr2 = reinterpret_cast<unsigned long long *>(wb + af + 2 * a4r + a8);
    void *out = wb + af + 2 * a4r + 2 * a8;  // one gathered column at a time (<= 8 bytes per item)
    auto *gidx = reinterpret_cast<uint32_t *>(wb + af + 2 * a4r + 3 * a8);
    auto *idx = reinterpret_cast<uint32_t *>(wb + af + 2 * a4r + 3 * a8 + a4);
    auto *idx2 = reinterpret_cast<uint32_t *>(wb + af + 2 * a4r + 3 * a8 + 2 * a4);
    auto *stats = reinterpret_cast<unsigned long long *>(wb + af + 2 * a4r + 3 * a8 + 3 * a4);
    void *tmp = wb + af + 2 * a4r + 3 * a8 + 3 * a4 + 256;
    VH_HIP(hipMemsetAsync(first, 0xff, 8 * range, st));
    VH_HIP(hipMemsetAsync(stats, 0, 16, st));
    thread_local PinnedBuf res_buf;
    res_buf.ensure(64);
    auto *hstats = res_buf.as<unsigned long long>();
    {
        TimedScope ts("dense_first");
        HaScratch &S = scratch();
        std::lock_guard<std::mutex> lk(S.mu);
        // every group's first row: the prefix scan of run heads of vh_dense_first_order
        uint64_t r0 = 0, chunk = std::max<uint64_t>(1u << 20, 4 * m);
        const bool aligned = (reinterpret_cast<uintptr_t>(keys) & 15) == 0;
        while (r0 < n) {
            const uint64_t r1 = std::min(n, r0 + (chunk & ~uint64_t(1023)));
            const void *kp = static_cast<const char *>(keys) + r0 * kisz;
            if (loc == VH_LOC_HOST || !aligned) {
                const uint64_t lead = std::min<uint64_t>(r0, 16 / kisz);
                S.stage.ensure((r1 - r0) * kisz + 64);
                char *d = S.stage.as<char>() + 16;
                VH_HIP(hipMemcpyAsync(d - lead * kisz, static_cast<const char *>(keys) + (r0 - lead) * kisz,
                                      (r1 - r0 + lead) * kisz, hipMemcpyDefault, st));
                kp = d;
            }
            VH_DISPATCH_DTYPE(key_dtype, K, {
                if constexpr (std::is_integral_v<K>) {
                    hipLaunchKernelGGL(k_dense_first<K>, dim3(blocks_for((r1 - r0) / (16 / sizeof(K)) + 1, 256, 8)), dim3(256),
                                       0, st, static_cast<const K *>(kp), r1 - r0, r0, vmin, range, first, stats);
                }
            });
            VH_HIP(hipGetLastError());
            VH_HIP(hipMemcpyAsync(hstats, stats, 16, hipMemcpyDeviceToHost, st));
            VH_HIP(hipStreamSynchronize(st));
            r0 = r1;
            if (hstats[0] >= m) break;
            chunk = hstats[1] * 16 > r0 ? chunk + chunk / 2 : chunk * 4;
        }
        if (hstats[0] < m) fail(VH_ERR_ARG, "dense_first_take: an occupied cell's key does not occur in the column");
    }
    // the occupied cells in key order (flags, exclusive scan, compaction), sorted by first row
    hipLaunchKernelGGL(k_nz_flags, dim3(blocks_for(range, 256, 8)), dim3(256), 0, st, counts, count_isz, range, flag);
    size_t sb = scan_bytes;
    VH_HIP(rocprim::exclusive_scan(tmp, sb, flag, pos, 0u, (size_t)range, rocprim::plus<uint32_t>(), st));
    hipLaunchKernelGGL(k_nz_compact, dim3(blocks_for(range, 256, 8)), dim3(256), 0, st, flag, pos, range, first, gidx, fr, idx);
    VH_HIP(hipGetLastError());
    size_t tbs = sort_bytes;
    VH_HIP(rocprim::radix_sort_pairs(tmp, tbs, fr, fr2, idx, idx2, (size_t)m, 0, 64, st));
    // gather every column (and the labels) in that order, read back into the caller's buffers
    for (int c = 0; c <= ncols; c++) {
        const bool lab = c == ncols;
        if (lab && !labels) break;
        const int z = lab ? label_isz : isz[c];
        hipLaunchKernelGGL(k_take_items, dim3(blocks_for(m, 256, 8)), dim3(256), 0, st, lab ? nullptr : src[c], z, gidx, idx2, m,
                           out, lab ? 1 : 0, vmin);
        VH_HIP(hipGetLastError());
        copy_to_host(lab ? labels : dst[c], out, (uint64_t)z * m, st);
    }
    VH_HIP(hipStreamSynchronize(st));
    VH_API_END
}

int vh_combine_keys(uint64_t n, int nkeys, const void *const *cols, const int *dtypes, const int64_t *mins,
                    const int64_t *mults, int64_t *out) {
    VH_API_BEGIN
    if (nkeys < 1 || nkeys > HC_MAX_KEYS) fail(VH_ERR_ARG, "combine_keys: 1..8 key columns");
    HcParams p{};
    p.nkeys = nkeys;
    for (int j = 0; j < nkeys; j++) {
        dtype_itemsize(dtypes[j]);
        if (!key_dtype_ok(dtypes[j])) fail(VH_ERR_ARG, "combine_keys: integer key columns only");
        if (resolve_loc(cols[j], VH_LOC_AUTO) != VH_LOC_DEVICE) fail(VH_ERR_ARG, "combine_keys: device columns only");
        p.col[j] = cols[j];
        p.dtype[j] = dtypes[j];
        p.min[j] = mins[j];
        p.mult[j] = mults[j];
    }
    if (resolve_loc(out, VH_LOC_AUTO) != VH_LOC_DEVICE) fail(VH_ERR_ARG, "combine_keys: device output only");
    if (n) {
        TimedScope ts("combine_keys");
        hipLaunchKernelGGL(k_combine_keys, dim3(blocks_for(n, 256, 8)), dim3(256), 0, stream(), p, n, out);
        VH_HIP(hipGetLastError());
    }
    VH_API_END
}

}  // extern "C"

namespace vh {
// ---- dense rank of int64 keys: (key, row) pairs radix-sorted, run heads flagged, an
// inclusive scan of the flags numbers the runs, each sorted row scatters its run number
// to its original row and every run head writes its key to the distinct list.
__global__ void k_dr_iota(uint32_t *idx, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        idx[i] = (uint32_t)i;
}

__global__ void k_dr_heads(const int64_t *sk, uint32_t *flag, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        flag[i] = (i == 0 || sk[i] != sk[i - 1]) ? 1u : 0u;
}

__global__ void k_dr_scatter(const int64_t *sk, const uint32_t *sidx, const uint32_t *flag, const uint32_t *scan,
                             int32_t *rank, int64_t *distinct, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t r = scan[i] - 1u;
        rank[sidx[i]] = (int32_t)r;
        if (flag[i]) distinct[r] = sk[i];
    }
}
// ---- labels of combined keys: key j of group i = (v / mult_j) % span_j + min_j, with
// v = table ? table[ck[i]] : ck[i] (the inverse of k_combine_keys, after a dense rank),
// stored in the label's width (values fit it by construction)
struct HdParams {
    void *out[HC_MAX_KEYS];
    int32_t itemsize[HC_MAX_KEYS];
    int64_t min[HC_MAX_KEYS];
    int64_t mult[HC_MAX_KEYS];
    int64_t span[HC_MAX_KEYS];
    int nkeys;
};

__global__ __launch_bounds__(256) void k_decode_keys(HdParams p, const int64_t *ck, const int64_t *table, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const int64_t v = table ? table[ck[i]] : ck[i];
        for (int j = 0; j < p.nkeys; j++) {
            const int64_t k = (v / p.mult[j]) % p.span[j] + p.min[j];
            switch (p.itemsize[j]) {
            case 1: static_cast<int8_t *>(p.out[j])[i] = (int8_t)k; break;
            case 2: static_cast<int16_t *>(p.out[j])[i] = (int16_t)k; break;
            case 4: static_cast<int32_t *>(p.out[j])[i] = (int32_t)k; break;
            default: static_cast<int64_t *>(p.out[j])[i] = k;
            }
        }
    }
}
}  // namespace vh

extern "C" {

int vh_decode_keys(uint64_t n, const int64_t *ck, const int64_t *table, int nkeys, const int64_t *mins,
                   const int64_t *mults, const int64_t *spans, const int *itemsizes, void *const *outs) {
    VH_API_BEGIN
    if (nkeys < 1 || nkeys > HC_MAX_KEYS) fail(VH_ERR_ARG, "decode_keys: 1..8 key columns");
    HdParams p{};
    p.nkeys = nkeys;
    for (int j = 0; j < nkeys; j++) {
        if (itemsizes[j] != 1 && itemsizes[j] != 2 && itemsizes[j] != 4 && itemsizes[j] != 8)
            fail(VH_ERR_ARG, "decode_keys: label itemsize must be 1, 2, 4 or 8");
        if (mults[j] < 1 || spans[j] < 1) fail(VH_ERR_ARG, "decode_keys: multipliers and spans must be >= 1");
        if (n && resolve_loc(outs[j], VH_LOC_AUTO) != VH_LOC_DEVICE) fail(VH_ERR_ARG, "decode_keys: device outputs only");
        p.out[j] = outs[j];
        p.itemsize[j] = itemsizes[j];
        p.min[j] = mins[j];
        p.mult[j] = mults[j];
        p.span[j] = spans[j];
    }
    if (n) {
        if (resolve_loc(ck, VH_LOC_AUTO) != VH_LOC_DEVICE || (table && resolve_loc(table, VH_LOC_AUTO) != VH_LOC_DEVICE))
            fail(VH_ERR_ARG, "decode_keys: device inputs only");
        TimedScope ts("decode_keys");
        hipLaunchKernelGGL(k_decode_keys, dim3(blocks_for(n, 256, 8)), dim3(256), 0, stream(), p, ck, table, n);
        VH_HIP(hipGetLastError());
    }
    VH_API_END
}

}  // extern "C"

// max of the keys, and whether any is negative (out[0] = max as uint64, out[1] = 1 if any < 0)
__global__ __launch_bounds__(256) void k_dr_keymax(const int64_t *keys, uint64_t n, unsigned long long *out) {
    uint64_t mx = 0;
    bool neg = false;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const int64_t k = keys[i];
        neg = neg || k < 0;
        mx = k > (int64_t)mx ? (uint64_t)k : mx;
    }
#pragma unroll
    for (int off = 32; off; off >>= 1) mx = max(mx, (uint64_t)__shfl_xor((unsigned long long)mx, off, 64));
    const bool any_neg = __any(neg);
    if ((threadIdx.x & 63) == 0) {
        if (mx) atomicMax(&out[0], (unsigned long long)mx);
        if (any_neg) atomicOr(&out[1], 1ull);
    }
}

namespace {
struct DrScratch {
    std::mutex mu;
    DevBuf sk, idx, sidx, flag, scan, tmp;
};
DrScratch &dr_scratch() {
    static std::mutex g;
    static std::map<int, std::unique_ptr<DrScratch>> m;
    std::lock_guard<std::mutex> lk(g);
    auto &p = m[current_device()];
    if (!p) p = std::make_unique<DrScratch>();
    return *p;
}
}  // namespace

namespace vh {
void dense_rank_scratch_release() {
    DrScratch &S = dr_scratch();
    std::lock_guard<std::mutex> lk(S.mu);
    for (DevBuf *b : {&S.sk, &S.idx, &S.sidx, &S.flag, &S.scan, &S.tmp}) b->release();
}
}  // namespace vh

extern "C" {

int vh_dense_rank_i64(uint64_t n, const int64_t *keys, int32_t *rank, int64_t *distinct, uint64_t *m) {
    VH_API_BEGIN
    if (!m) fail(VH_ERR_ARG, "dense_rank: m is null");
    *m = 0;
    if (n >= (uint64_t(1) << 31)) fail(VH_ERR_ARG, "dense_rank: at most 2^31 - 1 rows");
    if (!n) return VH_OK;
    for (const void *p : {(const void *)keys, (const void *)rank, (const void *)distinct})
        if (resolve_loc(p, VH_LOC_AUTO) != VH_LOC_DEVICE) fail(VH_ERR_ARG, "dense_rank: device buffers only");
    TimedScope ts("dense_rank");
    hipStream_t st = stream();
    // the sort's ~36 B per row of scratch (36 GB at 1e9 rows) is kept per device between
    // calls: allocating and freeing it per call ran into multi-second hipMalloc / hipFree
    // stalls every few h2o q10 queries (6.1 s instead of 0.31 s)
    DrScratch &S = dr_scratch();
    std::lock_guard<std::mutex> lk(S.mu);
    DevBuf &sk = S.sk, &idx = S.idx, &sidx = S.sidx, &flag = S.flag, &scan = S.scan, &tmp = S.tmp;
    sk.ensure(n * 8);
    idx.ensure(n * 4);
    sidx.ensure(n * 4);
    flag.ensure(n * 4);
    scan.ensure(n * 4);
    // non-negative keys (combined cartesian ordinals always are) sort as uint64 over only the
    // bits their maximum needs: q10's 47-bit keys take 6 radix passes instead of 8
    DevBuf kmx;
    kmx.ensure(16);
    VH_HIP(hipMemsetAsync(kmx.ptr, 0, 16, st));
    hipLaunchKernelGGL(k_dr_keymax, dim3(blocks_for(n, 256, 8)), dim3(256), 0, st, keys, n, kmx.as<unsigned long long>());
    uint64_t kinfo[2] = {0, 0};
    VH_HIP(hipMemcpyAsync(kinfo, kmx.ptr, 16, hipMemcpyDeviceToHost, st));
    VH_HIP(hipStreamSynchronize(st));
    const bool unsigned_sort = kinfo[1] == 0;
    unsigned end_bit = 64;
    if (unsigned_sort) {
        end_bit = 1;
        while (end_bit < 64 && (kinfo[0] >> end_bit)) end_bit++;
    }
    size_t t1 = 0, t2 = 0;
    if (unsigned_sort)
        VH_HIP(rocprim::radix_sort_pairs(nullptr, t1, (uint64_t *)nullptr, (uint64_t *)nullptr, (uint32_t *)nullptr,
                                         (uint32_t *)nullptr, (size_t)n, 0, end_bit, st));
    else
        VH_HIP(rocprim::radix_sort_pairs(nullptr, t1, (int64_t *)nullptr, (int64_t *)nullptr, (uint32_t *)nullptr,
                                         (uint32_t *)nullptr, (size_t)n, 0, 64, st));
    VH_HIP(rocprim::inclusive_scan(nullptr, t2, (uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)n,
                                   rocprim::plus<uint32_t>(), st));
    tmp.ensure(std::max<size_t>(std::max(t1, t2), 16));
    const unsigned g = blocks_for(n, 256, 8);
    hipLaunchKernelGGL(k_dr_iota, dim3(g), dim3(256), 0, st, idx.as<uint32_t>(), n);
    size_t tb = tmp.bytes;
    if (unsigned_sort)
        VH_HIP(rocprim::radix_sort_pairs(tmp.ptr, tb, reinterpret_cast<const uint64_t *>(keys), sk.as<uint64_t>(),
                                         idx.as<uint32_t>(), sidx.as<uint32_t>(), (size_t)n, 0, end_bit, st));
    else
        VH_HIP(rocprim::radix_sort_pairs(tmp.ptr, tb, keys, sk.as<int64_t>(), idx.as<uint32_t>(), sidx.as<uint32_t>(),
                                         (size_t)n, 0, 64, st));
    hipLaunchKernelGGL(k_dr_heads, dim3(g), dim3(256), 0, st, sk.as<int64_t>(), flag.as<uint32_t>(), n);
    tb = tmp.bytes;
    VH_HIP(rocprim::inclusive_scan(tmp.ptr, tb, flag.as<uint32_t>(), scan.as<uint32_t>(), (size_t)n,
                                   rocprim::plus<uint32_t>(), st));
    // (sorting (row, rank) pairs back to row order instead of this random scatter measured the
    // same at 1e9 rows: 331 vs 335 ms for h2o q10)
    hipLaunchKernelGGL(k_dr_scatter, dim3(g), dim3(256), 0, st, sk.as<int64_t>(), sidx.as<uint32_t>(),
                       flag.as<uint32_t>(), scan.as<uint32_t>(), rank, distinct, n);
    VH_HIP(hipGetLastError());
    uint32_t last = 0;
    VH_HIP(hipMemcpyAsync(&last, scan.as<uint32_t>() + (n - 1), 4, hipMemcpyDeviceToHost, st));
    VH_HIP(hipStreamSynchronize(st));
    *m = last;
    VH_API_END
}

}  // extern "C"

// ---- groupby results across ranks: hash-partition exchange on the device ------------------
// Every rank holds its shard's groups (key-sorted, vh_hashagg_finish).  Each group row
// [key, count, sum_v.., nonnull_v..] goes to owner splitmix64(key bits) % world
// (vaex_amd/distributed.py group_owner) in one RCCL all-to-all; the owner sorts what it
// received by key (stable: senders stay in rank order) and folds each run of equal keys
// in that order, so float sums add exactly as a merge of the ranks' parts in rank order
// would (superagg.cpp:354-361 reduce in part order).  With `gather` the owners' disjoint
// results are all-gathered and sorted again, so every rank holds the whole result.
namespace vh {

__host__ __device__ inline uint64_t xo_mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

constexpr int XO_MAX_WORLD = 64;

__global__ __launch_bounds__(256) void k_xo_owner(const int64_t *okey, uint64_t m, int world, uint32_t *owner,
                                                  uint32_t *idx, unsigned long long *hist) {
    __shared__ uint32_t h[XO_MAX_WORLD];
    if (threadIdx.x < XO_MAX_WORLD) h[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
        const uint32_t o = (uint32_t)(xo_mix((uint64_t)okey[j]) % (uint64_t)world);
        owner[j] = o;
        idx[j] = (uint32_t)j;
        atomicAdd(&h[o], 1u);
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)world && h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

// row j of the send buffer <- group sidx[j] (rows of one destination keep key order)
__global__ __launch_bounds__(256) void k_xo_pack(const char *res, uint64_t m, int nv, const uint32_t *sidx, uint64_t *rows) {
    const int R = 2 + 2 * nv;
    const uint64_t *col = reinterpret_cast<const uint64_t *>(res);
    for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
        const uint64_t i = sidx[j];
        for (int c = 0; c < R; c++) rows[j * R + c] = col[(uint64_t)c * m + i];
    }
}

// sortable key bits of received row j (signed keys: sign bit flipped) + its index
__global__ __launch_bounds__(256) void k_xo_keys(const uint64_t *rows, uint64_t M, int R, int is_signed, uint64_t *skey,
                                                 uint32_t *idx) {
    for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j < M; j += (uint64_t)gridDim.x * 256) {
        const uint64_t k = rows[j * R];
        skey[j] = is_signed ? (k ^ 0x8000000000000000ULL) : k;
        idx[j] = (uint32_t)j;
    }
}

__global__ __launch_bounds__(256) void k_xo_heads(const uint64_t *skey, uint64_t M, uint32_t *flag) {
    for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j < M; j += (uint64_t)gridDim.x * 256)
        flag[j] = (j == 0 || skey[j] != skey[j - 1]) ? 1u : 0u;
}

// one output group per run of equal keys, folded in sorted (= rank) order
__global__ __launch_bounds__(256) void k_xo_runs(const uint64_t *rows, const uint32_t *sidx, const uint32_t *flag,
                                                 const uint32_t *scan, uint64_t M, int nv, uint32_t vfloat,
                                                 uint64_t m_out, uint64_t *out) {
    const int R = 2 + 2 * nv;
    for (uint64_t p = blockIdx.x * 256ull + threadIdx.x; p < M; p += (uint64_t)gridDim.x * 256) {
        if (!flag[p]) continue;
        const uint64_t g = scan[p] - 1u;
        const uint64_t *r0 = rows + (uint64_t)sidx[p] * R;
        uint64_t acc[2 + 2 * HA_MAX_V];
        for (int c = 0; c < R; c++) acc[c] = r0[c];
        for (uint64_t q = p + 1; q < M && !flag[q]; q++) {
            const uint64_t *r = rows + (uint64_t)sidx[q] * R;
            acc[1] += r[1];
            for (int v = 0; v < nv; v++) {
                if ((vfloat >> v) & 1)
                    acc[2 + v] = __builtin_bit_cast(uint64_t, __builtin_bit_cast(double, acc[2 + v]) +
                                                                  __builtin_bit_cast(double, r[2 + v]));
                else
                    acc[2 + v] += r[2 + v];
                acc[2 + nv + v] += r[2 + nv + v];
            }
        }
        for (int c = 0; c < R; c++) out[(uint64_t)c * m_out + g] = acc[c];
    }
}

// fold M packed rows (any order within a key: stable sort keeps the given order) into
// key-sorted result columns in h->xres; returns the number of groups
static uint64_t xo_fold(vh_hashagg *h, const uint64_t *rows, uint64_t M) {
    hipStream_t st = stream();
    const int R = 2 + 2 * h->nv;
    if (!M) {
        h->xres.ensure(8);
        h->res = h->xres.as<char>();
        return 0;
    }
    if (M >= (1ull << 32)) fail(VH_ERR_RUNTIME, "hashagg exchange: too many group rows");
    DevBuf skey, skey2, idx, sidx, flag, scan, tmp;
    skey.ensure(8 * M);
    skey2.ensure(8 * M);
    idx.ensure(4 * M);
    sidx.ensure(4 * M);
    flag.ensure(4 * M);
    scan.ensure(4 * M);
    size_t t1 = 0, t2 = 0;
    VH_HIP(rocprim::radix_sort_pairs(nullptr, t1, (uint64_t *)nullptr, (uint64_t *)nullptr, (uint32_t *)nullptr,
                                     (uint32_t *)nullptr, (size_t)M, 0, 64, st));
    VH_HIP(rocprim::inclusive_scan(nullptr, t2, (uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)M,
                                   rocprim::plus<uint32_t>(), st));
    tmp.ensure(std::max<size_t>(std::max(t1, t2), 16));
    const unsigned g = blocks_for(M, 256, 8);
    hipLaunchKernelGGL(k_xo_keys, dim3(g), dim3(256), 0, st, rows, M, R, key_signed(h->key_dtype), skey.as<uint64_t>(),
                       idx.as<uint32_t>());
    size_t tb = tmp.bytes;
    VH_HIP(rocprim::radix_sort_pairs(tmp.ptr, tb, skey.as<uint64_t>(), skey2.as<uint64_t>(), idx.as<uint32_t>(),
                                     sidx.as<uint32_t>(), (size_t)M, 0, 64, st));
    hipLaunchKernelGGL(k_xo_heads, dim3(g), dim3(256), 0, st, skey2.as<uint64_t>(), M, flag.as<uint32_t>());
    tb = tmp.bytes;
    VH_HIP(rocprim::inclusive_scan(tmp.ptr, tb, flag.as<uint32_t>(), scan.as<uint32_t>(), (size_t)M,
                                   rocprim::plus<uint32_t>(), st));
    uint32_t mo = 0;
    VH_HIP(hipMemcpyAsync(&mo, scan.as<uint32_t>() + (M - 1), 4, hipMemcpyDeviceToHost, st));
    VH_HIP(hipStreamSynchronize(st));
    DevBuf out;
    out.ensure(8 * (uint64_t)mo * R + 8);
    hipLaunchKernelGGL(k_xo_runs, dim3(g), dim3(256), 0, st, rows, sidx.as<uint32_t>(), flag.as<uint32_t>(),
                       scan.as<uint32_t>(), M, h->nv, h->vfloat, (uint64_t)mo, out.as<uint64_t>());
    VH_HIP(hipGetLastError());
    VH_HIP(hipStreamSynchronize(st));
    std::swap(h->xres.ptr, out.ptr);
    std::swap(h->xres.bytes, out.bytes);
    h->res = h->xres.as<char>();
    return mo;
}

}  // namespace vh

extern "C" {

int vh_hashagg_exchange(vh_hashagg *h, vh_comm *c, int gather) {
    VH_API_BEGIN
    if (!h->finished) fail(VH_ERR_RUNTIME, "hashagg: exchange before finish");
    DeviceScope ds(comm_device(c));
    std::lock_guard<std::mutex> lk(comm_mutex(c));
    hipStream_t st = stream();
    const int world = comm_world(c), me = comm_rank(c);
    if (world > XO_MAX_WORLD) fail(VH_ERR_ARG, "hashagg exchange: at most 64 ranks");
    const int R = 2 + 2 * h->nv;
    const uint64_t m = h->ngroups;
    // ---- owners, rows packed by destination
    DevBuf owner, idx, sowner, sidx, tmp, hist, rows;
    owner.ensure(4 * std::max<uint64_t>(m, 1));
    idx.ensure(4 * std::max<uint64_t>(m, 1));
    sowner.ensure(4 * std::max<uint64_t>(m, 1));
    sidx.ensure(4 * std::max<uint64_t>(m, 1));
    hist.ensure(8 * (uint64_t)world * world + 8);
    rows.ensure(8 * (uint64_t)R * std::max<uint64_t>(m, 1));
    unsigned long long *d_hist = hist.as<unsigned long long>();  // [world] mine | [world][world] all
    VH_HIP(hipMemsetAsync(d_hist, 0, 8 * (uint64_t)world, st));
    if (m) {
        const unsigned g = blocks_for(m, 256, 8);
        hipLaunchKernelGGL(k_xo_owner, dim3(g), dim3(256), 0, st, reinterpret_cast<const int64_t *>(h->res), m, world,
                           owner.as<uint32_t>(), idx.as<uint32_t>(), d_hist);
        int bits = 1;
        while ((1 << bits) < world) bits++;
        size_t tb = 0;
        VH_HIP(rocprim::radix_sort_pairs(nullptr, tb, (uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                         (uint32_t *)nullptr, (size_t)m, 0, bits, st));
        tmp.ensure(std::max<size_t>(tb, 16));
        tb = tmp.bytes;
        VH_HIP(rocprim::radix_sort_pairs(tmp.ptr, tb, owner.as<uint32_t>(), sowner.as<uint32_t>(), idx.as<uint32_t>(),
                                         sidx.as<uint32_t>(), (size_t)m, 0, bits, st));
        hipLaunchKernelGGL(k_xo_pack, dim3(g), dim3(256), 0, st, h->res, m, h->nv, sidx.as<uint32_t>(),
                           rows.as<uint64_t>());
        VH_HIP(hipGetLastError());
    }
    // ---- every rank's send counts, then the rows
    comm_allgather_dev(c, d_hist, d_hist + world, 8 * (uint64_t)world);
    std::vector<uint64_t> all((uint64_t)world * world);
    VH_HIP(hipMemcpyAsync(all.data(), d_hist + world, 8 * all.size(), hipMemcpyDeviceToHost, st));
    VH_HIP(hipStreamSynchronize(st));
    std::vector<uint64_t> sb(world), rb(world);
    uint64_t M = 0;
    for (int r = 0; r < world; r++) {
        sb[r] = all[(uint64_t)me * world + r] * 8 * R;
        rb[r] = all[(uint64_t)r * world + me] * 8 * R;
        M += all[(uint64_t)r * world + me];
    }
    DevBuf recv;
    recv.ensure(8 * (uint64_t)R * std::max<uint64_t>(M, 1));
    {
        TimedScope ts("ha_exchange");
        comm_alltoallv_dev(c, rows.ptr, sb.data(), recv.ptr, rb.data());
    }
    uint64_t mine = xo_fold(h, recv.as<uint64_t>(), M);
    if (gather) {
        // owners' disjoint results to every rank (padded all-gather), sorted once more
        DevBuf cnt;
        cnt.ensure(8 * (uint64_t)(world + 1));
        VH_HIP(hipMemcpyAsync(cnt.as<uint64_t>(), &mine, 8, hipMemcpyHostToDevice, st));
        comm_allgather_dev(c, cnt.as<uint64_t>(), cnt.as<uint64_t>() + 1, 8);
        std::vector<uint64_t> sizes(world);
        VH_HIP(hipMemcpyAsync(sizes.data(), cnt.as<uint64_t>() + 1, 8 * (uint64_t)world, hipMemcpyDeviceToHost, st));
        VH_HIP(hipStreamSynchronize(st));
        uint64_t top = 0, tot = 0;
        for (auto v : sizes) {
            top = std::max(top, v);
            tot += v;
        }
        // my result as rows, padded to `top`
        DevBuf mrows, allrows, packed;
        mrows.ensure(8 * (uint64_t)R * std::max<uint64_t>(top, 1));
        if (mine) {
            DevBuf iota;
            iota.ensure(4 * mine);
            hipLaunchKernelGGL(k_dr_iota, dim3(blocks_for(mine, 256, 8)), dim3(256), 0, st, iota.as<uint32_t>(), mine);
            hipLaunchKernelGGL(k_xo_pack, dim3(blocks_for(mine, 256, 8)), dim3(256), 0, st, h->res, mine, h->nv,
                               iota.as<uint32_t>(), mrows.as<uint64_t>());
            VH_HIP(hipStreamSynchronize(st));
        }
        allrows.ensure(8 * (uint64_t)R * std::max<uint64_t>(top, 1) * world);
        comm_allgather_dev(c, mrows.ptr, allrows.ptr, 8 * (uint64_t)R * top);
        packed.ensure(8 * (uint64_t)R * std::max<uint64_t>(tot, 1));
        uint64_t at = 0;
        for (int r = 0; r < world; r++) {
            if (sizes[r])
                VH_HIP(hipMemcpyAsync(packed.as<uint64_t>() + at * R, allrows.as<uint64_t>() + (uint64_t)r * top * R,
                                      8 * (uint64_t)R * sizes[r], hipMemcpyDeviceToDevice, st));
            at += sizes[r];
        }
        mine = xo_fold(h, packed.as<uint64_t>(), tot);
    }
    h->ngroups = mine;
    VH_HIP(hipStreamSynchronize(st));
    VH_API_END
}

}  // extern "C"

// ---- stable argsort of a key column on the device (Grouper sort=True, groupby.py:137-156:
// ascending, NaN after every number; -0.0 and 0.0 compare equal, so they keep their order)
namespace vh {
template <typename T> __device__ inline uint64_t sortable_bits(T v) {
    if constexpr (std::is_same_v<T, double> || std::is_same_v<T, float>) {
        if (v != v) return ~0ULL;                        // NaN last
        const double d = (double)v == 0.0 ? 0.0 : (double)v;  // -0.0 == 0.0
        const uint64_t u = __builtin_bit_cast(uint64_t, d);
        return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
    } else if constexpr (std::is_same_v<T, vbool>) {
        return v.v ? 1 : 0;
    } else if constexpr (std::is_signed_v<T>) {
        return (uint64_t)(int64_t)v ^ 0x8000000000000000ULL;
    } else {
        return (uint64_t)v;
    }
}

template <typename T> __global__ __launch_bounds__(256) void k_sortkeys(const T *keys, uint64_t n, uint64_t *sk, uint32_t *idx) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        sk[i] = sortable_bits<T>(keys[i]);
        idx[i] = (uint32_t)i;
    }
}

__global__ __launch_bounds__(256) void k_widen_idx(const uint32_t *idx, uint64_t n, int64_t *out) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) out[i] = idx[i];
}
}  // namespace vh

extern "C" {

int vh_argsort(uint64_t n, const void *keys, int dtype, int64_t *order) {
    VH_API_BEGIN
    if (n >= (uint64_t(1) << 32)) fail(VH_ERR_ARG, "argsort: at most 2^32 - 1 keys");
    if (!n) return VH_OK;
    if (resolve_loc(keys, VH_LOC_AUTO) != VH_LOC_DEVICE || resolve_loc(order, VH_LOC_AUTO) != VH_LOC_DEVICE)
        fail(VH_ERR_ARG, "argsort: device buffers only");
    hipStream_t st = stream();
    DevBuf sk, sk2, idx, idx2, tmp;
    sk.ensure(8 * n);
    sk2.ensure(8 * n);
    idx.ensure(4 * n);
    idx2.ensure(4 * n);
    const unsigned g = blocks_for(n, 256, 8);
    VH_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(k_sortkeys<T>, dim3(g), dim3(256), 0, st, static_cast<const T *>(keys), n,
                                                   sk.as<uint64_t>(), idx.as<uint32_t>()));
    size_t tb = 0;
    VH_HIP(rocprim::radix_sort_pairs(nullptr, tb, (uint64_t *)nullptr, (uint64_t *)nullptr, (uint32_t *)nullptr,
                                     (uint32_t *)nullptr, (size_t)n, 0, 64, st));
    tmp.ensure(std::max<size_t>(tb, 16));
    tb = tmp.bytes;
    VH_HIP(rocprim::radix_sort_pairs(tmp.ptr, tb, sk.as<uint64_t>(), sk2.as<uint64_t>(), idx.as<uint32_t>(),
                                     idx2.as<uint32_t>(), (size_t)n, 0, 64, st));
    hipLaunchKernelGGL(k_widen_idx, dim3(g), dim3(256), 0, st, idx2.as<uint32_t>(), n, order);
    VH_HIP(hipGetLastError());
    VH_HIP(hipStreamSynchronize(st));
    VH_API_END
}

}  // extern "C"

namespace vh {
uint64_t stat_hashagg_overflow(bool reset) {
    unsigned long long v = 0;
    VH_HIP(hipStreamSynchronize(stream()));
    VH_HIP(hipMemcpyFromSymbol(&v, HIP_SYMBOL(d_ha_overflow_rows), sizeof(v)));
    if (reset) {
        const unsigned long long z = 0;
        VH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(d_ha_overflow_rows), &z, sizeof(z)));
    }
    return v;
}
}  // namespace vh
