// ordered_set_<dtype> on the GPU: the groupby key set of vaex-core
// (packages/vaex-core/src/hash_primitives.hpp:417-621, hash.hpp:124-257),
// rebuilt as one open-address table in HBM instead of nmaps mutex-guarded
// hopscotch maps:
//   update      -- every row inserts its key with a CAS on an EMPTY slot
//                  (linear probing from _hash64(bits), hash.hpp:25-30) and
//                  lowers the slot's first-seen row with atomicMin (only when
//                  the row is older than the slot's current one);
//   seal        -- occupied slots are compacted and ordinals assigned in
//                  first-appearance order (the order a single-threaded
//                  reference update assigns `ordinal = map.size()`,
//                  hash_primitives.hpp:453-461, with nmaps = 1);
//   map_ordinal -- one probe per row (hash_primitives.hpp:556-583).
// NaN and null keys get their own ordinals (nan_value / null_value,
// hash_primitives.hpp:436-450).  Rows are inserted in chunks that double while the
// table does not need to grow; inside a chunk an insert that would push the table past
// 3/4 full, or a probe sequence longer than SET_MAX_PROBE, is refused and flags overflow:
// the table then grows x4 and the chunk is re-run (inserts are idempotent).
#include <algorithm>
#include <cmath>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <type_traits>

#include "common.hpp"
#include "hashset.hpp"

using namespace vh;

enum { C_DISTINCT = 0, C_OVERFLOW, C_NAN_FIRST, C_NULL_FIRST, C_SPECIAL_FIRST, C_NAN_COUNT, C_NULL_COUNT, C_CURSOR, C_N };

struct vh_set {
    // ordered_set.update is called concurrently on ONE set by every worker thread of the
    // reference (cpu.py:147-195; per-map mutexes, hash_primitives.hpp:242-247): every entry
    // point holds this lock, so concurrent updates serialise whole (row numbering, staging
    // buffers, counters and the table stay consistent; ordinals follow the order in which
    // the calls ran, as the reference's follow its thread interleaving)
    std::recursive_mutex mu;
    int dtype = VH_I64;
    uint64_t cap = 0;
    DevBuf tab, lut, ctr;
    DevBuf stage_keys, stage_mask, stage_select;
    DevBuf c_slot, c_first, c_ord, c_bits;
    uint64_t rows_seen = 0;
    uint64_t nan_count_before = 0, null_count_before = 0;  // counters before the current chunk
    // the reference flushes NaN/null rows after the regular keys of the update call that
    // saw them first (hash_primitives.hpp:248-274): their ordinal position is the end of
    // that call, ties broken NaN before null
    uint64_t nan_pos = ~0ULL, null_pos = ~0ULL;
    bool sealed = false;
    int64_t length = 0, nan_count = 0, null_count = 0;
    int64_t nan_ord = -1, null_ord = -1, special_ord = -1;
    std::vector<uint64_t> key_bits;  // per ordinal (after seal)
    std::vector<int8_t> key_kind;    // 0 regular, 1 nan, 2 null, 3 special
};

namespace vh {
// pass-A rows that missed their region since the last reset (vh_stat_read)
__device__ unsigned long long d_si_overflow_rows;


// ---- update: hash-partitioned insert ------------------------------------------------------
// Per update chunk (hash_primitives.hpp:96-281 `_update` over one chunk of keys):
//   sample -- ~1 M evenly spaced rows: fine bucket histogram (top 12 bits of the key hash)
//             and a distinct-key estimate (Chao1) -> the HBM table is grown before the
//             pass, and P = 2^p buckets of <= ~SI_TARGET_KEYS keys are chosen;
//   pass A -- workgroup w owns a row range; per 4096-row batch it classifies the rows
//             (unselected / null / NaN / the EMPTY-bits key are counted in LDS, their
//             first rows kept), ranks the regular rows per bucket in LDS, counting-sorts
//             (key bits, row) by bucket and streams the runs to per-(w, bucket) regions;
//   pass B -- work unit = (bucket, range of pass-A workgroups): the unit's entries are
//             deduplicated in an LDS table keeping each key's smallest row (ds_min), then
//             each distinct key is inserted into the HBM table ONCE per unit (CAS on an
//             EMPTY slot, atomicMin of the first row) -- not once per row;
//   direct -- (P == 1, few keys) each workgroup dedups its raw rows in LDS, then merges.
// A key that finds its LDS table closed (full: a sampling miss), or a row whose pass-A
// region is full, goes straight to the HBM table.  An HBM insert past `limit` keys is
// refused and raises the overflow counter; the host then grows the table and re-runs the
// chunk (inserts are idempotent).  Two host round trips per chunk: the sample and the end.
constexpr int SI_THREADS = 512;
constexpr int SI_RPT = 8;
constexpr int SI_BATCH = SI_THREADS * SI_RPT;
constexpr int SB_THREADS = 1024;
constexpr int SB_M = 8;                   // entries per lane per pass-B step
constexpr uint32_t SI_LT_LOG2 = 13;
constexpr uint32_t SI_LT = 1u << SI_LT_LOG2;  // LDS table slots (+2 side records)
constexpr uint32_t SI_TARGET_KEYS = 4096;     // P: a bucket holds about this many keys
constexpr uint32_t SI_FINE_LOG2 = 12;
constexpr uint32_t SI_MAX_P_LOG2 = 11;
constexpr int SI_SAMPLE_BLOCKS = 128;
constexpr uint32_t SI_DEST_OVER = 0x80000000u;
constexpr uint32_t SI_ROW_NONE = 0xffffffffu;

template <typename T> using si_kb_t = std::conditional_t<sizeof(T) == 8, uint64_t, uint32_t>;

struct SiParams {
    const void *keys;
    const uint8_t *mask, *select;
    uint64_t n, row0;  // rows of the chunk; set row number of its first row
    uint32_t p_log2, P, W, pad;
    uint64_t rows_per_wg, wg_stride;
    const uint32_t *cap;   // [P]
    const uint64_t *toff;  // [P]
    uint32_t *fills;       // [P][W]
    void *ent;             // <= 4-byte keys: u64 (row << 32 | key bits); else u64 key bits
    uint32_t *ent_row;     // 8-byte keys: the rows
    uint32_t debug;        // experiment switches (VH_SI_DEBUG), 0 in production
};

struct SiTable {
    uint64_t *tab;
    uint64_t cap_mask, limit;
    uint64_t *ctr;
    uint32_t *wg_new;  // the workgroup's LDS count of keys it inserted (added to C_DISTINCT once)
};

struct SiUnit {
    uint32_t bucket, w_begin, w_end, pad;
};

// top p_log2 bits of the key hash's high word (fine histogram: top SI_FINE_LOG2 bits)
__device__ inline uint32_t si_h32(uint64_t kb) { return (uint32_t)(hash64(kb) >> 32); }
__device__ inline uint32_t si_bucket(uint64_t kb, uint32_t p_log2) {
    return (uint32_t)(((uint64_t)si_h32(kb) << p_log2) >> 32);
}

// One distinct key (and the smallest row it was seen at) into the HBM table.  The table was
// sized for the sampled estimate at <= 1/2 load; a probe sequence longer than SET_MAX_PROBE
// (the estimate missed and the table filled up) raises the overflow counter instead, and
// the host grows the table and re-runs the chunk.  New keys are counted per workgroup in
// LDS (one global add per workgroup: one counter bumped by every new key serialises).
__device__ inline void si_global(const SiTable &g, uint64_t kb, uint64_t row) {
    uint64_t pos = hash64(kb) & g.cap_mask;
    for (int p = 0; p <= SET_MAX_PROBE; p++) {
        const uint64_t k = __hip_atomic_load(&g.tab[2 * pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool mine = k == kb;
        if (!mine && k == SET_EMPTY) {
            const uint64_t old = atomicCAS((unsigned long long *)&g.tab[2 * pos], (unsigned long long)SET_EMPTY,
                                           (unsigned long long)kb);
            if (old == SET_EMPTY) atomicAdd(g.wg_new, 1u);
            mine = old == SET_EMPTY || old == kb;
        }
        if (mine) {
            if (__hip_atomic_load(&g.tab[2 * pos + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > row)
                atomicMin((unsigned long long *)&g.tab[2 * pos + 1], (unsigned long long)row);
            return;
        }
        pos = (pos + 1) & g.cap_mask;
    }
    atomicOr((unsigned long long *)&g.ctr[C_OVERFLOW], 1ULL);
}

// ---- LDS dedup table: key bits -> smallest row (chunk-relative) ---------------------------
// LDS slot hash: a 32-bit mixer (murmur3 fmix32), cheaper than hash64's 64-bit multiplies;
// independent of the bucket bits (which come from hash64)
__device__ inline uint32_t si_lds_hash(uint64_t kb) {
    uint32_t h = (uint32_t)kb ^ (uint32_t)(kb >> 32) * 0x9e3779b9u;
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

template <typename KB> __host__ __device__ constexpr KB si_empty() { return ~KB(0); }
template <typename KB> __host__ __device__ constexpr KB si_closed() { return ~KB(0) - 1; }

template <typename KB> struct SiLds {
    KB *keys;        // [SI_LT]
    uint32_t *rows;  // [SI_LT + 2]: +2 side records for the keys equal to CLOSED / EMPTY
    uint32_t *used;
};

__host__ __device__ constexpr size_t si_lt_bytes(int kbsize) { return (size_t)kbsize * SI_LT + 4 * (SI_LT + 2) + 16; }

template <typename KB> __device__ inline SiLds<KB> si_lt_layout(unsigned char *raw) {
    SiLds<KB> t;
    t.keys = reinterpret_cast<KB *>(raw);
    t.rows = reinterpret_cast<uint32_t *>(raw + sizeof(KB) * SI_LT);
    t.used = t.rows + SI_LT + 2;
    return t;
}

template <typename KB> __device__ inline void si_lt_init(const SiLds<KB> &t, int nthreads) {
    for (uint32_t i = threadIdx.x; i < SI_LT + 2; i += nthreads) {
        if (i < SI_LT) t.keys[i] = si_empty<KB>();
        t.rows[i] = SI_ROW_NONE;
    }
    if (threadIdx.x == 0) *t.used = 0;
}

template <typename KB> struct alignas(16) SiKB4 {
    KB v[4];
};

__device__ inline uint32_t si_cas(uint32_t *p, uint32_t cmp, uint32_t val) { return atomicCAS(p, cmp, val); }
__device__ inline uint64_t si_cas(uint64_t *p, uint64_t cmp, uint64_t val) {
    return atomicCAS(reinterpret_cast<unsigned long long *>(p), (unsigned long long)cmp, (unsigned long long)val);
}

// Two-choice LDS table (as hashagg.hip's pass B): a key lives in one of two 4-slot groups,
// g1 from its LDS hash and g2 from a second mix, both read at once (one ds_read_b128 each
// for 4-byte keys), so a hit almost never needs a second round trip; one-group linear
// probing displaced a few per cent of the keys, whose probe chains serialised every wave.
// A new key is CASed into the first EMPTY slot of the group with more room.  Two lanes that
// insert one key at once may place it in both groups: harmless, both records merge into the
// key's one HBM slot with atomicMin of the row.  A key whose groups are both full goes to
// the HBM table directly; keys whose bits are the top two patterns use the side records.
template <typename KB> __device__ inline void si_lt2_groups(KB kb, uint32_t &g1, uint32_t &g2) {
    const uint32_t h = si_lds_hash((uint64_t)kb);
    g1 = (h & (SI_LT - 1)) >> 2;
    g2 = ((h ^ 0x9e3779b9u) * 0x2545f491u) >> (32 - (SI_LT_LOG2 - 2));  // multiply-shift: top bits
}

template <typename KB>
__device__ inline uint32_t si_lt2_find(const SiKB4<KB> &q1, const SiKB4<KB> &q2, uint32_t g1, uint32_t g2, KB kb) {
    uint32_t slot = ~0u;
#pragma unroll
    for (int j = 3; j >= 0; j--) {
        if (q2.v[j] == kb) slot = 4 * g2 + j;
        if (q1.v[j] == kb) slot = 4 * g1 + j;
    }
    return slot;
}

template <typename KB>
__device__ inline void si_lt2_insert(const SiLds<KB> &t, const SiTable &g, uint64_t row0, KB kb, uint32_t row) {
    constexpr KB EMPTY = si_empty<KB>();
    uint32_t g1, g2;
    si_lt2_groups(kb, g1, g2);
    for (int it = 0; it < 64; it++) {
        const SiKB4<KB> q1 = *reinterpret_cast<const SiKB4<KB> *>(t.keys + 4 * g1);
        const SiKB4<KB> q2 = *reinterpret_cast<const SiKB4<KB> *>(t.keys + 4 * g2);
        const uint32_t hit = si_lt2_find(q1, q2, g1, g2, kb);
        if (hit != ~0u) {
            atomicMin(&t.rows[hit], row);
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
        const KB cur = si_cas(&t.keys[pos], EMPTY, kb);
        if (cur == EMPTY || cur == kb) {
            atomicMin(&t.rows[pos], row);
            return;
        }
    }
    si_global(g, (uint64_t)kb, row0 + row);
}

// M entries at once: both group reads of every entry issued before any is used, hits take
// their ds_min right away, only keys new to the table take si_lt2_insert
template <typename KB, int M>
__device__ inline void si_lt_add_many(const SiLds<KB> &t, const SiTable &g, uint64_t row0, const KB *kb,
                                      const uint32_t *row, const bool *valid) {
    SiKB4<KB> q1[M], q2[M];
    uint32_t g1[M], g2[M];
#pragma unroll
    for (int i = 0; i < M; i++) {
        si_lt2_groups(kb[i], g1[i], g2[i]);
        q1[i] = *reinterpret_cast<const SiKB4<KB> *>(t.keys + 4 * g1[i]);
        q2[i] = *reinterpret_cast<const SiKB4<KB> *>(t.keys + 4 * g2[i]);
    }
    bool slow[M];
#pragma unroll
    for (int i = 0; i < M; i++) {
        uint32_t slot = si_lt2_find(q1[i], q2[i], g1[i], g2[i], kb[i]);
        if (kb[i] >= si_closed<KB>()) slot = SI_LT + (uint32_t)(kb[i] - si_closed<KB>());
        slow[i] = valid[i] && slot == ~0u;
        if (valid[i] && slot != ~0u) atomicMin(&t.rows[slot], row[i]);
    }
#pragma unroll
    for (int i = 0; i < M; i++)
        if (slow[i]) si_lt2_insert<KB>(t, g, row0, kb[i], row[i]);
}

// every key the LDS table holds, with its smallest row, into the HBM table (after a barrier)
template <typename KB> __device__ inline void si_lt_merge(const SiLds<KB> &t, const SiTable &g, uint64_t row0, int nthreads) {
    for (uint32_t i = threadIdx.x; i < SI_LT + 2; i += nthreads) {
        const uint32_t r = t.rows[i];
        if (r == SI_ROW_NONE) continue;
        const KB kb = i < SI_LT ? t.keys[i] : (KB)(si_closed<KB>() + (i - SI_LT));
        si_global(g, (uint64_t)kb, row0 + r);
    }
}

// ---- per-workgroup counters of the rows that never enter the table -----------------------
struct SiSpecial {
    uint32_t nan_first, null_first, spec_first, pad;
    uint32_t nan_cnt, null_cnt;
};

__device__ inline void si_special_init(SiSpecial *sp) {
    if (threadIdx.x == 0) {
        sp->nan_first = sp->null_first = sp->spec_first = SI_ROW_NONE;
        sp->nan_cnt = sp->null_cnt = 0;
    }
}

__device__ inline void si_special_flush(const SiSpecial *sp, uint64_t row0, uint64_t *ctr) {
    if (threadIdx.x != 0) return;
    if (sp->nan_cnt) {
        atomicMin((unsigned long long *)&ctr[C_NAN_FIRST], (unsigned long long)(row0 + sp->nan_first));
        atomicAdd((unsigned long long *)&ctr[C_NAN_COUNT], (unsigned long long)sp->nan_cnt);
    }
    if (sp->null_cnt) {
        atomicMin((unsigned long long *)&ctr[C_NULL_FIRST], (unsigned long long)(row0 + sp->null_first));
        atomicAdd((unsigned long long *)&ctr[C_NULL_COUNT], (unsigned long long)sp->null_cnt);
    }
    if (sp->spec_first != SI_ROW_NONE)
        atomicMin((unsigned long long *)&ctr[C_SPECIAL_FIRST], (unsigned long long)(row0 + sp->spec_first));
}

// classify row i (chunk-relative): returns true with its key bits when it is a regular key
template <typename T>
__device__ inline bool si_row(const SiParams &sp, uint64_t i, SiSpecial *spec, si_kb_t<T> *kb) {
    if (sp.select && !sp.select[i]) return false;  // filtered out / not selected
    if (sp.mask && sp.mask[i]) {
        atomicMin(&spec->null_first, (uint32_t)i);
        atomicAdd(&spec->null_cnt, 1u);
        return false;
    }
    const T v = static_cast<const T *>(sp.keys)[i];
    if (is_nan_v(v)) {
        atomicMin(&spec->nan_first, (uint32_t)i);
        atomicAdd(&spec->nan_cnt, 1u);
        return false;
    }
    const uint64_t b = key_bits(v);
    if (b == SET_EMPTY) {  // 8-byte keys only: the side slot ("special")
        atomicMin(&spec->spec_first, (uint32_t)i);
        return false;
    }
    *kb = (si_kb_t<T>)b;
    return true;
}

// ---- sample -------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(SI_THREADS) void k_si_sample(SiParams sp, uint64_t block_stride,
                                                          unsigned long long *fine_hist, uint64_t *skeys, uint32_t *scnt,
                                                          uint64_t smask) {
    __shared__ uint32_t h[1u << SI_FINE_LOG2];
    __shared__ SiSpecial spec;  // discarded: the pass counts these rows
    for (uint32_t t = threadIdx.x; t < (1u << SI_FINE_LOG2); t += SI_THREADS) h[t] = 0;
    si_special_init(&spec);
    __syncthreads();
    // rows at pseudo-random positions: the distinct-key estimate holds for any row order
    // (evenly spaced blocks of a sorted column saw a few keys each)
    for (uint64_t r = threadIdx.x; r < SI_BATCH; r += SI_THREADS) {
        // a sample as large as the rows covers each row once (exact estimate)
        const uint64_t lin = blockIdx.x * (uint64_t)SI_BATCH + r;
        if ((uint64_t)gridDim.x * SI_BATCH >= sp.n && lin >= sp.n) break;
        const uint64_t i = (uint64_t)gridDim.x * SI_BATCH >= sp.n ? lin : hash64(block_stride * 0x9E3779B97F4A7C15ULL + lin) % sp.n;
        si_kb_t<T> kb;
        if (!si_row<T>(sp, i, &spec, &kb)) continue;
        atomicAdd(&h[si_h32(kb) >> (32 - SI_FINE_LOG2)], 1u);
        uint64_t pos = hash64(kb) & smask;
        for (int p = 0; p < 1 << 14; p++) {
            uint64_t cur = __hip_atomic_load(&skeys[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur == SET_EMPTY)
                cur = atomicCAS((unsigned long long *)&skeys[pos], (unsigned long long)SET_EMPTY, (unsigned long long)kb);
            if (cur == SET_EMPTY || cur == (uint64_t)kb) {
                atomicAdd(&scnt[pos], 1u);
                break;
            }
            pos = (pos + 1) & smask;
        }
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < (1u << SI_FINE_LOG2); t += SI_THREADS)
        if (h[t]) atomicAdd(&fine_hist[t], (unsigned long long)h[t]);
}

// distinct keys of the sample, and how many were seen once / twice (Chao1 inputs)
__global__ __launch_bounds__(256) void k_si_sample_stats(const uint32_t *scnt, uint64_t slots, unsigned long long *stats) {
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
__host__ __device__ constexpr size_t si_scatter_lds_bytes(uint32_t P) {
    return (size_t)(8 + 4 + 4) * (SI_BATCH + 1) + 16 * ((size_t)P + 1) + 64;
}

__device__ inline void si_lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ inline void si_new_init(uint32_t *s_new) {
    if (threadIdx.x == 0) *s_new = 0;
}
// after a workgroup barrier
__device__ inline void si_new_flush(const uint32_t *s_new, uint64_t *ctr) {
    if (threadIdx.x == 0 && *s_new) atomicAdd((unsigned long long *)&ctr[C_DISTINCT], (unsigned long long)*s_new);
}

template <typename T>
__global__ __launch_bounds__(SI_THREADS) void k_si_scatter(SiParams sp, SiTable g) {
    using KB = si_kb_t<T>;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    __shared__ SiSpecial spec;
    __shared__ uint32_t s_total, s_over, s_new;
    g.wg_new = &s_new;
    si_new_init(&s_new);
    uint64_t *skb = reinterpret_cast<uint64_t *>(lds_raw);           // [SI_BATCH + 1]
    uint32_t *srow = reinterpret_cast<uint32_t *>(skb + SI_BATCH + 1);  // [SI_BATCH + 1]
    uint32_t *sdst = srow + SI_BATCH + 1;                               // [SI_BATCH + 1]
    uint32_t *hist = sdst + SI_BATCH + 1;                               // [P + 1]: [P] = sink
    uint32_t *boff = hist + sp.P + 1, *base = boff + sp.P, *lim = base + sp.P, *wave_sums = lim + sp.P;
    for (uint32_t t = threadIdx.x; t <= sp.P; t += SI_THREADS) hist[t] = 0;
    for (uint32_t t = threadIdx.x; t < sp.P; t += SI_THREADS) {
        base[t] = (uint32_t)sp.toff[t];
        lim[t] = (uint32_t)sp.toff[t] + sp.cap[t];
    }
    si_special_init(&spec);
    __syncthreads();
    // batches w, w + W, w + 2W, ...: every workgroup's rows spread over the whole range
    const uint32_t w = blockIdx.x, P = sp.P;
    const uint64_t row_end = sp.n;
    const uint64_t region0 = (uint64_t)w * sp.wg_stride;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t novf = 0;
    for (uint64_t b0 = (uint64_t)w * SI_BATCH; b0 < row_end; b0 += (uint64_t)sp.W * SI_BATCH) {
        KB kb[SI_RPT];
        uint32_t bkt[SI_RPT];
        int32_t rank[SI_RPT];
#pragma unroll
        for (int r = 0; r < SI_RPT; r++) {
            const uint64_t i = b0 + (uint64_t)r * SI_THREADS + threadIdx.x;
            rank[r] = -1;
            bkt[r] = 0;
            kb[r] = 0;
            bool ok = i < row_end && si_row<T>(sp, i, &spec, &kb[r]);
            // a regular row whose key equals the previous row's (also regular) cannot be a
            // first appearance: dropped (a sorted or clustered key column sends one row per run)
            const bool pok = __shfl_up((int)ok, 1, 64) != 0;
            const KB pk = __shfl_up(kb[r], 1, 64);
            if (ok && pok && lane > 0 && pk == kb[r]) ok = false;
            if (ok) {
                bkt[r] = si_bucket((uint64_t)kb[r], sp.p_log2);
                rank[r] = (int32_t)atomicAdd(&hist[bkt[r]], 1u);
            }
        }
        // exclusive scan of the bucket histogram
        si_lds_barrier();
        {
            const uint32_t per = (P + SI_THREADS - 1) / SI_THREADS;
            const uint32_t t0 = threadIdx.x * per;
            uint32_t sum = 0;
            for (uint32_t t = t0; t < t0 + per && t < P; t++) sum += hist[t];
            uint32_t inc = sum;
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(inc, off, 64);
                if (lane >= off) inc += y;
            }
            if (lane == 63) wave_sums[wave] = inc;
            si_lds_barrier();
            uint32_t wave_base = 0, total = 0;
            for (int k = 0; k < SI_THREADS / 64; k++) {
                if (k < wave) wave_base += wave_sums[k];
                total += wave_sums[k];
            }
            uint32_t acc = wave_base + inc - sum;
            for (uint32_t t = t0; t < t0 + per && t < P; t++) {
                boff[t] = acc;
                acc += hist[t];
            }
            if (threadIdx.x == 0) {
                s_total = total;
                s_over = 0;
            }
        }
        si_lds_barrier();
        bool over = false;
#pragma unroll
        for (int r = 0; r < SI_RPT; r++) {
            if (rank[r] < 0) continue;
            const uint32_t t = bkt[r];
            const uint32_t pos = boff[t] + (uint32_t)rank[r];
            const uint32_t d = base[t] + (uint32_t)rank[r];
            const bool fits = d < lim[t];
            over |= !fits;
            sdst[pos] = fits ? d : SI_DEST_OVER;
            skb[pos] = (uint64_t)kb[r];
            srow[pos] = (uint32_t)(b0 + (uint64_t)r * SI_THREADS + threadIdx.x);
        }
        if (over) s_over = 1;
        si_lds_barrier();
        const uint32_t tot = s_total;
        for (uint32_t k = threadIdx.x; k < tot; k += SI_THREADS) {
            const uint32_t dst = sdst[k];
            if (dst & SI_DEST_OVER) continue;
            const uint64_t e = region0 + dst;
            if constexpr (sizeof(KB) == 4) {
                reinterpret_cast<uint64_t *>(sp.ent)[e] = ((uint64_t)srow[k] << 32) | (uint32_t)skb[k];
            } else {
                reinterpret_cast<uint64_t *>(sp.ent)[e] = skb[k];
                sp.ent_row[e] = srow[k];
            }
        }
        if (s_over) {  // a full region (sampling miss): those rows go to the HBM table
            for (uint32_t k = threadIdx.x; k < tot; k += SI_THREADS)
                if (sdst[k] & SI_DEST_OVER) {
                    si_global(g, skb[k], sp.row0 + srow[k]);
                    novf++;
                }
        }
        si_lds_barrier();
        for (uint32_t t = threadIdx.x; t < P; t += SI_THREADS) {
            base[t] += hist[t];
            hist[t] = 0;
        }
        si_lds_barrier();
    }
    if (novf) atomicAdd(&d_si_overflow_rows, (unsigned long long)novf);
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < P; t += SI_THREADS) sp.fills[(uint64_t)t * sp.W + w] = base[t] - (uint32_t)sp.toff[t];
    si_special_flush(&spec, sp.row0, g.ctr);
    si_new_flush(&s_new, g.ctr);
}

// Pass A for keys of <= 4 bytes, after the tile path's fast scatter: SB batches of 4096 rows
// are ranked before one commit, so a partition's run per commit is SB times longer (short
// runs are partial lines HBM receives twice: 9.9 GB written for 8 GB of entries with one
// batch per commit).  LDS holds the staged key bits and rows (8 B per row); a staged row's
// partition is recomputed from its key at stream-out; one wave's scan turns the histogram
// into sorted offsets, destination bases and advanced region bases (three LDS barriers).
__host__ __device__ constexpr size_t si_fast_lds_bytes(int sb, uint32_t P) {
    return (size_t)8 * sb * SI_BATCH + 20 * ((size_t)P + 1) + 64;
}

// PLAIN: 4-byte integer keys without mask / select, 16-byte aligned, n a multiple of 4 -- the
// keys are read as 16-byte quads and the next batch is prefetched in registers while this
// one is ranked (a quad is wholly inside a workgroup's range or wholly past it)
template <typename T, int SB, bool PLAIN>
__global__ __launch_bounds__(SI_THREADS) void k_si_scatter4(SiParams sp, SiTable g) {
    static_assert(sizeof(T) <= 4, "keys of at most 4 bytes");
    static_assert(!PLAIN || sizeof(T) == 4, "quad loads take 4-byte keys");
    constexpr uint32_t CAP = SB * SI_BATCH;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    __shared__ SiSpecial spec;
    __shared__ uint32_t s_new;
    g.wg_new = &s_new;
    si_new_init(&s_new);
    const uint32_t P = sp.P;
    uint32_t *sk = reinterpret_cast<uint32_t *>(lds_raw);
    uint32_t *srow = sk + CAP;
    uint32_t *hist = srow + CAP;  // [P + 1]: hist[P] takes the ranks of rows that are dropped
    uint32_t *boff = hist + P + 1, *dbase = boff + P, *base = dbase + P, *lim = base + P;
    uint32_t *wave_sums = lim + P;
    for (uint32_t t = threadIdx.x; t <= P; t += SI_THREADS) hist[t] = 0;
    for (uint32_t t = threadIdx.x; t < P; t += SI_THREADS) {
        base[t] = (uint32_t)sp.toff[t];
        lim[t] = (uint32_t)sp.toff[t] + sp.cap[t];
    }
    si_special_init(&spec);
    __syncthreads();
    // batches w, w + W, w + 2W, ...: every workgroup's rows spread over the whole range
    const uint32_t w = blockIdx.x;
    const uint64_t row_end = sp.n, bstep = (uint64_t)sp.W * SI_BATCH;
    const uint64_t region0 = (uint64_t)w * sp.wg_stride;
    const int lane = threadIdx.x & 63;
    uint64_t *ent = static_cast<uint64_t *>(sp.ent);
    constexpr int QUADS = SI_RPT / 4;
    // row of slot r (batch r / SI_RPT of the commit starting at b0): plain -- lane-owned
    // quads; else -- one row per lane per step
    auto row_of = [&](uint64_t b0, int r) -> uint64_t {
        const int sb = r / SI_RPT, rr = r % SI_RPT;
        if constexpr (PLAIN) {
            return b0 + (uint64_t)sb * bstep + 4 * ((uint64_t)(rr >> 2) * SI_THREADS + threadIdx.x) + (rr & 3);
        } else {
            return b0 + (uint64_t)sb * bstep + (uint64_t)rr * SI_THREADS + threadIdx.x;
        }
    };
    uint4 cur[QUADS], nxt[QUADS];
    auto load = [&](uint64_t b0, uint4 (&R)[QUADS]) {
#pragma unroll
        for (int q = 0; q < QUADS; q++) {
            const uint64_t i = b0 + 4 * ((uint64_t)q * SI_THREADS + threadIdx.x);
            const uint64_t is = i < sp.n - 4 ? i : sp.n - 4;
            R[q] = *reinterpret_cast<const uint4 *>(static_cast<const T *>(sp.keys) + is);
        }
    };
    uint32_t novf = 0;
    if constexpr (PLAIN) load((uint64_t)w * SI_BATCH, cur);
    for (uint64_t b0 = (uint64_t)w * SI_BATCH; b0 < row_end; b0 += SB * bstep) {
        uint32_t kb[SB * SI_RPT];
        int32_t rank[SB * SI_RPT];
        // a row whose key equals the previous row's cannot be a first appearance: dropped
        // (a sorted or clustered key column sends one row per run)
        if constexpr (PLAIN) {
#pragma unroll
            for (int sb = 0; sb < SB; sb++) {
                load(b0 + (uint64_t)(sb + 1) * bstep, nxt);
#pragma unroll
                for (int q = 0; q < QUADS; q++) {
                    const uint32_t w4[4] = {cur[q].x, cur[q].y, cur[q].z, cur[q].w};
                    const uint32_t prev3 = (uint32_t)__shfl_up((int)cur[q].w, 1, 64);
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int rr = 4 * q + j, r = sb * SI_RPT + rr;
                        kb[r] = w4[j];
                        const bool dup = j > 0 ? w4[j] == w4[j - 1] : (lane > 0 && w4[0] == prev3);
                        const bool ok = row_of(b0, r) < row_end && !dup;
                        const uint32_t rk = atomicAdd(&hist[ok ? si_bucket((uint64_t)kb[r], sp.p_log2) : P], 1u);
                        rank[r] = ok ? (int32_t)rk : -1;
                    }
                }
#pragma unroll
                for (int q = 0; q < QUADS; q++) cur[q] = nxt[q];
            }
        } else {
#pragma unroll
            for (int r = 0; r < SB * SI_RPT; r++) {
                const uint64_t i = row_of(b0, r);
                kb[r] = 0;
                bool ok = i < row_end && si_row<T>(sp, i, &spec, &kb[r]);
                const bool pok = __shfl_up((int)ok, 1, 64) != 0;
                const uint32_t pk = (uint32_t)__shfl_up((int)kb[r], 1, 64);
                if (ok && pok && lane > 0 && pk == kb[r]) ok = false;
                const uint32_t rk = atomicAdd(&hist[ok ? si_bucket((uint64_t)kb[r], sp.p_log2) : P], 1u);
                rank[r] = ok ? (int32_t)rk : -1;
            }
        }
        si_lds_barrier();
        if (threadIdx.x < 64) {
            const uint32_t lane = threadIdx.x;
            const uint32_t per = (P + 63) / 64;
            const uint32_t t0 = lane * per;
            uint32_t sum = 0;
            for (uint32_t t = t0; t < t0 + per && t < P; t++) sum += hist[t];
            uint32_t inc = sum;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(inc, off, 64);
                if ((int)lane >= off) inc += y;
            }
            uint32_t acc = inc - sum;
            for (uint32_t t = t0; t < t0 + per && t < P; t++) {
                const uint32_t hh = hist[t], bb = base[t];
                boff[t] = acc;
                dbase[t] = bb - acc;
                base[t] = bb + hh;
                hist[t] = 0;
                acc += hh;
            }
            if (lane == 0) hist[P] = 0;
            if (lane == 63) wave_sums[0] = inc;
        }
        si_lds_barrier();
        const uint32_t tot = wave_sums[0];
#pragma unroll
        for (int r = 0; r < SB * SI_RPT; r++) {
            if (rank[r] < 0) continue;
            const uint32_t pos = boff[si_bucket((uint64_t)kb[r], sp.p_log2)] + (uint32_t)rank[r];
            sk[pos] = kb[r];
            srow[pos] = (uint32_t)row_of(b0, r);
        }
        si_lds_barrier();
        for (uint32_t k = threadIdx.x; k < tot; k += SI_THREADS) {
            const uint32_t key = sk[k], row = srow[k];
            const uint32_t t = si_bucket((uint64_t)key, sp.p_log2);
            const uint32_t dest = dbase[t] + k;
            if (dest < lim[t]) {
                ent[region0 + dest] = ((uint64_t)row << 32) | key;
            } else {
                si_global(g, (uint64_t)key, sp.row0 + row);  // a full region (sampling miss)
                novf++;
            }
        }
    }
    if (novf) atomicAdd(&d_si_overflow_rows, (unsigned long long)novf);
    si_lds_barrier();
    for (uint32_t t = threadIdx.x; t < P; t += SI_THREADS) sp.fills[(uint64_t)t * sp.W + w] = base[t] - (uint32_t)sp.toff[t];
    si_special_flush(&spec, sp.row0, g.ctr);
    si_new_flush(&s_new, g.ctr);
}

// ---- pass B -------------------------------------------------------------------------------
template <typename KB>
__global__ __launch_bounds__(SB_THREADS) void k_si_reduce(SiParams sp, SiTable g, const SiUnit *units) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    __shared__ uint32_t s_fill[1024];
    __shared__ uint32_t s_pre[1025];
    __shared__ uint32_t s_new;
    g.wg_new = &s_new;
    si_new_init(&s_new);
    const SiUnit u = units[blockIdx.x];
    const uint32_t b = u.bucket;
    const uint32_t cap = sp.cap[b];
    const uint32_t nw = u.w_end - u.w_begin;  // <= 1024 (host checks)
    bool any = false;
    for (uint32_t k = threadIdx.x; k < nw; k += SB_THREADS) {
        const uint32_t f = min(sp.fills[(uint64_t)b * sp.W + u.w_begin + k], cap);
        s_fill[k] = f;
        any |= f != 0;
    }
    if (!__syncthreads_or(any)) return;
    const SiLds<KB> t = si_lt_layout<KB>(lds_raw);
    si_lt_init<KB>(t, SB_THREADS);
    if (threadIdx.x < 64) {  // exclusive scan of the region fills (16 regions per lane)
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
    const uint64_t toff_b = sp.toff[b];
    uint32_t kr = 0;  // region of this lane's current entry (entry indices of a lane only grow)
    for (uint32_t c0 = 0; c0 < E; c0 += SB_THREADS * SB_M) {
        KB kb[SB_M];
        uint32_t row[SB_M];
        bool valid[SB_M];
#pragma unroll
        for (int j = 0; j < SB_M; j++) {
            const uint32_t c = c0 + j * SB_THREADS + threadIdx.x;
            const uint32_t cc = c < E ? c : E - 1;
            while (s_pre[kr + 1] <= cc) kr++;
            const uint64_t e = (uint64_t)(u.w_begin + kr) * sp.wg_stride + toff_b + (cc - s_pre[kr]);
            valid[j] = c < E;
            if constexpr (sizeof(KB) == 4) {
                const uint64_t q = reinterpret_cast<const uint64_t *>(sp.ent)[e];
                kb[j] = (KB)(uint32_t)q;
                row[j] = (uint32_t)(q >> 32);
            } else {
                kb[j] = reinterpret_cast<const uint64_t *>(sp.ent)[e];
                row[j] = sp.ent_row[e];
            }
        }
        if (DBG(sp.debug) & 2) {
#pragma unroll
            for (int j = 0; j < SB_M; j++) asm volatile("" ::"v"(kb[j]), "v"(row[j]));
        } else {
            constexpr int MM = sizeof(KB) == 4 ? SB_M / 2 : SB_M / 4;  // 128 VGPRs at 1024 threads
#pragma unroll
            for (int h0 = 0; h0 < SB_M; h0 += MM) si_lt_add_many<KB, MM>(t, g, sp.row0, kb + h0, row + h0, valid + h0);
        }
    }
    __syncthreads();
    if (!(DBG(sp.debug) & 1)) si_lt_merge<KB>(t, g, sp.row0, SB_THREADS);
    __syncthreads();
    si_new_flush(&s_new, g.ctr);
}

// ---- direct (P == 1): each workgroup dedups its row range of the raw keys -----------------
template <typename T>
__global__ __launch_bounds__(SB_THREADS) void k_si_direct(SiParams sp, SiTable g) {
    using KB = si_kb_t<T>;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    __shared__ SiSpecial spec;
    __shared__ uint32_t s_new;
    g.wg_new = &s_new;
    si_new_init(&s_new);
    const SiLds<KB> t = si_lt_layout<KB>(lds_raw);
    si_lt_init<KB>(t, SB_THREADS);
    si_special_init(&spec);
    __syncthreads();
    const uint64_t row_begin = (uint64_t)blockIdx.x * sp.rows_per_wg;
    const uint64_t row_end = min(sp.n, row_begin + sp.rows_per_wg);
    constexpr int U = 4;
    for (uint64_t b0 = row_begin; b0 < row_end; b0 += (uint64_t)U * SB_THREADS) {
        KB kb[U];
        uint32_t row[U];
        bool valid[U];
#pragma unroll
        for (int r = 0; r < U; r++) {
            const uint64_t i = b0 + (uint64_t)r * SB_THREADS + threadIdx.x;
            kb[r] = 0;
            row[r] = (uint32_t)i;
            valid[r] = i < row_end && si_row<T>(sp, i, &spec, &kb[r]);
        }
        si_lt_add_many<KB, U>(t, g, sp.row0, kb, row, valid);
    }
    __syncthreads();
    si_lt_merge<KB>(t, g, sp.row0, SB_THREADS);
    __syncthreads();
    si_special_flush(&spec, sp.row0, g.ctr);
    si_new_flush(&s_new, g.ctr);
}

__global__ void k_set_rehash(const uint64_t *otab, uint64_t ocap, uint64_t *ntab, uint64_t ncap_mask) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ocap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t kb = otab[2 * i];
        if (kb == SET_EMPTY) continue;
        uint64_t pos = hash64(kb) & ncap_mask;
        for (;;) {
            uint64_t old = atomicCAS((unsigned long long *)&ntab[2 * pos], (unsigned long long)SET_EMPTY,
                                     (unsigned long long)kb);
            if (old == SET_EMPTY) break;
            pos = (pos + 1) & ncap_mask;
        }
        ntab[2 * pos + 1] = otab[2 * i + 1];
    }
}

__global__ __launch_bounds__(256) void k_set_compact(const uint64_t *tab, uint64_t cap, uint64_t *slot, uint64_t *first,
                                                     uint64_t *bits, uint64_t *ctr) {
    // 8 consecutive slots per thread; output positions reserved once per workgroup and tile
    // (one cursor add per wave was one same-address atomic per 64 slots)
    __shared__ uint32_t s_w[4];
    __shared__ unsigned long long s_base;
    constexpr int R = 8;
    const uint64_t tile = 256ull * R, step = (uint64_t)gridDim.x * tile;
    for (uint64_t t0 = blockIdx.x * tile; t0 < cap; t0 += step) {
        const uint64_t i0 = t0 + (uint64_t)threadIdx.x * R;
        uint64_t kb[R];
        uint32_t occ = 0;
#pragma unroll
        for (int r = 0; r < R; r++) {
            kb[r] = i0 + r < cap ? tab[2 * (i0 + r)] : SET_EMPTY;
            if (kb[r] != SET_EMPTY) occ |= 1u << r;
        }
        uint64_t j = block_reserve<256>((uint32_t)__popc(occ), s_w, &s_base,
                                        reinterpret_cast<unsigned long long *>(&ctr[C_CURSOR]));
#pragma unroll
        for (int r = 0; r < R; r++) {
            if (!((occ >> r) & 1)) continue;
            const uint64_t i = i0 + r;
            slot[j] = i;
            first[j] = tab[2 * i + 1];
            bits[j] = kb[r];
            j++;
        }
    }
}

// ---- first-appearance ranks without a sort: first rows are distinct, so the rank of key j
// is the number of set bits below first[j] in a row bitmap (per-word popcounts + scan)
__global__ void k_rank_mark(const uint64_t *first, uint64_t m, uint64_t *bitmap) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t f = first[j];
        atomicOr((unsigned long long *)&bitmap[f >> 6], 1ULL << (f & 63));
    }
}

constexpr int SCAN_THREADS = 256, SCAN_PER_THREAD = 16, SCAN_TILE = SCAN_THREADS * SCAN_PER_THREAD;

// inclusive block scan of one value per thread (wave64 shuffles + wave partials in LDS)
__device__ inline uint32_t block_scan_inclusive(uint32_t v, uint32_t *wsum, uint32_t *total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(v, off, 64);
        if (lane >= off) v += y;
    }
    if (lane == 63) wsum[wave] = v;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (int k = 0; k < SCAN_THREADS / 64; k++) {
        if (k < wave) base += wsum[k];
        tot += wsum[k];
    }
    __syncthreads();
    *total = tot;
    return base + v;
}

// phase 1: per-tile sums of popcount(bitmap words)
__global__ __launch_bounds__(SCAN_THREADS) void k_rank_tile_sums(const uint64_t *bitmap, uint64_t nw, uint32_t *tile_sum) {
    __shared__ uint32_t wsum[SCAN_THREADS / 64];
    const uint64_t w0 = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_PER_THREAD;
    uint32_t c = 0;
    for (int k = 0; k < SCAN_PER_THREAD; k++)
        if (w0 + k < nw) c += __popcll(bitmap[w0 + k]);
    uint32_t tot;
    block_scan_inclusive(c, wsum, &tot);
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = tot;
}

// phase 2: exclusive scan of the tile sums in place (one workgroup)
__global__ __launch_bounds__(SCAN_THREADS) void k_rank_scan_tiles(uint32_t *tile_sum, uint64_t ntiles) {
    __shared__ uint32_t wsum[SCAN_THREADS / 64];
    uint32_t carry = 0;
    for (uint64_t b = 0; b < ntiles; b += SCAN_THREADS) {
        const uint64_t i = b + threadIdx.x;
        const uint32_t v = i < ntiles ? tile_sum[i] : 0;
        uint32_t tot;
        const uint32_t inc = block_scan_inclusive(v, wsum, &tot);
        if (i < ntiles) tile_sum[i] = carry + inc - v;
        carry += tot;
    }
}

// phase 3: exclusive prefix of set bits per word
__global__ __launch_bounds__(SCAN_THREADS) void k_rank_word_prefix(const uint64_t *bitmap, uint64_t nw,
                                                                   const uint32_t *tile_base, uint32_t *word_prefix) {
    __shared__ uint32_t wsum[SCAN_THREADS / 64];
    const uint64_t w0 = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_PER_THREAD;
    uint32_t c[SCAN_PER_THREAD], sum = 0;
    for (int k = 0; k < SCAN_PER_THREAD; k++) {
        c[k] = w0 + k < nw ? __popcll(bitmap[w0 + k]) : 0;
        sum += c[k];
    }
    uint32_t tot;
    uint32_t acc = tile_base[blockIdx.x] + block_scan_inclusive(sum, wsum, &tot) - sum;
    for (int k = 0; k < SCAN_PER_THREAD; k++) {
        if (w0 + k < nw) word_prefix[w0 + k] = acc;
        acc += c[k];
    }
}

__device__ inline uint64_t rank_of_row(const uint64_t *bitmap, const uint32_t *word_prefix, uint64_t r) {
    const uint64_t w = r >> 6, b = r & 63;
    return word_prefix[w] + __popcll(bitmap[w] & ((1ULL << b) - 1));
}

struct SpecialKeys {
    uint64_t key[3];  // sort keys (2*row for the EMPTY-bits key, 2*end_of_call - 1 for NaN / null)
    int n;
};

// ordinal of compacted key j = its rank among the regular keys + the special keys before it;
// also records the key bits per ordinal
__global__ void k_rank_assign(const uint64_t *first, const uint64_t *bits, uint64_t m, const uint64_t *bitmap,
                              const uint32_t *word_prefix, SpecialKeys sk, int64_t *ord, uint64_t *bits_by_ord) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t f = first[j];
        uint64_t o = rank_of_row(bitmap, word_prefix, f);
        for (int s = 0; s < sk.n; s++) o += 2 * f > sk.key[s];
        ord[j] = (int64_t)o;
        bits_by_ord[o] = bits[j];
    }
}

// number of regular keys first seen before row r (r may be the end of the rows)
__global__ void k_rank_rows(const uint64_t *bitmap, const uint32_t *word_prefix, uint64_t nrows, uint64_t m,
                            SpecialKeys sk, uint64_t *out) {
    const int s = threadIdx.x;
    if (s >= sk.n) return;
    const uint64_t r = (sk.key[s] + 1) / 2;  // regular keys with 2 * first < key
    out[s] = r >= nrows ? m : rank_of_row(bitmap, word_prefix, r);
}

// lookup table slot j <- (key bits, ordinal) of compacted key j at its table position
__global__ void k_set_build_lut(const uint64_t *slot, const uint64_t *bits, const int64_t *ord, uint64_t m, int wide,
                                uint64_t *lut) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < m;
         j += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t pos = slot[j];
        if (wide) {
            lut[2 * pos] = bits[j];
            lut[2 * pos + 1] = (uint64_t)ord[j];
        } else {
            lut[pos] = ((uint64_t)ord[j] << 32) | (bits[j] & 0xffffffffULL);
        }
    }
}

template <typename T, typename O>
__global__ __launch_bounds__(256) void k_set_map_ordinal(const T *keys, uint64_t n, SetDev s, int64_t nan_value, O *out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const T v = keys[i];
        int64_t o = is_nan_v(v) ? nan_value : set_lookup_bits(s, key_bits(v));
        out[i] = (O)o;
    }
}

static void set_grow(vh_set *s, uint64_t new_cap) {
    DevBuf nt;
    nt.ensure(new_cap * 16);
    VH_HIP(hipMemsetAsync(nt.ptr, 0xff, new_cap * 16, stream()));
    if (s->cap) {
        hipLaunchKernelGGL(k_set_rehash, dim3(blocks_for(s->cap, 256)), dim3(256), 0, stream(), s->tab.as<uint64_t>(),
                           s->cap, nt.as<uint64_t>(), new_cap - 1);
        VH_HIP(hipGetLastError());
    }
    VH_HIP(hipStreamSynchronize(stream()));
    std::swap(s->tab.ptr, nt.ptr);
    std::swap(s->tab.bytes, nt.bytes);
    s->cap = new_cap;
    s->sealed = false;
}

static std::vector<uint64_t> read_ctr(vh_set *s) {
    std::vector<uint64_t> c(C_N);
    VH_HIP(hipMemcpyAsync(c.data(), s->ctr.ptr, 8 * C_N, hipMemcpyDeviceToHost, stream()));
    VH_HIP(hipStreamSynchronize(stream()));
    return c;
}

static void set_seal(vh_set *s) {
    if (s->sealed) return;
    auto c = read_ctr(s);
    const uint64_t cap = s->cap;
    s->c_slot.ensure(cap * 8);
    s->c_first.ensure(cap * 8);
    s->c_bits.ensure(cap * 8);
    s->c_ord.ensure(cap * 8);
    uint64_t zero = 0;
    VH_HIP(hipMemcpyAsync(s->ctr.as<uint64_t>() + C_CURSOR, &zero, 8, hipMemcpyHostToDevice, stream()));
    hipLaunchKernelGGL(k_set_compact, dim3(blocks_for((cap + 7) / 8, 256)), dim3(256), 0, stream(), s->tab.as<uint64_t>(), cap,
                       s->c_slot.as<uint64_t>(), s->c_first.as<uint64_t>(), s->c_bits.as<uint64_t>(),
                       s->ctr.as<uint64_t>());
    VH_HIP(hipGetLastError());
    c = read_ctr(s);
    const uint64_t m = c[C_CURSOR];
    // special keys (at most 3), ordered by (sort key, tie) as the reference flushes them
    struct Spec {
        uint64_t key;
        int tie;  // 0 EMPTY-bits key, 1 NaN, 2 null
    };
    std::vector<Spec> specs;
    if (c[C_SPECIAL_FIRST] != ~0ULL) specs.push_back({2 * c[C_SPECIAL_FIRST], 0});
    if (c[C_NAN_FIRST] != ~0ULL) specs.push_back({2 * s->nan_pos - 1, 1});
    if (c[C_NULL_FIRST] != ~0ULL) specs.push_back({2 * s->null_pos - 1, 2});
    std::sort(specs.begin(), specs.end(), [](const Spec &a, const Spec &b) {
        return a.key != b.key ? a.key < b.key : a.tie < b.tie;
    });
    SpecialKeys sk{};
    sk.n = (int)specs.size();
    for (int k = 0; k < sk.n; k++) sk.key[k] = specs[k].key;
    const uint64_t total = m + specs.size();
    const uint64_t nrows = std::max<uint64_t>(s->rows_seen, 1);
    const uint64_t nw = (nrows + 63) / 64;
    const uint64_t ntiles = (nw + SCAN_TILE - 1) / SCAN_TILE;
    DevBuf bitmap, prefix, tiles, bits_by_ord, spec_rank;
    bitmap.ensure(nw * 8);
    prefix.ensure(nw * 4);
    tiles.ensure(ntiles * 4);
    bits_by_ord.ensure(std::max<uint64_t>(total, 1) * 8);
    spec_rank.ensure(3 * 8);
    VH_HIP(hipMemsetAsync(bitmap.ptr, 0, nw * 8, stream()));
    VH_HIP(hipMemsetAsync(bits_by_ord.ptr, 0xff, std::max<uint64_t>(total, 1) * 8, stream()));
    {
        TimedScope ts("set_rank");
        if (m) hipLaunchKernelGGL(k_rank_mark, dim3(blocks_for(m, 256)), dim3(256), 0, stream(), s->c_first.as<uint64_t>(), m,
                                  bitmap.as<uint64_t>());
        hipLaunchKernelGGL(k_rank_tile_sums, dim3(ntiles), dim3(SCAN_THREADS), 0, stream(), bitmap.as<uint64_t>(), nw,
                           tiles.as<uint32_t>());
        hipLaunchKernelGGL(k_rank_scan_tiles, dim3(1), dim3(SCAN_THREADS), 0, stream(), tiles.as<uint32_t>(), ntiles);
        hipLaunchKernelGGL(k_rank_word_prefix, dim3(ntiles), dim3(SCAN_THREADS), 0, stream(), bitmap.as<uint64_t>(), nw,
                           tiles.as<uint32_t>(), prefix.as<uint32_t>());
        if (m) hipLaunchKernelGGL(k_rank_assign, dim3(blocks_for(m, 256)), dim3(256), 0, stream(), s->c_first.as<uint64_t>(),
                                  s->c_bits.as<uint64_t>(), m, bitmap.as<uint64_t>(), prefix.as<uint32_t>(), sk,
                                  s->c_ord.as<int64_t>(), bits_by_ord.as<uint64_t>());
        if (sk.n) hipLaunchKernelGGL(k_rank_rows, dim3(1), dim3(64), 0, stream(), bitmap.as<uint64_t>(), prefix.as<uint32_t>(),
                                     s->rows_seen, m, sk, spec_rank.as<uint64_t>());
        VH_HIP(hipGetLastError());
    }
    std::vector<uint64_t> srank(3, 0);
    s->key_bits.assign(total, 0);
    s->key_kind.assign(total, 0);
    if (total) VH_HIP(hipMemcpyAsync(s->key_bits.data(), bits_by_ord.ptr, total * 8, hipMemcpyDeviceToHost, stream()));
    if (sk.n) VH_HIP(hipMemcpyAsync(srank.data(), spec_rank.ptr, 3 * 8, hipMemcpyDeviceToHost, stream()));
    const int wide = dtype_itemsize(s->dtype) > 4;
    s->lut.ensure(cap * (wide ? 16 : 8));
    VH_HIP(hipMemsetAsync(s->lut.ptr, 0xff, cap * (wide ? 16 : 8), stream()));
    if (m) {
        hipLaunchKernelGGL(k_set_build_lut, dim3(blocks_for(m, 256)), dim3(256), 0, stream(), s->c_slot.as<uint64_t>(),
                           s->c_bits.as<uint64_t>(), s->c_ord.as<int64_t>(), m, wide, s->lut.as<uint64_t>());
        VH_HIP(hipGetLastError());
    }
    VH_HIP(hipStreamSynchronize(stream()));
    s->nan_ord = s->null_ord = s->special_ord = -1;
    for (int k = 0; k < sk.n; k++) {
        const int64_t o = (int64_t)srank[k] + k;  // regular keys before it + earlier specials
        if (specs[k].tie == 1) {
            s->nan_ord = o;
            s->key_kind[o] = 1;
        } else if (specs[k].tie == 2) {
            s->null_ord = o;
            s->key_kind[o] = 2;
        } else {
            s->special_ord = o;
            s->key_kind[o] = 3;
            s->key_bits[o] = SET_EMPTY;
        }
    }
    VH_HIP(hipStreamSynchronize(stream()));
    s->length = (int64_t)total;
    s->nan_count = (int64_t)c[C_NAN_COUNT];
    s->null_count = (int64_t)c[C_NULL_COUNT];
    s->sealed = true;
}

SetDev set_device_view(vh_set *s) {
    std::lock_guard<std::recursive_mutex> lk(s->mu);
    set_seal(s);
    SetDev d{};
    d.lut = s->lut.as<uint64_t>();
    d.wide = dtype_itemsize(s->dtype) > 4;
    d.cap_mask = s->cap - 1;
    d.nan_ord = s->nan_ord;
    d.null_ord = s->null_ord;
    d.special_ord = s->special_ord;
    return d;
}

int set_dtype(const vh_set *s) { return s->dtype; }

template <typename T> static void write_keys(vh_set *s, T *o) {
    for (int64_t i = 0; i < s->length; i++) {
        const int kind = s->key_kind[i];
        uint64_t b = s->key_bits[i];
        if (kind == 1) {  // NaNish<T>::value (hash_primitives.hpp:23-41)
            if constexpr (is_float_t<T>::value) o[i] = std::numeric_limits<T>::quiet_NaN();
            else memset(&o[i], 0xff, sizeof(T));
        } else if (kind == 2) {  // null -> -1 (:306-308)
            if constexpr (std::is_same<T, vbool>::value) o[i].v = 1;
            else if constexpr (is_float_t<T>::value) o[i] = (T)-1;
            else memset(&o[i], 0xff, sizeof(T));
        } else {
            memcpy(&o[i], &b, sizeof(T));
        }
    }
}

}  // namespace vh

extern "C" {

int vh_set_create(int dtype, vh_set **out) {
    VH_API_BEGIN
    dtype_itemsize(dtype);
    std::unique_ptr<vh_set> s(new vh_set());
    s->dtype = dtype;
    s->ctr.ensure(8 * C_N);
    std::vector<uint64_t> init(C_N, 0);
    init[C_NAN_FIRST] = init[C_NULL_FIRST] = init[C_SPECIAL_FIRST] = ~0ULL;
    VH_HIP(hipMemcpyAsync(s->ctr.ptr, init.data(), 8 * C_N, hipMemcpyHostToDevice, stream()));
    set_grow(s.get(), 1 << 16);
    *out = s.release();
    VH_API_END
}

int vh_set_destroy(vh_set *s) {
    VH_API_BEGIN
    if (s) (void)hipStreamSynchronize(stream());
    delete s;
    VH_API_END
}

namespace vh {

// partition scratch shared by the sets of a device (regions of a 2^28-row chunk are ~2 GB)
struct SiScratch {
    std::mutex mu;
    DevBuf sample, meta, ent, ent_row;
};
static SiScratch &si_scratch() {
    static std::mutex g;
    static std::map<int, std::unique_ptr<SiScratch>> m;
    std::lock_guard<std::mutex> lk(g);
    auto &p = m[current_device()];
    if (!p) p = std::make_unique<SiScratch>();
    return *p;
}

static uint64_t si_next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

static int si_blocks_per_cu(const void *kernel, int threads, size_t lds) {
    int nb = 0;
    VH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, threads, lds));
    return std::max(1, nb);
}

// one chunk of rows (device-resident, < 2^32) into the set; rows numbered from row0
static void si_chunk(vh_set *s, SiScratch &S, const void *keys, const uint8_t *mask, const uint8_t *select, uint64_t n,
                     uint64_t row0) {
    hipStream_t st = stream();
    const int isz = dtype_itemsize(s->dtype);
    const int kbs = isz == 8 ? 8 : 4;
    SiParams sp{};
    sp.keys = keys;
    sp.mask = mask;
    sp.select = select;
    sp.n = n;
    sp.row0 = row0;
#ifdef VH_ABLATION
    if (const char *dbg = getenv("VH_SI_DEBUG")) sp.debug = (uint32_t)atoi(dbg);
#endif
    // ---- sample: fine bucket histogram + distinct estimate, read back with the counters
    const uint64_t sslots = 1ull << 21;
    const uint64_t nbatch = (n + SI_BATCH - 1) / SI_BATCH;
    const uint64_t sblocks = std::min<uint64_t>(nbatch, SI_SAMPLE_BLOCKS);
    const uint64_t bstride = std::max<uint64_t>(SI_BATCH, n / sblocks);
    const uint32_t FINE = 1u << SI_FINE_LOG2;
    S.sample.ensure(sslots * 12 + 8 * FINE + 64);
    uint64_t *skeys = S.sample.as<uint64_t>();
    uint32_t *scnt = reinterpret_cast<uint32_t *>(skeys + sslots);
    unsigned long long *fine = reinterpret_cast<unsigned long long *>(scnt + sslots);
    unsigned long long *stats = fine + FINE;
    VH_HIP(hipMemsetAsync(skeys, 0xff, 8 * sslots, st));
    VH_HIP(hipMemsetAsync(scnt, 0, 4 * sslots + 8 * FINE + 64, st));
    {
        TimedScope ts("set_sample");
        VH_DISPATCH_DTYPE(s->dtype, T,
                          hipLaunchKernelGGL(k_si_sample<T>, dim3(sblocks), dim3(SI_THREADS), 0, st, sp, bstride, fine,
                                             skeys, scnt, sslots - 1));
        hipLaunchKernelGGL(k_si_sample_stats, dim3(blocks_for(sslots, 256, 4)), dim3(256), 0, st, scnt, sslots, stats);
        VH_HIP(hipGetLastError());
    }
    std::vector<uint64_t> fh(FINE + 3), c(C_N);
    VH_HIP(hipMemcpyAsync(fh.data(), fine, 8 * (FINE + 3), hipMemcpyDeviceToHost, st));
    VH_HIP(hipMemcpyAsync(c.data(), s->ctr.ptr, 8 * C_N, hipMemcpyDeviceToHost, st));
    VH_HIP(hipStreamSynchronize(st));
    uint64_t sampled = 0;
    for (uint32_t i = 0; i < FINE; i++) sampled += fh[i];
    const double ds = (double)fh[FINE], f1 = (double)fh[FINE + 1], f2 = (double)fh[FINE + 2];
    double dest;
    if (sampled >= n || sblocks == nbatch) dest = ds;  // every row sampled: exact
    else dest = f2 > 0 ? ds + f1 * f1 / (2 * f2) : ds + f1 * (f1 - 1) / 2;  // Chao1
    dest = std::min<double>(std::max(dest, 1.0), (double)n);
    // the HBM table at <= 1/2 load for what it holds plus the estimate
    const uint64_t need = c[C_DISTINCT] + (uint64_t)dest;
    if (2 * need > s->cap) set_grow(s, si_next_pow2(2 * need));
    uint32_t p_log2 = 0;
    while (p_log2 < SI_MAX_P_LOG2 && dest / (double)(1u << p_log2) > SI_TARGET_KEYS) p_log2++;
    sp.p_log2 = p_log2;
    sp.P = 1u << p_log2;
    const uint32_t P = sp.P;
    const size_t lt_lds = si_lt_bytes(kbs);

    const bool plain = (s->dtype == VH_I32 || s->dtype == VH_U32) && !mask && !select && n % 4 == 0 &&
                       (reinterpret_cast<uintptr_t>(keys) & 15) == 0;
    std::vector<SiUnit> units;
    std::vector<uint32_t> cap;
    std::vector<uint64_t> toff;
    uint32_t W = 0;
    int fast_sb = 0;
    size_t lds_scatter = 0;
    // f(kernel instance) of the multi-batch pass A for this key dtype and fast_sb
    auto with_fast = [&](auto &&f) {
        auto by_sb = [&](auto tc) {
            using T = decltype(tc);
            if (fast_sb == 4) f(k_si_scatter4<T, 4, false>);
            else if (fast_sb == 3) f(k_si_scatter4<T, 3, false>);
            else if (fast_sb == 2) f(k_si_scatter4<T, 2, false>);
            else f(k_si_scatter4<T, 1, false>);
        };
        auto by_sb_plain = [&](auto tc) {
            using T = decltype(tc);
            if (fast_sb == 4) f(k_si_scatter4<T, 4, true>);
            else if (fast_sb == 3) f(k_si_scatter4<T, 3, true>);
            else if (fast_sb == 2) f(k_si_scatter4<T, 2, true>);
            else f(k_si_scatter4<T, 1, true>);
        };
        if (plain) {
            if (s->dtype == VH_I32) by_sb_plain(int32_t());
            else by_sb_plain(uint32_t());
            return;
        }
        switch (s->dtype) {
        case VH_I32: by_sb(int32_t()); break;
        case VH_U32: by_sb(uint32_t()); break;
        case VH_F32: by_sb(float()); break;
        case VH_I16: by_sb(int16_t()); break;
        case VH_U16: by_sb(uint16_t()); break;
        case VH_I8: by_sb(int8_t()); break;
        case VH_U8: by_sb(uint8_t()); break;
        case VH_BOOL: by_sb(vbool()); break;
        default: fail(VH_ERR_RUNTIME, "internal: multi-batch set pass A takes keys of <= 4 bytes");
        }
    };
    if (P > 1) {
        std::vector<uint64_t> bh(P, 0);
        for (uint32_t i = 0; i < FINE; i++) bh[i >> (SI_FINE_LOG2 - p_log2)] += fh[i];
        // keys of <= 4 bytes take the multi-batch pass A (k_si_scatter4) with as many
        // batches per commit as the LDS holds (VH_SI_FAST=0: the one-batch kernel, A/B runs)
        static const bool fast_on = [] {
            const char *e = getenv("VH_SI_FAST");
            return !e || atoi(e) != 0;
        }();
        fast_sb = 0;
        // quad loads with a register prefetch hide the load latency at one workgroup per CU
        // (4 batches per commit: 3.9 ms vs 5.0 at one batch, C3 set); per-row loads need the
        // occupancy of one batch per commit (4 workgroups per CU)
        static const int sb_env = [] {
            const char *e = getenv("VH_SI_SB");
            return e ? std::min(4, std::max(1, atoi(e))) : 0;
        }();
        const int sb_max = sb_env ? sb_env : plain ? 4 : 1;
        if (fast_on && isz <= 4)
            for (fast_sb = sb_max; fast_sb > 1 && si_fast_lds_bytes(fast_sb, P) > 160 * 1024; fast_sb--) {
            }
        const size_t lds_a = fast_sb ? si_fast_lds_bytes(fast_sb, P) : si_scatter_lds_bytes(P);
        lds_scatter = lds_a;
        int bpc = 1;
        if (fast_sb)
            with_fast([&](auto kernel) { bpc = si_blocks_per_cu(reinterpret_cast<const void *>(kernel), SI_THREADS, lds_a); });
        else
            VH_DISPATCH_DTYPE(s->dtype, T,
                              bpc = si_blocks_per_cu(reinterpret_cast<const void *>(k_si_scatter<T>), SI_THREADS, lds_a));
        bpc = std::min(bpc, 4);
        W = std::min<uint32_t>(1024, (uint32_t)cu_count() * bpc);
        // pass-A workgroup w takes batches w, w + W, ...: at most ceil(batches / W) of them
        const uint64_t rows_per_wg = (nbatch + W - 1) / W * SI_BATCH;
        cap.resize(P);
        toff.resize(P);
        uint64_t stride = 0;
        for (uint32_t t = 0; t < P; t++) {
            const double e = (double)rows_per_wg * (double)bh[t] / (double)std::max<uint64_t>(sampled, 1);
            uint64_t cc = (uint64_t)(e * 1.04 + 6.0 * std::sqrt(e + 1.0)) + 32;
            cc = std::min<uint64_t>((cc + 7) & ~uint64_t(7), rows_per_wg + 8);
            cap[t] = (uint32_t)cc;
            toff[t] = stride;
            stride += cc;
        }
        if (stride + rows_per_wg >= (uint64_t)SI_DEST_OVER) fail(VH_ERR_RUNTIME, "ordered_set: region table too large");
        const uint64_t total = stride * W;
        S.ent.ensure(8 * total + 64);
        if (kbs == 8) S.ent_row.ensure(4 * total + 64);
        // pass-B units: a unit merges each of its keys into the HBM table once, so split a
        // bucket over ranges of workgroups only as far as the CUs need work
        const double target = std::max(1.0, (double)n / ((double)cu_count() * 2));
        for (uint32_t t = 0; t < P; t++) {
            const double e = (double)n * (double)bh[t] / (double)std::max<uint64_t>(sampled, 1);
            const uint32_t gq = (uint32_t)std::min<double>(W, std::max(1.0, std::ceil(e / target)));
            for (uint32_t k = 0; k < gq; k++)
                units.push_back({t, (uint32_t)((uint64_t)W * k / gq), (uint32_t)((uint64_t)W * (k + 1) / gq), 0});
        }
        const uint64_t meta_bytes = 8 * (uint64_t)P + sizeof(SiUnit) * units.size() + 4 * (uint64_t)P +
                                    4 * (uint64_t)P * W + 256;
        S.meta.ensure(meta_bytes);
        unsigned char *mb = S.meta.as<unsigned char>();
        uint64_t *d_toff = reinterpret_cast<uint64_t *>(mb);
        SiUnit *d_units = reinterpret_cast<SiUnit *>(d_toff + P);
        uint32_t *d_cap = reinterpret_cast<uint32_t *>(d_units + units.size());
        uint32_t *d_fills = d_cap + P;
        VH_HIP(hipMemcpyAsync(d_toff, toff.data(), 8 * (uint64_t)P, hipMemcpyHostToDevice, st));
        VH_HIP(hipMemcpyAsync(d_units, units.data(), sizeof(SiUnit) * units.size(), hipMemcpyHostToDevice, st));
        VH_HIP(hipMemcpyAsync(d_cap, cap.data(), 4 * (uint64_t)P, hipMemcpyHostToDevice, st));
        sp.W = W;
        sp.rows_per_wg = rows_per_wg;
        sp.wg_stride = stride;
        sp.cap = d_cap;
        sp.toff = d_toff;
        sp.fills = d_fills;
        sp.ent = S.ent.ptr;
        sp.ent_row = S.ent_row.as<uint32_t>();
    }
    for (int attempt = 0;; attempt++) {
        SiTable g{s->tab.as<uint64_t>(), s->cap - 1, s->cap / 4 * 3, s->ctr.as<uint64_t>(), nullptr};
        if (P == 1) {
            TimedScope ts("set_insert");
            int bpc = 1;
            VH_DISPATCH_DTYPE(s->dtype, T,
                              bpc = si_blocks_per_cu(reinterpret_cast<const void *>(k_si_direct<T>), SB_THREADS, lt_lds));
            const uint64_t Wd = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)cu_count() * bpc,
                                                                          (n + 4 * SB_THREADS - 1) / (4 * SB_THREADS)));
            sp.rows_per_wg = (n + Wd - 1) / Wd;
            VH_DISPATCH_DTYPE(s->dtype, T,
                              hipLaunchKernelGGL(k_si_direct<T>, dim3((unsigned)Wd), dim3(SB_THREADS), lt_lds, st, sp, g));
            VH_HIP(hipGetLastError());
        } else {
            {
                TimedScope ts("set_insert");
                if (fast_sb)
                    with_fast([&](auto kernel) {
                        hipLaunchKernelGGL(kernel, dim3(W), dim3(SI_THREADS), lds_scatter, st, sp, g);
                    });
                else
                    VH_DISPATCH_DTYPE(s->dtype, T,
                                      hipLaunchKernelGGL(k_si_scatter<T>, dim3(W), dim3(SI_THREADS), lds_scatter, st, sp,
                                                         g));
                VH_HIP(hipGetLastError());
            }
            {
                TimedScope ts("set_reduce");
                const SiUnit *d_units = reinterpret_cast<const SiUnit *>(S.meta.as<uint64_t>() + P);
                if (kbs == 8)
                    hipLaunchKernelGGL(k_si_reduce<uint64_t>, dim3((unsigned)units.size()), dim3(SB_THREADS), lt_lds, st,
                                       sp, g, d_units);
                else
                    hipLaunchKernelGGL(k_si_reduce<uint32_t>, dim3((unsigned)units.size()), dim3(SB_THREADS), lt_lds, st,
                                       sp, g, d_units);
                VH_HIP(hipGetLastError());
            }
        }
        VH_HIP(hipMemcpyAsync(c.data(), s->ctr.ptr, 8 * C_N, hipMemcpyDeviceToHost, st));
        VH_HIP(hipStreamSynchronize(st));
        if (!c[C_OVERFLOW]) {
            if (c[C_DISTINCT] * 2 > s->cap) set_grow(s, si_next_pow2(c[C_DISTINCT] * 2));
            break;
        }
        // the estimate missed: grow x4 and re-run the chunk (inserts are idempotent; the
        // special rows' counts of this chunk are taken back first)
        if (attempt > 16) fail(VH_ERR_RUNTIME, "hash set could not grow enough");
        set_grow(s, s->cap * 4);
        uint64_t reset[C_N];
        memcpy(reset, c.data(), sizeof(reset));
        reset[C_OVERFLOW] = 0;
        reset[C_NAN_COUNT] = s->nan_count_before;
        reset[C_NULL_COUNT] = s->null_count_before;
        VH_HIP(hipMemcpyAsync(s->ctr.ptr, reset, 8 * C_N, hipMemcpyHostToDevice, st));
        VH_HIP(hipStreamSynchronize(st));
    }
}

}  // namespace vh

static void set_update(vh_set *s, const void *keys, const uint8_t *mask, const uint8_t *select, uint64_t n, int loc) {
    loc = resolve_loc(keys, loc);
    const int isz = dtype_itemsize(s->dtype);
    // host keys are staged per 16 Mi rows; device keys are taken 2^30 rows at a time (the
    // pass-A regions of a chunk are ~8 B per row; each chunk merges every key once per unit)
    const uint64_t CH = loc == VH_LOC_HOST ? (uint64_t(1) << 24) : (uint64_t(1) << 30);
    SiScratch &S = si_scratch();
    std::lock_guard<std::mutex> lk(S.mu);
    for (uint64_t r0 = 0; r0 < n; r0 += CH) {
        const uint64_t len = std::min(CH, n - r0);
        const void *dk = reinterpret_cast<const char *>(keys) + r0 * isz;
        const uint8_t *dm = mask ? mask + r0 : nullptr;
        const uint8_t *ds = select ? select + r0 : nullptr;
        if (loc == VH_LOC_HOST) {
            s->stage_keys.ensure(len * isz);
            VH_HIP(hipMemcpyAsync(s->stage_keys.ptr, dk, len * isz, hipMemcpyHostToDevice, stream()));
            dk = s->stage_keys.ptr;
            if (mask) {
                s->stage_mask.ensure(len);
                VH_HIP(hipMemcpyAsync(s->stage_mask.ptr, dm, len, hipMemcpyHostToDevice, stream()));
                dm = s->stage_mask.as<uint8_t>();
            }
            if (select) {
                s->stage_select.ensure(len);
                VH_HIP(hipMemcpyAsync(s->stage_select.ptr, ds, len, hipMemcpyHostToDevice, stream()));
                ds = s->stage_select.as<uint8_t>();
            }
        }
        // the chunk's NaN / null counts, restored if the chunk must be re-run
        {
            std::vector<uint64_t> c(C_N);
            VH_HIP(hipMemcpyAsync(c.data(), s->ctr.ptr, 8 * C_N, hipMemcpyDeviceToHost, stream()));
            VH_HIP(hipStreamSynchronize(stream()));
            s->nan_count_before = c[C_NAN_COUNT];
            s->null_count_before = c[C_NULL_COUNT];
        }
        si_chunk(s, S, dk, dm, ds, len, s->rows_seen + r0);
    }
    s->rows_seen += n;
    {
        auto c = read_ctr(s);
        if (c[C_NAN_FIRST] != ~0ULL && s->nan_pos == ~0ULL) s->nan_pos = s->rows_seen;
        if (c[C_NULL_FIRST] != ~0ULL && s->null_pos == ~0ULL) s->null_pos = s->rows_seen;
    }
    s->sealed = false;
}

int vh_set_update(vh_set *s, const void *keys, const uint8_t *mask, uint64_t n, int loc) {
    VH_API_BEGIN
    std::lock_guard<std::recursive_mutex> lk(s->mu);
    set_update(s, keys, mask, nullptr, n, loc);
    VH_API_END
}

int vh_set_update_selected(vh_set *s, const void *keys, const uint8_t *mask, const uint8_t *select, uint64_t n,
                           int loc) {
    VH_API_BEGIN
    std::lock_guard<std::recursive_mutex> lk(s->mu);
    set_update(s, keys, mask, select, n, loc);
    VH_API_END
}

int vh_set_seal(vh_set *s) {
    VH_API_BEGIN
    std::lock_guard<std::recursive_mutex> lk(s->mu);
    set_seal(s);
    VH_API_END
}

int vh_set_info(vh_set *s, int64_t *length, int64_t *nan_count, int64_t *null_count, int64_t *nan_value,
                int64_t *null_value) {
    VH_API_BEGIN
    std::lock_guard<std::recursive_mutex> lk(s->mu);
    set_seal(s);
    if (length) *length = s->length;
    if (nan_count) *nan_count = s->nan_count;
    if (null_count) *null_count = s->null_count;
    if (nan_value) *nan_value = s->nan_ord >= 0 ? s->nan_ord : 0x7fffffff;
    if (null_value) *null_value = s->null_ord >= 0 ? s->null_ord : 0x7fffffff;
    VH_API_END
}

int vh_set_key_array(vh_set *s, void *out) {
    VH_API_BEGIN
    std::lock_guard<std::recursive_mutex> lk(s->mu);
    set_seal(s);
    VH_DISPATCH_DTYPE(s->dtype, T, write_keys<T>(s, reinterpret_cast<T *>(out)));
    VH_API_END
}

int vh_set_map_ordinal(vh_set *s, const void *keys, uint64_t n, int loc, void *out, int out_itemsize, int out_loc) {
    VH_API_BEGIN
    std::lock_guard<std::recursive_mutex> lk(s->mu);
    set_seal(s);
    if (out_itemsize != 1 && out_itemsize != 2 && out_itemsize != 4 && out_itemsize != 8)
        fail(VH_ERR_ARG, "out_itemsize must be 1, 2, 4 or 8");
    loc = resolve_loc(keys, loc);
    out_loc = resolve_loc(out, out_loc);
    const int isz = dtype_itemsize(s->dtype);
    DevBuf dkeys, dout;
    const void *dk = keys;
    void *dout_p = out;
    if (loc == VH_LOC_HOST && n) {
        dkeys.ensure(n * isz);
        VH_HIP(hipMemcpyAsync(dkeys.ptr, keys, n * isz, hipMemcpyHostToDevice, stream()));
        dk = dkeys.ptr;
    }
    if (out_loc == VH_LOC_HOST && n) {
        dout.ensure(n * out_itemsize);
        dout_p = dout.ptr;
    }
    SetDev sd = set_device_view(s);
    const int64_t nan_value = s->nan_ord >= 0 ? s->nan_ord : 0x7fffffff;
    if (n) {
        TimedScope ts("set_map_ordinal");
        dim3 grd(blocks_for(n, 256)), blk(256);
        VH_DISPATCH_DTYPE(s->dtype, T, {
            const T *kp = reinterpret_cast<const T *>(dk);
            switch (out_itemsize) {
            case 1: hipLaunchKernelGGL((k_set_map_ordinal<T, int8_t>), grd, blk, 0, stream(), kp, n, sd, nan_value, (int8_t *)dout_p); break;
            case 2: hipLaunchKernelGGL((k_set_map_ordinal<T, int16_t>), grd, blk, 0, stream(), kp, n, sd, nan_value, (int16_t *)dout_p); break;
            case 4: hipLaunchKernelGGL((k_set_map_ordinal<T, int32_t>), grd, blk, 0, stream(), kp, n, sd, nan_value, (int32_t *)dout_p); break;
            default: hipLaunchKernelGGL((k_set_map_ordinal<T, int64_t>), grd, blk, 0, stream(), kp, n, sd, nan_value, (int64_t *)dout_p);
            }
        });
        VH_HIP(hipGetLastError());
    }
    if (out_loc == VH_LOC_HOST && n)
        VH_HIP(hipMemcpyAsync(out, dout_p, n * out_itemsize, hipMemcpyDeviceToHost, stream()));
    VH_HIP(hipStreamSynchronize(stream()));
    VH_API_END
}

}  // extern "C"

namespace vh {
uint64_t stat_set_overflow(bool reset) {
    unsigned long long v = 0;
    VH_HIP(hipStreamSynchronize(stream()));
    VH_HIP(hipMemcpyFromSymbol(&v, HIP_SYMBOL(d_si_overflow_rows), sizeof(v)));
    if (reset) {
        const unsigned long long z = 0;
        VH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(d_si_overflow_rows), &z, sizeof(z)));
    }
    return v;
}
}  // namespace vh
