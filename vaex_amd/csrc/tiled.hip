// Tile-partitioned LDS aggregation for grids larger than one workgroup's LDS
// (the 1027x1027 grid of df.count(binby=[x, y], shape=1024), the 1e6-cell
// groupby grid).  Global atomics on a scattered 8 MB grid cost ~one 64-B
// atomic request per row (MI355X_MICROARCH.md §Global float atomics: "64 lanes
// in 64 different rows ~17x slower"); instead the rows are partitioned by grid
// tile and every tile is aggregated in LDS:
//
//   sample  -- per-tile row fractions p_t from ~1M evenly spaced rows (LDS
//              histogram per workgroup); they size the partition regions.
//   pass A  -- workgroup w owns a contiguous row range and, per tile t, a
//              private region of cap_t entries.  Per batch of 2048 rows it reads
//              the binby/value columns coalesced, computes the cell in
//              registers, ranks the rows per tile in an LDS histogram, counting-
//              sorts (entry, value) by tile into LDS and streams the sorted runs
//              to its regions (consecutive lanes -> consecutive addresses).  No
//              global atomics; a row beyond its region's capacity (an unlikely
//              sampling miss) is applied directly with global atomics.
//   pass B  -- work units (tile, range of pass-A workgroups) sized from p_t:
//              stream the regions' entries, aggregate into an LDS copy of the
//              tile (u32 counts, f64 sums), flush with coalesced global atomics.
//
// Entry formats: u16 local cell (counts unconditional or keyed on a carried
// value's NaN-ness) or u32 local cell | keep flags << 16.  Results equal
// AggCount/AggSum (superagg.cpp:168-191,362-388): counts exact, float sums in a
// different association order (within 1e-6 relative, north_star).
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cmath>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>

#include "binner_dev.hpp"
#include "common.hpp"
#include "engine.hpp"

namespace vh {

#ifndef VH_TA_THREADS
#define VH_TA_THREADS 512
#endif
#ifndef VH_TA_WAVES
#define VH_TA_WAVES 0  // amdgpu_waves_per_eu floor for pass A (0 = compiler's choice)
#endif
constexpr int TA_THREADS = VH_TA_THREADS;
#ifndef VH_TA_RPT
#define VH_TA_RPT 8
#endif
#ifndef VH_TA_NT
#define VH_TA_NT 0
#endif
#ifndef VH_TA_DRAIN
#define VH_TA_DRAIN 1  // fast pass A: the prefetched batch lands before the commit's stores
#endif
#ifndef VH_TB_THREADS
#define VH_TB_THREADS 1024
#endif
constexpr int TA_RPT = VH_TA_RPT;
constexpr int TA_BATCH = TA_THREADS * TA_RPT;
constexpr int TB_THREADS = VH_TB_THREADS;
#ifndef VH_TILE_LDS_KB
#define VH_TILE_LDS_KB 96
#endif
constexpr uint64_t TILE_LDS_BUDGET = VH_TILE_LDS_KB * 1024;
constexpr uint32_t TILE_MAX_TILES = 4096;
constexpr size_t LDS_MAX_BYTES = 160 * 1024;  // per workgroup on gfx950
constexpr int TA_WG_PER_CU = 4;
constexpr int SAMPLE_BLOCKS = 512;

enum : int32_t { CNT_ALWAYS = -2, CNT_FLAG = -1 };

struct TileParams {
    uint32_t s_log2, ntiles, flags_mode, nvals;
    uint64_t cells;
    uint32_t W;                // pass-A workgroups
    uint32_t pad;
    uint64_t rows_per_wg;
    uint64_t wg_stride;        // entries of one workgroup's regions
    const uint32_t *cap;       // [T]
    const uint64_t *toff;      // [T] region offset inside a workgroup's block
    uint32_t *fills;           // [T][W] entries produced (may exceed cap)
    void *entries;             // u16 / u32, W * wg_stride
    double *values[2];         // per value slot, W * wg_stride
    int32_t val_slot[MAX_FUSED_AGGS];  // sum agg k -> value slot
    int32_t cnt_slot[MAX_FUSED_AGGS];  // count agg k -> CNT_ALWAYS / CNT_FLAG / value slot
    const double *vdata[2];    // value slot -> source column (fast kernel)
    uint32_t debug;            // experiment switches (VH_TILE_DEBUG), 0 in production
    const uint32_t *tile_of;   // [T] region id -> grid tile (XCD-resident path), nullptr = identity
    const uint32_t *abort_word;  // XCD-resident path's state word: pass B skips an aborted launch
    // 4-byte value slots (every summed column <= 4 bytes: int8/16/32, uint8/16/32, bool,
    // float32 -- exact): slot s is float32 bits when bit s of vfloat is set, else the low 32
    // bits of the int64 slot, sign-extended back when bit s of vsigned is set
    uint32_t vnarrow, vfloat, vsigned, pad2;
    int32_t vdt[2];            // value slot -> column dtype (fast ordinal kernel)
};

// value of row h (0/1) of a loaded pair of a column of dtype dt, as the 8-byte slot pass A
// carries (float data as double, integer / bool data as int64 / uint64 bits); `pr` holds
// the pair's raw bits: both doubles for float64, else packed in pr.x from the low byte up
__host__ __device__ inline int dtype_itemsize_dev(int dt) {
    switch (dt) {
    case VH_F64: case VH_I64: case VH_U64: return 8;
    case VH_F32: case VH_I32: case VH_U32: return 4;
    case VH_I16: case VH_U16: return 2;
    default: return 1;
    }
}

__device__ __forceinline__ double pair_slot(const double2 &pr, int dt, int h) {
    if (dt == VH_F64 || dt == VH_I64 || dt == VH_U64) return h ? pr.y : pr.x;
    const uint64_t raw = __builtin_bit_cast(uint64_t, pr.x);
    switch (dt) {
    case VH_F32: return (double)__builtin_bit_cast(float, (uint32_t)(raw >> (32 * h)));
    case VH_I32: return __builtin_bit_cast(double, (int64_t)(int32_t)(uint32_t)(raw >> (32 * h)));
    case VH_U32: return __builtin_bit_cast(double, (uint64_t)(uint32_t)(raw >> (32 * h)));
    case VH_I16: return __builtin_bit_cast(double, (int64_t)(int16_t)(uint16_t)(raw >> (16 * h)));
    case VH_U16: return __builtin_bit_cast(double, (uint64_t)(uint16_t)(raw >> (16 * h)));
    case VH_I8: return __builtin_bit_cast(double, (int64_t)(int8_t)(uint8_t)(raw >> (8 * h)));
    case VH_BOOL: return __builtin_bit_cast(double, (uint64_t)(((raw >> (8 * h)) & 0xff) ? 1 : 0));
    default: return __builtin_bit_cast(double, (uint64_t)(uint8_t)(raw >> (8 * h)));  // VH_U8
    }
}

// a carried 8-byte slot value (double, or int64 / uint64 bits) as its 4-byte form and back
__device__ __forceinline__ uint32_t slot_narrow(double v, bool is_float) {
    return is_float ? __builtin_bit_cast(uint32_t, (float)v) : (uint32_t)__builtin_bit_cast(uint64_t, v);
}
__device__ __forceinline__ double slot_wide(uint32_t u, bool is_float, bool is_signed) {
    if (is_float) return (double)__builtin_bit_cast(float, u);
    return __builtin_bit_cast(double, is_signed ? (uint64_t)(int64_t)(int32_t)u : (uint64_t)u);
}

// ---- min / max in the tile path (AggMin / AggMax, superagg.cpp:195-285) ----------------
// Pass A carries the value slot like a sum's; pass B keeps an order-preserving 64-bit form
// per LDS cell (float: sign-flipped bits, ds_min/max_u64; signed: int64, ds_min/max_i64;
// unsigned: uint64), cells start at the kind's identity, and touched cells are flushed into
// the typed grid with the CAS min / max of the generic path (std::min/max semantics; NaN
// never enters, as the reference's comparisons skip it).
__host__ __device__ inline bool is_minmax(int kind) { return kind == VH_AGG_MIN || kind == VH_AGG_MAX; }
__device__ inline bool dt_float(int dt) { return dt == VH_F64 || dt == VH_F32; }
__device__ inline bool dt_signed(int dt) { return dt == VH_I64 || dt == VH_I32 || dt == VH_I16 || dt == VH_I8; }
__device__ inline uint64_t ord_bits(double d) {
    const uint64_t u = __builtin_bit_cast(uint64_t, d);
    return (u >> 63) ? ~u : (u | (1ull << 63));
}
__device__ inline double unord_bits(uint64_t o) {
    return __builtin_bit_cast(double, (o >> 63) ? (o & ~(1ull << 63)) : ~o);
}
__device__ inline uint64_t mm_identity(int dt, bool mx) {
    if (dt_signed(dt)) return mx ? (uint64_t)INT64_MIN : (uint64_t)INT64_MAX;
    return mx ? 0ull : ~0ull;  // float (ordered bits) and unsigned
}
// one carried slot value into an LDS cell
__device__ inline void mm_lds(uint64_t *cell, int dt, bool mx, double v) {
    if (dt_float(dt)) {
        if (v != v) return;
        const uint64_t o = ord_bits(v);
        if (mx) atomicMax((unsigned long long *)cell, (unsigned long long)o);
        else atomicMin((unsigned long long *)cell, (unsigned long long)o);
    } else if (dt_signed(dt)) {
        const long long x = (long long)__builtin_bit_cast(int64_t, v);
        if (mx) atomicMax((long long *)cell, x);
        else atomicMin((long long *)cell, x);
    } else {
        const unsigned long long x = __builtin_bit_cast(unsigned long long, v);
        if (mx) atomicMax((unsigned long long *)cell, x);
        else atomicMin((unsigned long long *)cell, x);
    }
}
// a value (LDS cell form when `cellform`, else a carried slot) into the typed grid
__device__ inline void mm_grid(void *grid, uint64_t c, int dt, bool mx, uint64_t x, bool cellform) {
    double d = 0.0;
    if (dt_float(dt)) {
        d = cellform ? unord_bits(x) : __builtin_bit_cast(double, x);
        if (d != d) return;
    }
    switch (dt) {
    case VH_F64: atomic_minmax<double>(static_cast<double *>(grid) + c, d, mx); break;
    case VH_F32: atomic_minmax<float>(static_cast<float *>(grid) + c, (float)d, mx); break;
    case VH_I64: atomic_minmax<int64_t>(static_cast<int64_t *>(grid) + c, (int64_t)x, mx); break;
    case VH_I32: atomic_minmax<int32_t>(static_cast<int32_t *>(grid) + c, (int32_t)(int64_t)x, mx); break;
    case VH_I16: atomic_minmax<int16_t>(static_cast<int16_t *>(grid) + c, (int16_t)(int64_t)x, mx); break;
    case VH_I8: atomic_minmax<int8_t>(static_cast<int8_t *>(grid) + c, (int8_t)(int64_t)x, mx); break;
    case VH_U64: atomic_minmax<uint64_t>(static_cast<uint64_t *>(grid) + c, x, mx); break;
    case VH_U32: atomic_minmax<uint32_t>(static_cast<uint32_t *>(grid) + c, (uint32_t)x, mx); break;
    case VH_U16: atomic_minmax<uint16_t>(static_cast<uint16_t *>(grid) + c, (uint16_t)x, mx); break;
    default: atomic_minmax<uint8_t>(static_cast<uint8_t *>(grid) + c, (uint8_t)x, mx); break;  // VH_U8
    }
}

struct WorkUnit {
    uint32_t tile, w_begin, w_end, pad;
};

template <int ND> __device__ inline uint64_t cell_of(const BinPlan &p, uint64_t i) {
    if constexpr (ND == 0) {
        return plan_index(p, i);
    } else {
        uint64_t c = 0;
#pragma unroll
        for (int d = 0; d < ND; d++) c += scalar_index<double>(p.b[d], i) * p.b[d].stride;
        return c;
    }
}

// a value as the 64-bit slot pass A carries: float data as float64 (NaN kept), integer
// and bool data as int64 / uint64 bits (the AggSum upcast, superagg.cpp:289-346)
__device__ inline double load_slot_value(const void *p, int dtype, uint64_t i, bool *nan) {
    *nan = false;
    switch (dtype) {
    case VH_F64: {
        const double d = static_cast<const double *>(p)[i];
        *nan = d != d;
        return d;
    }
    case VH_F32: {
        const double d = (double)static_cast<const float *>(p)[i];
        *nan = d != d;
        return d;
    }
    case VH_I64: return __builtin_bit_cast(double, static_cast<const int64_t *>(p)[i]);
    case VH_I32: return __builtin_bit_cast(double, (int64_t) static_cast<const int32_t *>(p)[i]);
    case VH_I16: return __builtin_bit_cast(double, (int64_t) static_cast<const int16_t *>(p)[i]);
    case VH_I8: return __builtin_bit_cast(double, (int64_t) static_cast<const int8_t *>(p)[i]);
    case VH_U64: return __builtin_bit_cast(double, static_cast<const uint64_t *>(p)[i]);
    case VH_U32: return __builtin_bit_cast(double, (uint64_t) static_cast<const uint32_t *>(p)[i]);
    case VH_U16: return __builtin_bit_cast(double, (uint64_t) static_cast<const uint16_t *>(p)[i]);
    default: {
        const uint8_t b = static_cast<const uint8_t *>(p)[i];
        return __builtin_bit_cast(double, (uint64_t)(dtype == VH_BOOL ? (b ? 1 : 0) : b));
    }
    }
}

// keep flags of a row (bit k: aggregator k takes the row) and the carried values
template <int NV>
__device__ inline uint32_t row_contrib(const FusedAggs &fa, const TileParams &tp, uint64_t i, double *vals) {
    uint32_t f = 0;
    #pragma unroll
    for (int k = 0; k < MAX_FUSED_AGGS; k++) {
        if (k >= fa.na) break;
        const FusedAgg &a = fa.a[k];
        bool keep = !a.mask || a.mask[i] == 1;
        double v = 0.0;
        if (a.data) {
            bool nan;
            v = load_slot_value(a.data, a.dtype, i, &nan);
            keep = keep && !nan;
        }
        if (keep) f |= 1u << k;
        if constexpr (NV > 0) {
            const int s = tp.val_slot[k];
            // a dropped row carries NaN (float sums skip it) or 0 (integer sums add nothing;
            // masks with integer data are not taken by the tile path)
            if (s >= 0 && s < NV) vals[s] = keep ? v : (a.vint ? 0.0 : __builtin_nan(""));
        }
    }
    return f;
}

// ---- sample: per-tile histogram of SAMPLE_BLOCKS evenly spaced row blocks ----
template <int ND>
__global__ __launch_bounds__(TA_THREADS) void k_tile_sample(BinPlan p, uint64_t n, uint32_t s_log2, uint32_t ntiles,
                                                            uint64_t block_stride, uint64_t *hist) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    uint32_t *h = reinterpret_cast<uint32_t *>(lds_raw);
    for (uint32_t t = threadIdx.x; t < ntiles; t += TA_THREADS) h[t] = 0;
    __syncthreads();
    const uint64_t row0 = blockIdx.x * block_stride;
    for (uint64_t r = threadIdx.x; r < TA_BATCH; r += TA_THREADS) {
        const uint64_t i = row0 + r;
        if (i >= n) break;
        atomicAdd(&h[cell_of<ND>(p, i) >> s_log2], 1u);
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < ntiles; t += TA_THREADS)
        if (h[t]) atomicAdd((unsigned long long *)&hist[t], (unsigned long long)h[t]);
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a workgroup fence +
// s_barrier, which waits vmcnt(0): it would drain the prefetched loads of the next batch
// and every outstanding region store at each of the batch's barriers
// (cdna_hip_programming.md "Pipelining across barriers").  Only LDS traffic is ordered here.
#if VH_TA_WAVES > 0
#define TA_ATTR __attribute__((amdgpu_waves_per_eu(VH_TA_WAVES)))
#else
#define TA_ATTR
#endif

__device__ inline void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// exclusive scan of in[0..T) into out[0..T), returns the total (all threads)
__device__ inline uint32_t block_exclusive_scan(const uint32_t *in, uint32_t *out, uint32_t T, uint32_t *wave_sums) {
    const uint32_t per = (T + TA_THREADS - 1) / TA_THREADS;
    const uint32_t t0 = threadIdx.x * per;
    uint32_t s = 0;
    for (uint32_t t = t0; t < t0 + per && t < T; t++) s += in[t];
    // inclusive scan of s across the workgroup (wave64 shuffles + 4 wave partials)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc = s;
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(inc, off, 64);
        if (lane >= off) inc += y;
    }
    if (lane == 63) wave_sums[wave] = inc;
    lds_barrier();
    uint32_t wave_base = 0, total = 0;
    for (int k = 0; k < TA_THREADS / 64; k++) {
        if (k < wave) wave_base += wave_sums[k];
        total += wave_sums[k];
    }
    uint32_t acc = wave_base + inc - s;
    for (uint32_t t = t0; t < t0 + per && t < T; t++) {
        out[t] = acc;
        acc += in[t];
    }
    return total;
}

// LDS layout of pass A: staged values | staged (destination, entry) pairs | per-tile
// hist | batch offsets | region write base | region limit | wave sums
struct ScatterLds {
    double *sv;
    uint64_t *sp;
    uint32_t *hist, *boff, *base, *lim, *dbase, *wave_sums;
};

// LDS bytes of pass A (must match scatter_lds)
__host__ __device__ inline size_t scatter_lds_bytes(int nv, uint32_t T) {
    return (size_t)8 * nv * TA_BATCH + (size_t)8 * TA_BATCH + 20 * (size_t)T + 64;
}

template <int NV> __device__ inline ScatterLds scatter_lds(unsigned char *raw, uint32_t T) {
    ScatterLds l;
    l.sv = reinterpret_cast<double *>(raw);
    l.sp = reinterpret_cast<uint64_t *>(raw + (size_t)8 * NV * TA_BATCH);
    l.hist = reinterpret_cast<uint32_t *>(l.sp + TA_BATCH);
    l.boff = l.hist + T;
    l.base = l.boff + T;
    l.lim = l.base + T;
    l.dbase = l.lim + T;
    l.wave_sums = l.dbase + T;
    return l;
}

// rows per thread of one commit of the fast f64 pass A: with sums, SB batches are ranked
// into one commit, so each (workgroup, tile) run is SB times longer (fewer, longer region
// stores; the kernel already runs one workgroup per CU on registers)
#ifndef VH_TA_SB
#define VH_TA_SB 3
#endif
#ifndef VH_TA_SB0
#define VH_TA_SB0 2  // count-only commits (same-process A/B: 1 -> 2 is 3.99 -> 3.87 ms, 3 is 4.08)
#endif
__host__ __device__ constexpr int fast_sb(int nv) { return nv == 0 ? VH_TA_SB0 : nv == 1 ? VH_TA_SB : (VH_TA_SB < 2 ? VH_TA_SB : 2); }

// LDS of the fast kernels: staged values | staged 4-byte keys | tile arrays
__host__ __device__ inline size_t fast_lds_bytes(int nv, uint32_t T, uint32_t cap) {
    return (size_t)8 * nv * cap + (size_t)4 * cap + 20 * (size_t)T + 64;
}

template <int NV> __device__ inline ScatterLds fast_lds(unsigned char *raw, uint32_t T, uint32_t cap) {
    ScatterLds l;
    l.sv = reinterpret_cast<double *>(raw);
    l.sp = reinterpret_cast<uint64_t *>(raw + (size_t)8 * NV * cap);
    l.hist = reinterpret_cast<uint32_t *>(raw + (size_t)8 * NV * cap + (size_t)4 * cap);
    l.boff = l.hist + T;
    l.base = l.boff + T;
    l.lim = l.base + T;
    l.dbase = l.lim + T;
    l.wave_sums = l.dbase + T;
    return l;
}

// per-workgroup init: zero the histogram; a tile's region of this workgroup is
// [toff, toff + cap) inside the workgroup's block, written from base upwards
__device__ inline void scatter_lds_init(const ScatterLds &l, const TileParams &tp, uint32_t T) {
    for (uint32_t t = threadIdx.x; t < T; t += TA_THREADS) {
        l.hist[t] = 0;
        l.base[t] = (uint32_t)tp.toff[t];
        l.lim[t] = (uint32_t)tp.toff[t] + tp.cap[t];
    }
}

constexpr uint32_t DEST_OVERFLOW = 0x80000000u;  // | tile: region full, global atomics

// phases 2-5 of a batch, after every row has its tile, entry, rank (-1 = drop) and
// carried values: exclusive scan of the tile histogram; every row computes its final
// destination (region base + rank, or overflow) and is counting-sorted into LDS as one
// (destination, entry) pair + its values; the sorted pairs are streamed out as runs;
// the region bases advance.
template <int NV>
__device__ inline void batch_commit(const ScatterLds &l, const FusedAggs &fa, const TileParams &tp, uint32_t T,
                                    uint64_t region0, const uint32_t *tile, const uint32_t *ent, const int32_t *rank,
                                    const double (*vals)[NV > 0 ? NV : 1], uint32_t *s_total) {
    lds_barrier();
    const uint32_t total = block_exclusive_scan(l.hist, l.boff, T, l.wave_sums);
    if (threadIdx.x == 0) *s_total = total;
    lds_barrier();
#pragma unroll
    for (int r = 0; r < TA_RPT; r++) {
        if (rank[r] < 0) continue;
        const uint32_t t = tile[r];
        const uint32_t pos = l.boff[t] + (uint32_t)rank[r];
        const uint32_t d = l.base[t] + (uint32_t)rank[r];
        const uint32_t dest = d < l.lim[t] ? d : (DEST_OVERFLOW | t);
        l.sp[pos] = ((uint64_t)dest << 32) | ent[r];
#pragma unroll
        for (int s = 0; s < NV; s++) l.sv[s * TA_BATCH + pos] = vals[r][s];
    }
    lds_barrier();
    const uint32_t tot = *s_total;
    for (uint32_t k = threadIdx.x; k < tot; k += TA_THREADS) {
        const uint64_t pk = l.sp[k];
        const uint32_t dest = (uint32_t)(pk >> 32), e32 = (uint32_t)pk;
        if (tp.debug & 1) {
            asm volatile("" :: "v"(e32), "v"(dest));
        } else if (!(dest & DEST_OVERFLOW)) {
            const uint64_t e = region0 + dest;
            if (tp.flags_mode) reinterpret_cast<uint32_t *>(tp.entries)[e] = e32;
            else reinterpret_cast<uint16_t *>(tp.entries)[e] = (uint16_t)(e32 & 0xffffu);
#pragma unroll
            for (int s = 0; s < NV; s++) {
                if (tp.vnarrow)
                    reinterpret_cast<uint32_t *>(tp.values[s])[e] = slot_narrow(l.sv[s * TA_BATCH + k], (tp.vfloat >> s) & 1);
                else
                    tp.values[s][e] = l.sv[s * TA_BATCH + k];
            }
        } else {
            // region overflow (a sampling miss): apply the staged row with global atomics
            const uint32_t t = dest & ~DEST_OVERFLOW;
            const uint64_t c = ((uint64_t)t << tp.s_log2) | (e32 & 0xffffu);
            const uint32_t f = e32 >> 16;
            #pragma unroll
            for (int a = 0; a < MAX_FUSED_AGGS; a++) {
                if (a >= fa.na) break;
                if (!((f >> a) & 1)) continue;
                if (fa.a[a].kind == VH_AGG_COUNT) {
                    atomicAdd((unsigned long long *)fa.a[a].grid + c, 1ULL);
                } else if (is_minmax(fa.a[a].kind)) {
                    if constexpr (NV > 0)
                        mm_grid(fa.a[a].grid, c, fa.a[a].dtype, fa.a[a].kind == VH_AGG_MAX,
                                __builtin_bit_cast(uint64_t, l.sv[tp.val_slot[a] * TA_BATCH + k]), false);
                } else if constexpr (NV > 0) {
                    const double v = l.sv[tp.val_slot[a] * TA_BATCH + k];
                    if (fa.a[a].vint)
                        atomicAdd(reinterpret_cast<unsigned long long *>(fa.a[a].grid) + c,
                                  __builtin_bit_cast(unsigned long long, v));
                    else
                        atomicAdd(reinterpret_cast<double *>(fa.a[a].grid) + c, v);
                }
            }
        }
    }
    lds_barrier();
    for (uint32_t t = threadIdx.x; t < T; t += TA_THREADS) {
        l.base[t] += l.hist[t];
        l.hist[t] = 0;
    }
}

// Batch commit of the fast kernels, three LDS barriers per batch:
//   B1 (every rank taken) -> wave 0 scans the tile histogram: boff = exclusive offsets,
//   dbase = region write base - boff (a row sorted to position k of tile t goes to
//   dbase[t] + k), then advances base and clears hist -> B2 -> rows stage their sorted
//   (tile << 16 | cell) key and values -> B3 -> sorted runs streamed to the regions.
// The next batch's ranking may start while slower waves still stream: it only touches
// hist, which the scan already cleared; boff/dbase/sp/sv are rewritten only after the next
// B1, which every wave reaches after its stream-out.
__device__ inline void fast_scan(const ScatterLds &l, uint32_t T) {
    if (threadIdx.x >= 64) return;
    const uint32_t lane = threadIdx.x;
    const uint32_t per = (T + 63) / 64;
    const uint32_t t0 = lane * per;
    uint32_t s = 0;
    for (uint32_t t = t0; t < t0 + per && t < T; t++) s += l.hist[t];
    uint32_t inc = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off, 64);
        if ((int)lane >= off) inc += y;
    }
    uint32_t acc = inc - s;
    for (uint32_t t = t0; t < t0 + per && t < T; t++) {
        const uint32_t h = l.hist[t], b = l.base[t];
        l.boff[t] = acc;
        l.dbase[t] = b - acc;
        l.base[t] = b + h;
        l.hist[t] = 0;
        acc += h;
    }
    if (lane == 63) l.wave_sums[0] = inc;
}

template <int NV, int R>
__device__ inline void batch_commit_fast(const ScatterLds &l, const FusedAggs &fa, const TileParams &tp, uint32_t T,
                                         uint64_t region0, const uint32_t *key, const int32_t *rank,
                                         const double (*vals)[NV > 0 ? NV : 1], uint32_t count_mask,
                                         const uint32_t *keyed_slot_of) {
    constexpr uint32_t CAP = R * TA_THREADS;
    uint32_t *sk = reinterpret_cast<uint32_t *>(l.sp);
    lds_barrier();
    fast_scan(l, T);
    lds_barrier();
    const uint32_t tot = l.wave_sums[0];
#pragma unroll
    for (int r = 0; r < R; r++) {
        if (rank[r] < 0) continue;
        const uint32_t pos = l.boff[key[r] >> 16] + (uint32_t)rank[r];
        sk[pos] = key[r];
#pragma unroll
        for (int s = 0; s < NV; s++) l.sv[s * CAP + pos] = vals[r][s];
    }
    lds_barrier();
    for (uint32_t k = threadIdx.x; k < tot; k += TA_THREADS) {
        const uint32_t kk = sk[k];
        const uint32_t t = kk >> 16;
        const uint32_t dest = l.dbase[t] + k;
        if (tp.debug & 128) {  // experiment: no region stores
            asm volatile("" ::"v"(kk), "v"(dest));
        } else if (dest < l.lim[t]) {
            const uint64_t e = region0 + dest;
            reinterpret_cast<uint16_t *>(tp.entries)[e] = (uint16_t)kk;
#pragma unroll
            for (int s = 0; s < NV; s++) {
                if (tp.vnarrow)
                    reinterpret_cast<uint32_t *>(tp.values[s])[e] = slot_narrow(l.sv[s * CAP + k], (tp.vfloat >> s) & 1);
                else
                    tp.values[s][e] = l.sv[s * CAP + k];
            }
        } else {
            // region overflow (a sampling miss): apply the staged row with global atomics
            const uint64_t c = ((uint64_t)t << tp.s_log2) | (kk & 0xffffu);
            #pragma unroll
            for (int a = 0; a < MAX_FUSED_AGGS; a++) {
                if (a >= fa.na) break;
                bool take = (count_mask >> a) & 1;
                if constexpr (NV > 0) {
                    if (!take) {
                        const double v = l.sv[keyed_slot_of[a] * CAP + k];
                        take = v == v;
                    }
                }
                if (!take) continue;
                if (fa.a[a].kind == VH_AGG_COUNT) {
                    atomicAdd((unsigned long long *)fa.a[a].grid + c, 1ULL);
                } else if (is_minmax(fa.a[a].kind)) {
                    if constexpr (NV > 0)
                        mm_grid(fa.a[a].grid, c, fa.a[a].dtype, fa.a[a].kind == VH_AGG_MAX,
                                __builtin_bit_cast(uint64_t, l.sv[tp.val_slot[a] * CAP + k]), false);
                } else if constexpr (NV > 0) {
                    const double v = l.sv[tp.val_slot[a] * CAP + k];
                    if (fa.a[a].vint)
                        atomicAdd(reinterpret_cast<unsigned long long *>(fa.a[a].grid) + c, __builtin_bit_cast(unsigned long long, v));
                    else
                        atomicAdd(reinterpret_cast<double *>(fa.a[a].grid) + c, v);
                }
            }
        }
    }
}

// The generic pass A's per-row work with the dtype dispatch hoisted out of the row loop:
// one switch per binner (or aggregator) per batch, then TA_RPT rows of plain typed loads
// and index math (per-row dispatch cost ~75 scalar + branch instructions per wave
// iteration, see DESIGN.md, small grids).
template <typename T> __device__ __forceinline__ void ta_dim(const BinnerDev &b, uint64_t b0, uint64_t row_end,
                                                             uint64_t (&cell)[TA_RPT]) {
    T raw[TA_RPT];
    bool m[TA_RPT];
#pragma unroll
    for (int r = 0; r < TA_RPT; r++) {
        const uint64_t i = b0 + (uint64_t)r * TA_THREADS + threadIdx.x;
        const bool in = i < row_end;
        raw[r] = in ? reinterpret_cast<const T *>(b.data)[i] : T{};
        m[r] = (in && b.mask) ? b.mask[i] == 1 : false;
    }
    if (b.kind == 0) {
#pragma unroll
        for (int r = 0; r < TA_RPT; r++) cell[r] += scalar_cell<T>(b, raw[r], m[r]) * b.stride;
    } else {
#pragma unroll
        for (int r = 0; r < TA_RPT; r++) cell[r] += ordinal_cell<T>(b, raw[r], m[r]) * b.stride;
    }
}

// load_slot_value on a loaded raw value
template <typename T> __device__ __forceinline__ double slot_of(T raw, bool *nan) {
    *nan = false;
    if constexpr (std::is_same_v<T, double> || std::is_same_v<T, float>) {
        const double d = (double)raw;
        *nan = d != d;
        return d;
    } else if constexpr (std::is_same_v<T, vbool>) {
        return __builtin_bit_cast(double, (uint64_t)(raw.v ? 1 : 0));
    } else if constexpr (is_signed_int_t<T>::value) {
        return __builtin_bit_cast(double, (int64_t)raw);
    } else {
        return __builtin_bit_cast(double, (uint64_t)raw);
    }
}

template <typename T, int NV>
__device__ __forceinline__ void ta_agg(const FusedAgg &a, int k, int slot, uint64_t b0, uint64_t row_end,
                                       uint32_t (&f)[TA_RPT], double (&vals)[TA_RPT][NV > 0 ? NV : 1]) {
    T raw[TA_RPT];
    bool m[TA_RPT];
#pragma unroll
    for (int r = 0; r < TA_RPT; r++) {
        const uint64_t i = b0 + (uint64_t)r * TA_THREADS + threadIdx.x;
        const bool in = i < row_end;
        raw[r] = (in && a.data) ? reinterpret_cast<const T *>(a.data)[i] : T{};
        m[r] = (in && a.mask) ? a.mask[i] == 1 : true;
    }
#pragma unroll
    for (int r = 0; r < TA_RPT; r++) {
        bool keep = m[r];
        double v = 0.0;
        if (a.data) {
            bool nan;
            v = slot_of<T>(raw[r], &nan);
            keep = keep && !nan;
        }
        if (keep) f[r] |= 1u << k;
        if constexpr (NV > 0) {
            const double carried = keep ? v : (a.vint ? 0.0 : __builtin_nan(""));
#pragma unroll
            for (int s = 0; s < NV; s++)  // compile-time slot index: the array stays in registers
                if (s == slot) vals[r][s] = carried;
        }
    }
}

// generic pass A: any binner kinds/dtypes, masks and keep flags
template <int ND, int NV>
__global__ __launch_bounds__(TA_THREADS) TA_ATTR void k_tile_scatter(BinPlan p, FusedAggs fa, TileParams tp, uint64_t n) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const uint32_t T = tp.ntiles;
    const ScatterLds l = scatter_lds<NV>(lds_raw, T);
    __shared__ uint32_t s_total;
    scatter_lds_init(l, tp, T);
    __syncthreads();
    const uint32_t w = blockIdx.x;
    const uint64_t row_begin = (uint64_t)w * tp.rows_per_wg;
    const uint64_t row_end = min(n, row_begin + tp.rows_per_wg);
    const uint32_t smask = (1u << tp.s_log2) - 1;
    const uint64_t region0 = (uint64_t)w * tp.wg_stride;
    for (uint64_t b0 = row_begin; b0 < row_end; b0 += TA_BATCH) {
        uint32_t tile[TA_RPT], ent[TA_RPT];
        int32_t rank[TA_RPT];
        double vals[TA_RPT][NV > 0 ? NV : 1];
        if constexpr (ND == -1) {
            // plans with a set-ordinal binner: per-row hash probe, per-row dispatch (the
            // hoisted form's register footprint made this case slower: 21.6 -> 27.1 ms C3)
#pragma unroll
            for (int r = 0; r < TA_RPT; r++) {
                const uint64_t i = b0 + (uint64_t)r * TA_THREADS + threadIdx.x;
                rank[r] = -1;
                if (i < row_end) {
                    const uint64_t c = plan_index(p, i);
                    const uint32_t f = row_contrib<NV>(fa, tp, i, vals[r]);
                    tile[r] = (uint32_t)(c >> tp.s_log2);
                    ent[r] = ((uint32_t)c & smask) | (f << 16);
                    if (f) rank[r] = (int32_t)atomicAdd(&l.hist[tile[r]], 1u);
                }
            }
        } else {
            uint64_t cell[TA_RPT];
            uint32_t fl[TA_RPT];
    #pragma unroll
            for (int r = 0; r < TA_RPT; r++) {
                cell[r] = 0;
                fl[r] = 0;
            }
            if constexpr (ND == 0) {
                for (int d = 0; d < p.nb; d++) {
                    const BinnerDev &b = p.b[d];
                    if (b.kind == 2) {  // set-ordinal binner: a hash probe per row
    #pragma unroll
                        for (int r = 0; r < TA_RPT; r++) {
                            const uint64_t i = b0 + (uint64_t)r * TA_THREADS + threadIdx.x;
                            if (i < row_end) cell[r] += binner_index(b, i) * b.stride;
                        }
                        continue;
                    }
                    VH_DEV_DISPATCH(b.dtype, T, ta_dim<T>(b, b0, row_end, cell); break)
                }
            } else {
    #pragma unroll
                for (int r = 0; r < TA_RPT; r++) {
                    const uint64_t i = b0 + (uint64_t)r * TA_THREADS + threadIdx.x;
                    if (i < row_end) cell[r] = cell_of<ND>(p, i);
                }
            }
    #pragma unroll
            for (int k = 0; k < MAX_FUSED_AGGS; k++) {
                if (k >= fa.na) break;
                const FusedAgg &a = fa.a[k];
                const int slot = tp.val_slot[k];
                if (!a.data) {
                    ta_agg<uint8_t, NV>(a, k, slot, b0, row_end, fl, vals);
                } else {
                    VH_DEV_DISPATCH(a.dtype, T, ta_agg<T, NV>(a, k, slot, b0, row_end, fl, vals); break)
                }
            }
    #pragma unroll
            for (int r = 0; r < TA_RPT; r++) {
                const uint64_t i = b0 + (uint64_t)r * TA_THREADS + threadIdx.x;
                rank[r] = -1;
                if (i < row_end) {
                    const uint64_t c = cell[r];
                    const uint32_t f = fl[r];
                    tile[r] = (uint32_t)(c >> tp.s_log2);
                    ent[r] = ((uint32_t)c & smask) | (f << 16);
                    if (f) rank[r] = (int32_t)atomicAdd(&l.hist[tile[r]], 1u);
                }
            }
        }
        batch_commit<NV>(l, fa, tp, T, region0, tile, ent, rank, vals, &s_total);
        lds_barrier();
    }
    for (uint32_t t = threadIdx.x; t < T; t += TA_THREADS) tp.fills[(uint64_t)t * tp.W + w] = l.base[t] - (uint32_t)tp.toff[t];
}

// BinnerScalar<double> index from a loaded value (superagg_binners.cpp:42-53),
// branch-free in 32 bits (the tile path has cells < 2^28): every candidate is computed
// and selected, so a wave runs no exec-masked branches.  The
// conversion of an out-of-range or NaN product is never selected.
__device__ inline uint32_t scalar_f64_index32(double v, double vmin, double scale, double bins_d, uint32_t bins2) {
    const double scaled = (v - vmin) * scale;
    const uint32_t inner = (uint32_t)((int)(scaled * bins_d) + 2);
    uint32_t idx = scaled >= 1 ? bins2 : inner;
    idx = scaled < 0 ? 1u : idx;
    return scaled != scaled ? 0u : idx;
}

// fast pass A: ND native float64 scalar binners without masks, NV float64 sums without
// masks, counts unconditional or keyed on a carried value (mean).  Rows are read as
// 16-byte pairs; the next batch loads into a second register buffer while the current
// one is ranked, sorted and written.
template <int ND, int NV, int SB>
__global__ __launch_bounds__(TA_THREADS) TA_ATTR void k_tile_scatter_f64(BinPlan p, FusedAggs fa, TileParams tp, uint64_t n) {
    constexpr int NC = ND + NV;
    constexpr int PAIRS = TA_RPT / 2;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const uint32_t T = tp.ntiles;
    const ScatterLds l = fast_lds<NV>(lds_raw, T, SB * TA_BATCH);
    scatter_lds_init(l, tp, T);
    __syncthreads();
    const double *col[NC];
    double vmin[ND > 0 ? ND : 1], scale[ND > 0 ? ND : 1], bins_d[ND > 0 ? ND : 1];
    uint32_t bins2[ND > 0 ? ND : 1], stride[ND > 0 ? ND : 1];
#pragma unroll
    for (int d = 0; d < ND; d++) {
        col[d] = reinterpret_cast<const double *>(p.b[d].data);
        vmin[d] = p.b[d].vmin;
        scale[d] = p.b[d].scale;
        bins_d[d] = (double)p.b[d].bins;
        bins2[d] = (uint32_t)p.b[d].bins + 2;
        stride[d] = (uint32_t)p.b[d].stride;
    }
#pragma unroll
    for (int s = 0; s < NV; s++) col[ND + s] = tp.vdata[s];
    // take flags: count(*) always; a sum, or a count keyed on a summed column, takes the
    // row when that value is not NaN (nan_keyed[s] = the aggregators keyed on slot s)
    uint32_t count_mask = 0, keyed_slot_of[MAX_FUSED_AGGS], nan_keyed[NV > 0 ? NV : 1] = {};
    #pragma unroll
    for (int k = 0; k < MAX_FUSED_AGGS; k++) {
        if (k >= fa.na) break;
        keyed_slot_of[k] = fa.a[k].kind == VH_AGG_COUNT ? (uint32_t)tp.cnt_slot[k] : (uint32_t)tp.val_slot[k];
        if (fa.a[k].kind == VH_AGG_COUNT && tp.cnt_slot[k] == CNT_ALWAYS) count_mask |= 1u << k;
        else
#pragma unroll
            for (int s = 0; s < NV; s++)
                if ((uint32_t)s == keyed_slot_of[k]) nan_keyed[s] |= 1u << k;
    }
    const uint32_t w = blockIdx.x;
    const uint64_t row_begin = (uint64_t)w * tp.rows_per_wg;
    const uint64_t row_end = min(n, row_begin + tp.rows_per_wg);
    const uint32_t smask = (1u << tp.s_log2) - 1, s_log2 = tp.s_log2;
    const uint64_t region0 = (uint64_t)w * tp.wg_stride;
    // Branch-free 16-byte loads: n is even on this path (the host bins an odd last row
    // separately) and workgroup ranges are multiples of TA_BATCH, so a pair is either
    // wholly inside [row_begin, row_end) or wholly past it; past-the-end pairs load the
    // clamped last pair and are dropped by the i < row_end test.  With no load behind an
    // exec branch the compiler counts vmcnt instead of draining to 0, so the prefetched
    // batch stays in flight.
    auto load = [&](uint64_t b0, double2 (&dst)[PAIRS][NC]) {
#pragma unroll
        for (int q = 0; q < PAIRS; q++) {
            const uint64_t i = b0 + 2 * ((uint64_t)q * TA_THREADS + threadIdx.x);
            const uint64_t is = i < n - 2 ? i : n - 2;
#pragma unroll
            for (int c = 0; c < NC; c++) {
#if VH_TA_NT  // experiment: non-temporal loads of the once-read columns
                typedef double v2d __attribute__((ext_vector_type(2)));
                const v2d t = __builtin_nontemporal_load(reinterpret_cast<const v2d *>(col[c] + is));
                dst[q][c] = make_double2(t.x, t.y);
#else
                dst[q][c] = *reinterpret_cast<const double2 *>(col[c] + is);
#endif
            }
        }
    };
    // rank the rows of one batch: cell, take flags, (tile << 16 | cell) key, rank in tile
    auto rows = [&](uint64_t b0, const double2 (&cur)[PAIRS][NC], uint32_t *key, int32_t *rank,
                    double (*vals)[NV > 0 ? NV : 1]) {
#pragma unroll
        for (int r = 0; r < TA_RPT; r++) {
            const int q = r >> 1, h = r & 1;
            const uint64_t i = b0 + 2 * ((uint64_t)q * TA_THREADS + threadIdx.x) + h;
            uint32_t c = 0;
#pragma unroll
            for (int d = 0; d < ND; d++) {
                const double v = h ? cur[q][d].y : cur[q][d].x;
                c += scalar_f64_index32(v, vmin[d], scale[d], bins_d[d], bins2[d]) * stride[d];
            }
            uint32_t f = count_mask;
#pragma unroll
            for (int s = 0; s < NV; s++) {
                vals[r][s] = h ? cur[q][ND + s].y : cur[q][ND + s].x;
                f |= vals[r][s] == vals[r][s] ? nan_keyed[s] : 0u;
            }
            f = i < row_end ? f : 0u;
            const uint32_t t = c >> s_log2;
            key[r] = (t << 16) | (c & smask);
            rank[r] = -1;
            if (tp.debug & 64) {  // experiment: no ranking
                asm volatile("" ::"v"(key[r]), "v"(f));
            } else if (f) {
                rank[r] = (int32_t)atomicAdd(&l.hist[t], 1u);
            }
        }
    };
    double2 cur[PAIRS][NC], nxt[PAIRS][NC];
    load(row_begin, cur);
    for (uint64_t b0 = row_begin; b0 < row_end; b0 += SB * TA_BATCH) {
        uint32_t key[SB * TA_RPT];
        int32_t rank[SB * TA_RPT];
        double vals[SB * TA_RPT][NV > 0 ? NV : 1];
        // the last prefetch stays in flight across the commit: it is moved into cur only
        // after the commit (a copy before it would wait for those loads)
#pragma unroll
        for (int sb = 0; sb < SB; sb++) {
            load(b0 + (sb + 1) * TA_BATCH, nxt);
            rows(b0 + sb * TA_BATCH, cur, key + sb * TA_RPT, rank + sb * TA_RPT, vals + sb * TA_RPT);
            if (sb + 1 < SB || VH_TA_DRAIN)
#pragma unroll
                for (int q = 0; q < PAIRS; q++)
#pragma unroll
                    for (int c = 0; c < NC; c++) cur[q][c] = nxt[q][c];
        }
        if (tp.debug & 32) {  // experiment: no commit (loads, cell math, ranking only)
#pragma unroll
            for (int r = 0; r < SB * TA_RPT; r++) asm volatile("" ::"v"(key[r]), "v"(rank[r]));
        } else {
            batch_commit_fast<NV, SB * TA_RPT>(l, fa, tp, T, region0, key, rank, vals, count_mask, keyed_slot_of);
        }
        if (!VH_TA_DRAIN)
#pragma unroll
            for (int q = 0; q < PAIRS; q++)
#pragma unroll
                for (int c = 0; c < NC; c++) cur[q][c] = nxt[q][c];
    }
    lds_barrier();
    for (uint32_t t = threadIdx.x; t < T; t += TA_THREADS) tp.fills[(uint64_t)t * tp.W + w] = l.base[t] - (uint32_t)tp.toff[t];
}

// BinnerOrdinal<int32_t> index of a loaded key, native byte order, no mask
// (superagg_binners.cpp:104-142 with T = int32: the uint64 min_value is subtracted first)
__device__ inline uint64_t ordinal_i32_index(int32_t raw, uint64_t min_value, uint64_t count) {
    const int32_t value = (int32_t)((uint64_t)(int64_t)raw - min_value);
    if (value < 0) return 1;
    if ((uint64_t)(int64_t)value >= count) return count + 2;
    return (uint64_t)((int64_t)value + 2);
}

// fast pass A of the groupby / categorical grid: one int32 BinnerOrdinal (native, no mask)
// and NV float64 sums without masks -- the C3 groupby(key).agg({sum, count}) shape.
// Keys are read as 8-byte pairs and values as 16-byte pairs, the next batch prefetched in
// registers (same row layout and pipelining as k_tile_scatter_f64).
// cell of a set ordinal (set_index, binner_dev.hpp): unknown keys -> 1, past the count -> count + 2
__device__ inline uint32_t set_ord_cell(int64_t o, uint64_t count) {
    if (o < 0) return 1;
    if ((uint64_t)o >= count) return (uint32_t)count + 2;
    return (uint32_t)o + 2;
}

// SET = false: one native int32 BinnerOrdinal.  SET = true: the fused set-ordinal binner
// (BinnerOrdinal over map_ordinal of a 4-byte integer key, no mask, packed LUT): the first
// LUT probe of every row of a batch is issued before any is used, so a lane keeps eight
// random lookups in flight instead of walking one probe chain at a time (the per-row form
// fetched ~114 B per row at ~2.4 TB/s of random lines: 27 ms for C3); the rare rows whose
// first slot holds another key continue their probe sequence afterwards.
// DT0 / DT1: value slot dtypes as compile-time constants (VH_F64 = the float64 kernel), or -1:
// any dtype through a run-time switch (slower: the branches around the prefetch loads)
template <int NV, int SB, bool SET = false, int DT0 = VH_F64, int DT1 = VH_F64>
__global__ __launch_bounds__(TA_THREADS) TA_ATTR void k_tile_scatter_ord(BinPlan p, FusedAggs fa, TileParams tp, uint64_t n) {
    constexpr int PAIRS = TA_RPT / 2;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const uint32_t T = tp.ntiles;
    const ScatterLds l = fast_lds<NV>(lds_raw, T, SB * TA_BATCH);
    scatter_lds_init(l, tp, T);
    __syncthreads();
    const int32_t *keys = reinterpret_cast<const int32_t *>(p.b[0].data);
    const double *col[NV > 0 ? NV : 1];
#pragma unroll
    for (int s = 0; s < NV; s++) col[s] = tp.vdata[s];
    const uint64_t min_value = p.b[0].min_value, count = p.b[0].ordinal_count;
    const uint32_t stride0 = (uint32_t)p.b[0].stride;
    uint32_t count_mask = 0, keyed_slot_of[MAX_FUSED_AGGS], nan_keyed[NV > 0 ? NV : 1] = {};
    #pragma unroll
    for (int k = 0; k < MAX_FUSED_AGGS; k++) {
        if (k >= fa.na) break;
        keyed_slot_of[k] = fa.a[k].kind == VH_AGG_COUNT ? (uint32_t)tp.cnt_slot[k] : (uint32_t)tp.val_slot[k];
        // count(*) and integer sums take every row (int64 bits are not NaN-tested)
        if ((fa.a[k].kind == VH_AGG_COUNT && tp.cnt_slot[k] == CNT_ALWAYS) || fa.a[k].vint ||
            (is_minmax(fa.a[k].kind) && fa.a[k].dtype != VH_F64 && fa.a[k].dtype != VH_F32))
            count_mask |= 1u << k;
        else
#pragma unroll
            for (int s = 0; s < NV; s++)
                if ((uint32_t)s == keyed_slot_of[k]) nan_keyed[s] |= 1u << k;
    }
    const uint32_t w = blockIdx.x;
    const uint64_t row_begin = (uint64_t)w * tp.rows_per_wg;
    const uint64_t row_end = min(n, row_begin + tp.rows_per_wg);
    const uint32_t smask = (1u << tp.s_log2) - 1, s_log2 = tp.s_log2;
    const uint64_t region0 = (uint64_t)w * tp.wg_stride;
    struct Regs {
        int2 k[PAIRS];
        double2 v[PAIRS][NV > 0 ? NV : 1];
    };
    int vsz[NV > 0 ? NV : 1];
#pragma unroll
    for (int s = 0; s < NV; s++) {
        const int dts = s == 0 ? DT0 : DT1;
        vsz[s] = dts >= 0 ? dtype_itemsize_dev(dts) : dtype_itemsize_dev(tp.vdt[s]);
    }
    // row pairs: keys as int2, values by item size (float64 16 B; narrower types' pair bits
    // packed into .x, decoded per row by pair_slot when used, so the prefetch stays in flight)
    auto load = [&](uint64_t b0, Regs &R) {
#pragma unroll
        for (int q = 0; q < PAIRS; q++) {
            const uint64_t i = b0 + 2 * ((uint64_t)q * TA_THREADS + threadIdx.x);
            const uint64_t is = i < n - 2 ? i : n - 2;
            R.k[q] = *reinterpret_cast<const int2 *>(keys + is);
#pragma unroll
            for (int s = 0; s < NV; s++) {
                const char *cb = reinterpret_cast<const char *>(col[s]);
                if (vsz[s] == 8) {
                    R.v[q][s] = *reinterpret_cast<const double2 *>(cb + is * 8);
                } else if (vsz[s] == 4) {
                    R.v[q][s].x = __builtin_bit_cast(double, *reinterpret_cast<const uint64_t *>(cb + is * 4));
                } else if (vsz[s] == 2) {
                    R.v[q][s].x = __builtin_bit_cast(double, (uint64_t)*reinterpret_cast<const uint32_t *>(cb + is * 2));
                } else {
                    R.v[q][s].x = __builtin_bit_cast(double, (uint64_t)*reinterpret_cast<const uint16_t *>(cb + is));
                }
            }
        }
    };
    const SetDev sd = p.b[0].set;
    auto rows = [&](uint64_t b0, const Regs &cur, uint32_t *key, int32_t *rank, double (*vals)[NV > 0 ? NV : 1]) {
        uint32_t scell[SET ? TA_RPT : 1];
        if constexpr (SET) {
            uint64_t e[TA_RPT], pos[TA_RPT];
#pragma unroll
            for (int r = 0; r < TA_RPT; r++) {
                const uint32_t kb = (uint32_t)(r & 1 ? cur.k[r >> 1].y : cur.k[r >> 1].x);
                pos[r] = hash64(kb) & sd.cap_mask;
                e[r] = sd.lut[pos[r]];
            }
#pragma unroll
            for (int r = 0; r < TA_RPT; r++) {
                const uint32_t kb = (uint32_t)(r & 1 ? cur.k[r >> 1].y : cur.k[r >> 1].x);
                int64_t o = -1;
                if (e[r] != SET_EMPTY && (uint32_t)e[r] == kb) {
                    o = (int64_t)(e[r] >> 32);
                } else if (e[r] != SET_EMPTY) {
                    uint64_t ps = pos[r];
                    for (int k = 0; k < SET_MAX_PROBE; k++) {
                        ps = (ps + 1) & sd.cap_mask;
                        const uint64_t x = sd.lut[ps];
                        if (x == SET_EMPTY) break;
                        if ((uint32_t)x == kb) {
                            o = (int64_t)(x >> 32);
                            break;
                        }
                    }
                }
                scell[r] = set_ord_cell(o, count) * stride0;
            }
        }
#pragma unroll
        for (int r = 0; r < TA_RPT; r++) {
            const int q = r >> 1, h = r & 1;
            const uint64_t i = b0 + 2 * ((uint64_t)q * TA_THREADS + threadIdx.x) + h;
            uint32_t c;
            if constexpr (SET) c = scell[r];
            else c = (uint32_t)ordinal_i32_index(h ? cur.k[q].y : cur.k[q].x, min_value, count) * stride0;
            uint32_t f = count_mask;
#pragma unroll
            for (int s = 0; s < NV; s++) {
                const int dts = s == 0 ? DT0 : DT1;
                vals[r][s] = pair_slot(cur.v[q][s], dts >= 0 ? dts : tp.vdt[s], h);
                f |= vals[r][s] == vals[r][s] ? nan_keyed[s] : 0u;
            }
            f = i < row_end ? f : 0u;
            const uint32_t t = c >> s_log2;
            key[r] = (t << 16) | (c & smask);
            rank[r] = -1;
            if (f) rank[r] = (int32_t)atomicAdd(&l.hist[t], 1u);
        }
    };
    Regs cur, nxt;
    load(row_begin, cur);
    for (uint64_t b0 = row_begin; b0 < row_end; b0 += SB * TA_BATCH) {
        uint32_t key[SB * TA_RPT];
        int32_t rank[SB * TA_RPT];
        double vals[SB * TA_RPT][NV > 0 ? NV : 1];
#pragma unroll
        for (int sb = 0; sb < SB; sb++) {
            load(b0 + (sb + 1) * TA_BATCH, nxt);
            rows(b0 + sb * TA_BATCH, cur, key + sb * TA_RPT, rank + sb * TA_RPT, vals + sb * TA_RPT);
            if (sb + 1 < SB || VH_TA_DRAIN) cur = nxt;
        }
        batch_commit_fast<NV, SB * TA_RPT>(l, fa, tp, T, region0, key, rank, vals, count_mask, keyed_slot_of);
        if (!VH_TA_DRAIN) cur = nxt;
    }
    lds_barrier();
    for (uint32_t t = threadIdx.x; t < T; t += TA_THREADS) tp.fills[(uint64_t)t * tp.W + w] = l.base[t] - (uint32_t)tp.toff[t];
}

template <int NV>
__device__ inline void reduce_entry(const FusedAggs &fa, const TileParams &tp, unsigned char *lds, uint32_t local,
                                    uint32_t fl, const double *v) {
    #pragma unroll
    for (int k = 0; k < MAX_FUSED_AGGS; k++) {
        if (k >= fa.na) break;
        if (fa.a[k].kind == VH_AGG_COUNT) {
            const int cs = tp.cnt_slot[k];
            bool take;
            if (cs == CNT_ALWAYS) take = true;
            else if (cs == CNT_FLAG) take = (fl >> k) & 1;
            else {
                take = false;
#pragma unroll
                for (int s = 0; s < NV; s++)
                    if (s == cs) take = v[s] == v[s];
            }
            if (take) atomicAdd(reinterpret_cast<uint32_t *>(lds + fa.a[k].lds_off) + local, 1u);
        } else if (is_minmax(fa.a[k].kind)) {
#pragma unroll
            for (int s = 0; s < NV; s++) {
                if (s != tp.val_slot[k]) continue;
                mm_lds(reinterpret_cast<uint64_t *>(lds + fa.a[k].lds_off) + local, fa.a[k].dtype, fa.a[k].kind == VH_AGG_MAX, v[s]);
            }
        } else {
#pragma unroll
            for (int s = 0; s < NV; s++) {
                if (s != tp.val_slot[k]) continue;
                if (fa.a[k].vint)  // integer sums: two's-complement 64-bit adds of the upcast value
                    atomicAdd(reinterpret_cast<unsigned long long *>(lds + fa.a[k].lds_off) + local,
                              __builtin_bit_cast(unsigned long long, v[s]));
                else if (v[s] == v[s])
                    atomicAdd(reinterpret_cast<double *>(lds + fa.a[k].lds_off) + local, v[s]);
            }
        }
    }
}

constexpr int TB_UNROLL = 8;
#ifndef VH_TB_VU
#define VH_TB_VU 0  // 8-entry chunks per lane per step (0 = by NV)
#endif
template <int NV> constexpr int tb_vu() { return VH_TB_VU ? VH_TB_VU : NV == 0 ? 8 : 2; }  // NV 1: 3 -> 2 was 2.17 -> 2.06 ms (same-process A/B, twice)

// Pass B: one work unit = one tile x a range of pass-A workgroups.  The unit's regions are
// read as one flat stream of 8-entry chunks (prefix sums of the region fills in LDS), so
// every step issues TB_THREADS * VU full 16-byte entry loads (+ their values) no matter how
// short the regions are; a lane finds the region of its chunk by a forward scan (chunk
// indices of a lane only grow).  Entries are reduced with LDS atomics, then the tile is
// flushed with coalesced global atomics.
template <int NV, bool NARROW = false>
__global__ __launch_bounds__(TB_THREADS) void k_tile_reduce(FusedAggs fa, TileParams tp, const WorkUnit *units) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    __shared__ uint32_t s_fill[1024];
    __shared__ uint32_t s_pre[1025];
    if (tp.abort_word && *tp.abort_word != 1u) return;  // resident launch not committed: rerun by the host
    const WorkUnit u = units[blockIdx.x];
    const uint32_t t = u.tile;
    const uint32_t cap = tp.cap[t];
    const uint32_t nw = u.w_end - u.w_begin;  // <= W <= 1024 (host checks)
    bool any = false;
    for (uint32_t k = threadIdx.x; k < nw; k += TB_THREADS) {
        const uint32_t f = min(tp.fills[(uint64_t)t * tp.W + u.w_begin + k], cap);
        s_fill[k] = f;
        any |= f != 0;
    }
    if (!__syncthreads_or(any)) return;
    uint32_t *lw = reinterpret_cast<uint32_t *>(lds_raw);
    for (uint32_t i = threadIdx.x; i < fa.lds_words; i += TB_THREADS) lw[i] = 0;
    if (!tp.flags_mode && threadIdx.x < 64) {
        // exclusive scan of the chunk counts by the first wave (16 regions per lane)
        const uint32_t lane = threadIdx.x, k0 = lane * 16;
        uint32_t sum = 0;
        for (uint32_t k = k0; k < k0 + 16 && k < nw; k++) sum += (s_fill[k] + 7) >> 3;
        uint32_t inc = sum;
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(inc, off, 64);
            if ((int)lane >= off) inc += y;
        }
        uint32_t acc = inc - sum;
        for (uint32_t k = k0; k < k0 + 16 && k < nw; k++) {
            s_pre[k] = acc;
            acc += (s_fill[k] + 7) >> 3;
        }
        if (lane == 63) s_pre[nw] = inc;
    }
    __syncthreads();
    bool any_mm = false;
    #pragma unroll
    for (int k = 0; k < MAX_FUSED_AGGS; k++)
        if (k < fa.na && is_minmax(fa.a[k].kind)) any_mm = true;
    if (any_mm) {  // min / max cells start at the kind's identity (after the zero fill)
        const uint32_t ncells = 1u << tp.s_log2;
        #pragma unroll
        for (int k = 0; k < MAX_FUSED_AGGS; k++) {
            if (k >= fa.na || !is_minmax(fa.a[k].kind)) continue;
            uint64_t *cells = reinterpret_cast<uint64_t *>(lds_raw + fa.a[k].lds_off);
            const uint64_t id = mm_identity(fa.a[k].dtype, fa.a[k].kind == VH_AGG_MAX);
            for (uint32_t i = threadIdx.x; i < ncells; i += TB_THREADS) cells[i] = id;
        }
        __syncthreads();
    }
    if (!tp.flags_mode) {
        constexpr int VU = tb_vu<NV>();
        const uint32_t C = s_pre[nw];
        const uint16_t *ent16 = reinterpret_cast<const uint16_t *>(tp.entries);
        const uint64_t toff_t = tp.toff[t];
        uint32_t kk = 0;  // region of this lane's current chunk
        for (uint32_t c0 = 0; c0 < C; c0 += TB_THREADS * VU) {
            uint4 ev[VU];
            double2 vv[VU][NV > 0 ? NV : 1][4];
            uint32_t rem[VU];
#pragma unroll
            for (int j = 0; j < VU; j++) {
                const uint32_t c = c0 + j * TB_THREADS + threadIdx.x;
                const uint32_t cc = c < C ? c : C - 1;
                while (s_pre[kk + 1] <= cc) kk++;
                const uint32_t q = (cc - s_pre[kk]) * 8;
                // regions start at multiples of 8 entries and hold a multiple of 8, so the
                // chunk never leaves its region (entries past the fill are ignored)
                const uint64_t e = (uint64_t)(u.w_begin + kk) * tp.wg_stride + toff_t + q;
                rem[j] = c < C ? min(8u, s_fill[kk] - q) : 0u;
                ev[j] = *reinterpret_cast<const uint4 *>(ent16 + e);
#pragma unroll
                for (int s = 0; s < NV; s++) {
                    if constexpr (NARROW) {  // 8 x 4-byte slots: two 16-byte loads, widened
                        const bool fl = (tp.vfloat >> s) & 1, sg = (tp.vsigned >> s) & 1;
                        const uint4 a = *reinterpret_cast<const uint4 *>(reinterpret_cast<const uint32_t *>(tp.values[s]) + e);
                        const uint4 b = *reinterpret_cast<const uint4 *>(reinterpret_cast<const uint32_t *>(tp.values[s]) + e + 4);
                        vv[j][s][0] = make_double2(slot_wide(a.x, fl, sg), slot_wide(a.y, fl, sg));
                        vv[j][s][1] = make_double2(slot_wide(a.z, fl, sg), slot_wide(a.w, fl, sg));
                        vv[j][s][2] = make_double2(slot_wide(b.x, fl, sg), slot_wide(b.y, fl, sg));
                        vv[j][s][3] = make_double2(slot_wide(b.z, fl, sg), slot_wide(b.w, fl, sg));
                    } else {
#pragma unroll
                        for (int h = 0; h < 4; h++) vv[j][s][h] = *reinterpret_cast<const double2 *>(tp.values[s] + e + 2 * h);
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < VU; j++) {
                const uint32_t words[4] = {ev[j].x, ev[j].y, ev[j].z, ev[j].w};
#pragma unroll
                for (int x = 0; x < 8; x++) {
                    if ((uint32_t)x >= rem[j]) break;
                    double v[NV > 0 ? NV : 1];
#pragma unroll
                    for (int s = 0; s < NV; s++) v[s] = (x & 1) ? vv[j][s][x >> 1].y : vv[j][s][x >> 1].x;
                    const uint32_t local = (words[x >> 1] >> (16 * (x & 1))) & 0xffffu;
                    if (tp.debug & 8) asm volatile("" :: "v"(local));
                    else reduce_entry<NV>(fa, tp, lds_raw, local, 0xfu, v);
                }
            }
        }
    } else {
        for (uint32_t k = 0; k < nw; k++) {
            const uint32_t cnt = s_fill[k];
            const uint64_t base = (uint64_t)(u.w_begin + k) * tp.wg_stride + tp.toff[t];
            for (uint32_t q0 = 0; q0 < cnt; q0 += TB_THREADS * TB_UNROLL) {
                uint32_t ent[TB_UNROLL];
                double v[TB_UNROLL][NV > 0 ? NV : 1];
#pragma unroll
                for (int j = 0; j < TB_UNROLL; j++) {
                    const uint32_t q = q0 + j * TB_THREADS + threadIdx.x;
                    if (q < cnt) {
                        const uint64_t e = base + q;
                        ent[j] = reinterpret_cast<const uint32_t *>(tp.entries)[e];
#pragma unroll
                        for (int s = 0; s < NV; s++) {
                            if constexpr (NARROW)
                                v[j][s] = slot_wide(reinterpret_cast<const uint32_t *>(tp.values[s])[e], (tp.vfloat >> s) & 1,
                                                    (tp.vsigned >> s) & 1);
                            else
                                v[j][s] = tp.values[s][e];
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < TB_UNROLL; j++) {
                    const uint32_t q = q0 + j * TB_THREADS + threadIdx.x;
                    if (q < cnt) reduce_entry<NV>(fa, tp, lds_raw, ent[j] & 0xffffu, ent[j] >> 16, v[j]);
                }
            }
        }
    }
    __syncthreads();
    if (tp.debug & 16) return;
    const uint64_t c0 = (uint64_t)(tp.tile_of ? tp.tile_of[t] : t) << tp.s_log2;
    const uint32_t ncell = (uint32_t)min((uint64_t)1 << tp.s_log2, tp.cells - c0);
    #pragma unroll
    for (int k = 0; k < MAX_FUSED_AGGS; k++) {
        if (k >= fa.na) break;
        for (uint32_t i = threadIdx.x; i < ncell; i += TB_THREADS) {
            if (fa.a[k].kind == VH_AGG_COUNT) {
                const uint32_t v = reinterpret_cast<const uint32_t *>(lds_raw + fa.a[k].lds_off)[i];
                if (v) atomicAdd((unsigned long long *)fa.a[k].grid + c0 + i, (unsigned long long)v);
            } else if (is_minmax(fa.a[k].kind)) {
                const bool mx = fa.a[k].kind == VH_AGG_MAX;
                const uint64_t v = reinterpret_cast<const uint64_t *>(lds_raw + fa.a[k].lds_off)[i];
                if (v != mm_identity(fa.a[k].dtype, mx)) mm_grid(fa.a[k].grid, c0 + i, fa.a[k].dtype, mx, v, true);
            } else if (fa.a[k].vint) {
                const unsigned long long v = reinterpret_cast<const unsigned long long *>(lds_raw + fa.a[k].lds_off)[i];
                if (v) atomicAdd(reinterpret_cast<unsigned long long *>(fa.a[k].grid) + c0 + i, v);
            } else {
                const double v = reinterpret_cast<const double *>(lds_raw + fa.a[k].lds_off)[i];
                if (v != 0.0) atomicAdd(reinterpret_cast<double *>(fa.a[k].grid) + c0 + i, v);
            }
        }
    }
}

// ---- XCD-resident hot tiles: one persistent launch replaces pass A + most of pass B ----
//
// The two-pass path moves every row through HBM twice more (pass A writes a 10-B entry,
// pass B reads it back): 44 B of traffic per 24-B count+sum row, and HBM read/write
// turnaround caps such a mix at ~3.6 TB/s of reads.  Here one workgroup
// per CU (8 XCDs x P) runs the whole query.  Each XCD keeps its own replica of the H
// densest tiles (sample histogram), spread over the LDS of its P workgroups (TPW tiles
// each).  A workgroup reads its row range like pass A, counting-sorts each batch by
// region id (hot tiles first, in owner order) and
//   * hands the hot prefix to the owners on its own XCD through a batch slot (K slots per
//     producer, plain stores that stay in the XCD's L2, read back with L1-bypassing `sc1`
//     loads by workgroups whose HW_REG_XCC_ID is the same), and
//   * streams the cold suffix to per-(workgroup, tile) regions for pass B, as pass A does.
// Between batches it consumes what the producers of its XCD published for its tiles (LDS
// atomics).  Flags: `sc1` stores / loads (ready[x][p] = batches published by p;
// cons[x][p][c] = batches of p consumed by c; a producer reuses slot b % K once every
// consumer acknowledged batch b - K).  No wait is unbounded: a workgroup that sees no
// progress for `timeout` ticks (or finds more workgroups on its XCD than slots) sets the
// state word to ABORT; the launch then writes nothing to the grids, pass B skips, and the
// host reruns the query on the two-pass path.  Otherwise the last workgroup to finish
// commits, every owner flushes its LDS tiles with coalesced global atomics and applies its
// few cold-region overflows.  Results are the same sums of the same rows (counts exact,
// float sums within 1e-6 relative).
#ifndef VH_RES_K
#define VH_RES_K 4
#endif
constexpr uint32_t RES_HDR = 64;   // run offsets per batch-slot header (P + 1 <= 64)
constexpr uint32_t RES_OVF = 2048; // cold-region overflow entries kept per workgroup
enum : uint32_t { RES_RUNNING = 0, RES_COMMIT = 1, RES_ABORT = 2 };

struct ResidentParams {
    uint32_t P, K, H, TPW, nb, G, wt, pad;
    uint64_t timeout;          // wall-clock ticks without progress before ABORT
    uint32_t *ctl;             // [0] state, [1] finished workgroups, [2 + x] slots taken on XCD x
    uint32_t *ready;           // [8][P]
    uint32_t *cons;            // [8][P producer][P consumer]
    uint32_t *hdr;             // [8][P][K][RES_HDR]
    uint32_t *skeys;           // [8][P][K][TA_BATCH] owner-local cell
    double *svals;             // [8][P][K][TA_BATCH]
    const uint32_t *tmap;      // [T] grid tile -> region id (hot ids 0..H-1)
    const uint32_t *tile_of;   // [T] region id -> grid tile
    uint32_t *ovf_key;         // [G][RES_OVF] id << 16 | cell in tile
    double *ovf_val;           // [G][RES_OVF]
};

__device__ __forceinline__ uint32_t ld_sc1(const uint32_t *p) {
    return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double *p) {
    return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<uint64_t *>(const_cast<double *>(p)),
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double *p, double v) {
    __hip_atomic_store(reinterpret_cast<uint64_t *>(p), __builtin_bit_cast(uint64_t, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// LDS of the resident kernel: owner tiles (fr.lds_words words) | pass-A staging | tmap[T]
__host__ __device__ inline size_t resident_lds_bytes(uint32_t tile_words, int nv, uint32_t T) {
    return (size_t)4 * tile_words + fast_lds_bytes(nv, T, TA_BATCH) + (size_t)4 * T;
}

// apply one staged row to the grids with global atomics (region overflow)
template <int NV>
__device__ inline void apply_row_global(const FusedAggs &fa, const TileParams &tp, uint64_t c, uint32_t count_mask,
                                        const uint32_t *keyed_slot_of, const double *v) {
    #pragma unroll
    for (int a = 0; a < MAX_FUSED_AGGS; a++) {
        if (a >= fa.na) break;
        bool take = (count_mask >> a) & 1;
        if constexpr (NV > 0) {
            if (!take) take = v[keyed_slot_of[a]] == v[keyed_slot_of[a]];
        }
        if (!take) continue;
        if (fa.a[a].kind == VH_AGG_COUNT) {
            atomicAdd((unsigned long long *)fa.a[a].grid + c, 1ULL);
        } else if constexpr (NV > 0) {
            atomicAdd(reinterpret_cast<double *>(fa.a[a].grid) + c, v[tp.val_slot[a]]);
        }
    }
}

// Roles inside the workgroup: waves 0..RES_PW-1 produce (pass-A pipeline, synchronised by
// an LDS counter barrier among themselves), RES_CW consumer waves poll the producers of
// their XCD independently (no workgroup barrier), so neither side waits on the other's
// memory latency.
constexpr int RES_PW = TA_THREADS / 64;
#ifndef VH_RES_CW
#define VH_RES_CW 4
#endif
constexpr int RES_CW = VH_RES_CW;
constexpr int RES_THREADS = TA_THREADS + 64 * RES_CW;
constexpr int RES_CU = 4;  // slot entries per consumer lane in flight

// barrier of the producer waves only: one lane per wave adds, then spins on the LDS counter
__device__ __forceinline__ void prod_barrier(uint32_t *ctr, uint32_t &target) {
    target += RES_PW;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63) == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target)
            __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

template <int ND, int NV>
__global__ __launch_bounds__(RES_THREADS) void k_tile_resident(BinPlan p, FusedAggs fa, FusedAggs fr, TileParams tp,
                                                               ResidentParams rp, uint64_t n) {
    constexpr int NC = ND + NV;
    constexpr int PAIRS = TA_RPT / 2;
    constexpr uint32_t CAP = TA_BATCH;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    __shared__ uint32_t s_ctl[8], s_bar;
    __shared__ uint32_t s_wpre[RES_CW][65], s_wbeg[RES_CW][64], s_wsb[RES_CW][64];
    const uint32_t T = tp.ntiles;
    unsigned char *tl = lds_raw;
    const ScatterLds l = fast_lds<NV>(lds_raw + (size_t)4 * fr.lds_words, T, CAP);
    uint32_t *s_tmap = reinterpret_cast<uint32_t *>(lds_raw + (size_t)4 * fr.lds_words + fast_lds_bytes(NV, T, CAP));
    uint32_t *sk = reinterpret_cast<uint32_t *>(l.sp);
    const uint32_t tid = threadIdx.x;
    {
        uint32_t *lw = reinterpret_cast<uint32_t *>(tl);
        for (uint32_t i = tid; i < fr.lds_words; i += RES_THREADS) lw[i] = 0;
    }
    for (uint32_t t = tid; t < T; t += RES_THREADS) s_tmap[t] = rp.tmap[t];
    for (uint32_t t = tid; t < T; t += RES_THREADS) {
        l.hist[t] = 0;
        l.base[t] = (uint32_t)tp.toff[t];
        l.lim[t] = (uint32_t)tp.toff[t] + tp.cap[t];
    }
    if (tid == 0) {
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        xcc &= 0xfu;
        const uint32_t slot = xcc < 8 ? atomicAdd(&rp.ctl[2 + xcc], 1u) : 0xffffffffu;
        bool ab = ld_sc1(&rp.ctl[0]) == RES_ABORT;
        if (slot >= rp.P) {  // placement the slots do not cover: the two-pass path reruns the query
            atomicCAS(&rp.ctl[0], RES_RUNNING, RES_ABORT);
            ab = true;
        }
        s_ctl[0] = xcc;
        s_ctl[1] = slot;
        s_ctl[3] = ab ? 1u : 0u;  // abort seen
        s_ctl[6] = 0;             // overflow entries
        s_ctl[7] = 0;             // overflow list full
        s_bar = 0;
    }
    __syncthreads();
    if (s_ctl[3]) return;
    const uint32_t xcc = s_ctl[0], me = s_ctl[1];
    const uint32_t P = rp.P, K = rp.K, H = rp.H, TPW = rp.TPW, nb = rp.nb;
    const uint32_t smask = (1u << tp.s_log2) - 1, s_log2 = tp.s_log2;
    const uint64_t xp0 = (uint64_t)xcc * P;
    const uint32_t w = blockIdx.x;
    uint32_t count_mask = 0, keyed_slot_of[MAX_FUSED_AGGS], nan_keyed[NV > 0 ? NV : 1] = {};
    #pragma unroll
    for (int k = 0; k < MAX_FUSED_AGGS; k++) {
        keyed_slot_of[k] = 0;
        if (k >= fa.na) break;
        keyed_slot_of[k] = fa.a[k].kind == VH_AGG_COUNT ? (uint32_t)tp.cnt_slot[k] : (uint32_t)tp.val_slot[k];
        if (fa.a[k].kind == VH_AGG_COUNT && tp.cnt_slot[k] == CNT_ALWAYS) count_mask |= 1u << k;
        else
#pragma unroll
            for (int s = 0; s < NV; s++)
                if ((uint32_t)s == keyed_slot_of[k]) nan_keyed[s] |= 1u << k;
    }
    uint32_t *ovf_key = rp.ovf_key + (uint64_t)w * RES_OVF;
    double *ovf_val = rp.ovf_val + (uint64_t)w * RES_OVF;

    if (tid < TA_THREADS) {
        // ================= producer waves =================
        const double *col[NC];
        double vmin[ND], scale[ND], bins_d[ND];
        uint32_t bins2[ND], stride[ND];
#pragma unroll
        for (int d = 0; d < ND; d++) {
            col[d] = reinterpret_cast<const double *>(p.b[d].data);
            vmin[d] = p.b[d].vmin;
            scale[d] = p.b[d].scale;
            bins_d[d] = (double)p.b[d].bins;
            bins2[d] = (uint32_t)p.b[d].bins + 2;
            stride[d] = (uint32_t)p.b[d].stride;
        }
#pragma unroll
        for (int s = 0; s < NV; s++) col[ND + s] = tp.vdata[s];
        const uint64_t row_begin = (uint64_t)w * tp.rows_per_wg;
        const uint64_t row_end = min(n, row_begin + tp.rows_per_wg);
        const uint64_t region0 = (uint64_t)w * tp.wg_stride;
        uint32_t bar = 0;
        uint32_t cmin = 0;  // wave 0: least batch count every consumer acknowledged (cached)
        uint64_t last = wall_clock64();
        auto load = [&](uint64_t b0, double2 (&dst)[PAIRS][NC]) {
#pragma unroll
            for (int q = 0; q < PAIRS; q++) {
                const uint64_t i = b0 + 2 * ((uint64_t)q * TA_THREADS + tid);
                const uint64_t is = i < n - 2 ? i : n - 2;
#pragma unroll
                for (int c = 0; c < NC; c++) dst[q][c] = *reinterpret_cast<const double2 *>(col[c] + is);
            }
        };
        // one batch: `cur` holds its rows (loaded one step earlier), `nxt` receives the next
        auto step = [&](uint32_t b, double2 (&cur)[PAIRS][NC], double2 (&nxt)[PAIRS][NC]) -> bool {
            const uint64_t b0 = row_begin + (uint64_t)b * CAP;
            // this batch's loads and the previous batch's stores complete; then the previous
            // batch is published (every producer wave's stores have reached L2)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            prod_barrier(&s_bar, bar);
            if (tid == 0 && b > 0) {
                if (rp.wt) st_sc1(&rp.ready[xp0 + me], b);
                else rp.ready[xp0 + me] = b;  // same XCD: the flag stays in the L2 the pollers read
            }
            if (b + 1 < nb) load(b0 + CAP, nxt);
            uint32_t key[TA_RPT];
            int32_t rank[TA_RPT];
            double vals[TA_RPT][NV > 0 ? NV : 1];
            if (tp.debug & 2048) {  // experiment: loads + cell math only, nothing published
                uint32_t acc = 0;
#pragma unroll
                for (int r = 0; r < TA_RPT; r++) {
                    const int q = r >> 1, h = r & 1;
                    uint32_t c = 0;
#pragma unroll
                    for (int d = 0; d < ND; d++)
                        c += scalar_f64_index32(h ? cur[q][d].y : cur[q][d].x, vmin[d], scale[d], bins_d[d], bins2[d]) * stride[d];
                    acc += c;
                }
                asm volatile("" ::"v"(acc));
                return true;
            }
#pragma unroll
            for (int r = 0; r < TA_RPT; r++) {
                const int q = r >> 1, h = r & 1;
                const uint64_t i = b0 + 2 * ((uint64_t)q * TA_THREADS + tid) + h;
                uint32_t c = 0;
#pragma unroll
                for (int d = 0; d < ND; d++) {
                    const double v = h ? cur[q][d].y : cur[q][d].x;
                    c += scalar_f64_index32(v, vmin[d], scale[d], bins_d[d], bins2[d]) * stride[d];
                }
                uint32_t f = count_mask;
#pragma unroll
                for (int s = 0; s < NV; s++) {
                    vals[r][s] = h ? cur[q][ND + s].y : cur[q][ND + s].x;
                    f |= vals[r][s] == vals[r][s] ? nan_keyed[s] : 0u;
                }
                f = i < row_end ? f : 0u;
                const uint32_t id = s_tmap[c >> s_log2];
                key[r] = (id << 16) | (c & smask);
                rank[r] = f ? (int32_t)atomicAdd(&l.hist[id], 1u) : -1;
            }
            prod_barrier(&s_bar, bar);
            fast_scan(l, T);
            prod_barrier(&s_bar, bar);
            const uint32_t tot = l.wave_sums[0];
            const uint32_t hot_n = H < T ? l.boff[H] : tot;
#pragma unroll
            for (int r = 0; r < TA_RPT; r++) {
                if (rank[r] < 0) continue;
                const uint32_t pos = l.boff[key[r] >> 16] + (uint32_t)rank[r];
                sk[pos] = key[r];
#pragma unroll
                for (int s = 0; s < NV; s++) l.sv[s * CAP + pos] = vals[r][s];
            }
            // wave 0: slot b % K is free once every owner acknowledged batch b - K
            if (tid < 64 && b >= K && cmin < b - K + 1) {
                const uint32_t target = b - K + 1;
                for (;;) {
                    const uint32_t v = tid < P ? ld_sc1(&rp.cons[(xp0 + me) * P + tid]) : 0xffffffffu;
                    uint32_t m = v;
#pragma unroll
                    for (int off = 32; off; off >>= 1) m = min(m, (uint32_t)__shfl_xor(m, off, 64));
                    if (m >= target) {
                        cmin = m;
                        last = wall_clock64();
                        break;
                    }
                    if (tid == 0) {
                        const uint64_t now = wall_clock64();
                        if (ld_sc1(&rp.ctl[0]) == RES_ABORT) s_ctl[3] = 1;
                        else if (now - last > rp.timeout) {
                            atomicCAS(&rp.ctl[0], RES_RUNNING, RES_ABORT);
                            s_ctl[3] = 1;
                        }
                    }
                    if (__shfl(s_ctl[3], 0, 64)) break;
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            // the stop decision every producer wave reads: written by lane 0 before the barrier
            // (s_ctl[3] may change under the consumer waves at any time)
            if (tid == 0) s_ctl[5] = s_ctl[3];
            prod_barrier(&s_bar, bar);
            if (s_ctl[5]) return false;
            const uint64_t sb = (xp0 + me) * K + b % K;
            uint32_t *dk = rp.skeys + sb * CAP;
            double *dv = rp.svals + sb * CAP;
            for (uint32_t k = tid; k < hot_n && !(tp.debug & 512); k += TA_THREADS) {  // 512: no slot stores
                const uint32_t kk = sk[k];
                const uint32_t loc = (((kk >> 16) % TPW) << s_log2) | (kk & smask);
                if (rp.wt) st_sc1(dk + k, loc);
                else dk[k] = loc;
#pragma unroll
                for (int s = 0; s < NV; s++) {
                    if (rp.wt) st_sc1(dv + k, l.sv[s * CAP + k]);
                    else dv[k] = l.sv[s * CAP + k];
                }
            }
            for (uint32_t o = tid; o <= P; o += TA_THREADS) {
                const uint32_t id = o * TPW;
                const uint32_t v = id < H ? l.boff[id] : hot_n;
                if (rp.wt) st_sc1(&rp.hdr[sb * RES_HDR + o], v);
                else rp.hdr[sb * RES_HDR + o] = v;
            }
            for (uint32_t k = hot_n + tid; k < tot && !(tp.debug & 1024); k += TA_THREADS) {  // 1024: no cold stores
                const uint32_t kk = sk[k];
                const uint32_t t = kk >> 16;
                const uint32_t dest = l.dbase[t] + k;
                if (dest < l.lim[t]) {
                    const uint64_t e = region0 + dest;
                    reinterpret_cast<uint16_t *>(tp.entries)[e] = (uint16_t)kk;
#pragma unroll
                    for (int s = 0; s < NV; s++) tp.values[s][e] = l.sv[s * CAP + k];
                } else {  // region overflow (a sampling miss): kept until the launch commits
                    const uint32_t pos = atomicAdd(&s_ctl[6], 1u);
                    if (pos < RES_OVF) {
                        ovf_key[pos] = kk;
                        if constexpr (NV > 0) ovf_val[pos] = l.sv[k];
                    } else {
                        s_ctl[7] = 1;
                    }
                }
            }
            return true;
        };
        double2 A[PAIRS][NC], B[PAIRS][NC];
        load(row_begin, A);
        bool ok = true;
        for (uint32_t b = 0; b < nb && ok; b += 2) {
            ok = step(b, A, B);
            if (ok && b + 1 < nb) ok = step(b + 1, B, A);
        }
        if (ok) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            prod_barrier(&s_bar, bar);
            if (tid == 0) {
                if (rp.wt) st_sc1(&rp.ready[xp0 + me], nb);
                else rp.ready[xp0 + me] = nb;
            }
        }
        for (uint32_t t = tid; t < T; t += TA_THREADS)
            tp.fills[(uint64_t)t * tp.W + w] = t < H ? 0u : l.base[t] - (uint32_t)tp.toff[t];
    } else {
        // ================= consumer waves =================
        const uint32_t cw = (tid - TA_THREADS) >> 6, lane = tid & 63;
        const uint32_t nq = P > cw ? (P - cw + RES_CW - 1) / RES_CW : 0;  // producers of this wave
        const uint32_t q = cw + lane * RES_CW;                             // this lane's producer
        uint32_t *wpre = s_wpre[cw], *wbeg = s_wbeg[cw], *wsb = s_wsb[cw];
        uint32_t nx = 0, idle = 0;
        uint64_t last = wall_clock64();
        for (;;) {
            const bool mine = lane < nq && nx < nb && !(tp.debug & 4096);  // 4096: experiment, no consumers
            if (!__any(mine)) break;
            bool av = false;
            uint32_t beg = 0, cnt = 0, sbq = 0;
            if (mine && ld_sc1(&rp.ready[xp0 + q]) > nx) {
                sbq = (uint32_t)((xp0 + q) * K + nx % K);
                beg = ld_sc1(&rp.hdr[(uint64_t)sbq * RES_HDR + me]);
                cnt = ld_sc1(&rp.hdr[(uint64_t)sbq * RES_HDR + me + 1]) - beg;
                av = true;
            }
            uint32_t inc = cnt;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(inc, off, 64);
                if ((int)lane >= off) inc += y;
            }
            const uint32_t total = __shfl(inc, 63, 64);
            if (total) {
                wpre[lane] = inc - cnt;
                wbeg[lane] = beg;
                wsb[lane] = sbq;
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
                for (uint32_t i0 = 0; i0 < total; i0 += 64 * RES_CU) {
                    uint32_t loc[RES_CU];
                    double v[RES_CU][NV > 0 ? NV : 1];
#pragma unroll
                    for (int u = 0; u < RES_CU; u++) {
                        const uint32_t i = i0 + u * 64 + lane;
                        loc[u] = 0xffffffffu;
                        if (i < total && !(tp.debug & 256)) {  // 256: experiment, consumers only acknowledge
                            uint32_t k = 0;
#pragma unroll
                            for (uint32_t stp = 8; stp; stp >>= 1)
                                if (k + stp < nq && wpre[k + stp] <= i) k += stp;
                            const uint64_t e = (uint64_t)wsb[k] * CAP + wbeg[k] + (i - wpre[k]);
                            loc[u] = ld_sc1(rp.skeys + e);
#pragma unroll
                            for (int s = 0; s < NV; s++) v[u][s] = ld_sc1(rp.svals + e);
                        }
                    }
#pragma unroll
                    for (int u = 0; u < RES_CU; u++)
                        if (loc[u] != 0xffffffffu) reduce_entry<NV>(fr, tp, tl, loc[u], 0xfu, v[u]);
                }
                __builtin_amdgcn_wave_barrier();
            }
            if (av) {
                nx++;
                if (rp.wt) st_sc1(&rp.cons[(xp0 + q) * P + me], nx);
                else rp.cons[(xp0 + q) * P + me] = nx;
            }
            if (__any(av)) {
                idle = 0;
                if (lane == 0) last = wall_clock64();
            } else {
                __builtin_amdgcn_s_sleep(4);
                if ((++idle & 15) == 0) {
                    uint32_t stop = 0;
                    if (lane == 0) {
                        if (s_ctl[3] || ld_sc1(&rp.ctl[0]) == RES_ABORT) stop = 1;
                        else if (wall_clock64() - last > rp.timeout) {
                            atomicCAS(&rp.ctl[0], RES_RUNNING, RES_ABORT);
                            stop = 1;
                        }
                        if (stop) s_ctl[3] = 1;
                    }
                    if (__shfl(stop, 0, 64)) break;
                }
            }
        }
    }
    // commit when every workgroup finished; abort otherwise
    __syncthreads();
    if (tid == 0) {
        if (!s_ctl[3]) {
            if (s_ctl[7]) atomicCAS(&rp.ctl[0], RES_RUNNING, RES_ABORT);
            atomicAdd(&rp.ctl[1], 1u);
            const uint64_t t0 = wall_clock64();
            for (;;) {
                if (ld_sc1(&rp.ctl[1]) >= rp.G) {
                    atomicCAS(&rp.ctl[0], RES_RUNNING, RES_COMMIT);
                    break;
                }
                if (ld_sc1(&rp.ctl[0]) != RES_RUNNING) break;
                if (wall_clock64() - t0 > rp.timeout) {
                    atomicCAS(&rp.ctl[0], RES_RUNNING, RES_ABORT);
                    break;
                }
                __builtin_amdgcn_s_sleep(8);
            }
        }
        s_ctl[2] = ld_sc1(&rp.ctl[0]) == RES_COMMIT ? 1u : 0u;
    }
    __syncthreads();
    if (!s_ctl[2]) return;
    // flush the owner tiles
    const uint32_t Sp = TPW << s_log2;
    #pragma unroll
    for (int k = 0; k < MAX_FUSED_AGGS; k++) {
        if (k >= fr.na) break;
        for (uint32_t i = tid; i < Sp; i += RES_THREADS) {
            const uint32_t id = me * TPW + (i >> s_log2);
            if (id >= H) continue;
            const uint64_t c = ((uint64_t)rp.tile_of[id] << s_log2) | (i & smask);
            if (c >= tp.cells) continue;
            if (fr.a[k].kind == VH_AGG_COUNT) {
                const uint32_t v = reinterpret_cast<const uint32_t *>(tl + fr.a[k].lds_off)[i];
                if (v) atomicAdd((unsigned long long *)fr.a[k].grid + c, (unsigned long long)v);
            } else {
                const double v = reinterpret_cast<const double *>(tl + fr.a[k].lds_off)[i];
                if (v != 0.0) atomicAdd(reinterpret_cast<double *>(fr.a[k].grid) + c, v);
            }
        }
    }
    const uint32_t novf = min(s_ctl[6], RES_OVF);
    for (uint32_t i = tid; i < novf; i += RES_THREADS) {
        const uint32_t kk = ovf_key[i];
        const uint64_t c = ((uint64_t)rp.tile_of[kk >> 16] << s_log2) | (kk & smask);
        double v[NV > 0 ? NV : 1];
        if constexpr (NV > 0) v[0] = ovf_val[i];
        apply_row_global<NV>(fa, tp, c, count_mask, keyed_slot_of, v);
    }
}

// fast: 0 = generic kernel, 1 = fast kernel one batch per commit, 2 = fast kernel with
// fast_sb(NV) batches per commit (when its LDS fits)
template <int ND, int NV>
static void launch_scatter(int fast, unsigned grid, size_t lds, const BinPlan &plan, const FusedAggs &fa,
                           const TileParams &tp, uint64_t n) {
    if constexpr (ND > 0) {
        if (fast == 2) {
            hipLaunchKernelGGL((k_tile_scatter_f64<ND, NV, fast_sb(NV)>), dim3(grid), dim3(TA_THREADS), lds, stream(), plan, fa, tp, n);
            return;
        }
        if (fast == 1) {
            hipLaunchKernelGGL((k_tile_scatter_f64<ND, NV, 1>), dim3(grid), dim3(TA_THREADS), lds, stream(), plan, fa, tp, n);
            return;
        }
    }
    hipLaunchKernelGGL((k_tile_scatter<ND, NV>), dim3(grid), dim3(TA_THREADS), lds, stream(), plan, fa, tp, n);
}

template <int NV>
static void launch_scatter_nd(int nd, int fast, unsigned grid, size_t lds, const BinPlan &plan, const FusedAggs &fa,
                              const TileParams &tp, uint64_t n) {
    switch (nd) {
    case 1: launch_scatter<1, NV>(fast, grid, lds, plan, fa, tp, n); break;
    case 2: launch_scatter<2, NV>(fast, grid, lds, plan, fa, tp, n); break;
    case 3: launch_scatter<3, NV>(fast, grid, lds, plan, fa, tp, n); break;
    case -1: launch_scatter<-1, NV>(0, grid, lds, plan, fa, tp, n); break;
    default: launch_scatter<0, NV>(0, grid, lds, plan, fa, tp, n);
    }
}

static bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

template <int ND, int NV> static int scatter_blocks_per_cu(int fast, size_t lds) {
    int nb = 0;
    if constexpr (ND > 0) {
        if (fast == 2) {
            VH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tile_scatter_f64<ND, NV, fast_sb(NV)>, TA_THREADS, lds));
            return nb;
        }
        if (fast == 1) {
            VH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tile_scatter_f64<ND, NV, 1>, TA_THREADS, lds));
            return nb;
        }
    }
    VH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tile_scatter<ND, NV>, TA_THREADS, lds));
    return nb;
}

template <int NV> static int scatter_blocks_per_cu_nd(int nd, int fast, size_t lds) {
    switch (nd) {
    case 1: return scatter_blocks_per_cu<1, NV>(fast, lds);
    case 2: return scatter_blocks_per_cu<2, NV>(fast, lds);
    case 3: return scatter_blocks_per_cu<3, NV>(fast, lds);
    case -1: return scatter_blocks_per_cu<-1, NV>(0, lds);
    default: return scatter_blocks_per_cu<0, NV>(0, lds);
    }
}

// value-dtype combinations with their own ordinal kernel (0: float64; h2o's int8 / float32
// sums; others take the run-time-switch kernel, -1)
template <int NV, int SB, bool SET, typename F> static void ord_by_dts(int dt0, int dt1, F &&f) {
#define VH_ORD_DT(a, b) if (dt0 == (a) && (NV < 2 || dt1 == (b))) return f(k_tile_scatter_ord<NV, SB, SET, (a), NV < 2 ? VH_F64 : (b)>);
    VH_ORD_DT(VH_F64, VH_F64)
    if constexpr (!SET) {
        VH_ORD_DT(VH_I8, VH_I8)
        VH_ORD_DT(VH_I8, VH_F32)
        VH_ORD_DT(VH_F32, VH_I8)
        VH_ORD_DT(VH_F32, VH_F32)
        VH_ORD_DT(VH_I32, VH_I32)
        VH_ORD_DT(VH_I32, VH_F64)
        VH_ORD_DT(VH_F32, VH_F64)
    }
#undef VH_ORD_DT
    f(k_tile_scatter_ord<NV, SB, SET, -1, -1>);
}
template <bool SET> static const void *ord_kernel_t(int nv, int fast_mode, int dt0, int dt1) {
    const void *k = nullptr;
    auto take = [&](auto kern) { k = reinterpret_cast<const void *>(kern); };
    if (nv == 0) ord_by_dts<0, 1, SET>(VH_F64, VH_F64, take);
    else if (nv == 1) {
        if (fast_mode == 2) ord_by_dts<1, fast_sb(1), SET>(dt0, dt1, take);
        else ord_by_dts<1, 1, SET>(dt0, dt1, take);
    } else {
        if (fast_mode == 2) ord_by_dts<2, fast_sb(2), SET>(dt0, dt1, take);
        else ord_by_dts<2, 1, SET>(dt0, dt1, take);
    }
    return k;
}
static const void *ord_kernel(int nv, int fast_mode, bool set, int dt0, int dt1) {
    return set ? ord_kernel_t<true>(nv, fast_mode, dt0, dt1) : ord_kernel_t<false>(nv, fast_mode, dt0, dt1);
}

// 0 = not tiled (caller takes another path), 1 = done, 2 = the XCD-resident launch aborted
// (nothing written to the grids): run again on the two-pass path
static int try_tiled_impl(const BinPlan &plan, const FusedAggs &fa_in, uint64_t n, uint64_t cells, int nd_f64,
                          Workspace &ws, bool allow_res);
static bool try_tiled_once(const BinPlan &plan, const FusedAggs &fa_in, uint64_t n, uint64_t cells, int nd_f64,
                           Workspace &ws) {
    const int r = try_tiled_impl(plan, fa_in, n, cells, nd_f64, ws, true);
    if (r == 2) return try_tiled_impl(plan, fa_in, n, cells, nd_f64, ws, false) == 1;
    return r == 1;
}

// the fast ordinal pass A applies: one native int32 BinnerOrdinal without mask, every
// sum a 16-byte aligned float64 column, no aggregator masks, no counts of other columns
static bool ord_fast_ok(const BinPlan &plan, const FusedAggs &fa) {
    if (plan.nb != 1) return false;
    const BinnerDev &b = plan.b[0];
    const bool set_ok = b.kind == 2 && (b.dtype == VH_I32 || b.dtype == VH_U32) && !b.set.wide;
    if (!(b.kind == 1 && b.dtype == VH_I32) && !set_ok) return false;
    if (b.flip || b.mask || (reinterpret_cast<uintptr_t>(b.data) & 7)) return false;
    for (int k = 0; k < fa.na; k++) {
        const FusedAgg &a = fa.a[k];
        if (a.mask) return false;
        if (a.kind != VH_AGG_COUNT) {
            // any native value dtype; pair loads need 2 x itemsize alignment
            if (!a.data) return false;
            const int isz = a.dtype == VH_F64 ? 16 : 2 * dtype_itemsize(a.dtype);
            if (reinterpret_cast<uintptr_t>(a.data) % isz) return false;
        } else if (a.data) {
            bool keyed = false;  // count(v) of a summed column rides on that sum's value
            for (int j = 0; j < fa.na; j++)
                if (fa.a[j].kind != VH_AGG_COUNT && fa.a[j].data == a.data) keyed = true;
            if (!keyed) return false;
        }
    }
    return true;
}

bool try_tiled(const BinPlan &plan, const FusedAggs &fa_in, uint64_t n, uint64_t cells, int nd_f64, Workspace &ws) {
    if (n < (1u << 20) || cells >= (1ull << 40)) return false;
    if ((n & 1) && !fa_in.generic_vals && (nd_f64 > 0 || ord_fast_ok(plan, fa_in))) {
        // the fast pass A reads row pairs: tile all rows but the last, which takes the
        // global-atomic path
        if (!try_tiled_once(plan, fa_in, n - 1, cells, nd_f64, ws)) return false;
        BinPlan p1 = plan;
        FusedAggs f1 = fa_in;
        for (int d = 0; d < p1.nb; d++) {
            p1.b[d].data = static_cast<const char *>(p1.b[d].data) + (n - 1) * dtype_itemsize(p1.b[d].dtype);
            if (p1.b[d].mask) p1.b[d].mask += n - 1;
        }
        for (int k = 0; k < f1.na; k++) {
            if (f1.a[k].data) f1.a[k].data += n - 1;
            if (f1.a[k].mask) f1.a[k].mask += n - 1;
        }
        launch_fused(p1, f1, 1, cells, nd_f64, ws);
        return true;
    }
    return try_tiled_once(plan, fa_in, n, cells, nd_f64, ws);
}

// Partition scratch shared by every grid of a device: a 1e9-row count+sum needs ~10 GB of
// regions, which a per-grid buffer would hipMalloc/hipFree for every query (a grid lives
// for one query).  Held under the device's lock while a bin is enqueued; reuse is ordered
// by the library stream.
struct TileScratch {
    std::mutex mu;
    DevBuf entries, values, meta, res;
};

// XCD-resident path switch (opt-in; measured slower than the two-pass path, DESIGN.md
// §5.1): VH_RESIDENT=0 off (default), 1 on (slot data and flags by plain stores kept in the
// XCD's L2), 2 on with write-through (`sc1`) stores; an aborted launch turns it off for the
// process
static std::atomic<bool> g_res_off{false};
static int res_mode() {
    if (g_res_off.load()) return 0;
    const char *e = getenv("VH_RESIDENT");
    return e ? atoi(e) : 0;
}
static bool getenv_flag_off(const char *name) {  // NAME=0 turns a default-on path off (A/B runs)
    const char *e = getenv(name);
    return e && atoi(e) == 0;
}
static uint64_t res_min_rows() {  // VH_RES_MIN_ROWS: tests run the path at small sizes
    const char *e = getenv("VH_RES_MIN_ROWS");
    return e ? strtoull(e, nullptr, 10) : (1ull << 24);
}
static uint64_t wall_clock_khz() {
    static std::mutex mu;
    static std::map<int, uint64_t> m;
    std::lock_guard<std::mutex> lk(mu);
    const int dev = current_device();
    auto it = m.find(dev);
    if (it != m.end()) return it->second;
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
    m[dev] = (uint64_t)khz;
    return (uint64_t)khz;
}
static TileScratch &tile_scratch() {
    static std::mutex g;
    static std::map<int, std::unique_ptr<TileScratch>> m;
    std::lock_guard<std::mutex> lk(g);
    auto &p = m[current_device()];
    if (!p) p = std::make_unique<TileScratch>();
    return *p;
}

static int try_tiled_impl(const BinPlan &plan, const FusedAggs &fa_in, uint64_t n, uint64_t cells, int nd_f64,
                          Workspace &, bool allow_res) {
    TileScratch &ws = tile_scratch();
    std::lock_guard<std::mutex> ws_lock(ws.mu);
    TileParams tp{};
    if (const char *dbg = getenv("VH_TILE_DEBUG")) tp.debug = (uint32_t)atoi(dbg);
    // carried values: one slot per distinct value column (sum / min / max of one column share
    // it: same data, mask, dtype and integer-sum encoding); counts keyed on a matching value
    int nv = 0;
    for (int k = 0; k < fa_in.na; k++) {
        tp.val_slot[k] = -1;
        tp.cnt_slot[k] = CNT_ALWAYS;
        if (fa_in.a[k].kind == VH_AGG_COUNT) continue;
        for (int j = 0; j < k && tp.val_slot[k] < 0; j++)
            if (tp.val_slot[j] >= 0 && same_value_slot(fa_in.a[j], fa_in.a[k])) tp.val_slot[k] = tp.val_slot[j];
        if (tp.val_slot[k] < 0) tp.val_slot[k] = nv++;
    }
    if (nv > 2) return false;
    bool flags_mode = false;
    for (int k = 0; k < fa_in.na; k++) {
        const FusedAgg &a = fa_in.a[k];
        if (a.kind != VH_AGG_COUNT || (!a.data && !a.mask)) continue;
        if (!a.mask && a.dtype != VH_F64 && a.dtype != VH_F32) continue;  // integers: never NaN
        tp.cnt_slot[k] = CNT_FLAG;
        for (int j = 0; j < fa_in.na; j++)
            if (fa_in.a[j].kind != VH_AGG_COUNT && fa_in.a[j].data == a.data && fa_in.a[j].mask == a.mask && a.data &&
                !fa_in.a[j].vint)
                tp.cnt_slot[k] = tp.val_slot[j];
        if (tp.cnt_slot[k] == CNT_FLAG) flags_mode = true;
    }
    if (flags_mode)
        for (int k = 0; k < fa_in.na; k++)
            if (fa_in.a[k].kind == VH_AGG_COUNT) tp.cnt_slot[k] = CNT_FLAG;
    uint64_t per_cell = 0;
    for (int k = 0; k < fa_in.na; k++) per_cell += fa_in.a[k].kind == VH_AGG_COUNT ? 4 : 8;
    uint32_t s_log2 = 0;
    while (s_log2 < 16 && ((uint64_t)2 << s_log2) * per_cell <= TILE_LDS_BUDGET) s_log2++;
    const uint64_t S = 1ull << s_log2;
    const uint64_t T64 = (cells + S - 1) / S;
    if (T64 > TILE_MAX_TILES || T64 < 2) return false;
    const uint32_t T = (uint32_t)T64;

    FusedAggs fa = fa_in;
    uint64_t off = 0;
    for (int k = 0; k < fa.na; k++) {
        off = (off + 7) & ~uint64_t(7);
        fa.a[k].lds_off = (uint32_t)off;
        off += S * (fa.a[k].kind == VH_AGG_COUNT ? 4 : 8);
    }
    const uint64_t lds_b = (off + 15) & ~uint64_t(15);
    fa.lds_words = (uint32_t)(lds_b / 4);
    hipStream_t st = stream();

    // ---- sample
    // the fast pass A: native f64 binners and sums, no masks, 16-byte aligned columns
    bool fast = nd_f64 > 0 && !flags_mode;
    // generic pass A flavour: -1 = a set-ordinal binner (per-row form), 0 = hoisted dispatch
    bool has_set = false;
    for (int d = 0; d < plan.nb; d++) has_set = has_set || plan.b[d].kind == 2;
    const int nd_k = nd_f64 > 0 ? nd_f64 : (has_set ? -1 : 0);
    for (int d = 0; d < plan.nb && fast; d++) fast = !plan.b[d].mask && aligned16(plan.b[d].data);
    for (int k = 0; k < fa.na; k++) {
        if (fa.a[k].mask) fast = false;
        if (fa.a[k].kind != VH_AGG_COUNT) {
            tp.vdata[tp.val_slot[k]] = fa.a[k].data;
            fast = fast && fa.a[k].data && fa.a[k].dtype == VH_F64 && aligned16(fa.a[k].data);
        }
        if (fa.a[k].kind == VH_AGG_COUNT && fa.a[k].data && fa.a[k].dtype != VH_F64) fast = false;
    }
    const bool ord = !fast && n % 2 == 0 && ord_fast_ok(plan, fa);
    tp.vdt[0] = tp.vdt[1] = VH_F64;
    if (ord) for (int k = 0; k < fa.na; k++)
        if (fa.a[k].kind != VH_AGG_COUNT) {
            tp.vdata[tp.val_slot[k]] = fa.a[k].data;
            tp.vdt[tp.val_slot[k]] = fa.a[k].dtype;
        }
    // fast kernel: several batches per commit when that staging fits the LDS
    const int fast_mode = !(fast || ord) ? 0 : fast_lds_bytes(nv, T, (uint32_t)(fast_sb(nv) * TA_BATCH)) <= LDS_MAX_BYTES ? 2 : 1;
    const size_t lds_a = fast_mode == 2   ? fast_lds_bytes(nv, T, (uint32_t)(fast_sb(nv) * TA_BATCH))
                         : fast_mode == 1 ? fast_lds_bytes(nv, T, (uint32_t)TA_BATCH)
                                          : scatter_lds_bytes(nv, T);
    if (lds_a > LDS_MAX_BYTES) return false;  // very many tiles: the global-atomic path
    int bpc;
    {
        static std::mutex mu;
        static std::map<std::tuple<int, int, int, int, size_t>, int> cache;
        std::lock_guard<std::mutex> lk(mu);
        const auto key = std::make_tuple(current_device(), ord ? (has_set ? -3 : -2) - 4 * (tp.vdt[0] + 32 * tp.vdt[1]) : nd_k, nv, fast_mode, lds_a);
        auto it = cache.find(key);
        if (it == cache.end()) {
            int v = 0;
            if (ord) {
                const void *kf = ord_kernel(nv, fast_mode, has_set, tp.vdt[0], tp.vdt[1]);
                VH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, kf, TA_THREADS, lds_a));
            } else {
                v = nv == 0 ? scatter_blocks_per_cu_nd<0>(nd_k, fast_mode, lds_a)
                            : nv == 1 ? scatter_blocks_per_cu_nd<1>(nd_k, fast_mode, lds_a)
                                      : scatter_blocks_per_cu_nd<2>(nd_k, fast_mode, lds_a);
            }
            it = cache.emplace(key, v).first;
        }
        bpc = it->second;
    }
    bpc = std::max(1, std::min(bpc, TA_WG_PER_CU));
    // XCD-resident variant: the fast f64 pass A with <= 1 value slot, one workgroup per CU,
    // P owners per XCD holding TPW tiles each in LDS (resident_lds_bytes + static arrays)
    bool res_kinds = true;  // the resident launch applies counts and sums only
    for (int k = 0; k < fa.na; k++) res_kinds = res_kinds && !is_minmax(fa.a[k].kind);
    const int rmode = allow_res && res_kinds && fast && nv <= 1 && nd_f64 >= 1 && nd_f64 <= 3 && n >= res_min_rows() ? res_mode() : 0;
    uint32_t rP = 0, rTPW = 0;
    if (rmode && cu_count() % 8 == 0 && cu_count() / 8 <= (int)RES_HDR - 1) {
        rP = (uint32_t)cu_count() / 8;
        for (uint32_t k = 1; (S * k) <= 65536; k++) {
            const uint64_t words = ((S * k * per_cell + 15) & ~uint64_t(15)) / 4;
            if (resident_lds_bytes((uint32_t)words, nv, T) + 4096 > LDS_MAX_BYTES) break;
            rTPW = k;
        }
    }
    bool res = rTPW > 0;
    const uint32_t W = res ? 8 * rP : std::min<uint32_t>(1024, (uint32_t)cu_count() * bpc);
    // pass-B work units: sum over tiles of ceil(e_t / target) <= T + 4 cu (target = n / 4 cu)
    const uint64_t max_units = (uint64_t)T + 4 * (uint64_t)cu_count() + 16;
    DevBuf &meta = ws.meta;
    const uint64_t meta_bytes = 8 * (uint64_t)T /*hist*/ + 4 * (uint64_t)T /*cap*/ + 8 * (uint64_t)T /*toff*/ +
                                4 * (uint64_t)T * W /*fills*/ + 16 * max_units /*units*/ + 8 * (uint64_t)T /*tmap, tile_of*/ + 256;
    meta.ensure(meta_bytes);
    unsigned char *mb = meta.as<unsigned char>();
    uint64_t *d_hist = reinterpret_cast<uint64_t *>(mb);
    uint64_t *d_toff = d_hist + T;
    uint32_t *d_cap = reinterpret_cast<uint32_t *>(d_toff + T);
    uint32_t *d_fills = d_cap + ((T + 3) & ~3u);
    WorkUnit *d_units = reinterpret_cast<WorkUnit *>(d_fills + (uint64_t)T * W + 4 - ((uint64_t)T * W) % 4);
    uint32_t *d_tmap = reinterpret_cast<uint32_t *>(d_units + max_units);
    uint32_t *d_tile_of = d_tmap + T;
    const uint64_t nb = (n + TA_BATCH - 1) / TA_BATCH;
    const uint64_t sblocks = std::min<uint64_t>(nb, SAMPLE_BLOCKS);
    const uint64_t bstride = std::max<uint64_t>(TA_BATCH, (n / sblocks));
    VH_HIP(hipMemsetAsync(d_hist, 0, 8 * (uint64_t)T, st));
    {
        TimedScope ts("tile_sample");
        const size_t lds = 4 * (size_t)T;
        switch (nd_f64) {
        case 1: hipLaunchKernelGGL(k_tile_sample<1>, dim3(sblocks), dim3(TA_THREADS), lds, st, plan, n, s_log2, T, bstride, d_hist); break;
        case 2: hipLaunchKernelGGL(k_tile_sample<2>, dim3(sblocks), dim3(TA_THREADS), lds, st, plan, n, s_log2, T, bstride, d_hist); break;
        case 3: hipLaunchKernelGGL(k_tile_sample<3>, dim3(sblocks), dim3(TA_THREADS), lds, st, plan, n, s_log2, T, bstride, d_hist); break;
        default: hipLaunchKernelGGL(k_tile_sample<0>, dim3(sblocks), dim3(TA_THREADS), lds, st, plan, n, s_log2, T, bstride, d_hist);
        }
        VH_HIP(hipGetLastError());
    }
    std::vector<uint64_t> hist(T);
    VH_HIP(hipMemcpyAsync(hist.data(), d_hist, 8 * (uint64_t)T, hipMemcpyDeviceToHost, st));
    VH_HIP(hipStreamSynchronize(st));
    uint64_t sampled = 0;
    for (auto h : hist) sampled += h;
    if (!sampled) return false;

    // ---- resident plan: the H densest tiles get region ids 0..H-1 (owner o holds ids
    // o*TPW .. o*TPW+TPW-1, dense and sparse ranks interleaved), cold tiles H..T-1
    std::vector<uint32_t> tile_of(T), tmap(T);
    for (uint32_t t = 0; t < T; t++) tile_of[t] = t;
    uint32_t H = 0;
    if (res) {
        std::vector<uint32_t> order(T);
        for (uint32_t t = 0; t < T; t++) order[t] = t;
        std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return hist[a] > hist[b]; });
        H = std::min<uint32_t>(T, rP * rTPW);
        uint64_t hot_mass = 0;
        for (uint32_t r = 0; r < H; r++) hot_mass += hist[order[r]];
        if (hot_mass * 4 < sampled) res = false;  // < 25 % of the rows would stay on chip
    }
    if (res) {
        std::vector<uint32_t> hot_ids(H);
        for (uint32_t r = 0; r < H; r++) {
            uint32_t id = r;
            if (H == rP * rTPW) {  // every owner full: balance dense and sparse tiles
                const uint32_t j = r / rP, q = r % rP;
                const uint32_t o = (j & 1) ? rP - 1 - q : q;
                id = o * rTPW + j;
            }
            hot_ids[r] = id;
        }
        std::vector<uint32_t> order(T);
        for (uint32_t t = 0; t < T; t++) order[t] = t;
        std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return hist[a] > hist[b]; });
        std::vector<char> hot(T, 0);
        for (uint32_t r = 0; r < H; r++) {
            tile_of[hot_ids[r]] = order[r];
            hot[order[r]] = 1;
        }
        uint32_t nid = H;
        for (uint32_t t = 0; t < T; t++)
            if (!hot[t]) tile_of[nid++] = t;
        for (uint32_t id = 0; id < T; id++) tmap[tile_of[id]] = id;
    }

    // ---- region capacities per workgroup (by region id; hot ids have none)
    const uint64_t rows_per_wg = ((n + W - 1) / W + TA_BATCH - 1) / TA_BATCH * TA_BATCH;
    std::vector<uint32_t> cap(T);
    std::vector<uint64_t> toff(T);
    uint64_t stride = 0;
    for (uint32_t id = 0; id < T; id++) {
        const uint32_t t = tile_of[id];
        const double e = (double)rows_per_wg * (double)hist[t] / (double)sampled;
        uint64_t c = (uint64_t)(e * 1.04 + 6.0 * std::sqrt(e + 1.0)) + 32;
        c = std::min<uint64_t>((c + 7) & ~uint64_t(7), rows_per_wg + 8);
        if (res && id < H) c = 0;
        cap[id] = (uint32_t)c;
        toff[id] = stride;
        stride += c;
    }
    // pass A keeps region positions in u32 (destination | overflow bit)
    if (stride + rows_per_wg >= (uint64_t)DEST_OVERFLOW) return false;
    const uint64_t total = stride * W;
    const int ebytes = flags_mode ? 4 : 2;
    ws.entries.ensure(total * ebytes);
    // 4-byte value slots when every summed column of a generic plan is <= 4 bytes (exact)
    bool vnarrow = fa.generic_vals && nv > 0 && !fast && !getenv_flag_off("VH_TILE_NARROW");
    uint32_t vfloat = 0, vsigned = 0;
    for (int k = 0; k < fa.na && vnarrow; k++) {
        if (fa.a[k].kind == VH_AGG_COUNT) continue;
        const int dt = fa.a[k].dtype, s = tp.val_slot[k];
        if (dtype_itemsize(dt) > 4) vnarrow = false;
        if (dt == VH_F32) vfloat |= 1u << s;
        if (dt == VH_I32 || dt == VH_I16 || dt == VH_I8) vsigned |= 1u << s;
    }
    if (nv) ws.values.ensure(total * (vnarrow ? 4 : 8) * nv + 64);
    tp.vnarrow = vnarrow ? 1u : 0u;
    tp.vfloat = vfloat;
    tp.vsigned = vsigned;
    tp.s_log2 = s_log2;
    tp.ntiles = T;
    tp.flags_mode = flags_mode ? 1 : 0;
    tp.nvals = nv;
    tp.cells = cells;
    tp.W = W;
    tp.rows_per_wg = rows_per_wg;
    tp.wg_stride = stride;
    tp.cap = d_cap;
    tp.toff = d_toff;
    tp.fills = d_fills;
    tp.entries = ws.entries.ptr;
    for (int s = 0; s < nv; s++)
        tp.values[s] = vnarrow ? reinterpret_cast<double *>(ws.values.as<uint32_t>() + (uint64_t)s * total)
                               : ws.values.as<double>() + (uint64_t)s * total;
    VH_HIP(hipMemcpyAsync(d_cap, cap.data(), 4 * (uint64_t)T, hipMemcpyHostToDevice, st));
    VH_HIP(hipMemcpyAsync(d_toff, toff.data(), 8 * (uint64_t)T, hipMemcpyHostToDevice, st));

    // ---- pass B work units: tiles split over ranges of pass-A workgroups by expected size
    std::vector<WorkUnit> units;
    const double target = std::max(1.0, (double)n / ((double)cu_count() * 4));
    for (uint32_t id = res ? H : 0; id < T; id++) {
        const double e = (double)n * (double)hist[tile_of[id]] / (double)sampled;
        uint32_t g = (uint32_t)std::min<double>(W, std::max(1.0, std::ceil(e / target)));
        for (uint32_t k = 0; k < g; k++) units.push_back({id, (uint32_t)((uint64_t)W * k / g), (uint32_t)((uint64_t)W * (k + 1) / g), 0});
    }
    if (units.size() > max_units) fail(VH_ERR_RUNTIME, "tiled binning: work-unit table overflow");
    if (!units.empty())
        VH_HIP(hipMemcpyAsync(d_units, units.data(), sizeof(WorkUnit) * units.size(), hipMemcpyHostToDevice, st));

    if (res) {
        // ---- XCD-resident launch (replaces pass A; pass B only for the cold tiles)
        const uint32_t P = rP, K = VH_RES_K, G = 8 * rP;
        FusedAggs fr = fa;  // owner tiles: TPW * S cells per aggregator
        uint64_t roff = 0;
        for (int k = 0; k < fr.na; k++) {
            roff = (roff + 7) & ~uint64_t(7);
            fr.a[k].lds_off = (uint32_t)roff;
            roff += S * rTPW * (fr.a[k].kind == VH_AGG_COUNT ? 4 : 8);
        }
        fr.lds_words = (uint32_t)(((roff + 15) & ~uint64_t(15)) / 4);
        const uint64_t ctl_b = 256, ready_b = 4ull * 8 * P, cons_b = 4ull * 8 * P * P;
        const uint64_t hdr_b = 4ull * 8 * P * K * RES_HDR, keys_b = 4ull * 8 * P * K * TA_BATCH;
        const uint64_t vals_b = 8ull * 8 * P * K * TA_BATCH * (nv ? 1 : 0);
        const uint64_t okey_b = 4ull * G * RES_OVF, oval_b = 8ull * G * RES_OVF;
        auto al = [](uint64_t b) { return (b + 255) & ~uint64_t(255); };
        const uint64_t flags_b = al(ctl_b) + al(ready_b) + al(cons_b);
        ws.res.ensure(flags_b + al(hdr_b) + al(keys_b) + al(vals_b) + al(okey_b) + al(oval_b));
        unsigned char *rb = ws.res.as<unsigned char>();
        ResidentParams rp{};
        rp.P = P;
        rp.K = K;
        rp.H = H;
        rp.TPW = rTPW;
        rp.nb = (uint32_t)(rows_per_wg / TA_BATCH);
        rp.G = G;
        rp.wt = rmode == 2 ? 1u : 0u;
        rp.timeout = 200 * wall_clock_khz();  // 200 ms without progress
        rp.ctl = reinterpret_cast<uint32_t *>(rb);
        rp.ready = reinterpret_cast<uint32_t *>(rb + al(ctl_b));
        rp.cons = reinterpret_cast<uint32_t *>(rb + al(ctl_b) + al(ready_b));
        unsigned char *q = rb + flags_b;
        rp.hdr = reinterpret_cast<uint32_t *>(q);
        q += al(hdr_b);
        rp.skeys = reinterpret_cast<uint32_t *>(q);
        q += al(keys_b);
        rp.svals = reinterpret_cast<double *>(q);
        q += al(vals_b);
        rp.ovf_key = reinterpret_cast<uint32_t *>(q);
        q += al(okey_b);
        rp.ovf_val = reinterpret_cast<double *>(q);
        rp.tmap = d_tmap;
        rp.tile_of = d_tile_of;
        tp.tile_of = d_tile_of;
        tp.abort_word = rp.ctl;
        VH_HIP(hipMemcpyAsync(d_tmap, tmap.data(), 4 * (uint64_t)T, hipMemcpyHostToDevice, st));
        VH_HIP(hipMemcpyAsync(d_tile_of, tile_of.data(), 4 * (uint64_t)T, hipMemcpyHostToDevice, st));
        VH_HIP(hipMemsetAsync(rb, 0, flags_b, st));
        const size_t lds = resident_lds_bytes(fr.lds_words, nv, T);
        {
            TimedScope ts("tile_resident");
            switch (nd_f64 * 2 + nv) {
            case 2: hipLaunchKernelGGL((k_tile_resident<1, 0>), dim3(G), dim3(RES_THREADS), lds, st, plan, fa, fr, tp, rp, n); break;
            case 3: hipLaunchKernelGGL((k_tile_resident<1, 1>), dim3(G), dim3(RES_THREADS), lds, st, plan, fa, fr, tp, rp, n); break;
            case 4: hipLaunchKernelGGL((k_tile_resident<2, 0>), dim3(G), dim3(RES_THREADS), lds, st, plan, fa, fr, tp, rp, n); break;
            case 5: hipLaunchKernelGGL((k_tile_resident<2, 1>), dim3(G), dim3(RES_THREADS), lds, st, plan, fa, fr, tp, rp, n); break;
            case 6: hipLaunchKernelGGL((k_tile_resident<3, 0>), dim3(G), dim3(RES_THREADS), lds, st, plan, fa, fr, tp, rp, n); break;
            default: hipLaunchKernelGGL((k_tile_resident<3, 1>), dim3(G), dim3(RES_THREADS), lds, st, plan, fa, fr, tp, rp, n);
            }
            VH_HIP(hipGetLastError());
        }
        if (!units.empty()) {
            TimedScope ts("tile_reduce");
            const unsigned g = (unsigned)units.size();
            if (nv == 0) hipLaunchKernelGGL(k_tile_reduce<0>, dim3(g), dim3(TB_THREADS), lds_b, st, fa, tp, d_units);
            else hipLaunchKernelGGL(k_tile_reduce<1>, dim3(g), dim3(TB_THREADS), lds_b, st, fa, tp, d_units);
            VH_HIP(hipGetLastError());
        }
        uint32_t state = 0;
        VH_HIP(hipMemcpyAsync(&state, rp.ctl, 4, hipMemcpyDeviceToHost, st));
        VH_HIP(hipStreamSynchronize(st));
        if (state != RES_COMMIT) {
            g_res_off.store(true);
            fprintf(stderr, "vaexhip: XCD-resident tile launch not committed (state %u); two-pass tile path from now on\n",
                    state);
            return 2;
        }
        return 1;
    }

    // ---- pass A
    {
        TimedScope ts(fast ? "tile_scatter_f64" : ord ? (has_set ? "tile_scatter_set" : "tile_scatter_ord") : "tile_scatter");
        const size_t lds = lds_a;
        if (ord) {
            const void *kf = ord_kernel(nv, fast_mode, has_set, tp.vdt[0], tp.vdt[1]);
            void *args[] = {(void *)&plan, (void *)&fa, (void *)&tp, (void *)&n};
            VH_HIP(hipLaunchKernel(kf, dim3(W), dim3(TA_THREADS), args, lds, st));
        } else {
            switch (nv) {
            case 0: launch_scatter_nd<0>(nd_k, fast_mode, W, lds, plan, fa, tp, n); break;
            case 1: launch_scatter_nd<1>(nd_k, fast_mode, W, lds, plan, fa, tp, n); break;
            default: launch_scatter_nd<2>(nd_k, fast_mode, W, lds, plan, fa, tp, n);
            }
        }
        VH_HIP(hipGetLastError());
    }
    // ---- pass B
    {
        TimedScope ts("tile_reduce");
        const unsigned g = (unsigned)units.size();
        switch (nv) {
        case 0: hipLaunchKernelGGL(k_tile_reduce<0>, dim3(g), dim3(TB_THREADS), lds_b, st, fa, tp, d_units); break;
        case 1:
            if (vnarrow) hipLaunchKernelGGL((k_tile_reduce<1, true>), dim3(g), dim3(TB_THREADS), lds_b, st, fa, tp, d_units);
            else hipLaunchKernelGGL(k_tile_reduce<1>, dim3(g), dim3(TB_THREADS), lds_b, st, fa, tp, d_units);
            break;
        default:
            if (vnarrow) hipLaunchKernelGGL((k_tile_reduce<2, true>), dim3(g), dim3(TB_THREADS), lds_b, st, fa, tp, d_units);
            else hipLaunchKernelGGL(k_tile_reduce<2>, dim3(g), dim3(TB_THREADS), lds_b, st, fa, tp, d_units);
        }
        VH_HIP(hipGetLastError());
    }
    return true;
}

}  // namespace vh
