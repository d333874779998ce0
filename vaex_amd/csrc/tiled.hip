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
#include <cstring>
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
// 1: the prefetched batch lands before the commit's stores; 0: it stays in flight across the
// commit.  Round 6, both instantiations on one scratch: C2 count+sum pass A 6.126 vs 6.147 ms
// (profiles/r06_drain_inproc.txt); a run-time choice cost the count-only kernel 48 spilled VGPRs
#define VH_TA_DRAIN 1
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
    uint64_t rows_per_wg;      // upper bound (region sizing): batches of a workgroup x TA_BATCH
    uint64_t wg_stride;        // entries of one workgroup's regions
    const uint32_t *cap;       // [T]
    const uint64_t *toff;      // [T] region offset inside a workgroup's block
    uint32_t *fills;           // [T][W] entries produced (may exceed cap)
    // spill areas: rows past their (workgroup, tile) region go to their tile's spill area
    // (one atomic reservation per tile and commit), read by pass B like one more region;
    // past the spill area too (should not happen): global atomics
    uint32_t *spill_fill;         // [T] entries reserved (may exceed spill_cap)
    const uint32_t *spill_cap;    // [T]
    const uint64_t *spill_start;  // [T] entry index of the area, relative to spill_base
    uint64_t spill_base;          // first entry of the spill areas (after the W regions)
    void *entries;             // u16 / u32, W * wg_stride
    double *values[2];         // per value slot, W * wg_stride
    int32_t val_slot[MAX_FUSED_AGGS];  // sum agg k -> value slot
    int32_t cnt_slot[MAX_FUSED_AGGS];  // count agg k -> CNT_ALWAYS / CNT_FLAG / value slot
    const double *vdata[2];    // value slot -> source column (fast kernel)
    uint32_t debug;            // experiment switches (VH_TILE_DEBUG), ablation build only (DBG)
    // 4-byte value slots (every summed column <= 4 bytes: int8/16/32, uint8/16/32, bool,
    // float32 -- exact): slot s is float32 bits when bit s of vfloat is set, else the low 32
    // bits of the int64 slot, sign-extended back when bit s of vsigned is set
    uint32_t vnarrow, vfloat, vsigned;
    // two narrow slots in one array: values[0] holds, per 8 entries, their 8 slot-0 values then
    // their 8 slot-1 values (the narrow ordinal pass A with two carried columns: one write
    // stream, not two; pass B still reads each slot as 32 contiguous bytes)
    uint32_t vpacked;
    int32_t vdt[2];            // value slot -> column dtype (fast ordinal kernel)
    // min / max aggregator k: pass B flushes its LDS cells with native global atomics into
    // mmtmp[k] (cells x 4 or 8 bytes of the LDS cell form, identity-filled), merged into the
    // typed grid afterwards by k_mm_merge (a CAS per cell on 1- and 2-byte grids serialised
    // on the shared words)
    void *mmtmp[MAX_FUSED_AGGS];
    // pass B with min / max / moment: mgeneric, a moment other than 2 (per-entry form); mmk, bit
    // k set when aggregator k is a min / max (its cells are read ahead of each chunk)
    uint32_t mgeneric, mmk;
    // wide stream-out of the fast kernels (batch_commit_fast): every (workgroup, tile) run of
    // a commit is padded to a multiple of 8 entries with DUMMY_CELL entries, so runs start
    // 8-aligned in the region and a lane stores 8 cells / 2 float64 values / 4 narrow slots
    // per 16-byte store; pass B skips the dummies.  lds_cap: staged entries per value slot
    uint32_t wide, lds_cap;
    // min / max pass B on one float64 value slot with at most one count, sum, min and max
    // aggregator of it (no moments, no integer sums): a branch-light entry loop (mm_simple);
    // LDS byte offsets of the count / sum / min / max cells (-1: absent), the count keyed on
    // the slot's non-NaN values (mm_cnt_nn) or on every entry
    uint32_t mm_simple, mm_cnt_nn;
    int32_t mm_off[4];
    // stream layout of the fast kernels (stream = 1): each pass-A workgroup appends every
    // commit's padded, tile-sorted entries to ONE contiguous stream (w * wg_stride on), instead
    // of T private per-tile regions, and records where each tile's run of the commit starts:
    // tab[(w * (T + 1) + t) * ncw + c] = stream offset of tile t's run of commit c (row T: the
    // commit's end; commits past a workgroup's last: its final offset, i.e. empty runs).  Pass B
    // gathers a tile's (workgroup, commit) segments through the table.  256-512 write streams
    // instead of T x W regions: the region pattern's cost and its dependence on where the
    // scratch lands in HBM (r05: 6.2-7.4 ms for one C2 pass A) go away (scripts/bw_probe6.hip)
    uint32_t stream, ncw;
    uint32_t *tab;
    // one keep mask shared by every aggregator (a selection or filter; 1 = keep) applied by the
    // fast pass A per row: masked rows are dropped before the exchange (MK instantiations)
    const uint8_t *rowmask;
};

// local cell of a padding entry (tiles hold at most 2^15 cells when runs are padded)
constexpr uint32_t DUMMY_CELL = 0xffffu;
typedef unsigned int vh_u32x4 __attribute__((ext_vector_type(4)));
typedef double vh_f64x2 __attribute__((ext_vector_type(2)));
// a 16-byte region store, non-temporal when nt (wave-uniform)
template <typename V> __device__ __forceinline__ void region_store(V *p, V v, bool nt) {
    if (nt) __builtin_nontemporal_store(v, p);
    else *p = v;
}

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

// row h of a loaded pair as its 4-byte slot directly (narrow kernels; dt <= 4 bytes): the
// same bits slot_narrow(pair_slot(...)) gives -- float32 bits, or the low word of the int64 /
// uint64 upcast
__device__ __forceinline__ uint32_t pair_slot32(const double2 &pr, int dt, int h) {
    const uint64_t raw = __builtin_bit_cast(uint64_t, pr.x);
    switch (dt) {
    case VH_F32: case VH_I32: case VH_U32: return (uint32_t)(raw >> (32 * h));
    case VH_I16: return (uint32_t)(int32_t)(int16_t)(uint16_t)(raw >> (16 * h));
    case VH_U16: return (uint32_t)(uint16_t)(raw >> (16 * h));
    case VH_I8: return (uint32_t)(int32_t)(int8_t)(uint8_t)(raw >> (8 * h));
    case VH_BOOL: return ((raw >> (8 * h)) & 0xff) ? 1u : 0u;
    default: return (uint32_t)(uint8_t)(raw >> (8 * h));  // VH_U8
    }
}
__device__ __forceinline__ bool slot32_is_nan(uint32_t u, bool is_float) { return is_float && (u & 0x7fffffffu) > 0x7f800000u; }

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
// one carried slot value into an LDS cell.  A plain read first: only a value that improves
// on the cell pays the atomic (a stale read only sends a no-op atomic; a cell of many rows
// improves ~ln(rows) times)
// (RF false: the caller has already compared against a read of the cell -- the atomic only)
template <bool RF = true>
__device__ inline void mm_lds(uint64_t *cell, int dt, bool mx, double v) {
    if (dt_float(dt)) {
        if (v != v) return;
        const uint64_t o = ord_bits(v), cur = RF ? *cell : 0;
        if (RF && (mx ? o <= cur : o >= cur)) return;
        if (mx) atomicMax((unsigned long long *)cell, (unsigned long long)o);
        else atomicMin((unsigned long long *)cell, (unsigned long long)o);
    } else if (dt_signed(dt)) {
        const long long x = (long long)__builtin_bit_cast(int64_t, v), cur = RF ? (long long)*cell : 0;
        if (RF && (mx ? x <= cur : x >= cur)) return;
        if (mx) atomicMax((long long *)cell, x);
        else atomicMin((long long *)cell, x);
    } else {
        const unsigned long long x = __builtin_bit_cast(unsigned long long, v), cur = RF ? *cell : 0;
        if (RF && (mx ? x <= cur : x >= cur)) return;
        if (mx) atomicMax((unsigned long long *)cell, x);
        else atomicMin((unsigned long long *)cell, x);
    }
}
// 4-byte LDS cells for min / max of <= 4-byte columns (ds_min/max_i32 / _u32: half the LDS
// of the 64-bit form, and 32-bit LDS atomics): signed as int32, unsigned as uint32, float32
// as order-preserving bits
__host__ __device__ inline bool mm_cell32(int dt) {
    return dt == VH_F32 || dt == VH_I32 || dt == VH_U32 || dt == VH_I16 || dt == VH_U16 || dt == VH_I8 || dt == VH_U8;
}
__device__ inline uint32_t mm_identity32(int dt, bool mx) {
    if (dt_signed(dt)) return mx ? (uint32_t)INT32_MIN : (uint32_t)INT32_MAX;
    return mx ? 0u : ~0u;
}
__device__ inline uint32_t ord_bits32(float f) {
    const uint32_t u = __builtin_bit_cast(uint32_t, f);
    return (u >> 31) ? ~u : (u | 0x80000000u);
}
__device__ inline float unord_bits32(uint32_t o) {
    return __builtin_bit_cast(float, (o >> 31) ? (o & 0x7fffffffu) : ~o);
}
// one carried slot value (double: float data as a double, integers as int64 / uint64 bits),
// with the same read-first filter
template <bool RF = true>
__device__ inline void mm_lds32(uint32_t *cell, int dt, bool mx, double v) {
    if (dt_float(dt)) {
        if (v != v) return;
        const uint32_t o = ord_bits32((float)v), cur = RF ? *cell : 0;
        if (RF && (mx ? o <= cur : o >= cur)) return;
        if (mx) atomicMax(cell, o);
        else atomicMin(cell, o);
    } else if (dt_signed(dt)) {
        const int x = (int)(int32_t)__builtin_bit_cast(int64_t, v), cur = RF ? (int)*cell : 0;
        if (RF && (mx ? x <= cur : x >= cur)) return;
        if (mx) atomicMax(reinterpret_cast<int *>(cell), x);
        else atomicMin(reinterpret_cast<int *>(cell), x);
    } else {
        const uint32_t x = (uint32_t)__builtin_bit_cast(uint64_t, v), cur = RF ? *cell : 0;
        if (RF && (mx ? x <= cur : x >= cur)) return;
        if (mx) atomicMax(cell, x);
        else atomicMin(cell, x);
    }
}
// a carried slot value as an order-preserving u64 (float data: ord_bits; signed: the sign bit
// flipped; unsigned: the bits) and back, for folding runs of min / max values in registers
__device__ inline uint64_t mm_okey(int dt, double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    if (dt_float(dt)) return ord_bits(v);
    return dt_signed(dt) ? b ^ (1ull << 63) : b;
}
__device__ inline double mm_unokey(int dt, uint64_t o) {
    if (dt_float(dt)) return unord_bits(o);
    return __builtin_bit_cast(double, dt_signed(dt) ? o ^ (1ull << 63) : o);
}

// a 4-byte cell as the carried-slot bits mm_grid takes
__device__ inline uint64_t mm_cell32_slot(int dt, uint32_t x) {
    if (dt_float(dt)) return __builtin_bit_cast(uint64_t, (double)unord_bits32(x));
    if (dt_signed(dt)) return (uint64_t)(int64_t)(int32_t)x;
    return (uint64_t)x;
}

// min / max scratch of the tile path (TileParams::mmtmp): identity fill, and the merge of the
// flushed cell forms into the typed grid (std::min / std::max, superagg.cpp:226,274)
__global__ __launch_bounds__(256) void k_mm_fill(void *tmp, uint64_t cells, int dt, int mx);
__global__ __launch_bounds__(256) void k_mm_merge(void *grid, const void *tmp, uint64_t cells, int dt, int mx);

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

__global__ __launch_bounds__(256) void k_mm_fill(void *tmp, uint64_t cells, int dt, int mx) {
    for (uint64_t c = blockIdx.x * 256ull + threadIdx.x; c < cells; c += (uint64_t)gridDim.x * 256) {
        if (mm_cell32(dt)) static_cast<uint32_t *>(tmp)[c] = mm_identity32(dt, mx);
        else static_cast<uint64_t *>(tmp)[c] = mm_identity(dt, mx);
    }
}

template <typename T> __device__ inline void mm_merge_cell(T *g, T v, bool mx) { *g = minmax_apply(*g, v, mx); }

__global__ __launch_bounds__(256) void k_mm_merge(void *grid, const void *tmp, uint64_t cells, int dt, int mx) {
    for (uint64_t c = blockIdx.x * 256ull + threadIdx.x; c < cells; c += (uint64_t)gridDim.x * 256) {
        uint64_t x;
        if (mm_cell32(dt)) {
            const uint32_t v = static_cast<const uint32_t *>(tmp)[c];
            if (v == mm_identity32(dt, mx)) continue;
            x = mm_cell32_slot(dt, v);
        } else {
            x = static_cast<const uint64_t *>(tmp)[c];
            if (x == mm_identity(dt, mx)) continue;
            if (dt_float(dt)) x = __builtin_bit_cast(uint64_t, unord_bits(x));
        }
        const double d = __builtin_bit_cast(double, x);
        switch (dt) {
        case VH_F64: mm_merge_cell<double>(static_cast<double *>(grid) + c, d, mx); break;
        case VH_F32: mm_merge_cell<float>(static_cast<float *>(grid) + c, (float)d, mx); break;
        case VH_I64: mm_merge_cell<int64_t>(static_cast<int64_t *>(grid) + c, (int64_t)x, mx); break;
        case VH_I32: mm_merge_cell<int32_t>(static_cast<int32_t *>(grid) + c, (int32_t)(int64_t)x, mx); break;
        case VH_I16: mm_merge_cell<int16_t>(static_cast<int16_t *>(grid) + c, (int16_t)(int64_t)x, mx); break;
        case VH_I8: mm_merge_cell<int8_t>(static_cast<int8_t *>(grid) + c, (int8_t)(int64_t)x, mx); break;
        case VH_U64: mm_merge_cell<uint64_t>(static_cast<uint64_t *>(grid) + c, x, mx); break;
        case VH_U32: mm_merge_cell<uint32_t>(static_cast<uint32_t *>(grid) + c, (uint32_t)x, mx); break;
        case VH_U16: mm_merge_cell<uint16_t>(static_cast<uint16_t *>(grid) + c, (uint16_t)x, mx); break;
        default: mm_merge_cell<uint8_t>(static_cast<uint8_t *>(grid) + c, (uint8_t)x, mx); break;
        }
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
// rows of the whole launch that missed their pass-A region (applied with global atomics);
// read and reset by vh_stat_read("tile_overflow_rows")
__device__ unsigned long long d_tile_overflow_rows;

template <int ND>
__global__ __launch_bounds__(TA_THREADS) void k_tile_sample(BinPlan p, uint64_t n, uint32_t s_log2, uint32_t ntiles,
                                                            uint64_t block_stride, uint64_t *hist, uint64_t *hist2,
                                                            uint32_t *brange) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    uint32_t *h = reinterpret_cast<uint32_t *>(lds_raw);
    __shared__ uint32_t s_lo, s_hi;
    for (uint32_t t = threadIdx.x; t < ntiles; t += TA_THREADS) h[t] = 0;
    if (threadIdx.x == 0) {
        s_lo = ~0u;
        s_hi = 0;
    }
    __syncthreads();
    const uint64_t row0 = blockIdx.x * block_stride;
    uint32_t lo = ~0u, hi = 0;
    for (uint64_t r = threadIdx.x; r < TA_BATCH; r += TA_THREADS) {
        const uint64_t i = row0 + r;
        if (i >= n) break;
        const uint32_t t = (uint32_t)(cell_of<ND>(p, i) >> s_log2);
        atomicAdd(&h[t], 1u);
        lo = min(lo, t);
        hi = max(hi, t);
    }
    atomicMin(&s_lo, lo);  // the block's tile range: sorted rows give ranges in order
    atomicMax(&s_hi, hi);
    __syncthreads();
    if (threadIdx.x == 0) {
        brange[2 * blockIdx.x] = s_lo;
        brange[2 * blockIdx.x + 1] = s_hi;
    }
    for (uint32_t t = threadIdx.x; t < ntiles; t += TA_THREADS)
        if (h[t]) {  // per-tile count and its square: the block-to-block spread (clustering)
            atomicAdd((unsigned long long *)&hist[t], (unsigned long long)h[t]);
            atomicAdd((unsigned long long *)&hist2[t], (unsigned long long)h[t] * h[t]);
        }
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
// the count-only f64 pass A (NV = 0, ND <= 2): VH_TA_WPE0 waves per SIMD at least (4 caps it at
// 128 VGPRs: two 512-thread workgroups per CU instead of one at 129; the 3-d kernel would spill)
#ifndef VH_TA_WPE0
#define VH_TA_WPE0 4  // same-process A/B (C2 count-only, 1e9 rows): 3.77 -> 3.45 ms (profiles/r06_ab1.txt)
#endif
#if VH_TA_WAVES > 0
#define TA_ATTR_F64(NV) TA_ATTR
#else
#define TA_ATTR_F64(NV) __attribute__((amdgpu_waves_per_eu(((NV) == 0 && ND <= 2 && VH_TA_WPE0 > 0) ? VH_TA_WPE0 : 1)))
#endif

__device__ inline void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// rank of a row in its tile's LDS histogram (common.hpp wave_rank)
__device__ __forceinline__ int32_t tile_rank(uint32_t *hist, uint32_t t, bool take) { return wave_rank(hist, t, take); }

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
    uint32_t *hist, *boff, *base, *lim, *dbase, *soff, *wave_sums;
};

// LDS bytes of pass A (must match scatter_lds)
__host__ __device__ inline size_t scatter_lds_bytes(int nv, uint32_t T) {
    return (size_t)8 * nv * TA_BATCH + (size_t)8 * TA_BATCH + 24 * (size_t)T + 64;
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
    l.soff = l.dbase + T;
    l.wave_sums = l.soff + T;
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
// the 3-d f64 pass A carries a third binner column: fewer batches per commit keep its
// registers out of scratch memory (three batches of one value slot spilled 17 VGPRs)
__host__ __device__ constexpr int fast_sb_nd(int nv, int nd) {
    return nd < 3 ? fast_sb(nv) : nv >= 2 ? 1 : (fast_sb(nv) < 2 ? fast_sb(nv) : 2);
}
// narrow (4-byte) value slots staged as 4 bytes: two carried columns still fit three batches
__host__ __device__ constexpr int fast_sb_narrow(int nv) { return nv == 0 ? VH_TA_SB0 : VH_TA_SB; }

// LDS of the fast kernels: staged values (vbytes each: 8, or 4 for narrow slots) | staged
// 4-byte keys | tile arrays
__host__ __device__ inline size_t fast_lds_bytes(int nv, uint32_t T, uint32_t cap, int vbytes = 8) {
    return (size_t)vbytes * nv * cap + (size_t)4 * cap + 24 * (size_t)T + 64;
}

template <int NV> __device__ inline ScatterLds fast_lds(unsigned char *raw, uint32_t T, uint32_t cap, int vbytes = 8) {
    ScatterLds l;
    l.sv = reinterpret_cast<double *>(raw);
    l.sp = reinterpret_cast<uint64_t *>(raw + (size_t)vbytes * NV * cap);
    l.hist = reinterpret_cast<uint32_t *>(raw + (size_t)vbytes * NV * cap + (size_t)4 * cap);
    l.boff = l.hist + T;
    l.base = l.boff + T;
    l.lim = l.base + T;
    l.dbase = l.lim + T;
    l.soff = l.dbase + T;
    l.wave_sums = l.soff + T;
    return l;
}

// per-workgroup init: zero the histogram; a tile's region of this workgroup is
// [toff, toff + cap) inside the workgroup's block, written from base upwards
__device__ inline void scatter_lds_init(const ScatterLds &l, const TileParams &tp, uint32_t T) {
    for (uint32_t t = threadIdx.x; t < T; t += TA_THREADS) {
        l.hist[t] = 0;
        l.base[t] = tp.stream ? 0u : (uint32_t)tp.toff[t];
        l.lim[t] = tp.stream ? ~0u : (uint32_t)tp.toff[t] + tp.cap[t];  // the stream is sized exactly
    }
    if (threadIdx.x == 0) {  // stream layout: write cursor and commit index of this workgroup
        l.wave_sums[1] = 0;
        l.wave_sums[2] = 0;
    }
}

// stream layout: the table rows of the commits a workgroup did not have (empty runs at its
// final offset); after the pass-A loop, behind an LDS barrier
__device__ inline void stream_tab_tail(const ScatterLds &l, const TileParams &tp, uint32_t T) {
    if (!tp.stream) return;
    const uint32_t cend = l.wave_sums[1], c0 = l.wave_sums[2], ncw = tp.ncw;
    if (c0 >= ncw) return;
    const uint64_t row0 = (uint64_t)blockIdx.x * (T + 1);
    const uint32_t per = ncw - c0;
    for (uint32_t i = threadIdx.x; i < (T + 1) * per; i += TA_THREADS)
        tp.tab[(row0 + i / per) * ncw + c0 + i % per] = cend;
}

constexpr uint32_t DEST_OVERFLOW = 0x80000000u;  // | tile: region and spill full, global atomics
constexpr uint32_t DEST_SPILL = 0x40000000u;     // | entry of the spill areas

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
    // a tile whose rows run past its region reserves the excess in its spill area
    for (uint32_t t = threadIdx.x; t < T; t += TA_THREADS) {
        const uint32_t b = l.base[t], h = l.hist[t], lim = l.lim[t];
        if (b + h > lim) {
            const uint32_t first = max(b, lim);
            l.soff[t] = atomicAdd(&tp.spill_fill[t], b + h - first) - first;
        }
    }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < TA_RPT; r++) {
        if (rank[r] < 0) continue;
        const uint32_t t = tile[r];
        const uint32_t pos = l.boff[t] + (uint32_t)rank[r];
        const uint32_t d = l.base[t] + (uint32_t)rank[r];
        // past the region: the tile's spill area (DEST_SPILL | entry relative to
        // spill_base), past that too: global atomics (DEST_OVERFLOW | tile)
        uint32_t dest = d;
        if (d >= l.lim[t]) {
            const uint32_t si = d + l.soff[t];
            dest = si < tp.spill_cap[t] ? (DEST_SPILL | (uint32_t)(tp.spill_start[t] + si)) : (DEST_OVERFLOW | t);
        }
        l.sp[pos] = ((uint64_t)dest << 32) | ent[r];
#pragma unroll
        for (int s = 0; s < NV; s++) l.sv[s * TA_BATCH + pos] = vals[r][s];
    }
    lds_barrier();
    const uint32_t tot = *s_total;
    for (uint32_t k = threadIdx.x; k < tot; k += TA_THREADS) {
        const uint64_t pk = l.sp[k];
        const uint32_t dest = (uint32_t)(pk >> 32), e32 = (uint32_t)pk;
        if (DBG(tp.debug) & 1) {
            asm volatile("" :: "v"(e32), "v"(dest));
        } else if (!(dest & DEST_OVERFLOW)) {
            const uint64_t e = (dest & DEST_SPILL) ? tp.spill_base + (dest & ~DEST_SPILL) : region0 + dest;
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
            // past the region and the spill area: apply the staged row with global atomics
            const uint32_t t = dest & ~DEST_OVERFLOW;
            const uint64_t c = ((uint64_t)t << tp.s_log2) | (e32 & 0xffffu);
            atomicAdd(&d_tile_overflow_rows, 1ull);
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
                    if (fa.a[a].kind == VH_AGG_SUM_MOMENT) {
                        if (v == v) atomicAdd(reinterpret_cast<double *>(fa.a[a].grid) + c, moment_term(v, fa.a[a].moment));
                    } else if (fa.a[a].vint)
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
// Wide stream-out (tp.wide): a tile's staged run is padded to hp = roundup8(h) entries with
// DUMMY_CELL keys, so boff, the region bases and dbase stay multiples of 8.
// Stream layout (tp.stream): every tile's dbase is the workgroup's stream cursor, so staged
// entry k goes to cursor + k (the commit is written as one contiguous block), the tile's run
// start is recorded in the table, and the cursor advances by the commit's padded total.
__device__ inline void fast_scan(const ScatterLds &l, const TileParams &tp, uint32_t T) {
    if (threadIdx.x >= 64) return;
    const uint32_t lane = threadIdx.x;
    const uint32_t per = (T + 63) / 64;
    const uint32_t t0 = lane * per;
    const uint32_t pad = tp.wide ? 7u : 0u;
    const bool stream = tp.stream != 0;
    // (read by every lane before lane 63 advances them below: one wave, program order)
    const uint32_t cur = stream ? l.wave_sums[1] : 0u, ci = stream ? l.wave_sums[2] : 0u;
    uint32_t *tab = stream ? tp.tab + ((uint64_t)blockIdx.x * (T + 1)) * tp.ncw + ci : nullptr;
    uint32_t *sk = reinterpret_cast<uint32_t *>(l.sp);
    uint32_t s = 0;
    for (uint32_t t = t0; t < t0 + per && t < T; t++) s += (l.hist[t] + pad) & ~pad;
    uint32_t inc = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off, 64);
        if ((int)lane >= off) inc += y;
    }
    uint32_t acc = inc - s;
    for (uint32_t t = t0; t < t0 + per && t < T; t++) {
        const uint32_t h0 = l.hist[t], h = (h0 + pad) & ~pad, b = l.base[t], lim = l.lim[t];
        l.boff[t] = acc;
        l.dbase[t] = stream ? cur : b - acc;
        l.base[t] = b + h;
        l.hist[t] = 0;
        for (uint32_t x = h0; x < h; x++) sk[acc + x] = (t << 16) | DUMMY_CELL;
        if (stream) tab[(uint64_t)t * tp.ncw] = cur + acc;
        acc += h;
        if (b + h > lim) {  // rows past the region: reserve them in the tile's spill area
            const uint32_t first = max(b, lim);
            l.soff[t] = atomicAdd(&tp.spill_fill[t], b + h - first) - first;
        }
    }
    if (lane == 63) {
        l.wave_sums[0] = inc;
        if (stream) {
            tab[(uint64_t)T * tp.ncw] = cur + inc;
            l.wave_sums[1] = cur + inc;
            l.wave_sums[2] = ci + 1;
        }
    }
}

// VT: the carried value type -- double (8-byte slots, or narrowed at the store when
// tp.vnarrow), or uint32_t (narrow slots computed from the raw column: staged and stored as
// 4 bytes; widened only for the rare overflow row)
template <typename VT> __device__ __forceinline__ double vt_wide(VT v, const TileParams &tp, int s) {
    if constexpr (sizeof(VT) == 8) return v;
    else return slot_wide(v, (tp.vfloat >> s) & 1, (tp.vsigned >> s) & 1);
}

template <int NV, int R, typename VT = double>
__device__ inline void batch_commit_fast(const ScatterLds &l, const FusedAggs &fa, const TileParams &tp, uint32_t T,
                                         uint64_t region0, const uint32_t *key, const int32_t *rank,
                                         const VT (*vals)[NV > 0 ? NV : 1], uint32_t count_mask,
                                         const uint32_t *keyed_slot_of) {
    const uint32_t CAP = tp.lds_cap;  // staged entries per value slot (R * TA_THREADS, + 8 T when wide)
    uint32_t *sk = reinterpret_cast<uint32_t *>(l.sp);
    VT *sv = reinterpret_cast<VT *>(l.sv);
    lds_barrier();
    fast_scan(l, tp, T);
    lds_barrier();
    const uint32_t tot = l.wave_sums[0];
#pragma unroll
    for (int r = 0; r < R; r++) {
        if (rank[r] < 0) continue;
        const uint32_t pos = l.boff[key[r] >> 16] + (uint32_t)rank[r];
        sk[pos] = key[r];
#pragma unroll
        for (int s = 0; s < NV; s++) sv[s * CAP + pos] = vals[r][s];
    }
    lds_barrier();
    // staged entry k to its region / spill slot, or (past both) to the grid with global
    // atomics; padding entries (DUMMY_CELL) are stored like rows but never applied
    auto entry = [&](uint32_t k, uint32_t kk) __attribute__((always_inline)) {
        const uint32_t t = kk >> 16;
        const uint32_t dest = l.dbase[t] + k;
        if (DBG(tp.debug) & 128) {  // experiment: no region stores
            asm volatile("" ::"v"(kk), "v"(dest));
        } else if (dest < l.lim[t] || dest + l.soff[t] < tp.spill_cap[t]) {
            // the region, or past it the tile's spill area
            const uint64_t e = dest < l.lim[t] ? region0 + dest : tp.spill_base + tp.spill_start[t] + (dest + l.soff[t]);
            reinterpret_cast<uint16_t *>(tp.entries)[e] = (uint16_t)kk;
            if constexpr (sizeof(VT) == 4 && NV == 2) {
                if (tp.vpacked) {  // blocked by 8 entries: [8 x slot 0 | 8 x slot 1] per 64 bytes
                    uint32_t *vb = reinterpret_cast<uint32_t *>(tp.values[0]) + (e & ~uint64_t(7)) * 2 + (e & 7);
                    vb[0] = sv[k];
                    vb[8] = sv[CAP + k];
                    return;
                }
            }
#pragma unroll
            for (int s = 0; s < NV; s++) {
                if constexpr (sizeof(VT) == 4)
                    reinterpret_cast<uint32_t *>(tp.values[s])[e] = sv[s * CAP + k];
                else if (tp.vnarrow)
                    reinterpret_cast<uint32_t *>(tp.values[s])[e] = slot_narrow(sv[s * CAP + k], (tp.vfloat >> s) & 1);
                else
                    tp.values[s][e] = sv[s * CAP + k];
            }
        } else if ((kk & 0xffffu) != DUMMY_CELL) {
            // past the region and the spill area: apply the staged row with global atomics
            const uint64_t c = ((uint64_t)t << tp.s_log2) | (kk & 0xffffu);
            atomicAdd(&d_tile_overflow_rows, 1ull);
            #pragma unroll
            for (int a = 0; a < MAX_FUSED_AGGS; a++) {
                if (a >= fa.na) break;
                bool take = (count_mask >> a) & 1;
                if constexpr (NV > 0) {
                    if (!take) {
                        const double v = vt_wide<VT>(sv[keyed_slot_of[a] * CAP + k], tp, keyed_slot_of[a]);
                        take = v == v;
                    }
                }
                if (!take) continue;
                if (fa.a[a].kind == VH_AGG_COUNT) {
                    atomicAdd((unsigned long long *)fa.a[a].grid + c, 1ULL);
                } else if (is_minmax(fa.a[a].kind)) {
                    if constexpr (NV > 0)
                        mm_grid(fa.a[a].grid, c, fa.a[a].dtype, fa.a[a].kind == VH_AGG_MAX,
                                __builtin_bit_cast(uint64_t, vt_wide<VT>(sv[tp.val_slot[a] * CAP + k], tp, tp.val_slot[a])), false);
                } else if constexpr (NV > 0) {
                    const double v = vt_wide<VT>(sv[tp.val_slot[a] * CAP + k], tp, tp.val_slot[a]);
                    if (fa.a[a].kind == VH_AGG_SUM_MOMENT) {
                        if (v == v) atomicAdd(reinterpret_cast<double *>(fa.a[a].grid) + c, moment_term(v, fa.a[a].moment));
                    } else if (fa.a[a].vint)
                        atomicAdd(reinterpret_cast<unsigned long long *>(fa.a[a].grid) + c, __builtin_bit_cast(unsigned long long, v));
                    else
                        atomicAdd(reinterpret_cast<double *>(fa.a[a].grid) + c, v);
                }
            }
        }
    };
    if (!tp.wide) {
        for (uint32_t k = threadIdx.x; k < tot; k += TA_THREADS) entry(k, sk[k]);
        return;
    }
    // Wide stream-out: runs are padded to 8 entries and start 8-aligned in their regions
    // (tot, boff, dbase, region bases and region limits are multiples of 8), so an aligned
    // group of 8 staged entries lies in one tile and wholly inside or wholly past its region.
    // Cells: one 16-byte store of 8 u16 cells per group; groups past the region take the
    // per-entry path (spill area / atomics), which also stores their values.
    uint16_t *ent16 = reinterpret_cast<uint16_t *>(tp.entries);
    const bool nt_cells = (tp.wide >> 1) & 1, nt_vals = (tp.wide >> 2) & 1;
    for (uint32_t g = threadIdx.x; g < (tot >> 3); g += TA_THREADS) {
        const uint32_t k = g << 3;
        const uint4 a = *reinterpret_cast<const uint4 *>(sk + k), b = *reinterpret_cast<const uint4 *>(sk + k + 4);
        const uint32_t t = a.x >> 16;
        const uint32_t dest = l.dbase[t] + k;
        if (DBG(tp.debug) & 128) {
            asm volatile("" ::"v"(a.y), "v"(dest));
        } else if (dest < l.lim[t]) {
            vh_u32x4 c;
            c.x = (a.x & 0xffffu) | (a.y << 16);
            c.y = (a.z & 0xffffu) | (a.w << 16);
            c.z = (b.x & 0xffffu) | (b.y << 16);
            c.w = (b.z & 0xffffu) | (b.w << 16);
            region_store(reinterpret_cast<vh_u32x4 *>(ent16 + region0 + dest), c, nt_cells);
        } else {
#pragma unroll 1
            for (uint32_t x = 0; x < 8; x++) entry(k + x, sk[k + x]);
        }
    }
    if constexpr (NV > 0) {
        if (DBG(tp.debug) & 128) return;
        if constexpr (sizeof(VT) == 8) {
            if (!tp.vnarrow) {
                // float64 slots: one 16-byte store of 2 values per pair of staged entries; UV
                // pairs per lane and step, their LDS lookups (key -> tile -> region base)
                // issued together
                constexpr int UV = 4;
                const uint32_t np = tot >> 1;
                for (uint32_t q0 = threadIdx.x; q0 < np; q0 += UV * TA_THREADS) {
                    uint32_t kk[UV], dst[UV];
                    bool ok[UV];
#pragma unroll
                    for (int u = 0; u < UV; u++) kk[u] = sk[(q0 + u * TA_THREADS < np ? q0 + u * TA_THREADS : q0) << 1];
#pragma unroll
                    for (int u = 0; u < UV; u++) {
                        const uint32_t t = kk[u] >> 16;
                        dst[u] = l.dbase[t] + ((q0 + u * TA_THREADS) << 1);
                        ok[u] = q0 + u * TA_THREADS < np && dst[u] < l.lim[t];  // else: the per-entry path
                    }
#pragma unroll
                    for (int s = 0; s < NV; s++) {
                        double2 v[UV];
#pragma unroll
                        for (int u = 0; u < UV; u++)
                            v[u] = *reinterpret_cast<const double2 *>(sv + s * CAP + (ok[u] ? (q0 + u * TA_THREADS) << 1 : 0u));
#pragma unroll
                        for (int u = 0; u < UV; u++)
                            if (ok[u]) region_store(reinterpret_cast<vh_f64x2 *>(tp.values[s] + region0 + dst[u]), vh_f64x2{v[u].x, v[u].y}, nt_vals);
                    }
                }
                return;
            }
        }
        // 4-byte slots: one 16-byte store of 4 slots per quad of staged entries
        for (uint32_t q = threadIdx.x; q < (tot >> 2); q += TA_THREADS) {
            const uint32_t k = q << 2;
            const uint32_t t = sk[k] >> 16;
            const uint32_t dest = l.dbase[t] + k;
            if (dest >= l.lim[t]) continue;
            const uint64_t e = region0 + dest;
            vh_u32x4 w[NV];
#pragma unroll
            for (int s = 0; s < NV; s++) {
                if constexpr (sizeof(VT) == 4) {
                    const uint4 u = *reinterpret_cast<const uint4 *>(sv + s * CAP + k);
                    w[s] = vh_u32x4{u.x, u.y, u.z, u.w};
                } else {
                    const bool fl = (tp.vfloat >> s) & 1;
                    w[s] = vh_u32x4{slot_narrow(sv[s * CAP + k], fl), slot_narrow(sv[s * CAP + k + 1], fl),
                                    slot_narrow(sv[s * CAP + k + 2], fl), slot_narrow(sv[s * CAP + k + 3], fl)};
                }
            }
            if constexpr (sizeof(VT) == 4 && NV == 2) {
                if (tp.vpacked) {  // [8 x slot 0 | 8 x slot 1] per 8 entries: e & 7 is 0 or 4
                    uint32_t *vb = reinterpret_cast<uint32_t *>(tp.values[0]) + (e & ~uint64_t(7)) * 2 + (e & 7);
                    region_store(reinterpret_cast<vh_u32x4 *>(vb), w[0], nt_vals);
                    region_store(reinterpret_cast<vh_u32x4 *>(vb + 8), w[1], nt_vals);
                    continue;
                }
            }
#pragma unroll
            for (int s = 0; s < NV; s++) region_store(reinterpret_cast<vh_u32x4 *>(reinterpret_cast<uint32_t *>(tp.values[s]) + e), w[s], nt_vals);
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
    // batches w, w + W, w + 2W, ... (tile distribution of every workgroup = the global one)
    const uint32_t w = blockIdx.x;
    const uint64_t row_end = n;
    const uint32_t smask = (1u << tp.s_log2) - 1;
    const uint64_t region0 = (uint64_t)w * tp.wg_stride;
    for (uint64_t b0 = (uint64_t)w * TA_BATCH; b0 < n; b0 += (uint64_t)tp.W * TA_BATCH) {
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
                const uint64_t c = cell[r];
                const uint32_t f = i < row_end ? fl[r] : 0u;
                tile[r] = (uint32_t)(c >> tp.s_log2);
                ent[r] = ((uint32_t)c & smask) | (f << 16);
                rank[r] = tile_rank(l.hist, tile[r], f != 0);
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
// CT = float: the same over float32 columns (binners and sums): rows read as 8-byte pairs,
// the binner value widened to double before the index math (BinnerScalar<float>::to_bins,
// superagg_binners.cpp:14-56, scales the value as double), sums carried, staged and stored
// as their 4-byte float32 bits (narrow slots, widened exactly in pass B)
// MK: the plan's aggregators share one keep mask (tp.rowmask): two mask bytes per row pair
// load with the pair, and a row whose byte is not 1 takes no aggregator (dropped from the
// exchange, as the generic pass A drops a row no aggregator takes)
// VT != CT (mixed plans: float64 binners with float32 sums, float32 binners with float64
// sums): the value columns load into a second register array of their own pair type.
// CT = int32_t / int64_t: integer binner columns (BinnerScalar<int>: the value widened to
// double before the same index math, superagg_binners.cpp:14-56)
template <typename T> struct PairOf;
template <> struct PairOf<double> { using type = double2; };
template <> struct PairOf<float> { using type = float2; };
template <> struct PairOf<int32_t> { using type = int2; };
template <> struct PairOf<int64_t> { using type = longlong2; };
template <int ND, int NV, int SB, typename CT = double, bool MK = false, typename VT = CT>
__global__ __launch_bounds__(TA_THREADS) TA_ATTR_F64(NV) void k_tile_scatter_f64(BinPlan p, FusedAggs fa, TileParams tp, uint64_t n) {
    constexpr bool F32 = std::is_same_v<CT, float>;
    constexpr bool MIX = !std::is_same_v<CT, VT>;
    constexpr bool VF32 = std::is_same_v<VT, float>;
    using P2 = typename PairOf<CT>::type;
    using VP2 = std::conditional_t<VF32, float2, double2>;
    using VS = std::conditional_t<VF32, uint32_t, double>;  // carried / staged value slot
    constexpr int NC = ND + (MIX ? 0 : NV);  // columns in the CT pair array
    constexpr int NVX = MIX ? NV : 0;        // value columns in the VT pair array
    constexpr int PAIRS = TA_RPT / 2;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const uint32_t T = tp.ntiles;
    const ScatterLds l = fast_lds<NV>(lds_raw, T, tp.lds_cap, VF32 ? 4 : 8);
    scatter_lds_init(l, tp, T);
    __syncthreads();
    const CT *col[NC > 0 ? NC : 1];
    const VT *vcol[NVX > 0 ? NVX : 1];
    double vmin[ND > 0 ? ND : 1], scale[ND > 0 ? ND : 1], bins_d[ND > 0 ? ND : 1];
    uint32_t bins2[ND > 0 ? ND : 1], stride[ND > 0 ? ND : 1];
#pragma unroll
    for (int d = 0; d < ND; d++) {
        col[d] = reinterpret_cast<const CT *>(p.b[d].data);
        vmin[d] = p.b[d].vmin;
        scale[d] = p.b[d].scale;
        bins_d[d] = (double)p.b[d].bins;
        bins2[d] = (uint32_t)p.b[d].bins + 2;
        stride[d] = (uint32_t)p.b[d].stride;
    }
#pragma unroll
    for (int s = 0; s < NV; s++) {
        if constexpr (MIX) vcol[s] = reinterpret_cast<const VT *>(tp.vdata[s]);
        else col[ND + s] = reinterpret_cast<const CT *>(tp.vdata[s]);
    }
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
    // batches w, w + W, w + 2W, ... of TA_BATCH rows (tile distribution of every workgroup
    // = the global one, whatever the row order)
    const uint32_t w = blockIdx.x;
    const uint64_t row_end = n, bstep = (uint64_t)tp.W * TA_BATCH;
    const uint32_t smask = (1u << tp.s_log2) - 1, s_log2 = tp.s_log2;
    const uint64_t region0 = (uint64_t)w * tp.wg_stride;
    // Branch-free 16-byte loads: n is even on this path (the host bins an odd last row
    // separately) and batches start at multiples of TA_BATCH, so a pair is either wholly
    // inside [0, n) or wholly past it; past-the-end pairs load the clamped last pair and
    // are dropped by the i < n test.  With no load behind an exec branch the compiler
    // counts vmcnt instead of draining to 0, so the prefetched batch stays in flight.
    const uint8_t *rowmask = tp.rowmask;
    auto load = [&](uint64_t b0, P2 (&dst)[PAIRS][NC > 0 ? NC : 1], VP2 (&vdst)[PAIRS][NVX > 0 ? NVX : 1],
                    uint32_t (&mdst)[MK ? PAIRS : 1]) {
#pragma unroll
        for (int q = 0; q < PAIRS; q++) {
            const uint64_t i = b0 + 2 * ((uint64_t)q * TA_THREADS + threadIdx.x);
            const uint64_t is = i < n - 2 ? i : n - 2;
            if constexpr (MK) mdst[q] = *reinterpret_cast<const uint16_t *>(rowmask + is);
#pragma unroll
            for (int s = 0; s < NVX; s++) vdst[q][s] = *reinterpret_cast<const VP2 *>(vcol[s] + is);
#pragma unroll
            for (int c = 0; c < NC; c++) {
#if VH_TA_NT  // experiment: non-temporal loads of the once-read columns
                if constexpr (std::is_same_v<CT, double>) {
                    typedef double v2d __attribute__((ext_vector_type(2)));
                    const v2d t = __builtin_nontemporal_load(reinterpret_cast<const v2d *>(col[c] + is));
                    dst[q][c] = make_double2(t.x, t.y);
                    continue;
                }
#endif
                dst[q][c] = *reinterpret_cast<const P2 *>(col[c] + is);
            }
        }
    };
    // rank the rows of one batch: cell, take flags, (tile << 16 | cell) key, rank in tile
    auto rows = [&](uint64_t b0, const P2 (&cur)[PAIRS][NC > 0 ? NC : 1], const VP2 (&vcur)[PAIRS][NVX > 0 ? NVX : 1],
                    const uint32_t (&mcur)[MK ? PAIRS : 1], uint32_t *key, int32_t *rank, VS (*vals)[NV > 0 ? NV : 1]) {
#pragma unroll
        for (int r = 0; r < TA_RPT; r++) {
            const int q = r >> 1, h = r & 1;
            const uint64_t i = b0 + 2 * ((uint64_t)q * TA_THREADS + threadIdx.x) + h;
            uint32_t c = 0;
#pragma unroll
            for (int d = 0; d < ND; d++) {
                const double v = (double)(h ? cur[q][d].y : cur[q][d].x);
                c += scalar_f64_index32(v, vmin[d], scale[d], bins_d[d], bins2[d]) * stride[d];
            }
            uint32_t f = count_mask;
#pragma unroll
            for (int s = 0; s < NV; s++) {
                VT v;
                if constexpr (MIX) v = h ? vcur[q][s].y : vcur[q][s].x;
                else v = h ? cur[q][ND + s].y : cur[q][ND + s].x;
                if constexpr (VF32) vals[r][s] = __builtin_bit_cast(uint32_t, v);
                else vals[r][s] = v;
                f |= v == v ? nan_keyed[s] : 0u;
            }
            if constexpr (MK) f = ((h ? mcur[q] >> 8 : mcur[q]) & 0xffu) == 1u ? f : 0u;
            f = i < row_end ? f : 0u;
            const uint32_t t = c >> s_log2;
            key[r] = (t << 16) | (c & smask);
            rank[r] = -1;
            if (DBG(tp.debug) & 64) {  // experiment: no ranking
                asm volatile("" ::"v"(key[r]), "v"(f));
            } else {
                rank[r] = tile_rank(l.hist, t, f != 0);
            }
        }
    };
    constexpr bool drain = VH_TA_DRAIN != 0;
    P2 cur[PAIRS][NC > 0 ? NC : 1], nxt[PAIRS][NC > 0 ? NC : 1];
    VP2 vcur[PAIRS][NVX > 0 ? NVX : 1], vnxt[PAIRS][NVX > 0 ? NVX : 1];
    uint32_t mcur[MK ? PAIRS : 1] = {}, mnxt[MK ? PAIRS : 1] = {};
    load((uint64_t)w * TA_BATCH, cur, vcur, mcur);
    for (uint64_t b0 = (uint64_t)w * TA_BATCH; b0 < n; b0 += SB * bstep) {
        uint32_t key[SB * TA_RPT];
        int32_t rank[SB * TA_RPT];
        VS vals[SB * TA_RPT][NV > 0 ? NV : 1];
        // the last prefetch stays in flight across the commit: it is moved into cur only
        // after the commit (a copy before it would wait for those loads)
#pragma unroll
        for (int sb = 0; sb < SB; sb++) {
            load(b0 + (sb + 1) * bstep, nxt, vnxt, mnxt);
            rows(b0 + sb * bstep, cur, vcur, mcur, key + sb * TA_RPT, rank + sb * TA_RPT, vals + sb * TA_RPT);
            if (sb + 1 < SB || drain)
#pragma unroll
                for (int q = 0; q < PAIRS; q++) {
#pragma unroll
                    for (int c = 0; c < NC; c++) cur[q][c] = nxt[q][c];
#pragma unroll
                    for (int c = 0; c < NVX; c++) vcur[q][c] = vnxt[q][c];
                    if constexpr (MK) mcur[q] = mnxt[q];
                }
        }
        if (DBG(tp.debug) & 32) {  // experiment: no commit (loads, cell math, ranking only)
#pragma unroll
            for (int r = 0; r < SB * TA_RPT; r++) asm volatile("" ::"v"(key[r]), "v"(rank[r]));
        } else {
            batch_commit_fast<NV, SB * TA_RPT, VS>(l, fa, tp, T, region0, key, rank, vals, count_mask, keyed_slot_of);
        }
        if (!drain)
#pragma unroll
            for (int q = 0; q < PAIRS; q++) {
#pragma unroll
                for (int c = 0; c < NC; c++) cur[q][c] = nxt[q][c];
#pragma unroll
                for (int c = 0; c < NVX; c++) vcur[q][c] = vnxt[q][c];
                if constexpr (MK) mcur[q] = mnxt[q];
            }
    }
    lds_barrier();
    for (uint32_t t = threadIdx.x; t < T; t += TA_THREADS) tp.fills[(uint64_t)t * tp.W + w] = l.base[t] - (uint32_t)tp.toff[t];
    stream_tab_tail(l, tp, T);
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
// VN: every carried column is <= 4 bytes (narrow slots): values are carried, staged and
// stored as their 4-byte slot bits (half the LDS staging: two columns still commit three
// batches at once)
// MK: a keep mask shared by the aggregators (tp.rowmask; a filtered frame's groupby), applied
// per row like the fast scalar kernels' MK instantiations
template <int NV, int SB, bool SET = false, int DT0 = VH_F64, int DT1 = VH_F64, bool VN = false, bool MK = false>
__global__ __launch_bounds__(TA_THREADS) TA_ATTR void k_tile_scatter_ord(BinPlan p, FusedAggs fa, TileParams tp, uint64_t n) {
    constexpr int PAIRS = TA_RPT / 2;
    using VT = std::conditional_t<VN, uint32_t, double>;
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const uint32_t T = tp.ntiles;
    const ScatterLds l = fast_lds<NV>(lds_raw, T, tp.lds_cap, VN ? 4 : 8);
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
    // batches w, w + W, w + 2W, ... (as k_tile_scatter_f64)
    const uint32_t w = blockIdx.x;
    const uint64_t row_end = n, bstep = (uint64_t)tp.W * TA_BATCH;
    const uint32_t smask = (1u << tp.s_log2) - 1, s_log2 = tp.s_log2;
    const uint64_t region0 = (uint64_t)w * tp.wg_stride;
    struct Regs {
        int2 k[PAIRS];
        double2 v[PAIRS][NV > 0 ? NV : 1];
        uint32_t m[MK ? PAIRS : 1];
    };
    const uint8_t *rowmask = tp.rowmask;
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
            if constexpr (MK) R.m[q] = *reinterpret_cast<const uint16_t *>(rowmask + is);
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
    auto rows = [&](uint64_t b0, const Regs &cur, uint32_t *key, int32_t *rank, VT (*vals)[NV > 0 ? NV : 1]) {
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
                if constexpr (VN) {
                    vals[r][s] = pair_slot32(cur.v[q][s], dts >= 0 ? dts : tp.vdt[s], h);
                    f |= slot32_is_nan(vals[r][s], (tp.vfloat >> s) & 1) ? 0u : nan_keyed[s];
                } else {
                    vals[r][s] = pair_slot(cur.v[q][s], dts >= 0 ? dts : tp.vdt[s], h);
                    f |= vals[r][s] == vals[r][s] ? nan_keyed[s] : 0u;
                }
            }
            if constexpr (MK) f = ((h ? cur.m[q] >> 8 : cur.m[q]) & 0xffu) == 1u ? f : 0u;
            f = i < row_end ? f : 0u;
            const uint32_t t = c >> s_log2;
            key[r] = (t << 16) | (c & smask);
            if (DBG(tp.debug) & 64) {  // experiment: no ranking
                asm volatile("" ::"v"(key[r]), "v"(f));
                rank[r] = -1;
            } else {
                rank[r] = tile_rank(l.hist, t, f != 0);
            }
        }
    };
    constexpr bool drain = VH_TA_DRAIN != 0;
    Regs cur, nxt;
    load((uint64_t)w * TA_BATCH, cur);
    for (uint64_t b0 = (uint64_t)w * TA_BATCH; b0 < n; b0 += SB * bstep) {
        uint32_t key[SB * TA_RPT];
        int32_t rank[SB * TA_RPT];
        VT vals[SB * TA_RPT][NV > 0 ? NV : 1];
#pragma unroll
        for (int sb = 0; sb < SB; sb++) {
            load(b0 + (sb + 1) * bstep, nxt);
            rows(b0 + sb * bstep, cur, key + sb * TA_RPT, rank + sb * TA_RPT, vals + sb * TA_RPT);
            if (sb + 1 < SB || drain) cur = nxt;
        }
        if (DBG(tp.debug) & 32) {  // experiment: no commit (loads, cell math, ranking only)
#pragma unroll
            for (int r = 0; r < SB * TA_RPT; r++) asm volatile("" ::"v"(key[r]), "v"(rank[r]));
        } else {
            batch_commit_fast<NV, SB * TA_RPT, VT>(l, fa, tp, T, region0, key, rank, vals, count_mask, keyed_slot_of);
        }
        if (!drain) cur = nxt;
    }
    lds_barrier();
    for (uint32_t t = threadIdx.x; t < T; t += TA_THREADS) tp.fills[(uint64_t)t * tp.W + w] = l.base[t] - (uint32_t)tp.toff[t];
    stream_tab_tail(l, tp, T);
}

template <int NV, bool MM>
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
            if constexpr (!MM) continue;
#pragma unroll
            for (int s = 0; s < NV; s++) {
                if (s != tp.val_slot[k]) continue;
                if (mm_cell32(fa.a[k].dtype))
                    mm_lds32(reinterpret_cast<uint32_t *>(lds + fa.a[k].lds_off) + local, fa.a[k].dtype, fa.a[k].kind == VH_AGG_MAX, v[s]);
                else
                    mm_lds(reinterpret_cast<uint64_t *>(lds + fa.a[k].lds_off) + local, fa.a[k].dtype, fa.a[k].kind == VH_AGG_MAX, v[s]);
            }
        } else if (fa.a[k].kind == VH_AGG_SUM_MOMENT) {
            if constexpr (!MM) continue;
#pragma unroll
            for (int s = 0; s < NV; s++)
                if (s == tp.val_slot[k] && v[s] == v[s])
                    atomicAdd(reinterpret_cast<double *>(lds + fa.a[k].lds_off) + local, moment_term(v[s], fa.a[k].moment));
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

// a run of entries of one LDS cell (count / sum aggregators): entries, and per value slot
// the non-NaN count, the float sum of non-NaN values and the 64-bit integer sum
// X: the plan also has min / max and moment-2 aggregators (var / std): per value slot the
// run's sum of squares (min / max entries are committed one by one, see k_tile_reduce)
template <int NV, bool X = false> struct TileRun {
    uint32_t cnt, nn[NV > 0 ? NV : 1];
    double sum[NV > 0 ? NV : 1];
    unsigned long long isum[NV > 0 ? NV : 1];
    double sum2[X && NV > 0 ? NV : 1];
    __device__ void clear() {
        cnt = 0;
#pragma unroll
        for (int s = 0; s < NV; s++) {
            nn[s] = 0;
            sum[s] = 0.0;
            isum[s] = 0;
            if constexpr (X) sum2[s] = 0.0;
        }
    }
    __device__ __attribute__((always_inline)) void add(const TileParams &tp, const double *v) {
        cnt++;
#pragma unroll
        for (int s = 0; s < NV; s++) {
            isum[s] += __builtin_bit_cast(unsigned long long, v[s]);
            if (v[s] == v[s]) {
                nn[s]++;
                sum[s] += v[s];
                if constexpr (X) sum2[s] += v[s] * v[s];
            }

        }
    }
    // the run into the LDS tile, as reduce_entry would add its entries one by one
    // add / flush always inlined: out of line they take fa / tp / the run by address, which
    // puts all three in scratch memory (the two-slot min / max kernel did)
    __device__ __attribute__((always_inline)) void flush(const FusedAggs &fa, const TileParams &tp, unsigned char *lds,
                                                         uint32_t local) const {
#pragma unroll
        for (int k = 0; k < MAX_FUSED_AGGS; k++) {
            if (k >= fa.na) break;
            const int kind = fa.a[k].kind;
            if (kind == VH_AGG_COUNT) {
                const int cs = tp.cnt_slot[k];
                uint32_t c = cs == CNT_ALWAYS || cs == CNT_FLAG ? cnt : 0u;
#pragma unroll
                for (int s = 0; s < NV; s++)
                    if (s == cs) c = nn[s];
                if (c) atomicAdd(reinterpret_cast<uint32_t *>(lds + fa.a[k].lds_off) + local, c);
                continue;
            }
#pragma unroll
            for (int s = 0; s < NV; s++) {
                if (s != tp.val_slot[k]) continue;
                if constexpr (X) {
                    if (kind == VH_AGG_SUM_MOMENT) {
                        if (nn[s]) atomicAdd(reinterpret_cast<double *>(lds + fa.a[k].lds_off) + local, sum2[s]);
                        continue;
                    }
                    if (is_minmax(kind)) continue;  // committed per entry by the caller
                }
                if (fa.a[k].vint)
                    atomicAdd(reinterpret_cast<unsigned long long *>(lds + fa.a[k].lds_off) + local, isum[s]);
                else if (nn[s])
                    atomicAdd(reinterpret_cast<double *>(lds + fa.a[k].lds_off) + local, sum[s]);
            }
        }
    }
};

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
// MG: a moment other than 2 (per-entry form; its own instantiation, so the run form's
// registers are not sized for it)
template <int NV, bool NARROW = false, bool MM = false, bool PK = false, bool MG = false, int TBT = TB_THREADS>
__global__ __launch_bounds__(TBT) void k_tile_reduce(FusedAggs fa, TileParams tp, const WorkUnit *units) {
    static_assert(!PK || (NV == 2 && NARROW), "packed pairs of narrow slots");
    extern __shared__ __align__(16) unsigned char lds_raw[];
    // per region (one round) / stream segment (rounds of SEGS): entries, chunk prefix, and the
    // first entry -- regions: absolute (u64 s_rbase); segments: the offset in their pass-A
    // workgroup's stream (u32 s_a; the workgroup follows from the segment index)
    constexpr uint32_t SEGS = 2 * TBT;
    __shared__ uint32_t s_fill[SEGS + 1];
    __shared__ uint32_t s_pre[SEGS + 2];
    __shared__ uint64_t s_b64[1024 + 1];  // s_rbase and s_a share it (one mode per launch)
    uint64_t *s_rbase = s_b64;
    uint32_t *s_a = reinterpret_cast<uint32_t *>(s_b64);
    static_assert(2 * (1024 + 1) >= SEGS + 1, "s_a fits s_b64");
    const WorkUnit u = units[blockIdx.x];
    const uint32_t t = u.tile;
    const uint32_t cap = tp.cap[t];
    // regions of pass-A workgroups w_begin .. w_end - 1 (<= W <= 1024, host checks), then
    // region nwr: this unit's slice `part` of `parts` of the tile's spill area (8-aligned)
    const uint32_t nwr = u.w_end - u.w_begin, nw = nwr + 1;
    const uint32_t part = u.pad & 0xffffu, parts = u.pad >> 16;
    const uint32_t F = min(tp.spill_fill[t], tp.spill_cap[t]);
    const uint32_t s0 = part == 0 ? 0u : min(F, (uint32_t)((uint64_t)F * part / parts) & ~7u);
    const uint32_t s1 = part + 1 >= parts ? F : min(F, (uint32_t)((uint64_t)F * (part + 1) / parts) & ~7u);
    const uint64_t spill0 = tp.spill_base + tp.spill_start[t] + s0;  // first entry of the slice
    // Stream layout: the unit's segments are (workgroup, commit) pairs, w_begin <= w < w_end and
    // c < ncw, taken in rounds of SEGS; segment g of the unit is w = w_begin + g / ncw,
    // c = g % ncw, its run [tab[row], tab[row + ncw]) with row = (w (T + 1) + t) ncw + c
    // (consecutive lanes read consecutive commits).  Regions: one round of nw regions.
    // two consecutive segments per thread and round; the next round's table entries are
    // fetched into registers while this round's chunks are processed
    static_assert(TBT <= 1024, "segments per round");
    const bool stream = tp.stream != 0;
    const uint32_t T = tp.ntiles, ncw = tp.ncw;
    const uint32_t nseg = stream ? nwr * ncw : nw;
    const uint32_t rounds = stream ? (nseg + SEGS - 1) / SEGS : 1u;
    uint32_t pf_f[2] = {0, 0}, pf_a[2] = {0, 0};
    auto fetch = [&](uint32_t r) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint32_t g = r * SEGS + 2 * threadIdx.x + h;
            pf_f[h] = 0;
            if (g < nseg) {
                const uint32_t w = u.w_begin + g / ncw, c = g % ncw;
                const uint64_t row = ((uint64_t)w * (T + 1) + t) * ncw + c;
                const uint32_t a = tp.tab[row], e = tp.tab[row + ncw];
                pf_f[h] = e - a;
                pf_a[h] = a;
            }
        }
    };
    // stream layout: the fetched segments into LDS and the block-wide exclusive scan of their
    // chunk counts (wave shuffles + wave totals; one barrier inside); returns whether this
    // thread's segments hold entries.  Segments past the unit's count 0 chunks, so s_pre[cnt]
    // is the round's total for any cnt <= SEGS.
    __shared__ uint32_t s_wsum[TBT / 64];
    auto stream_round = [&](uint32_t r) -> bool {
        const uint32_t k = 2 * threadIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        const uint32_t f0 = r * SEGS + k < nseg ? pf_f[0] : 0u, f1 = r * SEGS + k + 1 < nseg ? pf_f[1] : 0u;
        const uint32_t ch0 = (f0 + 7) >> 3, ch = ch0 + ((f1 + 7) >> 3);
        s_fill[k] = f0;
        s_fill[k + 1] = f1;
        s_a[k] = pf_a[0];
        s_a[k + 1] = pf_a[1];
        uint32_t inc = ch;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(inc, off, 64);
            if ((int)lane >= off) inc += y;
        }
        if (lane == 63) s_wsum[wave] = inc;
        __syncthreads();
        uint32_t before = 0, tot = 0;
#pragma unroll
        for (uint32_t v = 0; v < TBT / 64; v++) {
            const uint32_t x = s_wsum[v];
            before += v < wave ? x : 0u;
            tot += x;
        }
        s_pre[k] = before + inc - ch;
        s_pre[k + 1] = before + inc - ch + ch0;
        if (threadIdx.x == 0) s_pre[SEGS] = tot;
        return (f0 | f1) != 0;
    };
    auto load_round = [&]() -> bool {  // regions
        bool any = false;
        for (uint32_t k = threadIdx.x; k < nw; k += TBT) {
            const uint32_t f = k < nwr ? min(tp.fills[(uint64_t)t * tp.W + u.w_begin + k], cap) : (s1 > s0 ? s1 - s0 : 0u);
            s_fill[k] = f;
            s_rbase[k] = k < nwr ? (uint64_t)(u.w_begin + k) * tp.wg_stride + tp.toff[t] : spill0;
            any |= f != 0;
        }
        return any;
    };
    // exclusive scan of the round's chunk counts by the first wave (per segments per lane)
    auto scan_round = [&]() {  // regions
        if (threadIdx.x >= 64) return;
        const uint32_t cnt = nw;
        const uint32_t lane = threadIdx.x, per = (cnt + 63) / 64, k0 = lane * per;
        uint32_t sum = 0;
        for (uint32_t k = k0; k < k0 + per && k < cnt; k++) sum += (s_fill[k] + 7) >> 3;
        uint32_t inc = sum;
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(inc, off, 64);
            if ((int)lane >= off) inc += y;
        }
        uint32_t acc = inc - sum;
        for (uint32_t k = k0; k < k0 + per && k < cnt; k++) {
            s_pre[k] = acc;
            acc += (s_fill[k] + 7) >> 3;
        }
        if (lane == 63) s_pre[cnt] = inc;
    };
    bool any0;
    if (stream) {
        fetch(0);
        any0 = stream_round(0);
    } else {
        any0 = load_round();
    }
    if (!__syncthreads_or(any0 || (stream && rounds > 1))) return;
    uint32_t *lw = reinterpret_cast<uint32_t *>(lds_raw);
    for (uint32_t i = threadIdx.x; i < fa.lds_words; i += TBT) lw[i] = 0;
    if (!tp.flags_mode && !stream) scan_round();
    __syncthreads();
    // MM: the plan has min / max aggregators (a separate instantiation: their code would
    // raise the count / sum kernel's registers past the 1024-thread budget)
    if constexpr (MM) {  // min / max cells start at the kind's identity (after the zero fill)
        const uint32_t ncells = 1u << tp.s_log2;
        #pragma unroll
        for (int k = 0; k < MAX_FUSED_AGGS; k++) {
            if (k >= fa.na || !is_minmax(fa.a[k].kind)) continue;
            if (mm_cell32(fa.a[k].dtype)) {
                uint32_t *cells = reinterpret_cast<uint32_t *>(lds_raw + fa.a[k].lds_off);
                const uint32_t id = mm_identity32(fa.a[k].dtype, fa.a[k].kind == VH_AGG_MAX);
                for (uint32_t i = threadIdx.x; i < ncells; i += TBT) cells[i] = id;
                continue;
            }
            uint64_t *cells = reinterpret_cast<uint64_t *>(lds_raw + fa.a[k].lds_off);
            const uint64_t id = mm_identity(fa.a[k].dtype, fa.a[k].kind == VH_AGG_MAX);
            for (uint32_t i = threadIdx.x; i < ncells; i += TBT) cells[i] = id;
        }
        __syncthreads();
    }
    // per value slot: the dtype of a min / max aggregator on it (-1: none)
    int mmdt[NV > 0 ? NV : 1];
#pragma unroll
    for (int s = 0; s < NV; s++) {
        mmdt[s] = -1;
#pragma unroll
        for (int k = 0; k < MAX_FUSED_AGGS; k++)
            if (k < fa.na && ((tp.mmk >> k) & 1u) && tp.val_slot[k] == s) mmdt[s] = fa.a[k].dtype;
    }
    if (!tp.flags_mode) {
        // the run form of min / max / moment plans: one chunk per lane (128 VGPRs at 1024
        // threads; a 512-thread form with two chunks and the entry loop unrolled kept 176 B per
        // lane in scratch memory and ran pass B at 10.6 against 5.5 ms)
        constexpr int VU = MM ? 1 : tb_vu<NV>();
        const uint16_t *ent16 = reinterpret_cast<const uint16_t *>(tp.entries);
        for (uint32_t r = 0; r < rounds; r++) {
        if (r > 0) {  // the next round's segments (every lane is done with this round's)
            __syncthreads();
            stream_round(r);
            __syncthreads();
        }
        if (stream && r + 1 < rounds) fetch(r + 1);
        const uint32_t cnt = stream ? min(SEGS, nseg - r * SEGS) : nw;
        const uint32_t C = s_pre[cnt];
        // wave-major chunks: wave v takes the contiguous chunk block [cb, ce), 64 consecutive
        // chunks per load instruction, so a lane's chunks only grow and its segment cursor
        // walks forward over the block's few segments (an interleaved assignment skipped
        // TBT chunks, i.e. dozens of short segments, per step)
        const uint32_t lane = threadIdx.x & 63, nwv = TBT / 64;
        const uint32_t per_wave = ((C + nwv - 1) / nwv + 63) & ~63u;
        const uint32_t cb = min(C, (threadIdx.x >> 6) * per_wave), ce = min(C, cb + per_wave);
        uint32_t kk = 0;  // segment of this lane's current chunk: the last k with s_pre[k] <= cb
        if (cb < ce) {
            uint32_t lo = 0, hi = cnt;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_pre[mid] <= cb) lo = mid;
                else hi = mid;
            }
            kk = lo;
        }
        for (uint32_t c0 = cb; c0 < ce; c0 += 64 * VU) {
            uint4 ev[VU];
            double2 vv[VU][NV > 0 ? NV : 1][4];
            uint32_t rem[VU];
#pragma unroll
            for (int j = 0; j < VU; j++) {
                const uint32_t c = c0 + j * 64 + lane;
                const uint32_t cc = c < ce ? c : ce - 1;
                while (s_pre[kk + 1] <= cc) kk++;
                const uint32_t q = (cc - s_pre[kk]) * 8;
                // regions / segments start at multiples of 8 entries and hold a multiple of 8,
                // so the chunk never leaves its segment (entries past the fill are ignored)
                const uint64_t e = (stream ? (uint64_t)(u.w_begin + (r * SEGS + kk) / ncw) * tp.wg_stride + s_a[kk] : s_rbase[kk]) + q;
                rem[j] = c < ce ? min(8u, s_fill[kk] - q) : 0u;
                ev[j] = *reinterpret_cast<const uint4 *>(ent16 + e);
#pragma unroll
                for (int s = 0; s < NV; s++) {
                    if constexpr (PK) {
                        {  // tp.vpacked: the chunk's 8 x slot s at 64 * (e / 8) + 32 * s bytes
                            const bool fl = (tp.vfloat >> s) & 1, sg = (tp.vsigned >> s) & 1;
                            const uint4 *pp = reinterpret_cast<const uint4 *>(reinterpret_cast<const uint32_t *>(tp.values[0]) + e * 2 + 8 * s);
                            const uint4 a = pp[0], b = pp[1];
                            vv[j][s][0] = make_double2(slot_wide(a.x, fl, sg), slot_wide(a.y, fl, sg));
                            vv[j][s][1] = make_double2(slot_wide(a.z, fl, sg), slot_wide(a.w, fl, sg));
                            vv[j][s][2] = make_double2(slot_wide(b.x, fl, sg), slot_wide(b.y, fl, sg));
                            vv[j][s][3] = make_double2(slot_wide(b.z, fl, sg), slot_wide(b.w, fl, sg));
                            continue;
                        }
                    }
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
            if constexpr (!MG) {
                // consecutive entries of one cell (sorted / clustered rows) are added up in
                // registers first: one LDS atomic per run of a chunk, not per entry (min / max /
                // moment-2 plans: the extended run); a moment other than 2 takes the per-entry
                // form below
#pragma unroll
                for (int j = 0; j < VU; j++) {
                    const uint32_t words[4] = {ev[j].x, ev[j].y, ev[j].z, ev[j].w};
                    if constexpr (MM && NV == 1 && !NARROW) {
                        if (tp.mm_simple) {
                            // one float64 slot, count / sum / min / max of it: the run of one
                            // cell folds all four in registers (min / max as order-preserving
                            // bits) and commits with one LDS atomic per aggregator at its end
                            const double vx[8] = {vv[j][0][0].x, vv[j][0][0].y, vv[j][0][1].x, vv[j][0][1].y,
                                                  vv[j][0][2].x, vv[j][0][2].y, vv[j][0][3].x, vv[j][0][3].y};
                            const int oc = tp.mm_off[0], osm = tp.mm_off[1], omn = tp.mm_off[2], omx = tp.mm_off[3];
                            const bool cnn = tp.mm_cnt_nn;
                            uint32_t cur = ~0u, rc = 0, rn = 0;
                            double rs = 0.0;
                            uint64_t rlo = ~0ull, rhi = 0;
                            auto commit = [&]() __attribute__((always_inline)) {
                                if (oc >= 0 && (cnn ? rn : rc)) atomicAdd(reinterpret_cast<uint32_t *>(lds_raw + oc) + cur, cnn ? rn : rc);
                                if (rn) {
                                    if (osm >= 0) atomicAdd(reinterpret_cast<double *>(lds_raw + osm) + cur, rs);
                                    if (omn >= 0) atomicMin(reinterpret_cast<unsigned long long *>(lds_raw + omn) + cur, (unsigned long long)rlo);
                                    if (omx >= 0) atomicMax(reinterpret_cast<unsigned long long *>(lds_raw + omx) + cur, (unsigned long long)rhi);
                                }
                            };
#pragma unroll
                            for (int x = 0; x < 8; x++) {
                                const uint32_t local = (words[x >> 1] >> (16 * (x & 1))) & 0xffffu;
                                if ((uint32_t)x >= rem[j] || local == DUMMY_CELL) continue;
                                if (local != cur) {
                                    if (cur != ~0u) commit();
                                    cur = local;
                                    rc = rn = 0;
                                    rs = 0.0;
                                    rlo = ~0ull;
                                    rhi = 0;
                                }
                                const double v = vx[x];
                                rc++;
                                if (v == v) {
                                    const uint64_t o = ord_bits(v);
                                    rn++;
                                    rs += v;
                                    rlo = o < rlo ? o : rlo;
                                    rhi = o > rhi ? o : rhi;
                                }
                            }
                            if (cur != ~0u) commit();
                            continue;
                        }
                    }
                    if constexpr (MM) {
                        // min / max: a lane folds each run of one cell in its chunk (an entry
                        // whose successor is another cell, or the chunk's last, ends the run) in
                        // an order-preserving u64 form per value slot, and commits the run's
                        // min / max with one non-returning LDS atomic per aggregator: sorted /
                        // clustered rows stop paying an atomic per entry on one address, random
                        // rows (runs of one) pay what a per-entry atomic did.  The extended
                        // run's flush is large: one copy of the entry body in a run-time loop
                        // that takes the head of shift registers (an unrolled loop spills; a
                        // run-time index into the chunk's arrays goes through scratch memory)
                        double sv[NV > 0 ? NV : 1][8];
#pragma unroll
                        for (int s = 0; s < NV; s++)
#pragma unroll
                            for (int h = 0; h < 4; h++) {
                                sv[s][2 * h] = vv[j][s][h].x;
                                sv[s][2 * h + 1] = vv[j][s][h].y;
                            }
                        uint32_t w0 = words[0], w1 = words[1], w2 = words[2], w3 = words[3];
                        TileRun<NV, true> run;
                        uint32_t cur = ~0u;
                        uint64_t lo[NV > 0 ? NV : 1], hi[NV > 0 ? NV : 1];
                        bool open = false;  // a fold of two or more entries is in progress
                        auto entry = [&](uint32_t x) __attribute__((always_inline)) {
                            const uint32_t local = w0 & 0xffffu, next = (w0 >> 16) & 0xffffu;
                            double v[NV > 0 ? NV : 1];
#pragma unroll
                            for (int s = 0; s < NV; s++) v[s] = sv[s][0];
                            if (local != DUMMY_CELL) {  // (DUMMY_CELL: run padding of the wide pass A)
                                if (local != cur) {
                                    if (cur != ~0u) run.flush(fa, tp, lds_raw, cur);
                                    cur = local;
                                    run.clear();
                                }
                                run.add(tp, v);
                                const bool end = x + 1 >= rem[j] || next != local;
                                if (!open && end) {
                                    // a run of one entry (random rows): its value goes straight
                                    // to the cells, one non-returning atomic per aggregator
#pragma unroll
                                    for (int k = 0; k < MAX_FUSED_AGGS; k++) {
                                        if (!((tp.mmk >> k) & 1u)) continue;
                                        const FusedAgg &a = fa.a[k];
                                        const bool m = a.kind == VH_AGG_MAX;
#pragma unroll
                                        for (int s = 0; s < NV; s++) {
                                            if (s != tp.val_slot[k]) continue;
                                            if (mm_cell32(a.dtype))
                                                mm_lds32<false>(reinterpret_cast<uint32_t *>(lds_raw + a.lds_off) + local, a.dtype, m, v[s]);
                                            else
                                                mm_lds<false>(reinterpret_cast<uint64_t *>(lds_raw + a.lds_off) + local, a.dtype, m, v[s]);
                                        }
                                    }
                                } else {
                                    // a longer run: folded in registers, committed at its end
#pragma unroll
                                    for (int s = 0; s < NV; s++) {
                                        if (mmdt[s] < 0) continue;
                                        const bool ok = !dt_float(mmdt[s]) || v[s] == v[s];  // NaN never enters
                                        const uint64_t o = mm_okey(mmdt[s], v[s]);
                                        const uint64_t l0 = open ? lo[s] : ~0ull, h0 = open ? hi[s] : 0ull;
                                        lo[s] = ok && o < l0 ? o : l0;
                                        hi[s] = ok && o > h0 ? o : h0;
                                    }
                                    open = !end;
                                    if (end) {
#pragma unroll
                                        for (int k = 0; k < MAX_FUSED_AGGS; k++) {
                                            if (!((tp.mmk >> k) & 1u)) continue;
                                            const FusedAgg &a = fa.a[k];
                                            const bool m = a.kind == VH_AGG_MAX;
#pragma unroll
                                            for (int s = 0; s < NV; s++) {
                                                if (s != tp.val_slot[k]) continue;
                                                const uint64_t o = m ? hi[s] : lo[s];
                                                if (o == (m ? 0ull : ~0ull)) continue;  // the cell's identity: a no-op
                                                const double r = mm_unokey(a.dtype, o);
                                                if (mm_cell32(a.dtype))
                                                    mm_lds32<false>(reinterpret_cast<uint32_t *>(lds_raw + a.lds_off) + local, a.dtype, m, r);
                                                else
                                                    mm_lds<false>(reinterpret_cast<uint64_t *>(lds_raw + a.lds_off) + local, a.dtype, m, r);
                                            }
                                        }
                                    }
                                }
                            }
                            w0 = (w0 >> 16) | (w1 << 16);
                            w1 = (w1 >> 16) | (w2 << 16);
                            w2 = (w2 >> 16) | (w3 << 16);
                            w3 >>= 16;
#pragma unroll
                            for (int s = 0; s < NV; s++)
#pragma unroll
                                for (int h = 0; h < 7; h++) sv[s][h] = sv[s][h + 1];
                        };
#pragma unroll 1
                        for (uint32_t x = 0; x < rem[j]; x++) entry(x);
                        if (cur != ~0u) run.flush(fa, tp, lds_raw, cur);
                    } else {
                        TileRun<NV, false> run;
                        uint32_t cur = ~0u;
#pragma unroll
                        for (int x = 0; x < 8; x++) {
                            const uint32_t local = (words[x >> 1] >> (16 * (x & 1))) & 0xffffu;
                            if ((uint32_t)x < rem[j] && local != DUMMY_CELL) {
                                if (local != cur) {
                                    if (cur != ~0u) run.flush(fa, tp, lds_raw, cur);
                                    cur = local;
                                    run.clear();
                                }
                                double v[NV > 0 ? NV : 1];
#pragma unroll
                                for (int s = 0; s < NV; s++) v[s] = (x & 1) ? vv[j][s][x >> 1].y : vv[j][s][x >> 1].x;
                                run.add(tp, v);
                            }
                        }
                        if (cur != ~0u) run.flush(fa, tp, lds_raw, cur);
                    }
                }
            } else {
                // chunk j as a compile-time index (the unroller gave up on this body, and a
                // run-time j indexed vv through scratch memory)
                auto chunk = [&](auto jc) {
                    constexpr int j = decltype(jc)::value;
                    const uint32_t words[4] = {ev[j].x, ev[j].y, ev[j].z, ev[j].w};
#pragma unroll
                    for (int x = 0; x < 8; x++) {
                        // a guard, not a break: the loop stays unrolled and vv in registers
                        if ((uint32_t)x < rem[j]) {
                            double v[NV > 0 ? NV : 1];
#pragma unroll
                            for (int s = 0; s < NV; s++) v[s] = (x & 1) ? vv[j][s][x >> 1].y : vv[j][s][x >> 1].x;
                            const uint32_t local = (words[x >> 1] >> (16 * (x & 1))) & 0xffffu;
                            if (DBG(tp.debug) & 8) asm volatile("" :: "v"(local));
                            else if (local != DUMMY_CELL) reduce_entry<NV, MM>(fa, tp, lds_raw, local, 0xfu, v);
                        }
                    }
                };
                static_assert(VU <= 8, "chunks per step");
                chunk(std::integral_constant<int, 0>{});
                if constexpr (VU > 1) chunk(std::integral_constant<int, 1>{});
                if constexpr (VU > 2) chunk(std::integral_constant<int, 2>{});
                if constexpr (VU > 3) chunk(std::integral_constant<int, 3>{});
                if constexpr (VU > 4) chunk(std::integral_constant<int, 4>{});
                if constexpr (VU > 5) chunk(std::integral_constant<int, 5>{});
                if constexpr (VU > 6) chunk(std::integral_constant<int, 6>{});
                if constexpr (VU > 7) chunk(std::integral_constant<int, 7>{});
            }
        }
        }  // rounds
    } else {
        for (uint32_t k = 0; k < nw; k++) {
            const uint32_t cnt = s_fill[k];
            const uint64_t base = k < nwr ? (uint64_t)(u.w_begin + k) * tp.wg_stride + tp.toff[t] : spill0;
            // min / max plans: fewer entries in flight (8 inlined reduce_entry bodies of two
            // slots spill)
            constexpr int UN = MM && NV > 1 ? 2 : TB_UNROLL;
            for (uint32_t q0 = 0; q0 < cnt; q0 += TBT * UN) {
                uint32_t ent[UN];
                double v[UN][NV > 0 ? NV : 1];
#pragma unroll
                for (int j = 0; j < UN; j++) {
                    const uint32_t q = q0 + j * TBT + threadIdx.x;
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
                for (int j = 0; j < UN; j++) {
                    const uint32_t q = q0 + j * TBT + threadIdx.x;
                    if (q < cnt) reduce_entry<NV, MM>(fa, tp, lds_raw, ent[j] & 0xffffu, ent[j] >> 16, v[j]);
                }
            }
        }
    }
    __syncthreads();
    if (DBG(tp.debug) & 16) return;
    const uint64_t c0 = (uint64_t)t << tp.s_log2;
    const uint32_t ncell = (uint32_t)min((uint64_t)1 << tp.s_log2, tp.cells - c0);
    #pragma unroll
    for (int k = 0; k < MAX_FUSED_AGGS; k++) {
        if (k >= fa.na) break;
        for (uint32_t i = threadIdx.x; i < ncell; i += TBT) {
            if (fa.a[k].kind == VH_AGG_COUNT) {
                const uint32_t v = reinterpret_cast<const uint32_t *>(lds_raw + fa.a[k].lds_off)[i];
                if (v) atomicAdd((unsigned long long *)fa.a[k].grid + c0 + i, (unsigned long long)v);
            } else if (is_minmax(fa.a[k].kind)) {
                if constexpr (MM) {
                    const bool mx = fa.a[k].kind == VH_AGG_MAX;
                    const int dt = fa.a[k].dtype;
                    void *tmp = tp.mmtmp[k];
                    if (mm_cell32(dt)) {
                        const uint32_t v = reinterpret_cast<const uint32_t *>(lds_raw + fa.a[k].lds_off)[i];
                        if (v == mm_identity32(dt, mx)) continue;
                        if (!tmp) mm_grid(fa.a[k].grid, c0 + i, dt, mx, mm_cell32_slot(dt, v), false);
                        else if (dt_signed(dt)) mx ? atomicMax(static_cast<int *>(tmp) + c0 + i, (int)v) : atomicMin(static_cast<int *>(tmp) + c0 + i, (int)v);
                        else mx ? atomicMax(static_cast<unsigned *>(tmp) + c0 + i, v) : atomicMin(static_cast<unsigned *>(tmp) + c0 + i, v);
                        continue;
                    }
                    const uint64_t v = reinterpret_cast<const uint64_t *>(lds_raw + fa.a[k].lds_off)[i];
                    if (v == mm_identity(dt, mx)) continue;
                    if (!tmp) mm_grid(fa.a[k].grid, c0 + i, dt, mx, v, true);
                    else if (dt_signed(dt))
                        mx ? atomicMax(static_cast<long long *>(tmp) + c0 + i, (long long)v) : atomicMin(static_cast<long long *>(tmp) + c0 + i, (long long)v);
                    else
                        mx ? atomicMax(static_cast<unsigned long long *>(tmp) + c0 + i, (unsigned long long)v)
                           : atomicMin(static_cast<unsigned long long *>(tmp) + c0 + i, (unsigned long long)v);
                }
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

// integer binner kernels (fast modes 8-11): int32 / int64 binners, float64 (or no) / float32 values
template <int ND, int NV, typename F> static void int_kernel(int fast, F &&f) {
    if constexpr (NV == 0) {
        if (fast == 8) f(k_tile_scatter_f64<ND, 0, fast_sb_nd(0, ND), int32_t, false, double>);
        else f(k_tile_scatter_f64<ND, 0, fast_sb_nd(0, ND), int64_t, false, double>);
    } else {
        switch (fast) {
        case 8: f(k_tile_scatter_f64<ND, NV, fast_sb_nd(NV, ND), int32_t, false, double>); break;
        case 9: f(k_tile_scatter_f64<ND, NV, fast_sb_narrow(NV), int32_t, false, float>); break;
        case 10: f(k_tile_scatter_f64<ND, NV, fast_sb_nd(NV, ND), int64_t, false, double>); break;
        default: f(k_tile_scatter_f64<ND, NV, fast_sb_narrow(NV), int64_t, false, float>);
        }
    }
}
template <int ND, int NV>
static void launch_scatter_int(int fast, unsigned grid, size_t lds, const BinPlan &plan, const FusedAggs &fa,
                               const TileParams &tp, uint64_t n) {
    int_kernel<ND, NV>(fast, [&](auto kern) {
        BinPlan p = plan;
        FusedAggs f = fa;
        TileParams t = tp;
        uint64_t nn = n;
        void *args[] = {(void *)&p, (void *)&f, (void *)&t, (void *)&nn};
        VH_HIP(hipLaunchKernel(reinterpret_cast<const void *>(kern), dim3(grid), dim3(TA_THREADS), args, lds, stream()));
    });
}
template <int ND, int NV> static int scatter_int_blocks(int fast, size_t lds) {
    int nb = 0;
    int_kernel<ND, NV>(fast, [&](auto kern) {
        VH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void *>(kern), TA_THREADS, lds));
    });
    return nb;
}

// fast: 0 = generic kernel, 1 = fast kernel one batch per commit, 2 = fast kernel with
// fast_sb(NV) batches per commit (when its LDS fits)
template <int ND, int NV>
static void launch_scatter(int fast, unsigned grid, size_t lds, const BinPlan &plan, const FusedAggs &fa,
                           const TileParams &tp, uint64_t n) {
    if constexpr (ND > 0) {
        if (fast == 5 && tp.rowmask) {
            hipLaunchKernelGGL((k_tile_scatter_f64<ND, NV, fast_sb_narrow(NV), float, true>), dim3(grid), dim3(TA_THREADS), lds, stream(), plan, fa, tp, n);
            return;
        }
        if (fast == 2 && tp.rowmask) {
            hipLaunchKernelGGL((k_tile_scatter_f64<ND, NV, fast_sb_nd(NV, ND), double, true>), dim3(grid), dim3(TA_THREADS), lds, stream(), plan, fa, tp, n);
            return;
        }
        if (fast == 5) {
            hipLaunchKernelGGL((k_tile_scatter_f64<ND, NV, fast_sb_narrow(NV), float>), dim3(grid), dim3(TA_THREADS), lds, stream(), plan, fa, tp, n);
            return;
        }
        if constexpr (ND <= 2) {
            if (fast >= 8 && fast <= 11) {
                launch_scatter_int<ND, NV>(fast, grid, lds, plan, fa, tp, n);
                return;
            }
        }
        if constexpr (NV > 0) {
            if (fast == 6) {
                hipLaunchKernelGGL((k_tile_scatter_f64<ND, NV, fast_sb_nd(NV, ND), float, false, double>), dim3(grid), dim3(TA_THREADS), lds, stream(), plan, fa, tp, n);
                return;
            }
            if (fast == 7) {
                hipLaunchKernelGGL((k_tile_scatter_f64<ND, NV, fast_sb_narrow(NV), double, false, float>), dim3(grid), dim3(TA_THREADS), lds, stream(), plan, fa, tp, n);
                return;
            }
        }
        if (fast == 2) {
            hipLaunchKernelGGL((k_tile_scatter_f64<ND, NV, fast_sb_nd(NV, ND)>), dim3(grid), dim3(TA_THREADS), lds, stream(), plan, fa, tp, n);
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
static bool aligned8(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 7) == 0; }

template <int ND, int NV> static int scatter_blocks_per_cu(int fast, size_t lds, bool mk) {
    int nb = 0;
    if constexpr (ND > 0) {
        if (fast == 5 && mk) {
            VH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tile_scatter_f64<ND, NV, fast_sb_narrow(NV), float, true>, TA_THREADS, lds));
            return nb;
        }
        if (fast == 2 && mk) {
            VH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tile_scatter_f64<ND, NV, fast_sb_nd(NV, ND), double, true>, TA_THREADS, lds));
            return nb;
        }
        if (fast == 5) {
            VH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tile_scatter_f64<ND, NV, fast_sb_narrow(NV), float>, TA_THREADS, lds));
            return nb;
        }
        if constexpr (ND <= 2) {
            if (fast >= 8 && fast <= 11) return scatter_int_blocks<ND, NV>(fast, lds);
        }
        if constexpr (NV > 0) {
            if (fast == 6) {
                VH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tile_scatter_f64<ND, NV, fast_sb_nd(NV, ND), float, false, double>, TA_THREADS, lds));
                return nb;
            }
            if (fast == 7) {
                VH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tile_scatter_f64<ND, NV, fast_sb_narrow(NV), double, false, float>, TA_THREADS, lds));
                return nb;
            }
        }
        if (fast == 2) {
            VH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tile_scatter_f64<ND, NV, fast_sb_nd(NV, ND)>, TA_THREADS, lds));
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

template <int NV> static int scatter_blocks_per_cu_nd(int nd, int fast, size_t lds, bool mk) {
    switch (nd) {
    case 1: return scatter_blocks_per_cu<1, NV>(fast, lds, mk);
    case 2: return scatter_blocks_per_cu<2, NV>(fast, lds, mk);
    case 3: return scatter_blocks_per_cu<3, NV>(fast, lds, mk);
    case -1: return scatter_blocks_per_cu<-1, NV>(0, lds, false);
    default: return scatter_blocks_per_cu<0, NV>(0, lds, false);
    }
}

// value-dtype combinations with their own ordinal kernel (0: float64; h2o's int8 / float32
// sums; others take the run-time-switch kernel, -1)
// narrow (VN) kernels: h2o's int8 / float32 combinations and the run-time switch
template <int NV, int SB, typename F> static void ord_by_dts_narrow(int dt0, int dt1, F &&f) {
#define VH_ORD_DT(a, b) if (dt0 == (a) && (NV < 2 || dt1 == (b))) return f(k_tile_scatter_ord<NV, SB, false, (a), NV < 2 ? VH_F64 : (b), true>);
    VH_ORD_DT(VH_I8, VH_I8)
    VH_ORD_DT(VH_I8, VH_F32)
    VH_ORD_DT(VH_F32, VH_I8)
    VH_ORD_DT(VH_F32, VH_F32)
    VH_ORD_DT(VH_I32, VH_I32)
#undef VH_ORD_DT
    f(k_tile_scatter_ord<NV, SB, false, -1, -1, true>);
}
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
template <bool SET> static const void *ord_kernel_t(int nv, int fast_mode, int dt0, int dt1, bool mk) {
    const void *k = nullptr;
    auto take = [&](auto kern) { k = reinterpret_cast<const void *>(kern); };
    if (mk) {  // shared keep mask: int32 key, float64 values (or none), batched commits
        if constexpr (!SET) {
            if (nv == 0) return reinterpret_cast<const void *>(k_tile_scatter_ord<0, 1, false, VH_F64, VH_F64, false, true>);
            if (fast_mode != 2 || dt0 != VH_F64 || (nv > 1 && dt1 != VH_F64)) return nullptr;
            return nv == 1 ? reinterpret_cast<const void *>(k_tile_scatter_ord<1, fast_sb(1), false, VH_F64, VH_F64, false, true>)
                           : reinterpret_cast<const void *>(k_tile_scatter_ord<2, fast_sb(2), false, VH_F64, VH_F64, false, true>);
        }
        return nullptr;
    }
    if constexpr (!SET) {
        if (fast_mode == 3) {  // narrow slots, fast_sb_narrow(nv) batches per commit
            if (nv == 1) ord_by_dts_narrow<1, fast_sb_narrow(1)>(dt0, dt1, take);
            else ord_by_dts_narrow<2, fast_sb_narrow(2)>(dt0, dt1, take);
            return k;
        }
    }
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
static const void *ord_kernel(int nv, int fast_mode, bool set, int dt0, int dt1, bool mk = false) {
    return set ? ord_kernel_t<true>(nv, fast_mode, dt0, dt1, mk) : ord_kernel_t<false>(nv, fast_mode, dt0, dt1, mk);
}

static bool try_tiled_impl(const BinPlan &plan, const FusedAggs &fa_in, uint64_t n, uint64_t cells, int nd_f64);

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
        if (!try_tiled_impl(plan, fa_in, n - 1, cells, nd_f64)) return false;
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
    return try_tiled_impl(plan, fa_in, n, cells, nd_f64);
}

// Partition scratch shared by every grid of a device: a 1e9-row count+sum needs ~10 GB of
// regions, which a per-grid buffer would hipMalloc/hipFree for every query (a grid lives
// for one query).  Held under the device's lock while a bin is enqueued; reuse is ordered
// by the library stream.
struct TileScratch {
    std::mutex mu;
    DevBuf entries, values, meta, mmtmp, tab;
};

static bool getenv_flag_off(const char *name) {  // NAME=0 turns a default-on path off (A/B runs)
    const char *e = getenv(name);
    return e && atoi(e) == 0;
}
static TileScratch &tile_scratch() {
    static std::mutex g;
    static std::map<int, std::unique_ptr<TileScratch>> m;
    std::lock_guard<std::mutex> lk(g);
    auto &p = m[current_device()];
    if (!p) p = std::make_unique<TileScratch>();
    return *p;
}

static bool try_tiled_core(const BinPlan &plan, const FusedAggs &fa_in, uint64_t n, uint64_t cells, int nd_f64,
                           const uint8_t *rowmask);

// A plan whose aggregators all carry the same keep mask (a selection / filter) and whose
// binners have none: the fast pass A applies the mask per row (MK kernels) and the rest of
// the plan runs as unmasked -- counts of every kept row, no flag entries.  Only when a fast
// kernel takes the plan; otherwise the masks go to the generic pass A as before.  (C2 with a
// selection: generic pass A 12.0 ms, profiles/r06_mask.txt.)  VH_TILE_ROWMASK=0: off.
static bool try_tiled_impl(const BinPlan &plan, const FusedAggs &fa_in, uint64_t n, uint64_t cells, int nd_f64) {
    const uint8_t *m = fa_in.na > 0 ? fa_in.a[0].mask : nullptr;
    for (int k = 1; k < fa_in.na && m; k++)
        if (fa_in.a[k].mask != m) m = nullptr;
    for (int d = 0; d < plan.nb && m; d++)
        if (plan.b[d].mask) m = nullptr;
    if (m && !getenv_flag_off("VH_TILE_ROWMASK")) {
        FusedAggs f2 = fa_in;
        for (int k = 0; k < f2.na; k++) f2.a[k].mask = nullptr;
        if (try_tiled_core(plan, f2, n, cells, nd_f64, m)) return true;
    }
    return try_tiled_core(plan, fa_in, n, cells, nd_f64, nullptr);
}

static bool try_tiled_core(const BinPlan &plan, const FusedAggs &fa_in, uint64_t n, uint64_t cells, int nd_f64,
                           const uint8_t *rowmask) {
    TileScratch &ws = tile_scratch();
    std::lock_guard<std::mutex> ws_lock(ws.mu);
    TileParams tp{};
    tp.rowmask = rowmask;
#ifdef VH_ABLATION
    if (const char *dbg = getenv("VH_TILE_DEBUG")) tp.debug = (uint32_t)atoi(dbg);
#endif
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
    // LDS bytes per cell of pass B: u32 counts, 8-byte sums, min / max 4 or 8 (mm_cell32)
    auto cell_bytes = [](const FusedAgg &a) -> uint64_t {
        return a.kind == VH_AGG_COUNT || (is_minmax(a.kind) && mm_cell32(a.dtype)) ? 4 : 8;
    };
    uint64_t per_cell = 0;
    for (int k = 0; k < fa_in.na; k++) per_cell += cell_bytes(fa_in.a[k]);
    // pass B's LDS tile: 96 KB for count / sum plans; wider cells (min / max / moment) get up
    // to 128 KB so their tiles keep 4096 cells (fewer tiles: longer pass-A runs per region)
    const uint64_t budget = per_cell > 12 ? std::max<uint64_t>(TILE_LDS_BUDGET, 128 * 1024) : TILE_LDS_BUDGET;
    uint32_t s_log2 = 0;
    while (s_log2 < 16 && ((uint64_t)2 << s_log2) * per_cell <= budget) s_log2++;
    const uint64_t S = 1ull << s_log2;
    const uint64_t T64 = (cells + S - 1) / S;
    if (T64 > TILE_MAX_TILES || T64 < 2) return false;
    const uint32_t T = (uint32_t)T64;

    FusedAggs fa = fa_in;
    uint64_t off = 0;
    for (int k = 0; k < fa.na; k++) {
        off = (off + 7) & ~uint64_t(7);
        fa.a[k].lds_off = (uint32_t)off;
        off += S * cell_bytes(fa.a[k]);
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
    for (int d = 0; d < plan.nb && fast; d++) fast = !plan.b[d].mask && aligned16(plan.b[d].data);
    for (int k = 0; k < fa.na; k++) {
        if (fa.a[k].mask) fast = false;
        if (fa.a[k].kind != VH_AGG_COUNT) {
            tp.vdata[tp.val_slot[k]] = fa.a[k].data;
            fast = fast && fa.a[k].data && fa.a[k].dtype == VH_F64 && aligned16(fa.a[k].data);
        }
        if (fa.a[k].kind == VH_AGG_COUNT && fa.a[k].data && fa.a[k].dtype != VH_F64) fast = false;
    }
    // the fast float32 pass A (k_tile_scatter_f64<ND, NV, SB, float>): native float32 scalar
    // binners without masks, float32 sums and counts (of every row, or keyed on a summed
    // column), no aggregator masks, 8-byte aligned columns, n even (row pairs).  It replaces
    // the generic pass A's per-dimension dtype dispatch, whose loads wait at every switch join
    // (C2 on float32 columns: 11.3 ms generic pass A, profiles/r06_f32.txt)
    // Mixed plans take the same kernel with a second value-pair array (modes 6 / 7 below).
    int nd_f32 = 0, mix_mode = 0;  // 5: float32 / float32, 6: float32 binners + float64 values, 7: the reverse
    if (!fast && !flags_mode && n % 2 == 0 && plan.nb >= 1 && plan.nb <= 3 && !getenv_flag_off("VH_TILE_F32")) {
        bool ok = true;
        int bt = -1, vt = -1;
        for (int d = 0; d < plan.nb; d++) {
            const BinnerDev &b = plan.b[d];
            const int dt = b.dtype;
            ok = ok && b.kind == 0 && (dt == VH_F32 || dt == VH_F64 || dt == VH_I32 || dt == VH_I64) && (bt < 0 || dt == bt) &&
                 !b.flip && !b.mask && (dt == VH_F64 || dt == VH_I64 ? aligned16(b.data) : aligned8(b.data));
            bt = dt;
        }
        for (int k = 0; k < fa.na; k++) {
            const FusedAgg &a = fa.a[k];
            ok = ok && !a.mask;
            if (a.kind == VH_AGG_COUNT) continue;
            ok = ok && a.kind == VH_AGG_SUM && a.data && (a.dtype == VH_F32 || a.dtype == VH_F64) && (vt < 0 || a.dtype == vt) &&
                 (a.dtype == VH_F64 ? aligned16(a.data) : aligned8(a.data));
            vt = a.dtype;
        }
        if (vt < 0) vt = bt;
        for (int k = 0; k < fa.na; k++)  // counts of a column: the summed one (flags_mode otherwise)
            if (fa.a[k].kind == VH_AGG_COUNT && fa.a[k].data) ok = ok && fa.a[k].dtype == vt;
        if (vt == VH_I32 || vt == VH_I64) vt = VH_F64;  // integer binners, no values: the float64 form
        if (ok) {
            if (bt == VH_I32 || bt == VH_I64)  // integer binners (1- and 2-d): 8 / 9 int32, 10 / 11 int64
                mix_mode = plan.nb > 2 ? 0 : (bt == VH_I32 ? 8 : 10) + (vt == VH_F32 ? 1 : 0);
            else
                mix_mode = bt == VH_F32 ? (vt == VH_F32 ? 5 : 6) : (vt == VH_F32 ? 7 : 0);
            if (mix_mode) nd_f32 = plan.nb;
        }
    }
    const bool ord = !fast && n % 2 == 0 && ord_fast_ok(plan, fa);
    tp.vdt[0] = tp.vdt[1] = VH_F64;
    if (ord) for (int k = 0; k < fa.na; k++)
        if (fa.a[k].kind != VH_AGG_COUNT) {
            tp.vdata[tp.val_slot[k]] = fa.a[k].data;
            tp.vdt[tp.val_slot[k]] = fa.a[k].dtype;
        }
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
    // fast kernel: several batches per commit when that staging fits the LDS; the ordinal
    // kernel with narrow slots stages 4-byte values (mode 3); the float32 kernel too (mode 5:
    // its sums are float32 bits in narrow slots)
    const bool narrow_ord = ord && vnarrow &&
                            fast_lds_bytes(nv, T, (uint32_t)(fast_sb_narrow(nv) * TA_BATCH), 4) <= LDS_MAX_BYTES;
    const bool vf32 = mix_mode == 5 || mix_mode == 7 || mix_mode == 9 || mix_mode == 11;
    const int sb_mix = vf32 ? fast_sb_narrow(nv) : fast_sb_nd(nv, plan.nb);
    const bool f32_ok = mix_mode != 0 && (nv == 0 || vnarrow == vf32) &&
                        fast_lds_bytes(nv, T, (uint32_t)(sb_mix * TA_BATCH), vf32 ? 4 : 8) <= LDS_MAX_BYTES;
    const int fast_mode = f32_ok ? mix_mode
                          : !(fast || ord) ? 0
                          : narrow_ord  ? 3
                          : fast_lds_bytes(nv, T, (uint32_t)(fast_sb_nd(nv, fast ? nd_f64 : 1) * TA_BATCH)) <= LDS_MAX_BYTES ? 2 : 1;
    // the scatter kernels' ND: float64 binner dimensions (fast or generic kernels read them as
    // float64), the float32 / mixed kernels' dimensions only when one of them runs, else the
    // generic dispatch (0) or the set-ordinal form (-1) -- a float32 plan the fast kernels do
    // not take must not reach an ND > 0 generic kernel, which would read its columns as float64
    const int nd_k = nd_f64 > 0 ? nd_f64 : fast_mode >= 5 ? nd_f32 : (has_set ? -1 : 0);
    // a shared keep mask runs only on the fast f64 / f32 kernels' MK instantiations
    if (rowmask && !((fast && fast_mode == 2) || fast_mode == 5 ||
                     (ord && ord_kernel(nv, fast_mode, has_set, tp.vdt[0], tp.vdt[1], true) != nullptr)))
        return false;
    // wide stream-out (batch_commit_fast): runs padded to 8 entries, 16-byte region stores;
    // needs 8 T more staged entries of LDS and tiles below 2^16 - 1 cells (DUMMY_CELL).
    // VH_TILE_WIDE: bit 0 wide, bit 1 non-temporal cell stores, bit 2 non-temporal value stores
    const int sb_k = fast_mode >= 5 ? sb_mix : fast_mode == 3 ? fast_sb_narrow(nv) : fast_mode == 2 ? fast_sb_nd(nv, fast ? nd_f64 : 1) : 1;
    const uint32_t cap0 = (uint32_t)(sb_k * TA_BATCH);
    const int vbytes = fast_mode == 3 || (fast_mode >= 5 && vf32) ? 4 : 8;
    uint32_t wide_mode = 7;
    if (const char *e = getenv("VH_TILE_WIDE")) wide_mode = (uint32_t)atoi(e);
    const bool wide = (wide_mode & 1) && fast_mode != 0 && !flags_mode && S < DUMMY_CELL &&
                      fast_lds_bytes(nv, T, cap0 + 8 * T, vbytes) <= LDS_MAX_BYTES;
    tp.wide = wide ? wide_mode : 0u;
    tp.lds_cap = wide ? cap0 + 8 * T : cap0;
    const size_t lds_a = fast_mode != 0 ? fast_lds_bytes(nv, T, tp.lds_cap, vbytes) : scatter_lds_bytes(nv, T);
    if (lds_a > LDS_MAX_BYTES) return false;  // very many tiles: the global-atomic path
    int bpc;
    {
        static std::mutex mu;
        static std::map<std::tuple<int, int, int, int, size_t>, int> cache;
        std::lock_guard<std::mutex> lk(mu);
        const auto key = std::make_tuple(current_device(), ord ? (has_set ? -3 : -2) - 4 * (tp.vdt[0] + 32 * tp.vdt[1]) : nd_k, nv,
                                         fast_mode + (rowmask ? 16 : 0), lds_a);
        auto it = cache.find(key);
        if (it == cache.end()) {
            int v = 0;
            if (ord) {
                const void *kf = ord_kernel(nv, fast_mode, has_set, tp.vdt[0], tp.vdt[1], rowmask != nullptr);
                VH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, kf, TA_THREADS, lds_a));
            } else {
                v = nv == 0 ? scatter_blocks_per_cu_nd<0>(nd_k, fast_mode, lds_a, rowmask != nullptr)
                            : nv == 1 ? scatter_blocks_per_cu_nd<1>(nd_k, fast_mode, lds_a, rowmask != nullptr)
                                      : scatter_blocks_per_cu_nd<2>(nd_k, fast_mode, lds_a, rowmask != nullptr);
            }
            it = cache.emplace(key, v).first;
        }
        bpc = it->second;
    }
    bpc = std::max(1, std::min(bpc, TA_WG_PER_CU));
    const uint32_t W = std::min<uint32_t>(1024, (uint32_t)cu_count() * bpc);
    const uint64_t nb = (n + TA_BATCH - 1) / TA_BATCH;
    const uint64_t kbat = (nb + W - 1) / W;  // batches per workgroup (at most)
    const uint64_t rows_per_wg = kbat * TA_BATCH;
    const uint64_t ncw = (kbat + sb_k - 1) / sb_k;  // commits per workgroup (at most)
    // stream layout (TileParams::stream): one exactly sized stream per workgroup, no sampled
    // capacities, spill areas or overflow rows; VH_TILE_STREAM=0 keeps the per-tile regions
    // count-only plans keep the per-tile regions: their 2-byte entries make a stream segment's
    // partial lines a large share of pass B's reads (C2 count-only, same-process A/B: pass A
    // unchanged, pass B 0.8 -> 1.2 ms), while value-carrying plans gain in pass A (C2 count+sum
    // 7.56 -> 6.93 ms, C3 4.68 -> 4.14 ms; scripts/exp_stream.py, profiles/r06_stream.txt)
    const bool stream_layout = wide && nv > 0 && !getenv_flag_off("VH_TILE_STREAM") &&
                               (uint64_t)W * (T + 1) * ncw < (1ull << 31);
    // stream layout: a pass-B unit walks (workgroup, commit) segments in rounds of
    // TB_THREADS; at most TB_ROUNDS rounds per unit (a cold tile's single unit would walk all
    // W x ncw segments in one workgroup while the rest of the chip idles)
#ifndef VH_TB_ROUNDS
#define VH_TB_ROUNDS 6
#endif
    constexpr uint64_t TB_ROUNDS = VH_TB_ROUNDS;
    const uint64_t wpu = std::max<uint64_t>(1, (uint64_t)TB_THREADS * TB_ROUNDS / std::max<uint64_t>(ncw, 1));
    const uint64_t g_min = stream_layout ? (W + wpu - 1) / wpu : 1;
    // pass-B work units: sum over tiles of max(g_min, ceil(e_t / target)) <= T g_min + 4 cu
    // (target = n / 4 cu)
    const uint64_t max_units = (uint64_t)T * g_min + 4 * (uint64_t)cu_count() + 16;
    DevBuf &meta = ws.meta;
    const uint64_t meta_bytes = 8 * (uint64_t)T /*hist*/ + 8 * (uint64_t)T /*hist2*/ + 8 * (uint64_t)T /*toff*/ +
                                8 * (uint64_t)T /*spill_start*/ + 4 * (uint64_t)T /*spill_cap*/ + 4 * (uint64_t)T /*spill_fill*/ +
                                4 * (uint64_t)T /*cap*/ + 4 * (uint64_t)T * W /*fills*/ + 16 * max_units /*units*/ +
                                8 * (uint64_t)SAMPLE_BLOCKS /*brange*/ + 256;
    meta.ensure(meta_bytes);
    unsigned char *mb = meta.as<unsigned char>();
    uint64_t *d_hist = reinterpret_cast<uint64_t *>(mb);
    uint64_t *d_hist2 = d_hist + T;
    uint64_t *d_toff = d_hist2 + T;
    uint64_t *d_sstart = d_toff + T;
    uint32_t *d_scap = reinterpret_cast<uint32_t *>(d_sstart + T);
    uint32_t *d_sfill = d_scap + T;
    uint32_t *d_cap = d_sfill + T;
    uint32_t *d_fills = d_cap + ((T + 3) & ~3u);
    WorkUnit *d_units = reinterpret_cast<WorkUnit *>(d_fills + (uint64_t)T * W + 4 - ((uint64_t)T * W) % 4);
    uint32_t *d_brange = reinterpret_cast<uint32_t *>(d_units + max_units);
    const uint64_t sblocks = std::min<uint64_t>(nb, SAMPLE_BLOCKS);
    const uint64_t bstride = std::max<uint64_t>(TA_BATCH, (n / sblocks));
    VH_HIP(hipMemsetAsync(d_hist, 0, 16 * (uint64_t)T, st));
    {
        TimedScope ts("tile_sample");
        const size_t lds = 4 * (size_t)T;
        switch (nd_f64) {
        case 1: hipLaunchKernelGGL(k_tile_sample<1>, dim3(sblocks), dim3(TA_THREADS), lds, st, plan, n, s_log2, T, bstride, d_hist, d_hist2, d_brange); break;
        case 2: hipLaunchKernelGGL(k_tile_sample<2>, dim3(sblocks), dim3(TA_THREADS), lds, st, plan, n, s_log2, T, bstride, d_hist, d_hist2, d_brange); break;
        case 3: hipLaunchKernelGGL(k_tile_sample<3>, dim3(sblocks), dim3(TA_THREADS), lds, st, plan, n, s_log2, T, bstride, d_hist, d_hist2, d_brange); break;
        default: hipLaunchKernelGGL(k_tile_sample<0>, dim3(sblocks), dim3(TA_THREADS), lds, st, plan, n, s_log2, T, bstride, d_hist, d_hist2, d_brange);
        }
        VH_HIP(hipGetLastError());
    }
    // scratch and parameters of the partition exchange (regions: after the sample sized them)
    auto setup = [&](uint64_t stride, uint64_t stotal) {
        const uint64_t total = stride * W + stotal + 16;  // regions | spill areas | padding
        const int ebytes = flags_mode ? 4 : 2;
        ws.entries.ensure(total * ebytes);
        if (nv) ws.values.ensure(total * (vnarrow ? 4 : 8) * nv + 64);
        tp.vnarrow = vnarrow ? 1u : 0u;
        // the narrow ordinal pass A with two carried columns stores both in values[0], blocked
        // by 8 entries (values[0] spans both slot arrays; values[1] is unused)
        tp.vpacked = ((fast_mode == 3 || (fast_mode >= 5 && vf32)) && nv == 2 && !flags_mode && !getenv_flag_off("VH_TILE_PACK")) ? 1u : 0u;
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
        tp.spill_fill = d_sfill;
        tp.spill_cap = d_scap;
        tp.spill_start = d_sstart;
        tp.spill_base = stride * W;
        tp.entries = ws.entries.ptr;
        if (stream_layout) {
            tp.stream = 1;
            tp.ncw = (uint32_t)ncw;
            ws.tab.ensure((uint64_t)W * (T + 1) * ncw * 4 + 256);
            tp.tab = ws.tab.as<uint32_t>();
        }
        for (int s = 0; s < nv; s++)
            tp.values[s] = vnarrow ? reinterpret_cast<double *>(ws.values.as<uint32_t>() + (uint64_t)s * total)
                                   : ws.values.as<double>() + (uint64_t)s * total;
        VH_HIP(hipMemsetAsync(d_sfill, 0, 4 * (uint64_t)T, st));
    };
    bool a_launched = false;
    auto launch_pass_a = [&]() {
        TimedScope ts(fast ? "tile_scatter_f64" : fast_mode == 5 ? "tile_scatter_f32" : fast_mode >= 8 ? "tile_scatter_int" : fast_mode >= 6 ? "tile_scatter_mixed" : ord ? (has_set ? "tile_scatter_set" : "tile_scatter_ord") : "tile_scatter");
        const size_t lds = lds_a;
        if (ord) {
            const void *kf = ord_kernel(nv, fast_mode, has_set, tp.vdt[0], tp.vdt[1], rowmask != nullptr);
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
        a_launched = true;
    };
    // the sample comes back and the plan goes out through a page-locked block (pageable
    // copies are staged by the runtime, each one a host wait): [download | upload]; reuse is
    // safe because every call waits on the stream for its download before writing the block
    thread_local PinnedBuf tstage;
    thread_local hipEvent_t sample_ev = nullptr;
    if (!sample_ev) VH_HIP(hipEventCreateWithFlags(&sample_ev, hipEventDisableTiming));
    const uint64_t dl_bytes = (16 * (uint64_t)T + 8 * sblocks + 255) & ~uint64_t(255);
    tstage.ensure(dl_bytes + 24 * (uint64_t)T + sizeof(WorkUnit) * max_units + 1024);
    VH_HIP(hipMemcpyAsync(tstage.ptr, d_hist, 16 * (uint64_t)T, hipMemcpyDeviceToHost, st));
    VH_HIP(hipMemcpyAsync(tstage.as<char>() + 16 * (uint64_t)T, d_brange, 8 * sblocks, hipMemcpyDeviceToHost, st));
    VH_HIP(hipEventRecord(sample_ev, st));
    // stream layout: the streams are sized exactly without the sample (it only plans pass B),
    // so pass A is queued right behind the sample's read-back and the host plans pass B while
    // pass A runs (no host round trip between the two kernels)
    if (stream_layout) {
        uint64_t sstride = (rows_per_wg + 7 * ncw * T + 8 + 7) & ~uint64_t(7);
        if (const char *e = getenv("VH_TILE_WGPAD")) sstride += ((uint64_t)strtoull(e, nullptr, 10) + 7) & ~uint64_t(7);
        setup(sstride, 0);
        launch_pass_a();
    }
    VH_HIP(hipEventSynchronize(sample_ev));
    const uint64_t *hist = tstage.as<uint64_t>();
    const uint32_t *brange = reinterpret_cast<const uint32_t *>(tstage.as<char>() + 16 * (uint64_t)T);
    // sample blocks whose tile ranges follow each other (a column sorted, up or down, along
    // the grid index): each workgroup's evenly spaced batches then meet a tile floor or ceil
    // of K p_t times, and p_t is exact to a block
    uint64_t up = 0, down = 0;
    for (uint64_t b = 0; b + 1 < sblocks; b++) {
        up += brange[2 * b + 1] > brange[2 * b + 2];    // block b ends past block b + 1's start
        down += brange[2 * b] < brange[2 * b + 3];
    }
    const bool monotone = sblocks > 8 && std::min(up, down) * 100 <= sblocks;
    uint64_t sampled = 0;
    for (uint32_t t = 0; t < T; t++) sampled += hist[t];
    if (!sampled) return false;

    // ---- region capacities per workgroup.  Pass-A workgroup w takes batches w, w + W,
    // w + 2W, ... (TA_BATCH rows each), so every workgroup's rows are spread over the whole
    // row range and its tile distribution is the global one whatever the row order (a sorted
    // or clustered column would otherwise send a contiguous range's rows to a few tiles and
    // overflow their regions).  Regions are sized for shuffled rows (Poisson spread); a
    // workgroup's rows past its region go to the tile's spill area, sized from the spread the
    // sample measures per batch-sized block (clustered rows: each block all in or all out of
    // a tile) -- half the tile's expected rows when the rows are clustered.
    // wide stream-out: up to 7 padding entries per (workgroup, tile) and commit
    const uint64_t pad_wg = wide ? 7 * ncw : 0;
    std::vector<uint32_t> cap(T), scap(T);
    std::vector<uint64_t> toff(T), sstart(T);
    uint64_t stride = 0, stotal = 0;
    for (uint32_t t = 0; t < T && stream_layout; t++) cap[t] = scap[t] = 0, toff[t] = sstart[t] = 0;
    const double blocks = (double)sblocks;  // every sample block is TA_BATCH rows, like a batch
    // clustered rows (block variance well above the Poisson value: each sample block all in
    // or all out of a tile) anywhere in the sample
    bool any_clustered = false;
    for (uint32_t t = 0; t < T; t++) {
        const double m = (double)hist[t] / blocks, var_b = std::max(0.0, (double)hist[T + t] / blocks - m * m);
        any_clustered = any_clustered || var_b > 4.0 * m + 1.0;
    }
    for (uint32_t t = 0; t < T && !stream_layout; t++) {
        const double p = (double)hist[t] / (double)sampled, e = (double)rows_per_wg * p;
        const double m = (double)hist[t] / blocks, var_b = std::max(0.0, (double)hist[T + t] / blocks - m * m);
        const bool clustered = var_b > 4.0 * m + 1.0;
        // a clustered tile gets one batch of slack: a workgroup's evenly spaced batches meet a
        // sorted column's tile floor or ceil of K p_t times
        uint64_t c = (uint64_t)(e * 1.04 + 6.0 * std::sqrt(e + 1.0)) + 32 + (clustered ? TA_BATCH : 0) + pad_wg;
        c = std::min<uint64_t>((c + 7) & ~uint64_t(7), rows_per_wg + pad_wg + 8);
        cap[t] = (uint32_t)c;
        toff[t] = stride;
        stride += c;
        uint64_t sc = (uint64_t)(0.02 * (double)n * p) + TA_BATCH;
        // a tile the sample missed between two clustered sample blocks holds at most the rows
        // between them
        if (any_clustered && hist[t] == 0) sc = std::min<uint64_t>(n, bstride) + TA_BATCH;
        if (clustered && !monotone) {
            // whole batches land in a tile: a workgroup's batches in tile t ~ Poisson(K p_hi)
            // (p_hi: p plus two standard errors of a block sample); spill = the expected
            // excess over the region, x 2, for all workgroups (<= 1.25 n p_hi)
            const double p_hi = std::min(1.0, p + 2.0 * std::sqrt(p * (1.0 - p) / blocks));
            const double lam = (double)kbat * p_hi;
            double excess = 0.0, pk = std::exp(-lam);
            for (uint64_t x = 0; x <= kbat && (double)x <= lam + 12.0 * std::sqrt(lam) + 12.0; x++) {
                if (x) pk *= lam / (double)x;
                excess += pk * std::max(0.0, (double)x * TA_BATCH - (double)c);
            }
            sc = (uint64_t)std::min(1.25 * (double)n * p_hi, 2.0 * (double)W * excess) + 4 * TA_BATCH;
        }
        if (wide) sc += sc / 4 + 8 * (uint64_t)W;  // padding of the spilled runs
        scap[t] = (uint32_t)std::min<uint64_t>((sc + 7) & ~uint64_t(7), (uint64_t)n + 8 * (uint64_t)W + 8);
        sstart[t] = stotal;
        stotal += scap[t];
    }
    // pass A keeps region positions in u32 (destination | overflow bit), spill entries below
    // DEST_SPILL
    if (stride + rows_per_wg + pad_wg >= (uint64_t)DEST_SPILL) return false;
    if (stotal >= (uint64_t)DEST_SPILL) {  // very large launches: shrink the spill areas
        const double f = (double)(DEST_SPILL - 8 * (uint64_t)T) / (double)stotal;
        stotal = 0;
        for (uint32_t t = 0; t < T; t++) {
            scap[t] = (uint32_t)(((uint64_t)(scap[t] * f)) & ~uint64_t(7));
            sstart[t] = stotal;
            stotal += scap[t];
        }
    }
    if (!stream_layout) setup(stride, stotal);
    char *upl = tstage.as<char>() + dl_bytes;  // upload region: cap | toff | sstart | scap | units
    auto upload = [&](void *dst, const void *src, uint64_t bytes) {
        memcpy(upl, src, bytes);
        VH_HIP(hipMemcpyAsync(dst, upl, bytes, hipMemcpyHostToDevice, st));
        upl += (bytes + 15) & ~uint64_t(15);
    };
    upload(d_cap, cap.data(), 4 * (uint64_t)T);
    upload(d_toff, toff.data(), 8 * (uint64_t)T);
    upload(d_sstart, sstart.data(), 8 * (uint64_t)T);
    upload(d_scap, scap.data(), 4 * (uint64_t)T);

    // ---- pass B work units: tiles split over ranges of pass-A workgroups by expected size;
    // unit k of g of a tile also reads slice k of g of the tile's spill area
    std::vector<WorkUnit> units;
    const double target = std::max(1.0, (double)n / ((double)cu_count() * 4));
    std::vector<double> unit_rows;
    for (uint32_t t = 0; t < T; t++) {
        const double e = (double)n * (double)hist[t] / (double)sampled;
        uint32_t g = (uint32_t)std::min<double>(W, std::max((double)g_min, std::ceil(e / target)));
        for (uint32_t k = 0; k < g; k++) {
            units.push_back({t, (uint32_t)((uint64_t)W * k / g), (uint32_t)((uint64_t)W * (k + 1) / g), k | (g << 16)});
            unit_rows.push_back(e / g);
        }
    }
    if (stream_layout) {
        // largest units first (they start before the small ones fill the chip's tail)
        std::vector<uint32_t> ord(units.size());
        for (uint32_t i = 0; i < ord.size(); i++) ord[i] = i;
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return unit_rows[a] > unit_rows[b]; });
        std::vector<WorkUnit> sorted(units.size());
        for (uint32_t i = 0; i < ord.size(); i++) sorted[i] = units[ord[i]];
        units.swap(sorted);
    }
    if (units.size() > max_units) fail(VH_ERR_RUNTIME, "tiled binning: work-unit table overflow");
    if (!units.empty()) upload(d_units, units.data(), sizeof(WorkUnit) * units.size());

    // ---- pass A (launched before the sample comes back in the stream layout)
    if (!a_launched) launch_pass_a();
    // ---- pass B
    {
        TimedScope ts("tile_reduce");
        // MM: min / max cells or moment terms in pass B (the extended run form; a moment
        // other than 2 takes the per-entry form)
        bool mm = false;
        for (int k = 0; k < fa.na; k++) {
            const FusedAgg &a = fa.a[k];
            mm = mm || is_minmax(a.kind) || a.kind == VH_AGG_SUM_MOMENT;
            if (a.kind == VH_AGG_SUM_MOMENT && a.moment != 2) tp.mgeneric = 1;
            if (is_minmax(a.kind)) tp.mmk |= 1u << k;
        }
        // the branch-light form: one float64 value slot (8-byte), at most one count, sum, min and
        // max of it, count(*) or the count of its non-NaN values
        {
            bool simple = mm && !tp.mgeneric && nv == 1 && !vnarrow && !flags_mode;
            int off[4] = {-1, -1, -1, -1};
            uint32_t cnn = 0;
            for (int k = 0; k < fa.na && simple; k++) {
                const FusedAgg &a = fa.a[k];
                const int slot = a.kind == VH_AGG_COUNT ? -1 : tp.val_slot[k];
                int r = -1;
                if (a.kind == VH_AGG_COUNT) {
                    r = 0;
                    if (tp.cnt_slot[k] == 0) cnn = 1;
                    else if (tp.cnt_slot[k] != CNT_ALWAYS) simple = false;
                } else if (a.kind == VH_AGG_SUM && !a.vint && a.dtype == VH_F64 && slot == 0) r = 1;
                else if (a.kind == VH_AGG_MIN && a.dtype == VH_F64 && slot == 0) r = 2;
                else if (a.kind == VH_AGG_MAX && a.dtype == VH_F64 && slot == 0) r = 3;
                else simple = false;
                if (r >= 0) {
                    if (off[r] >= 0) simple = false;  // two of one kind
                    else off[r] = (int)a.lds_off;
                }
            }
            tp.mm_simple = simple ? 1u : 0u;
            tp.mm_cnt_nn = cnn;
            for (int r = 0; r < 4; r++) tp.mm_off[r] = off[r];
        }
        uint64_t mm_bytes = 0;
        for (int k = 0; k < fa.na; k++)
            if (is_minmax(fa.a[k].kind)) mm_bytes += ((cells * (mm_cell32(fa.a[k].dtype) ? 4 : 8)) + 255) & ~uint64_t(255);
        if (mm && mm_bytes <= (1ull << 30)) {
            // min / max: native-atomic scratch in the LDS cell form, merged after pass B (past
            // 1 GiB of scratch the flush takes the typed CAS into the grid instead)
            uint64_t off = 0;
            ws.mmtmp.ensure(mm_bytes + 256);
            off = 0;
            for (int k = 0; k < fa.na; k++) {
                if (!is_minmax(fa.a[k].kind)) continue;
                tp.mmtmp[k] = ws.mmtmp.as<char>() + off;
                off += ((cells * (mm_cell32(fa.a[k].dtype) ? 4 : 8)) + 255) & ~uint64_t(255);
                hipLaunchKernelGGL(k_mm_fill, dim3(blocks_for(cells, 256, 8)), dim3(256), 0, st, tp.mmtmp[k], cells,
                                   fa.a[k].dtype, (int)(fa.a[k].kind == VH_AGG_MAX));
                VH_HIP(hipGetLastError());
            }
        }
        const unsigned g = (unsigned)units.size();
#define VH_TB(NV_, NAR_)                                                                                      \
    do {                                                                                                      \
        if (mm && tp.mgeneric) hipLaunchKernelGGL((k_tile_reduce<NV_, NAR_, true, false, true>), dim3(g), dim3(TB_THREADS), lds_b, st, fa, tp, d_units); \
        else if (mm) hipLaunchKernelGGL((k_tile_reduce<NV_, NAR_, true>), dim3(g), dim3(TB_THREADS), lds_b, st, fa, tp, d_units); \
        else hipLaunchKernelGGL((k_tile_reduce<NV_, NAR_, false>), dim3(g), dim3(TB_THREADS), lds_b, st, fa, tp, d_units); \
    } while (0)
        switch (nv) {
        case 0: hipLaunchKernelGGL((k_tile_reduce<0, false, false>), dim3(g), dim3(TB_THREADS), lds_b, st, fa, tp, d_units); break;
        case 1:
            if (vnarrow) VH_TB(1, true);
            else VH_TB(1, false);
            break;
        default:
            if (tp.vpacked) {
                if (mm && tp.mgeneric) hipLaunchKernelGGL((k_tile_reduce<2, true, true, true, true>), dim3(g), dim3(TB_THREADS), lds_b, st, fa, tp, d_units);
                else if (mm) hipLaunchKernelGGL((k_tile_reduce<2, true, true, true>), dim3(g), dim3(TB_THREADS), lds_b, st, fa, tp, d_units);
                else hipLaunchKernelGGL((k_tile_reduce<2, true, false, true>), dim3(g), dim3(TB_THREADS), lds_b, st, fa, tp, d_units);
            } else if (vnarrow) {
                VH_TB(2, true);
            } else {
                VH_TB(2, false);
            }
        }
#undef VH_TB
        VH_HIP(hipGetLastError());
        for (int k = 0; k < fa.na; k++) {
            if (!tp.mmtmp[k]) continue;
            hipLaunchKernelGGL(k_mm_merge, dim3(blocks_for(cells, 256, 8)), dim3(256), 0, st, fa.a[k].grid, tp.mmtmp[k], cells,
                               fa.a[k].dtype, (int)(fa.a[k].kind == VH_AGG_MAX));
            VH_HIP(hipGetLastError());
        }
    }
    return true;
}

uint64_t stat_tile_overflow(bool reset) {
    unsigned long long v = 0;
    VH_HIP(hipStreamSynchronize(stream()));
    VH_HIP(hipMemcpyFromSymbol(&v, HIP_SYMBOL(d_tile_overflow_rows), sizeof(v)));
    if (reset) {
        const unsigned long long z = 0;
        VH_HIP(hipMemcpyToSymbol(HIP_SYMBOL(d_tile_overflow_rows), &z, sizeof(z)));
    }
    return v;
}

}  // namespace vh
