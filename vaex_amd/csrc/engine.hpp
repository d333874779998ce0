// Internal structures of the binning engine shared by binning.hip and tiled.hip.
#pragma once
#include <memory>
#include <mutex>
#include <vector>

#include "common.hpp"
#include "hashset.hpp"

struct vh_grid;
struct vh_agg;


namespace vh {

constexpr int MAX_DIM = 16;          // agg.hpp:25
constexpr int MAX_FUSED_AGGS = 4;
constexpr uint64_t LDS_FUSED_MAX = 64 * 1024;  // per-workgroup privatised grid budget

// one column as handed over by set_data / set_data_mask
struct ColumnRef {
    const void *ptr = nullptr;
    uint64_t size = 0;
    int itemsize = 0;
    int loc = VH_LOC_HOST;
    bool set = false;
};

// a binner as the kernels see it (chunk-relative pointers)
struct BinnerDev {
    int32_t kind, dtype, flip, pad;
    const void *data;
    const uint8_t *mask;
    double vmin, scale;
    uint64_t bins;
    uint64_t ordinal_count, min_value;
    uint64_t stride;
    SetDev set;
};

struct BinPlan {
    int32_t nb, pad;
    BinnerDev b[MAX_DIM];
};

struct AggDev {
    int32_t kind, dtype, flip;
    uint32_t moment;
    int32_t has_selection, pad;
    const void *data;
    const void *data2;
    const uint8_t *mask;
    void *grid;
    void *grid2;
    void *s_key;
    void *s_row;
};

// exact std::min/std::max(value, grid) semantics (superagg.cpp:226,274) with CAS
template <typename T> __device__ inline T minmax_apply(T g, T value, bool is_max) {
    return is_max ? ((value < g) ? g : value) : ((g < value) ? g : value);
}

template <typename T> __device__ inline void atomic_minmax(T *addr, T value, bool is_max) {
    if constexpr (sizeof(T) == 8 || sizeof(T) == 4) {
        using W = typename std::conditional<sizeof(T) == 8, unsigned long long, unsigned int>::type;
        W *a = reinterpret_cast<W *>(addr);
        W old = __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (;;) {
            T g;
            __builtin_memcpy(&g, &old, sizeof(T));
            T nv = minmax_apply(g, value, is_max);
            W nb;
            __builtin_memcpy(&nb, &nv, sizeof(T));
            if (nb == old) return;
            W prev = atomicCAS(a, old, nb);
            if (prev == old) return;
            old = prev;
        }
    } else {
        uintptr_t addr_u = reinterpret_cast<uintptr_t>(addr);
        unsigned int *word = reinterpret_cast<unsigned int *>(addr_u & ~(uintptr_t)3);
        const unsigned shift = (unsigned)(addr_u & 3) * 8;
        const unsigned mask = (sizeof(T) == 2 ? 0xffffu : 0xffu) << shift;
        unsigned int old = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (;;) {
            unsigned cur_bits = (old & mask) >> shift;
            T g;
            if constexpr (sizeof(T) == 2) {
                uint16_t cb = (uint16_t)cur_bits;
                __builtin_memcpy(&g, &cb, 2);
            } else {
                uint8_t cb = (uint8_t)cur_bits;
                __builtin_memcpy(&g, &cb, 1);
            }
            T nv = minmax_apply(g, value, is_max);
            unsigned nbits;
            if constexpr (sizeof(T) == 2) {
                uint16_t t;
                __builtin_memcpy(&t, &nv, 2);
                nbits = t;
            } else {
                uint8_t t;
                __builtin_memcpy(&t, &nv, 1);
                nbits = t;
            }
            if (nbits == cur_bits) return;
            unsigned int nw = (old & ~mask) | (nbits << shift);
            unsigned int prev = atomicCAS(word, old, nw);
            if (prev == old) return;
            old = prev;
        }
    }
}

// count / sum(float64) aggregators of the fused path
struct FusedAgg {
    int32_t kind;
    uint32_t lds_off;
    const double *data;   // nullptr for count(*); of `dtype` (float64 unless generic_vals)
    const uint8_t *mask;  // 1 = keep
    void *grid;           // int64 counts / upcast sums (float64, int64 or uint64), length1d cells
    int32_t dtype;        // data dtype code
    int32_t vint;         // the sum accumulates 64-bit integers (integer / bool data), not float64
    uint32_t moment;      // AggSumMoment: the power summed (float data only on the tile path)
    uint32_t pad;
};

// AggSumMoment's term of a non-NaN float value (superagg.cpp:400-433: pow(value, moment) in
// double; moment 2 as value * value, which pow rounds identically)
// pow out of line: inlined at every call site of an unrolled kernel it is ~7000 instructions
// each, for a moment that is rarely above 2
__device__ __noinline__ inline double moment_pow(double v, uint32_t m) { return pow(v, (double)m); }
__device__ inline double moment_term(double v, uint32_t m) {
    if (m == 0) return 1.0;
    if (m == 1) return v;
    if (m == 2) return v * v;
    return moment_pow(v, m);
}

// two value-carrying aggregators (sum / min / max) read the same column the same way: the tile
// path carries that column once per row for both
static inline bool same_value_slot(const FusedAgg &a, const FusedAgg &b) {
    return a.data && a.data == b.data && a.mask == b.mask && a.dtype == b.dtype && a.vint == b.vint;
}

struct FusedAggs {
    int32_t na;
    uint32_t lds_words;
    int32_t generic_vals;  // some data is not float64: tile path with per-dtype loads only
    int32_t pad;
    FusedAgg a[MAX_FUSED_AGGS];
};

// Double-buffered H2D pipeline for host (numpy) columns, replacing the ExecutorLocal
// chunk loop's in-place reads (execution.py:299-377): chunk i+1 is memcpy'd by host
// threads into a pinned bounce buffer and DMA'd on the copy stream while chunk i is binned
// on the compute stream; events order buffer reuse in both directions.
struct HostPipe {
    std::vector<const void *> cols;  // distinct host columns of this bin() call
    std::vector<int> isz;
    std::vector<uint64_t> off;       // byte offset of each column inside a chunk buffer
    uint64_t chunk = 0, bytes = 0;
    PinnedBuf pinned[2];
    DevBuf dev[2];
    hipEvent_t copied[2] = {nullptr, nullptr}, consumed[2] = {nullptr, nullptr};
    bool pending_copy[2] = {false, false}, pending_use[2] = {false, false};
    // page-aligned column ranges registered with the runtime for a direct DMA (memory-mapped
    // files: the page cache is the DMA source, no bounce copy), per buffer until its copy ends
    std::vector<void *> registered[2];
    ~HostPipe();
    void release_registered(int b);
    void add(const ColumnRef &c);
    void plan(uint64_t chunk_rows);
    void issue(uint64_t ci, uint64_t row0, uint64_t len);  // stage chunk ci into buffer ci & 1
    void wait_copied(int b);                                // compute stream waits for buffer b
    void mark_consumed(int b);                              // after the chunk's kernels
    int find(const void *ptr) const;
};

// per-grid device scratch, reused across bin() calls
struct Workspace {
    DevBuf idx;                                   // generic path indices1d
    DevBuf cells;                                 // small-grid path: u16 cell per row
    DevBuf first_part;                            // small-grid AggFirst: per-workgroup (key, row) partials
    HostPipe pipe;                                // host-column staging
    DevBuf tile_entries, tile_values, tile_meta;  // tiled path
    ~Workspace();
};

void run_bin(vh_grid *g, vh_agg *const *aggs, int naggs, uint64_t length);
void launch_fused(const BinPlan &plan, FusedAggs &fa, uint64_t n, uint64_t cells, int nd_f64, Workspace &ws);
// tile-partitioned LDS aggregation for grids too large for one workgroup's LDS
// (tiled.hip); returns false when the plan is not eligible
bool try_tiled(const BinPlan &plan, const FusedAggs &fa, uint64_t n, uint64_t cells, int nd_f64, Workspace &ws);
// rows of the partitioned engines' pass A that missed their region since the last reset
// (tiled.hip: applied with global atomics; hashagg.hip / hashset.hip: their overflow paths)
uint64_t stat_tile_overflow(bool reset);
uint64_t stat_hashagg_overflow(bool reset);
uint64_t stat_set_overflow(bool reset);
// AggFirst over a grid too large for LDS through the tile-partitioned exchange (first.hip):
// fills the aggregator's s_key / s_row scratch for rows [0, n) of this chunk (global rows
// row0 + j); false when not eligible or when its resolve list overflowed (scratch reset)
bool try_tiled_first(const BinPlan &plan, const AggDev &ad, uint64_t n, uint64_t cells, uint64_t row0, int nd_f64);
uint64_t stat_first_tiled(bool reset);  // chunks binned by try_tiled_first
// a set-ordinal grid (one set-ordinal binner over an integer key) with count / float64 sum
// aggregators through the fused hash aggregation (hashagg.hip); false when not eligible
bool hashagg_bin_set_ordinal(const BinPlan &plan, const FusedAggs &fa, uint64_t n);

}  // namespace vh

struct vh_grid {
    // one TaskPart uses a grid at a time (execution.py:358-375), but a C caller may bin
    // different grids -- or, by mistake, the same one -- from several threads: bin and
    // reduce hold the grid's lock (grids of different parts run concurrently)
    std::mutex mu;
    std::vector<vh_binner *> binners;
    std::vector<uint64_t> shapes, strides;
    uint64_t length1d = 1;
    vh::Workspace ws;
};

struct vh_agg {
    vh_grid *grid = nullptr;
    int kind = 0, dtype = VH_F64, flip = 0;
    uint32_t moment = 0;   // AggSumMoment moment; AggNUnique: bit 0 dropmissing, bit 1 dropnan
    int grid_dtype = VH_I64;
    int grid_isz = 8;
    vh::DevBuf g, g2;          // grid, AggFirst order grid / AggNUnique per-cell null counts
    vh::DevBuf s_key, s_row;   // AggFirst per-chunk scratch / AggNUnique per-cell nan counts
    vh::ColumnRef data, data2, mask;
    // AggNUnique (agg_hash_primitive.cpp:6-102): the (cell, value) pairs seen so far, kept
    // as an unordered list, deduplicated by sort when the grid is read or the list grows
    bool has_selection = false;
    bool nu_dirty = false;
    uint64_t L = 0;        // grid length1d
    uint64_t nu_n = 0;
    vh::DevBuf nu_cell, nu_val;
};

namespace vh {
// AggNUnique (nunique.hip)
void nunique_init(vh_agg *a);
void nunique_collect(vh_agg *a, const AggDev &ad, const uint64_t *idx, uint64_t len);
void nunique_merge(vh_agg *a, vh_agg *o);
void nunique_finalize(vh_agg *a);
}  // namespace vh
