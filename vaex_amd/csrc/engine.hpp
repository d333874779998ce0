// Internal structures of the binning engine shared by binning.hip and tiled.hip.
#pragma once
#include <memory>
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
    const void *data;
    const void *data2;
    const uint8_t *mask;
    void *grid;
    void *grid2;
    void *s_key;
    void *s_row;
};

// count / sum(float64) aggregators of the fused path
struct FusedAgg {
    int32_t kind;
    uint32_t lds_off;
    const double *data;   // nullptr for count(*)
    const uint8_t *mask;  // 1 = keep
    void *grid;           // int64 counts / float64 sums, length1d cells
};

struct FusedAggs {
    int32_t na;
    uint32_t lds_words;
    FusedAgg a[MAX_FUSED_AGGS];
};

// per-grid device scratch, reused across bin() calls
struct Workspace {
    DevBuf idx;                                   // generic path indices1d
    std::vector<std::unique_ptr<DevBuf>> stage;   // host-column staging
    DevBuf tile_entries, tile_values, tile_meta;  // tiled path
    ~Workspace();
    DevBuf &stage_buf(int slot, uint64_t bytes);
};

void run_bin(vh_grid *g, vh_agg *const *aggs, int naggs, uint64_t length);
void launch_fused(const BinPlan &plan, FusedAggs &fa, uint64_t n, uint64_t cells, int nd_f64, Workspace &ws);
// tile-partitioned LDS aggregation for grids too large for one workgroup's LDS
// (tiled.hip); returns false when the plan is not eligible
bool try_tiled(const BinPlan &plan, const FusedAggs &fa, uint64_t n, uint64_t cells, int nd_f64, Workspace &ws);

}  // namespace vh
