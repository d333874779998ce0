/*
 * vaexhip.h -- C-ABI of libvaexhip.so, the MI355X (gfx950) implementation of
 * vaex-core's binned-statistics and groupby-aggregation hot path.
 *
 * The boundary is plain C: opaque handles, raw pointers + sizes, int status
 * codes and a thread-local last-error string.  No torch / pybind11 types.
 * Every entry point names the reference interface it replaces
 * (paths relative to the reference root, packages/vaex-core/src unless noted).
 *
 * Pointer arguments tagged `loc` may point to host memory (VH_LOC_HOST: staged
 * to HBM by the library, pipelined per chunk) or to HBM (VH_LOC_DEVICE: read in
 * place); VH_LOC_AUTO asks the HIP runtime.  Like the reference (which stores
 * raw pointers from py::buffer without incref, superagg_binners.cpp:63-73),
 * the caller keeps column buffers alive until vh_grid_bin returns.
 */
#ifndef VAEXHIP_H
#define VAEXHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VH_ABI_VERSION 1

/* status codes; VH_ERR_RUNTIME mirrors the std::runtime_error the reference
 * throws ("Expected a 1d array", "Itemsize of data and binner are not equal",
 * "data not set", "data2 not set", "no binners set and no length given"). */
enum vh_status {
    VH_OK = 0,
    VH_ERR_RUNTIME = 1,
    VH_ERR_HIP = 2,
    VH_ERR_NOMEM = 3,
    VH_ERR_ARG = 4
};

/* dtype codes, same order as the reference's per-dtype bindings
 * (superagg_binners.cpp:279-303, superagg.cpp:614-624) */
enum vh_dtype {
    VH_F64 = 0, VH_F32 = 1, VH_I64 = 2, VH_I32 = 3, VH_I16 = 4, VH_I8 = 5,
    VH_U64 = 6, VH_U32 = 7, VH_U16 = 8, VH_U8 = 9, VH_BOOL = 10
};

enum vh_loc { VH_LOC_AUTO = 0, VH_LOC_HOST = 1, VH_LOC_DEVICE = 2 };

/* aggregator kinds (superagg.cpp:547-555) */
enum vh_agg_kind {
    VH_AGG_COUNT = 0,      /* AggCount_<t>      superagg.cpp:155-192 */
    VH_AGG_SUM = 1,        /* AggSum_<t>        superagg.cpp:349-389 */
    VH_AGG_MIN = 2,        /* AggMin_<t>        superagg.cpp:241-287 */
    VH_AGG_MAX = 3,        /* AggMax_<t>        superagg.cpp:194-239 */
    VH_AGG_FIRST = 4,      /* AggFirst_<t>      superagg.cpp:436-511 */
    VH_AGG_SUM_MOMENT = 5, /* AggSumMoment_<t>  superagg.cpp:391-434 */
    VH_AGG_NUNIQUE = 6     /* AggNUnique_<t>    agg_hash_primitive.cpp:6-102; create arg: bit 0
                              dropmissing, bit 1 dropnan */
};

/* reductions of the multi-GPU collectives */
enum vh_op { VH_OP_SUM = 0, VH_OP_MIN = 1, VH_OP_MAX = 2 };

typedef struct vh_binner vh_binner;
typedef struct vh_grid vh_grid;
typedef struct vh_agg vh_agg;
typedef struct vh_set vh_set;

/* ---- library / device plumbing ---------------------------------------- */
const char *vh_last_error(void);
int vh_abi_version(void);
int vh_device_count(int *count);
int vh_set_device(int device);
int vh_get_device(int *device);
int vh_synchronize(void);
int vh_malloc(void **dptr, uint64_t bytes);
int vh_free(void *dptr);
/* page-locked host blocks (cached; result arrays are read back through them) */
int vh_host_alloc(void **ptr, uint64_t bytes);
int vh_host_free(void *ptr, uint64_t bytes);
/* Register a page-aligned host range (typically a column memory-mapped from a file) for
 * direct DMA: host columns whose chunks lie inside it stream to HBM with no bounce copy.
 * The range must stay mapped until vh_host_unregister(ptr) (which drains the device). */
/* free the page-locked blocks the library caches for read-backs and pipeline buffers
 * (capped per process: VAEX_AMD_PINNED_CACHE_MB, else 8 GiB / LOCAL_WORLD_SIZE) */
int vh_host_cache_trim(void);
/* free the device blocks the library keeps for reuse on the calling thread's device
 * (freed scratch and DeviceArray buffers, at most 1/8 of the device's memory; the dense
 * rank's sort scratch); the next query allocates afresh */
int vh_device_cache_trim(void);
int vh_host_register(void *ptr, uint64_t bytes);
int vh_host_unregister(void *ptr);
int vh_memcpy_htod(void *dst, const void *src, uint64_t bytes);
int vh_memcpy_dtoh(void *dst, const void *src, uint64_t bytes);
int vh_memcpy_dtod(void *dst, const void *src, uint64_t bytes);
int vh_memset(void *dptr, int value, uint64_t bytes);
/* synthetic columns generated in HBM (bench/test data; counter-based
 * splitmix64, so any sub-range can be regenerated on the host):
 * dist 0 = uniform [a, b), 1 = normal(mean a, sd b): F64, or F32 (the
 *      float64 draw rounded),
 *      2 = uniform integer [a, b) stored as `dtype` (I8/I32/I64),
 *      3 = sorted: a + b * normal quantile of (i + 0.5) / n (f64, ascending),
 *      4 = sorted integers [a, b) in equal consecutive runs (I32/I64). */
int vh_fill_random(void *dptr, uint64_t n, int dtype, int dist, uint64_t seed, double a, double b);
/* kernel timing with hipEvents on the library stream (bench roofline) */
int vh_timing_enable(int on);
int vh_timing_reset(void);
int vh_timing_read(const char *kernel, uint64_t *launches, double *total_ms);
int vh_stream(void **stream);
/* engine statistics since the last reset (this device): "tile_overflow_rows" (tile path rows
 * that missed their pass-A region and took global atomics), "hashagg_overflow_rows",
 * "set_overflow_rows" (the groupby / ordered_set partition overflow paths) */
int vh_stat_read(const char *name, uint64_t *value, int reset);

/* ---- Binners: superagg_binners.cpp ------------------------------------- */
/* BinnerScalar_<dtype>[_non_native](expression, vmin, vmax, bins)
 * superagg_binners.cpp:5-93 (ctor :9, to_bins :14-56) */
int vh_binner_scalar_create(const char *expression, int dtype, int flip_endian, double vmin,
                            double vmax, uint64_t bins, vh_binner **out);
/* BinnerOrdinal_<dtype>[_non_native](expression, ordinal_count, min_value)
 * superagg_binners.cpp:95-184; both arguments already converted to uint64_t
 * the way the C++ ctor converts its T arguments (:99). */
int vh_binner_ordinal_create(const char *expression, int dtype, int flip_endian,
                             uint64_t ordinal_count, uint64_t min_value, vh_binner **out);
/* BinnerOrdinal over _ordinal_values(key, set) (functions.py:2441-2448 +
 * hash_primitives.hpp:556-583) fused into one binner: reads the raw key
 * column and probes the GPU set inside the bin kernel. */
int vh_binner_set_ordinal_create(const char *expression, vh_set *set, uint64_t ordinal_count,
                                 vh_binner **out);
int vh_binner_copy(const vh_binner *binner, vh_binner **out);   /* .copy() */
int vh_binner_destroy(vh_binner *binner);
/* set_data(buf): ndim must be 1 ("Expected a 1d array"), itemsize must match
 * ("Itemsize of data and binner are not equal"), superagg_binners.cpp:63-73 */
int vh_binner_set_data(vh_binner *binner, const void *ptr, uint64_t length, int itemsize, int ndim,
                       int loc);
int vh_binner_set_data_mask(vh_binner *binner, const uint8_t *mask, uint64_t length, int ndim,
                            int loc);                           /* :78-85, 1 = masked */
int vh_binner_clear_data_mask(vh_binner *binner);             /* :74-77 */
int vh_binner_shape(const vh_binner *binner, uint64_t *shape); /* bins+3 / count+3 */
int vh_binner_size(const vh_binner *binner, uint64_t *size);

/* ---- Grid: agg.hpp:50-143 ----------------------------------------------- */
int vh_grid_create(vh_binner *const *binners, int nbinners, vh_grid **out);
int vh_grid_destroy(vh_grid *grid);
/* shapes/strides must hold >= dims entries (agg.hpp:54-69: strides[0] = 1) */
int vh_grid_info(const vh_grid *grid, int *dims, uint64_t *shapes, uint64_t *strides,
                 uint64_t *length1d);
/* Grid.bin(aggs[, length]) agg.hpp:76-105; has_length = 0 takes the first
 * binner's size and fails with "no binners set and no length given". */
int vh_grid_bin(vh_grid *grid, vh_agg *const *aggs, int naggs, uint64_t length, int has_length);

/* ---- Aggregators: superagg.cpp ----------------------------------------- */
/* Agg<Kind>_<dtype>[_non_native](grid[, moment]) -- `arg` is the moment of
 * AggSumMoment, ignored otherwise.  The grid lives in HBM. */
int vh_agg_create(vh_grid *grid, int kind, int dtype, int flip_endian, uint32_t arg, vh_agg **out);
int vh_agg_destroy(vh_agg *agg);
/* set_data(buf, index): index 1 = the order column of AggFirst (:449-461) */
int vh_agg_set_data(vh_agg *agg, const void *ptr, uint64_t length, int itemsize, int ndim, int index,
                    int loc);
int vh_agg_set_data_mask(vh_agg *agg, const uint8_t *mask, uint64_t length, int ndim, int loc); /* 1 = keep */
int vh_agg_clear_data_mask(vh_agg *agg);
/* AggNUnique::set_selection_mask (agg_hash_primitive.cpp:82-89): with a selection set, rows
 * whose data mask is 0 are outside the selection (skipped), not missing values */
int vh_agg_set_selection_mask(vh_agg *agg, const uint8_t *mask, uint64_t length, int ndim, int loc);
/* AggNUnique state to / from host memory (multi-GPU combine, counter::merge
 * hash_primitives.hpp:393-415): export with null arrays returns the deduplicated pair
 * count in *n; nulls / nans hold one count per grid cell; import appends and adds */
int vh_agg_nunique_export(vh_agg *agg, uint64_t *n, uint64_t *cells, uint64_t *vals, uint64_t *nulls, uint64_t *nans);
int vh_agg_nunique_import(vh_agg *agg, uint64_t n, const uint64_t *cells, const uint64_t *vals, const uint64_t *nulls,
                          const uint64_t *nans);
/* __sizeof__ (grid bytes, agg.hpp:162-164), grid dtype and itemsize */
int vh_agg_info(const vh_agg *agg, uint64_t *bytes, int *grid_dtype, uint64_t *itemsize);
/* buffer protocol (agg.hpp:166-179): the grid is copied to/from a host image */
int vh_agg_download(vh_agg *agg, void *host, uint64_t bytes);
int vh_agg_upload(vh_agg *agg, const void *host, uint64_t bytes);
int vh_agg_download_order(vh_agg *agg, void *host, uint64_t bytes); /* AggFirst order grid */
/* Nonzero cells of grid items [begin, end): out3 = {count, first index, last index} relative to
 * begin ({0, -1, -1} when none) -- the occupied range of a dense groupby's count(*) grid, found
 * on the device (groupby.py:484-533 keeps the cells with count > 0). */
int vh_agg_occupancy(vh_agg *agg, uint64_t begin, uint64_t end, int64_t *out3);
int vh_agg_upload_order(vh_agg *agg, const void *host, uint64_t bytes);   /* (new) combine across ranks */
int vh_agg_device_ptr(vh_agg *agg, void **grid_dptr, void **grid2_dptr);
/* Aggregator.reduce(list) superagg.cpp:160-167, 205-212, 252-259, 354-361, 470-480 */
int vh_agg_reduce(vh_agg *agg, vh_agg *const *others, int nothers);

/* ---- ordered_set_<dtype>: hash_primitives.hpp:417-621 ------------------- */
int vh_set_create(int dtype, vh_set **out);
int vh_set_destroy(vh_set *set);
/* update(keys[, mask]) hash_primitives.hpp:96-281 (mask: 1 = null) */
int vh_set_update(vh_set *set, const void *keys, const uint8_t *mask, uint64_t n, int loc);
/* update with only the rows where select[i] != 0 (a filtered / selected chunk, without
 * compacting it first; ordinals follow the first selected occurrence) */
int vh_set_update_selected(vh_set *set, const void *keys, const uint8_t *mask, const uint8_t *select, uint64_t n,
                           int loc);
/* assigns ordinals (first-appearance order); called implicitly by the readers */
int vh_set_seal(vh_set *set);
/* len(set), nan_count, null_count, nan_value, null_value (ordinals; 0x7fffffff if absent) */
int vh_set_info(vh_set *set, int64_t *length, int64_t *nan_count, int64_t *null_count,
                int64_t *nan_value, int64_t *null_value);
/* key_array() hash_primitives.hpp:289-312 -- out has `length` items of the key dtype */
int vh_set_key_array(vh_set *set, void *out_host);
/* map_ordinal(keys) hash_primitives.hpp:543-583: out_itemsize 1/2/4/8; -1 = unknown key */
int vh_set_map_ordinal(vh_set *set, const void *keys, uint64_t n, int loc, void *out, int out_itemsize,
                       int out_loc);

/* ---- limits pre-pass: vaexfast.cpp:1043-1055 (op_min_max) --------------- */
int vh_minmax(const void *data, uint64_t n, int dtype, int flip_endian, const uint8_t *mask, int loc,
              double *out_min, double *out_max);
/* min / max (as double, NaN ignored) of `nsample` evenly spaced rows (row j * n / nsample) of
 * a native, unmasked HBM column: the speculative key range of a dense single-key groupby
 * (vaex_amd/groupby.py _dense_range).  No reference counterpart: the reference's Grouper
 * builds an ordered_set instead (groupby.py:97-168); the caller verifies the guess with the
 * grid's under/overflow cells (superagg_binners.cpp:104-142 bins out-of-range keys there)
 * and redoes the query with the exact vh_minmax range when they are not empty. */
int vh_minmax_sample(const void *data, uint64_t n, int dtype, uint64_t nsample, double *out_min, double *out_max);

/* ---- fused hash groupby (hashagg.hip) ------------------------------------
 * groupby(key).agg({count(*), count(v), sum(v), mean(v)}) for one integer key column
 * (any width) and up to 2 value columns, in one hash-partitioned pass.  Replaces, for that
 * query shape, Grouper pass 1 (ordered_set update, hash_primitives.hpp:96-281) +
 * _ordinal_values/map_ordinal (hash_primitives.hpp:543-583) + BinnerOrdinal
 * (superagg_binners.cpp:104-142) + AggCount/AggSum (superagg.cpp:155-192,349-389), as
 * driven by groupby.py:97-168,484-533.  Groups come out sorted by key. */
typedef struct vh_hashagg vh_hashagg;
/* nonnull_mask: bit v set = the non-NaN count of value column v is read (count(v), mean);
 * the counts of other float columns are left undefined */
int vh_hashagg_create(int key_dtype, int nvals, const int *val_dtypes, uint32_t nonnull_mask, vh_hashagg **out);
int vh_hashagg_destroy(vh_hashagg *h);
/* one chunk of rows (may be called repeatedly); VH_ERR_RUNTIME on a table overflow
 * (the caller then falls back to the ordered_set path) */
int vh_hashagg_update(vh_hashagg *h, const void *keys, const void *const *vals, uint64_t n, int loc);
int vh_hashagg_finish(vh_hashagg *h, uint64_t *ngroups);
/* outputs, ngroups items each: keys as int64, count(*) int64, per value column its sum
 * (8 bytes: double for float columns, int64/uint64 for integers) and non-NaN count int64;
 * any output may be host or HBM memory (a caller that decodes combined multi-key keys on the
 * device keeps them there) */
int vh_hashagg_read(vh_hashagg *h, int64_t *keys, int64_t *counts, void *const *sums, int64_t *const *nonnull);
/* after vh_hashagg_finish: reorder the groups by the row each key first appears at -- the
 * ordinal order of an ordered_set built over the same keys (hash_primitives.hpp:96-281,289-312;
 * groupby(key, assume_sparse=True, sort=False), groupby.py:97-168) -- so vh_hashagg_read
 * returns them in that order.  `keys` is the whole key column the updates saw, in order (n =
 * their total rows).  A prefix of the rows is scanned until every group has its first row
 * (run heads only); keys that first appear late fall back to an ordered_set over all rows. */
int vh_hashagg_order_first(vh_hashagg *h, const void *keys, uint64_t n, int loc);
/* the same first-appearance order for the groups of a dense integer key range (the grid
 * route of groupby(key, assume_sparse=True)): labels[0..m) are the keys of the result groups
 * (int64, host or HBM; every one occurs in `keys`, all within [vmin, vmin + span)), and
 * perm[i] (host, int64) is the label index of the i-th group in the order the keys first
 * appear in the key column (n rows, host or HBM) -- an ordered_set's ordinal order
 * (hash_primitives.hpp:96-281).  A prefix of run heads is scanned until every label is seen. */
int vh_dense_first_order(const void *keys, uint64_t n, int loc, int key_dtype, int64_t vmin, uint64_t span,
                         const int64_t *labels, uint64_t m, int64_t *perm);
/* groupby(int key, assume_sparse=True) over a dense key range, finished on the device: the
 * occupied cells of the count(*) grid slice `counts` (range cells, count_isz-byte integers;
 * cell j is key vmin + j; m of them occupied), ordered by the row each key first appears at
 * (the ordered_set grouper's order, groupby.py:97-168), each of ncols device columns src[c]
 * (the aggregators' grid slices, isz[c]-byte items) gathered in that order into the host
 * buffer dst[c] (m items), and the keys written to labels (m items of label_isz bytes). */
int vh_dense_first_take(const void *keys, uint64_t n, int loc, int key_dtype, int64_t vmin, uint64_t range,
                        const void *counts, int count_isz, uint64_t m, int ncols, const void *const *src,
                        const int *isz, void *const *dst, int label_isz, void *labels);
/* host: dsts[c][i] = srcs[c][idx[i]] for ncols columns of itemsizes[c] (1/2/4/8) bytes, i < n,
 * on up to `threads` threads */
int vh_host_take(int ncols, void *const *dsts, const void *const *srcs, const int *itemsizes, const int64_t *idx,
                 uint64_t n, int threads);
/* ---- multi-GPU (comm.hip): RCCL bound by the library, one process per GPU ----------
 * The reference has no multi-process path; its ExecutorLocal reduces per-thread task
 * parts serially (execution.py:285, Aggregator::reduce superagg.cpp:160-167,205-212,
 * 252-259,354-361,470-480).  Across GPUs the same reductions run as collectives on the
 * library stream.  The caller distributes rank 0's unique id (128 bytes)
 * to every rank before vh_comm_init (vaex_amd/comm.py does it over its host channel). */
typedef struct vh_comm vh_comm;
int vh_comm_unique_id(void *out128);
int vh_comm_init(const void *id128, int world, int rank, vh_comm **out); /* on the current device;
  every vh_comm_* call (and vh_hashagg_exchange) runs on that device, from any thread */
/* `world` loopback ranks in this process on the current GPU, out[0..world): one host
 * thread per rank calls the same collectives (a rendezvous; the last thread to arrive moves
 * every rank's bytes with device copies, all-reduce = all-gather + rank-order device fold).
 * A test backend: the device code around the collectives runs with N ranks' data on one
 * GPU, where RCCL refuses two ranks on one device.  Destroy each handle. */
int vh_comm_loopback(int world, vh_comm **out);
int vh_comm_destroy(vh_comm *comm);
/* in-place all-reduce of `count` items of `dtype` (host or HBM buffer) with vh_op */
int vh_comm_allreduce(vh_comm *comm, void *buf, uint64_t count, int dtype, int op, int loc);
/* recv = every rank's `bytes` of send, rank-major */
int vh_comm_allgather(vh_comm *comm, const void *send, void *recv, uint64_t bytes, int loc);
/* send / recv hold per-rank segments back to back in rank order (sizes in bytes) */
int vh_comm_alltoallv(vh_comm *comm, const void *send, const uint64_t *send_bytes, void *recv,
                      const uint64_t *recv_bytes, int loc);
int vh_comm_barrier(vh_comm *comm);
/* an aggregator's HBM grid combined across ranks in place: SUM for count / sum / moment,
 * MIN / MAX for min / max, AggFirst by (order, rank) on the device (superagg.cpp:470-480) */
int vh_comm_agg_allreduce(vh_comm *comm, vh_agg *agg);
/* groupby results across ranks (after vh_hashagg_finish): every group row to its owner
 * rank splitmix64(key bits) % world over RCCL, owners fold equal keys in rank order; with
 * `gather` every rank then holds the whole key-sorted result (read with vh_hashagg_read) */
int vh_hashagg_exchange(vh_hashagg *h, vh_comm *comm, int gather);

/* ---- expressions on HBM columns (expr.hip) ----------------------------------
 * out[i] = program(cols[.][i]) for i < n: the device evaluation of a virtual column,
 * selection or filter (the reference evaluates them with numpy per chunk, cpu.py:542-581,
 * execution.py:337-341).  code: stack program compiled by vaex_amd/expr.py (op | arg << 8),
 * consts: 64-bit constant bit patterns; HBM columns and output. */
int vh_expr_eval(const uint32_t *code, int ncode, const uint64_t *consts, int nconsts, const void *const *cols,
                 const int *col_dtypes, int ncols, uint64_t n, int out_dtype, void *out);

/* combined int64 key of a multi-key groupby, out[i] = sum_j (cols[j][i] - mins[j]) * mults[j]
 * (the cartesian ordinal of groupby.py:248-288 _combine, first key most significant);
 * HBM columns and output, up to 8 integer key columns */
int vh_combine_keys(uint64_t n, int nkeys, const void *const *cols, const int *dtypes, const int64_t *mins,
                    const int64_t *mults, int64_t *out);

/* dense rank of an int64 HBM column: rank[i] = number of distinct keys below keys[i], the
 * distinct keys ascending in distinct[0..*m) (capacity n); n < 2^31.  Replaces the
 * GrouperCombined set of a combined key (groupby.py:248-288, ordered_set::create +
 * map_ordinal, hash_primitives.hpp:468-516,543-583) with sorted ordinals. */
int vh_dense_rank_i64(uint64_t n, const int64_t *keys, int32_t *rank, int64_t *distinct, uint64_t *m);

/* stable ascending argsort of an HBM key column of `dtype` (order: int64, HBM): the Grouper
 * sort=True order (groupby.py:137-156 sorts the set's keys; NaN after every number, -0.0 ==
 * 0.0 keep their order); n < 2^32 */
int vh_argsort(uint64_t n, const void *keys, int dtype, int64_t *order);

/* group labels of combined keys (the inverse of vh_combine_keys; groupby.py:248-288 decodes
 * the GrouperCombined bins back to per-key labels): v = table ? table[ck[i]] : ck[i],
 * outs[j][i] = (v / mults[j]) % spans[j] + mins[j] stored in itemsizes[j] bytes; HBM buffers */
int vh_decode_keys(uint64_t n, const int64_t *ck, const int64_t *table, int nkeys, const int64_t *mins,
                   const int64_t *mults, const int64_t *spans, const int *itemsizes, void *const *outs);

#ifdef __cplusplus
}
#endif
#endif /* VAEXHIP_H */
