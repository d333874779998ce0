// AggFirst on the tile-partitioned path (superagg.cpp:436-511): first(v, order=o,
// binby=...) over a grid too large for one workgroup's LDS, with no per-row global atomics.
//
// AggFirst keeps, per cell, the value at the row whose order value is smallest (strict `<`:
// among equal order values the row a serial pass meets first, i.e. the lowest row), over
// rows whose value and order are both non-NaN (masks are ignored, as the reference's
// "TODO: masked support").  The generic path (binning.hip k_first_a/b/c) finds, per chunk,
// the minimum order key of every cell (s_key) and the lowest row holding it (s_row) with two
// passes of scattered 64-bit global atomics, then k_first_c merges them into the grid.  This
// engine fills the same s_key / s_row scratch through the partition exchange instead:
//
//   sample  -- per-tile row fractions from ~1M evenly spaced rows (4096 cells per tile)
//   pass A  -- batches of 4096 rows dealt round-robin to the workgroups; a row's cell, its
//              order key (order_key: order-preserving u64) and its row are ranked per tile in
//              LDS, counting-sorted, and streamed as runs into per-(workgroup, tile) regions
//              sized from the sample (tiled.hip's layout; a run past its region reserves the
//              tile's spill area).  4 + 8 bytes per row: the order key and one u32 packing
//              the cell (12 bits), the row's offset in its 4096-row batch (12 bits) and the
//              low 8 bits of the workgroup's commit index; the row is implied by the region
//              (workgroup w), the commit index k and the offset: (k W + w) 4096 + offset, with
//              k's high bits from the region positions where k crossed a multiple of 256
//              (recorded per (workgroup, tile)).  Spill-area entries also store their row.
//              (Per-(XCD, tile) streams with one reservation atomic per tile and batch were
//              tried: the returning atomics cost 4.5 of 17 ms of pass A at 1e9 rows.)
//   pass B  -- unit = (tile, range of pass-A workgroups) + a slice of the tile's spill area,
//              read as one stream of 8-entry chunks: per 8192-entry step, phase 1 lowers the
//              LDS order key of each cell (a row that lowers it resets the cell's row), phase
//              2 lowers the cell's row among entries equal to the key; the unit's (key, row)
//              per touched cell is merged with a global atomicMin of s_key, and appended to a
//              resolve list when it may win.
//   resolve -- list entries whose key equals the final s_key lower s_row (global rows).
// Rows past a stream and its spill area (sampling miss) go to s_key + the list directly; a
// full list sets a flag and the chunk is redone by the generic path (s_key / s_row reset).
#include <algorithm>
#include <cmath>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "binner_dev.hpp"
#include "common.hpp"
#include "engine.hpp"

namespace vh {

#ifndef VH_TF_THREADS
#define VH_TF_THREADS 512
#endif
constexpr int TF_THREADS = VH_TF_THREADS;
constexpr int TF_RPT = 8;
constexpr int TF_BATCH = TF_THREADS * TF_RPT;  // 4096 rows per batch
#ifndef VH_TF_LG
#define VH_TF_LG 2
#endif
constexpr int TF_LG = VH_TF_LG;  // rows per load group of the float64-binner pass A
static_assert(TF_RPT % TF_LG == 0, "load groups tile the rows of a lane");
#ifndef VH_TFB_THREADS
#define VH_TFB_THREADS 1024
#endif
constexpr int TFB_THREADS = VH_TFB_THREADS;  // pass B threads (512: two workgroups per CU)
static_assert((1 << 12) / TFB_THREADS <= 8, "merge: at most 8 cells of a 4096-cell tile per thread");
constexpr uint32_t TF_S_LOG2 = 12;  // 4096 cells per tile: pass B LDS 8-B key + 4-B row = 48 KB
constexpr uint32_t TF_MAX_TILES = 2048;
constexpr int TF_SAMPLE_BLOCKS = 512;

struct FirstParams {
    uint32_t T, W, s_log2, pad;
    uint64_t n, cells;
    const uint32_t *cap;          // [T] region capacity of (workgroup, t), the same for every workgroup; multiple of 8
    const uint32_t *toff;         // [T] region offset inside a workgroup's block; multiple of 8
    uint64_t xstride;             // entries of one workgroup's block
    uint32_t *sfill;              // [W * T] entries produced per (workgroup, tile) (may exceed cap)
    uint32_t *spill_fill;         // [T]
    const uint32_t *spill_cap;    // [T]
    const uint64_t *spill_start;  // [T] relative to spill_base
    uint64_t spill_base;
    uint32_t *epack;  // cell | batch offset << 12 | commit index (low 8 bits) << 24
    unsigned long long *eokey;
    uint32_t *erow;   // spill-area entries only: the chunk row
    uint32_t *kbound; // [W][T][kh]: region position where the commit index reached 256 (j + 1)
    uint32_t kh;
    uint32_t unmasked;  // float64 binners (ND > 0) without masks: the batch's loads go first
    unsigned long long *s_key, *s_row;  // the aggregator's per-cell scratch (AggDev)
    uint4 *list;                        // (cell, row, key lo, key hi)
    unsigned long long *list_fill;
    uint64_t list_cap;
    unsigned *flag;  // list overflow: the host redoes the chunk on the generic path
    uint32_t debug;  // ablation build only (VH_FIRST_DEBUG, results wrong): 2 = no stream-out
                     // stores, 4 = no staging / stream-out, 8 = value / order columns not loaded,
                     // 16 = one LDS atomic per kept row for the rank, 32 = no rank, 64 = no scan
};

template <int ND> __device__ __forceinline__ uint64_t tf_cell(const BinPlan &p, uint64_t i) {
    if constexpr (ND == 0) {
        return plan_index(p, i);
    } else {
        uint64_t c = 0;
#pragma unroll
        for (int d = 0; d < ND; d++) c += scalar_index<double>(p.b[d], i) * p.b[d].stride;
        return c;
    }
}

__device__ inline void tf_lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ inline void tf_list_push(const FirstParams &fp, uint64_t slot, uint32_t cell, uint32_t row, uint64_t key) {
    if (slot < fp.list_cap) fp.list[slot] = make_uint4(cell, row, (uint32_t)key, (uint32_t)(key >> 32));
    else atomicOr(fp.flag, 1u);
}

// per-tile histogram of TF_SAMPLE_BLOCKS evenly spaced batch-sized row blocks (count and
// square: the block-to-block spread tells clustered rows)
template <int ND>
__global__ __launch_bounds__(TF_THREADS) void k_first_sample(BinPlan p, uint64_t n, uint32_t s_log2, uint32_t T,
                                                             uint64_t block_stride, unsigned long long *hist) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    uint32_t *h = reinterpret_cast<uint32_t *>(lds_raw);
    for (uint32_t t = threadIdx.x; t < T; t += TF_THREADS) h[t] = 0;
    __syncthreads();
    const uint64_t r0 = blockIdx.x * block_stride;
    for (uint64_t r = threadIdx.x; r < TF_BATCH && r0 + r < n; r += TF_THREADS)
        atomicAdd(&h[(uint32_t)(tf_cell<ND>(p, r0 + r) >> s_log2)], 1u);
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < T; t += TF_THREADS)
        if (h[t]) {
            atomicAdd(&hist[t], (unsigned long long)h[t]);
            atomicAdd(&hist[T + t], (unsigned long long)h[t] * h[t]);
        }
}

// pass A (see the file comment).  LDS: staged keys u32 | order keys u64 | rows u32 (one batch)
// | per tile: hist, boff, sbase, soff, fill, cap, toff
template <int ND, typename T>
__global__ __launch_bounds__(TF_THREADS) void k_first_scatter(BinPlan p, AggDev a, FirstParams fp) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    __shared__ uint32_t s_tot;
    const uint32_t NT = fp.T;
    unsigned long long *sokey = reinterpret_cast<unsigned long long *>(lds_raw);
    uint32_t *skey = reinterpret_cast<uint32_t *>(sokey + TF_BATCH);
    uint32_t *srow = skey + TF_BATCH;
    uint32_t *hist = srow + TF_BATCH;
    uint32_t *boff = hist + NT, *sbase = boff + NT, *soff = sbase + NT, *fill = soff + NT, *cap = fill + NT, *toff = cap + NT;
    for (uint32_t t = threadIdx.x; t < NT; t += TF_THREADS) {
        hist[t] = 0;
        fill[t] = 0;
        cap[t] = fp.cap[t];
        toff[t] = fp.toff[t];
    }
    const uint64_t wblock = (uint64_t)blockIdx.x * fp.xstride;
    const uint32_t smask = (1u << fp.s_log2) - 1;
    const int lane = threadIdx.x & 63;
    __syncthreads();
    const uint64_t n = fp.n;
    // batches w, w + W, w + 2W, ...: every workgroup's rows spread over the whole range; the
    // trip count is uniform within the workgroup (every thread meets every barrier)
    static_assert(TF_S_LOG2 <= 12 && TF_BATCH <= 4096, "12-bit cells and batch offsets");
    uint32_t kc = 0;  // this workgroup's commit index: batch b0 = (kc W + w) TF_BATCH
    for (uint64_t b0 = (uint64_t)blockIdx.x * TF_BATCH; b0 < n; b0 += (uint64_t)gridDim.x * TF_BATCH, kc++) {
        uint32_t key[TF_RPT];
        int32_t rank[TF_RPT];
        unsigned long long ok[TF_RPT];
        // float64 binners without masks (UNMASKED): every column of the batch's rows is loaded
        // before any is used -- one memory round trip per batch, not three per row (a load
        // behind a binner's branches or a rank waits for the one before it)
        // (in groups of TF_LG rows: fewer registers held, TF_RPT / TF_LG round trips)
        double xr[ND > 0 ? ND : 1][TF_LG];
        T vr[TF_LG], orr[TF_LG];
#pragma unroll
        for (int r = 0; r < TF_RPT; r++) {
            if constexpr (ND > 0) {
                if (fp.unmasked && r % TF_LG == 0) {
#pragma unroll
                    for (int g = 0; g < TF_LG; g++) {
                        const uint64_t i = b0 + (uint64_t)(r + g) * TF_THREADS + threadIdx.x;
                        const uint64_t is = i < n ? i : n - 1;
#pragma unroll
                        for (int d = 0; d < ND; d++) xr[d][g] = static_cast<const double *>(p.b[d].data)[is];
                        vr[g] = load_v<T>(a.data, is, a.flip);
                        orr[g] = load_v<T>(a.data2, is, a.flip);
                    }
                }
            }
            const uint64_t i = b0 + (uint64_t)r * TF_THREADS + threadIdx.x;
            const bool in = i < n;
            uint64_t c = 0;
            bool keep = false;
            ok[r] = 0;
            bool done = false;
            if constexpr (ND > 0) {
                if (fp.unmasked) {
                    done = true;
                    if (in) {
#pragma unroll
                        for (int d = 0; d < ND; d++) c += scalar_cell<double>(p.b[d], xr[d][r % TF_LG], false) * p.b[d].stride;
                        keep = !is_nan_v(vr[r % TF_LG]) && !is_nan_v(orr[r % TF_LG]);
                        ok[r] = order_key(orr[r % TF_LG]);
                    }
                }
            }
            if (in && !done) {
                c = tf_cell<ND>(p, i);
                T v{}, o{};
                if (DBG(fp.debug) & 8) {
                    if constexpr (std::is_arithmetic<T>::value) {
                        v = (T)1;
                        o = (T)(i & 1023);
                    }
                } else {
                    v = load_v<T>(a.data, i, a.flip);
                    o = load_v<T>(a.data2, i, a.flip);
                }
                keep = !is_nan_v(v) && !is_nan_v(o);
                ok[r] = order_key(o);
            }
            const uint32_t t = (uint32_t)(c >> fp.s_log2);
            key[r] = (t << 16) | ((uint32_t)c & smask);
            if (DBG(fp.debug) & 32) {
                rank[r] = -1;
                asm volatile("" ::"v"(t), "v"(keep));
            } else if (DBG(fp.debug) & 16) {
                rank[r] = keep ? (int32_t)atomicAdd(&hist[t], 1u) : -1;
            } else {
                rank[r] = wave_rank(hist, t, keep);
            }
        }
        // B1: every rank taken -> wave 0 scans the histogram (clearing it for the next batch)
        // and advances this workgroup's regions; a run past a region's capacity reserves the
        // excess in the tile's spill area
        tf_lds_barrier();
        if (threadIdx.x < 64 && !(DBG(fp.debug) & 64)) {
            const uint32_t per = (NT + 63) / 64, t0 = lane * per;
            uint32_t s = 0;
            for (uint32_t t = t0; t < t0 + per && t < NT; t++) s += hist[t];
            uint32_t inc = s;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(inc, off, 64);
                if (lane >= off) inc += y;
            }
            uint32_t acc = inc - s;
            const bool kb = kc && !(kc & 255u) && (kc >> 8) <= fp.kh;  // k crosses a multiple of 256
            for (uint32_t t = t0; t < t0 + per && t < NT; t++) {
                const uint32_t h = hist[t], b = fill[t], c = cap[t];
                if (kb) fp.kbound[((uint64_t)blockIdx.x * NT + t) * fp.kh + (kc >> 8) - 1] = b;
                boff[t] = acc;
                sbase[t] = b;
                fill[t] = b + h;
                hist[t] = 0;
                acc += h;
                if (b + h > c) {
                    const uint32_t first = max(b, c);
                    soff[t] = atomicAdd(&fp.spill_fill[t], b + h - first) - first;
                }
            }
            if (lane == 63) s_tot = inc;
        }
        // B2: rows stage at their sorted positions
        tf_lds_barrier();
        if (DBG(fp.debug) & 4) continue;
#pragma unroll
        for (int r = 0; r < TF_RPT; r++) {
            if (rank[r] < 0) continue;
            const uint32_t pos = boff[key[r] >> 16] + (uint32_t)rank[r];
            skey[pos] = key[r];
            sokey[pos] = ok[r];
            srow[pos] = (uint32_t)r * TF_THREADS + threadIdx.x;  // offset in the batch
        }
        // B3: the sorted runs stream out to the regions
        tf_lds_barrier();
        const uint32_t tot = s_tot;
        const uint32_t packk = (kc & 255u) << 24;
        for (uint32_t k = threadIdx.x; k < tot; k += TF_THREADS) {
            const uint32_t kk = skey[k];
            const uint32_t t = kk >> 16;
            const uint32_t d = sbase[t] + (k - boff[t]);
            const uint32_t off = srow[k];
            const uint32_t row = (uint32_t)b0 + off;  // chunk row (< 2^32)
            uint64_t e;
            if (d < cap[t]) {
                e = wblock + toff[t] + d;
            } else {
                const uint32_t si = d + soff[t];
                if (si >= fp.spill_cap[t]) {
                    // past the region and the spill area: straight to s_key and the list
                    const uint32_t c = (t << fp.s_log2) | (kk & 0xffffu);
                    atomicMin(&fp.s_key[c], sokey[k]);
                    tf_list_push(fp, atomicAdd(fp.list_fill, 1ull), c, row, sokey[k]);
                    continue;
                }
                e = fp.spill_base + fp.spill_start[t] + si;
                fp.erow[e] = row;  // spill entries carry their row (any workgroup, any commit)
            }
            if (DBG(fp.debug) & 2) {
                asm volatile("" ::"v"(e), "v"(kk), "v"(off), "v"(sokey[k]));
                continue;
            }
            fp.epack[e] = (kk & 0xfffu) | (off << 12) | packk;
            fp.eokey[e] = sokey[k];
        }
    }
    tf_lds_barrier();
    for (uint32_t t = threadIdx.x; t < NT; t += TF_THREADS) fp.sfill[(uint64_t)blockIdx.x * NT + t] = fill[t];
}

struct FirstUnit {
    uint32_t tile, w0, w1, parts;  // parts: slice (low 16 bits) of parts (high 16) of the spill area
};

// pass B (see the file comment): the unit's regions (pass-A workgroups w0 .. w1 - 1) and its
// slice of the tile's spill area, read as one flat stream of 8-entry chunks (prefix sums of
// the region fills in LDS)
__global__ __launch_bounds__(TFB_THREADS) void k_first_reduce(FirstParams fp, const FirstUnit *units) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    __shared__ uint32_t s_w[TFB_THREADS / 64];
    __shared__ unsigned long long s_base;
    __shared__ uint32_t s_fill[1024 + 1];
    __shared__ uint32_t s_pre[1024 + 2];
    const uint32_t S = 1u << fp.s_log2;
    unsigned long long *lkey = reinterpret_cast<unsigned long long *>(lds_raw);
    uint32_t *lrow = reinterpret_cast<uint32_t *>(lkey + S);
    const FirstUnit u = units[blockIdx.x];
    const uint32_t t = u.tile;
    for (uint32_t i = threadIdx.x; i < S; i += TFB_THREADS) {
        lkey[i] = ~0ull;
        lrow[i] = ~0u;
    }
    const uint32_t part = u.parts & 0xffffu, parts = u.parts >> 16;
    const uint32_t SF = min(fp.spill_fill[t], fp.spill_cap[t]);
    const uint32_t q0 = part == 0 ? 0u : (uint32_t)((uint64_t)SF * part / parts) & ~7u;
    const uint32_t q1 = part + 1 >= parts ? SF : (uint32_t)((uint64_t)SF * (part + 1) / parts) & ~7u;
    const uint64_t eB = fp.spill_base + fp.spill_start[t] + q0;
    const uint32_t nwr = u.w1 - u.w0, nw = nwr + 1, cap_t = fp.cap[t];
    for (uint32_t k = threadIdx.x; k < nw; k += TFB_THREADS)
        s_fill[k] = k < nwr ? min(fp.sfill[(uint64_t)(u.w0 + k) * fp.T + t], cap_t) : (q1 > q0 ? q1 - q0 : 0u);
    __syncthreads();
    if (threadIdx.x < 64) {  // exclusive scan of the chunk counts
        const uint32_t lane = threadIdx.x, per = (nw + 63) / 64, k0 = lane * per;
        uint32_t sum = 0;
        for (uint32_t k = k0; k < k0 + per && k < nw; k++) sum += (s_fill[k] + 7) >> 3;
        uint32_t inc = sum;
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(inc, off, 64);
            if ((int)lane >= off) inc += y;
        }
        uint32_t acc = inc - sum;
        for (uint32_t k = k0; k < k0 + per && k < nw; k++) {
            s_pre[k] = acc;
            acc += (s_fill[k] + 7) >> 3;
        }
        if (lane == 63) s_pre[nw] = inc;
    }
    __syncthreads();
    const uint32_t C = s_pre[nw];
    const uint64_t toff_t = fp.toff[t];
    uint32_t kk = 0;  // region of this lane's current chunk (chunk indices of a lane only grow)
    // One chunk of 8 entries per lane and step; the next step's chunk (its packed entries,
    // order keys, and either its rows (spill area) or its region's commit-index boundaries)
    // is loaded while this step's two LDS phases run (r05: every step waited for its own
    // loads behind two barriers, 3.2 ms for 12 GB).
    constexpr uint32_t KHM = 4;  // boundaries carried in registers (more: read per chunk)
    struct Chunk {
        uint32_t rem, w, q0;
        bool spill;
        uint4 p0, p1, r0, r1;
        ulonglong2 k[4];
        uint32_t kb[KHM];
    };
    auto load = [&](uint32_t c, Chunk &x) __attribute__((always_inline)) {
        x.rem = 0;
        x.spill = false;
        x.p0 = x.p1 = x.r0 = x.r1 = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int h = 0; h < 4; h++) x.k[h] = ulonglong2{0, 0};
#pragma unroll
        for (uint32_t h = 0; h < KHM; h++) x.kb[h] = ~0u;
        if (c >= C) return;
        while (s_pre[kk + 1] <= c) kk++;
        const uint32_t q = (c - s_pre[kk]) * 8;
        const uint64_t e = kk < nwr ? (uint64_t)(u.w0 + kk) * fp.xstride + toff_t + q : eB + q;
        x.rem = min(8u, s_fill[kk] - q);
        x.spill = kk >= nwr;
        x.w = u.w0 + kk;
        x.q0 = q;
        x.p0 = *reinterpret_cast<const uint4 *>(fp.epack + e);
        x.p1 = *reinterpret_cast<const uint4 *>(fp.epack + e + 4);
#pragma unroll
        for (int h = 0; h < 4; h++) x.k[h] = *reinterpret_cast<const ulonglong2 *>(fp.eokey + e + 2 * h);
        if (x.spill) {
            x.r0 = *reinterpret_cast<const uint4 *>(fp.erow + e);
            x.r1 = *reinterpret_cast<const uint4 *>(fp.erow + e + 4);
        } else {
            const uint32_t *kb = fp.kbound + ((uint64_t)x.w * fp.T + t) * fp.kh;
#pragma unroll
            for (uint32_t h = 0; h < KHM; h++)
                if (h < fp.kh) x.kb[h] = kb[h];
        }
    };
    Chunk cur, nxt;
    load(threadIdx.x, nxt);
    __syncthreads();
    for (uint32_t c0 = 0; c0 < C; c0 += TFB_THREADS) {  // uniform trip count: barriers inside
        cur = nxt;
        load(c0 + TFB_THREADS + threadIdx.x, nxt);
        const uint32_t rem = cur.rem;
        const uint32_t pk[8] = {cur.p0.x, cur.p0.y, cur.p0.z, cur.p0.w, cur.p1.x, cur.p1.y, cur.p1.z, cur.p1.w};
        uint32_t rows[8] = {cur.r0.x, cur.r0.y, cur.r0.z, cur.r0.w, cur.r1.x, cur.r1.y, cur.r1.z, cur.r1.w};
        if (rem && !cur.spill) {
            // region entries: row = (k W + w) TF_BATCH + offset, k's high bits from the region
            // positions where the commit index crossed multiples of 256: boundaries at or below
            // the chunk's first position, and the first one above it (a boundary inside the
            // chunk -- a region with fewer than 8 entries in 256 commits -- takes the per-entry
            // count; more than KHM boundaries: read from memory)
            const uint32_t q0 = cur.q0, w = cur.w;
            const uint32_t *kb = fp.kbound + ((uint64_t)w * fp.T + t) * fp.kh;
            uint32_t hi0 = 0, nb = ~0u;
#pragma unroll
            for (uint32_t h = 0; h < KHM; h++) {
                const uint32_t b = cur.kb[h];
                hi0 += q0 >= b;
                nb = b > q0 && b < nb ? b : nb;
            }
            for (uint32_t h = KHM; h < fp.kh; h++) {
                const uint32_t b = kb[h];
                hi0 += q0 >= b;
                nb = b > q0 && b < nb ? b : nb;
            }
            const bool inside = nb <= q0 + 7;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                uint32_t hi = hi0;
                if (inside) {
                    hi = 0;
                    for (uint32_t h = 0; h < fp.kh; h++) hi += q0 + j >= kb[h];
                }
                const uint32_t kcj = (hi << 8) | (pk[j] >> 24);
                rows[j] = (kcj * fp.W + w) * (uint32_t)TF_BATCH + ((pk[j] >> 12) & 0xfffu);
            }
        }
        // phase 1: lower the cell's order key; the row that lowers it clears the cell's row
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if ((uint32_t)j >= rem) continue;
            const uint32_t cl = pk[j] & 0xfffu;
            const unsigned long long kj = (j & 1) ? cur.k[j >> 1].y : cur.k[j >> 1].x;
            const unsigned long long old = atomicMin(&lkey[cl], kj);
            if (kj < old) lrow[cl] = ~0u;
        }
        tf_lds_barrier();
        // phase 2: the lowest row among the entries holding the cell's key
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if ((uint32_t)j >= rem) continue;
            const uint32_t cl = pk[j] & 0xfffu;
            const unsigned long long kj = (j & 1) ? cur.k[j >> 1].y : cur.k[j >> 1].x;
            if (kj == lkey[cl]) atomicMin(&lrow[cl], rows[j]);
        }
        tf_lds_barrier();
    }
    __syncthreads();
    // merge: global minimum key per cell, and the candidates for its row into the list (one
    // list reservation per workgroup)
    const uint64_t cbase = (uint64_t)t << fp.s_log2;
    constexpr int PER = 8;  // S / TFB_THREADS cells per thread (S <= 8192)
    uint32_t push = 0;
    unsigned long long kept[PER];
    uint32_t kc[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const uint32_t i = q * TFB_THREADS + threadIdx.x;
        kept[q] = ~0ull;
        kc[q] = 0;
        if (i >= S || cbase + i >= fp.cells) continue;
        const unsigned long long kk = lkey[i];
        if (kk == ~0ull) continue;
        const unsigned long long old = atomicMin(&fp.s_key[cbase + i], kk);
        if (kk <= old) {
            kept[q] = kk;
            kc[q] = i;
            push++;
        }
    }
    const uint64_t base = block_reserve<TFB_THREADS>(push, s_w, &s_base, fp.list_fill);
    uint64_t j = base;
#pragma unroll
    for (int q = 0; q < PER; q++) {
        if (kept[q] == ~0ull) continue;
        tf_list_push(fp, j++, (uint32_t)(cbase + kc[q]), lrow[kc[q]], kept[q]);
    }
}

// resolve: candidates holding the final key lower the cell's (global) row
__global__ __launch_bounds__(256) void k_first_resolve(FirstParams fp, uint64_t row0) {
    if (*fp.flag) return;
    const uint64_t m = min(*fp.list_fill, fp.list_cap);
    for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
        const uint4 e = fp.list[j];
        const unsigned long long kk = (unsigned long long)e.z | ((unsigned long long)e.w << 32);
        if (kk == fp.s_key[e.x]) atomicMin(&fp.s_row[e.x], (unsigned long long)(row0 + e.y));
    }
}

struct FirstScratch {
    std::mutex mu;
    DevBuf epack, eokey, erow, meta, list;
};

static FirstScratch &first_scratch() {
    static std::mutex g;
    static std::map<int, std::unique_ptr<FirstScratch>> m;
    std::lock_guard<std::mutex> lk(g);
    auto &p = m[current_device()];
    if (!p) p = std::make_unique<FirstScratch>();
    return *p;
}

template <int ND> static void tf_launch_a(int dtype, unsigned grid, size_t lds, const BinPlan &plan, const AggDev &ad,
                                          const FirstParams &fp) {
    VH_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL((k_first_scatter<ND, T>), dim3(grid), dim3(TF_THREADS), lds, stream(), plan, ad, fp));
}

template <int ND> static int tf_blocks_per_cu(int dtype, size_t lds) {
    int nb = 1;
    VH_DISPATCH_DTYPE(dtype, T, VH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_first_scatter<ND, T>, TF_THREADS, lds)));
    return nb;
}

static uint64_t g_first_tiled_chunks = 0;  // chunks the engine binned (vh_stat_read("first_tiled_chunks"))

uint64_t stat_first_tiled(bool reset) {
    return reset ? __atomic_exchange_n(&g_first_tiled_chunks, 0ull, __ATOMIC_RELAXED)
                 : __atomic_load_n(&g_first_tiled_chunks, __ATOMIC_RELAXED);
}

bool try_tiled_first(const BinPlan &plan, const AggDev &ad, uint64_t n, uint64_t cells, uint64_t row0, int nd_f64) {
    if (n < (1u << 20) || n >= (1ull << 32) || !ad.data || !ad.data2 || !ad.s_key || !ad.s_row) return false;
    const uint32_t s_log2 = TF_S_LOG2;
    const uint64_t S = 1ull << s_log2;
    const uint64_t T64 = (cells + S - 1) / S;
    if (T64 < 2 || T64 > TF_MAX_TILES) return false;
    const uint32_t T = (uint32_t)T64;
    const int nd = nd_f64 >= 1 && nd_f64 <= 3 ? nd_f64 : 0;
    FirstScratch &ws = first_scratch();
    std::lock_guard<std::mutex> lock(ws.mu);
    hipStream_t st = stream();
    const size_t lds_a = (size_t)16 * TF_BATCH + (size_t)7 * 4 * T + 64;
    if (lds_a > 160 * 1024) return false;
    int bpc = 1;
    {
        static std::mutex mu;
        static std::map<std::tuple<int, int, int, size_t>, int> cache;
        std::lock_guard<std::mutex> lk(mu);
        const auto key = std::make_tuple(current_device(), nd, ad.dtype, lds_a);
        auto it = cache.find(key);
        if (it == cache.end()) {
            int v = nd == 1 ? tf_blocks_per_cu<1>(ad.dtype, lds_a) : nd == 2 ? tf_blocks_per_cu<2>(ad.dtype, lds_a)
                    : nd == 3 ? tf_blocks_per_cu<3>(ad.dtype, lds_a) : tf_blocks_per_cu<0>(ad.dtype, lds_a);
            it = cache.emplace(key, std::max(1, std::min(v, 4))).first;
        }
        bpc = it->second;
    }
    uint32_t W = std::min<uint32_t>(1024, (uint32_t)cu_count() * (uint32_t)bpc);
    // fewer pass-A workgroups (tests: hundreds of commits per workgroup, the commit-index
    // boundaries, at a few million rows; same results)
    if (const char *e = getenv("VH_FIRST_MAX_WG")) W = std::max<uint32_t>(1, std::min<uint32_t>(W, (uint32_t)atoi(e)));
    // meta: hist (2T u64) | cap | toff | spill_cap (T u32 each) | spill_start (T u64) | fills
    // (W T u32) | spill_fill (T u32) | list_fill | flag | units
    const uint64_t nb = (n + TF_BATCH - 1) / TF_BATCH;
    const uint64_t sblocks = std::min<uint64_t>(nb, TF_SAMPLE_BLOCKS);
    const uint64_t bstride = std::max<uint64_t>(TF_BATCH, n / sblocks);
    const double target = std::max(1.0, (double)n / ((double)cu_count() * 4));
    const uint64_t max_units = (uint64_t)T + 4 * (uint64_t)cu_count() + 16;
    const uint64_t kbat0 = (nb + W - 1) / W;                   // commits per workgroup (at most)
    const uint32_t kh = (uint32_t)std::max<uint64_t>(1, (kbat0 + 255) / 256);  // commit-index high parts
    const uint64_t meta_bytes = 16 * (uint64_t)T + 4 * 3 * (uint64_t)T + 8 * (uint64_t)T + 4 * (uint64_t)W * T +
                                4 * (uint64_t)T + 64 + sizeof(FirstUnit) * max_units + 4 * (uint64_t)W * T * kh + 4096;
    ws.meta.ensure(meta_bytes);
    char *mb = ws.meta.as<char>();
    auto carve = [&](uint64_t bytes) {
        char *p = mb;
        mb += (bytes + 255) & ~uint64_t(255);
        return p;
    };
    auto *d_hist = reinterpret_cast<unsigned long long *>(carve(16 * (uint64_t)T));
    auto *d_cap = reinterpret_cast<uint32_t *>(carve(4 * (uint64_t)T));
    auto *d_toff = reinterpret_cast<uint32_t *>(carve(4 * (uint64_t)T));
    auto *d_scap = reinterpret_cast<uint32_t *>(carve(4 * (uint64_t)T));
    auto *d_sstart = reinterpret_cast<uint64_t *>(carve(8 * (uint64_t)T));
    auto *d_sfill = reinterpret_cast<uint32_t *>(carve(4 * (uint64_t)W * T));
    auto *d_spfill = reinterpret_cast<uint32_t *>(carve(4 * (uint64_t)T));
    auto *d_misc = reinterpret_cast<unsigned long long *>(carve(64));  // [0] list fill, [1] flag
    auto *d_units = reinterpret_cast<FirstUnit *>(carve(sizeof(FirstUnit) * max_units));
    auto *d_kbound = reinterpret_cast<uint32_t *>(carve(4 * (uint64_t)W * T * kh));
    (void)mb;
    VH_HIP(hipMemsetAsync(d_hist, 0, 16 * (uint64_t)T, st));
    {
        TimedScope ts("first_sample");
        const size_t lds = 4 * (size_t)T;
        switch (nd) {
        case 1: hipLaunchKernelGGL(k_first_sample<1>, dim3(sblocks), dim3(TF_THREADS), lds, st, plan, n, s_log2, T, bstride, d_hist); break;
        case 2: hipLaunchKernelGGL(k_first_sample<2>, dim3(sblocks), dim3(TF_THREADS), lds, st, plan, n, s_log2, T, bstride, d_hist); break;
        case 3: hipLaunchKernelGGL(k_first_sample<3>, dim3(sblocks), dim3(TF_THREADS), lds, st, plan, n, s_log2, T, bstride, d_hist); break;
        default: hipLaunchKernelGGL(k_first_sample<0>, dim3(sblocks), dim3(TF_THREADS), lds, st, plan, n, s_log2, T, bstride, d_hist);
        }
        VH_HIP(hipGetLastError());
    }
    thread_local PinnedBuf stage;
    const uint64_t up_bytes = 4 * 3 * (uint64_t)T + 8 * (uint64_t)T + sizeof(FirstUnit) * max_units + 256;
    stage.ensure(16 * (uint64_t)T + up_bytes + 256);
    VH_HIP(hipMemcpyAsync(stage.ptr, d_hist, 16 * (uint64_t)T, hipMemcpyDeviceToHost, st));
    VH_HIP(hipStreamSynchronize(st));
    const unsigned long long *hist = stage.as<unsigned long long>();
    uint64_t sampled = 0;
    for (uint32_t t = 0; t < T; t++) sampled += hist[t];
    if (!sampled) return false;
    // region capacities per (workgroup, tile) (tiled.hip's plan): workgroup w takes batches
    // w, w + W, ... so its tile distribution is the global one; Poisson room for shuffled rows,
    // one batch of slack for clustered tiles (whole batch-sized blocks in or out, per the
    // sample's spread); past a region, the tile's spill area (for clustered tiles the expected
    // excess of a workgroup's Poisson batch count over its region, for all workgroups)
    const uint64_t kbat = (nb + W - 1) / W;
    const double rows_w = (double)kbat * TF_BATCH;
    std::vector<uint32_t> cap(T), toff(T), scap(T);
    std::vector<uint64_t> sstart(T);
    uint64_t xstride = 0, stotal = 0;
    for (uint32_t t = 0; t < T; t++) {
        const double p = (double)hist[t] / (double)sampled;
        const double m = (double)hist[t] / (double)sblocks, var_b = std::max(0.0, (double)hist[T + t] / (double)sblocks - m * m);
        const bool clustered = var_b > 4.0 * m + 1.0;
        const double e = rows_w * p;
        const double c = e * 1.04 + 6.0 * std::sqrt(e + 1.0) + 32 + (clustered ? TF_BATCH : 0);
        const uint64_t ci = std::min<uint64_t>(((uint64_t)c + 7) & ~uint64_t(7), ((uint64_t)rows_w + 15) & ~uint64_t(7));
        cap[t] = (uint32_t)ci;
        toff[t] = (uint32_t)xstride;
        xstride += ci;
        double sc = 0.02 * (double)n * p + TF_BATCH;
        if (clustered) {
            const double p_hi = std::min(1.0, p + 2.0 * std::sqrt(p * (1.0 - p) / (double)sblocks));
            const double lam = (double)kbat * p_hi;
            double excess = 0.0, pk = std::exp(-lam);
            for (uint64_t x = 0; x <= kbat && (double)x <= lam + 12.0 * std::sqrt(lam) + 12.0; x++) {
                if (x) pk *= lam / (double)x;
                excess += pk * std::max(0.0, (double)x * TF_BATCH - (double)ci);
            }
            sc = std::min(1.25 * (double)n * p_hi, 2.0 * (double)W * excess) + 4.0 * TF_BATCH;
        }
        if (hist[t] == 0) sc = std::min<double>((double)n, (double)bstride) + 2.0 * TF_BATCH;  // a tile the sample missed
        scap[t] = (uint32_t)std::min<uint64_t>(((uint64_t)sc + 7) & ~uint64_t(7), (n + 15) & ~uint64_t(7));
        sstart[t] = stotal;
        stotal += scap[t];
    }
    if (xstride >= (1ull << 32) - TF_BATCH || stotal >= (1ull << 32)) return false;
    const uint64_t total = (uint64_t)W * xstride + stotal + 16;
    // pass-B units: tiles split over ranges of pass-A workgroups by expected entries; unit k
    // of g of a tile also reads slice k of g of the tile's spill area
    std::vector<FirstUnit> units;
    for (uint32_t t = 0; t < T; t++) {
        const double e = (double)n * (double)hist[t] / (double)sampled;
        const uint32_t g = (uint32_t)std::min<double>(W, std::max(1.0, std::ceil(e / target)));
        for (uint32_t k = 0; k < g; k++)
            units.push_back({t, (uint32_t)((uint64_t)W * k / g), (uint32_t)((uint64_t)W * (k + 1) / g), k | (g << 16)});
    }
    if (units.size() > max_units) return false;
    const uint64_t list_cap = (uint64_t)units.size() * S + (1u << 20);
    ws.epack.ensure(total * 4);
    ws.eokey.ensure(total * 8);
    ws.erow.ensure(total * 4);  // spill-area entries only
    ws.list.ensure(list_cap * 16);
    char *upl = stage.as<char>() + 16 * (uint64_t)T;
    auto upload = [&](void *dst, const void *src, uint64_t bytes) {
        memcpy(upl, src, bytes);
        VH_HIP(hipMemcpyAsync(dst, upl, bytes, hipMemcpyHostToDevice, st));
        upl += (bytes + 15) & ~uint64_t(15);
    };
    upload(d_cap, cap.data(), 4 * (uint64_t)T);
    upload(d_toff, toff.data(), 4 * (uint64_t)T);
    upload(d_scap, scap.data(), 4 * (uint64_t)T);
    upload(d_sstart, sstart.data(), 8 * (uint64_t)T);
    upload(d_units, units.data(), sizeof(FirstUnit) * units.size());
    VH_HIP(hipMemsetAsync(d_sfill, 0, 4 * (uint64_t)W * T, st));
    VH_HIP(hipMemsetAsync(d_spfill, 0, 4 * (uint64_t)T, st));
    VH_HIP(hipMemsetAsync(d_misc, 0, 64, st));
    VH_HIP(hipMemsetAsync(d_kbound, 0xff, 4 * (uint64_t)W * T * kh, st));  // boundaries never reached: none
    FirstParams fp{};
    fp.T = T;
    fp.W = W;
    fp.s_log2 = s_log2;
    fp.n = n;
    fp.cells = cells;
    fp.cap = d_cap;
    fp.toff = d_toff;
    fp.xstride = xstride;
    fp.sfill = d_sfill;
    fp.spill_fill = d_spfill;
    fp.spill_cap = d_scap;
    fp.spill_start = d_sstart;
    fp.spill_base = (uint64_t)W * xstride;
    fp.epack = ws.epack.as<uint32_t>();
    fp.eokey = ws.eokey.as<unsigned long long>();
    fp.erow = ws.erow.as<uint32_t>();
    fp.kbound = d_kbound;
    fp.kh = kh;
    fp.unmasked = 0;
    if (nd >= 1) {
        fp.unmasked = 1;
        for (int d = 0; d < nd; d++)
            if (plan.b[d].mask) fp.unmasked = 0;
    }
    if (const char *e = getenv("VH_FIRST_LOADS_FIRST")) fp.unmasked = fp.unmasked && atoi(e) != 0;  // A/B
    fp.s_key = static_cast<unsigned long long *>(ad.s_key);
    fp.s_row = static_cast<unsigned long long *>(ad.s_row);
    fp.list = ws.list.as<uint4>();
    fp.list_fill = d_misc;
    fp.list_cap = list_cap;
    fp.flag = reinterpret_cast<unsigned *>(d_misc + 1);
#ifdef VH_ABLATION
    if (const char *dbg = getenv("VH_FIRST_DEBUG")) fp.debug = (uint32_t)atoi(dbg);
#endif
    {
        TimedScope ts("first_scatter");
        switch (nd) {
        case 1: tf_launch_a<1>(ad.dtype, W, lds_a, plan, ad, fp); break;
        case 2: tf_launch_a<2>(ad.dtype, W, lds_a, plan, ad, fp); break;
        case 3: tf_launch_a<3>(ad.dtype, W, lds_a, plan, ad, fp); break;
        default: tf_launch_a<0>(ad.dtype, W, lds_a, plan, ad, fp);
        }
        VH_HIP(hipGetLastError());
    }
    {
        TimedScope ts("first_reduce");
        hipLaunchKernelGGL(k_first_reduce, dim3((unsigned)units.size()), dim3(TFB_THREADS), (size_t)12 * S, st, fp, d_units);
        VH_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_first_resolve, dim3(blocks_for(list_cap, 256, 4)), dim3(256), 0, st, fp, row0);
        VH_HIP(hipGetLastError());
    }
    unsigned long long *res = reinterpret_cast<unsigned long long *>(stage.as<char>());
    VH_HIP(hipMemcpyAsync(res, d_misc, 16, hipMemcpyDeviceToHost, st));
    VH_HIP(hipStreamSynchronize(st));
    if ((unsigned)res[1]) {
        // the resolve list overflowed: the generic path redoes this chunk from clean scratch
        VH_HIP(hipMemsetAsync(ad.s_key, 0xff, cells * 8, st));
        VH_HIP(hipMemsetAsync(ad.s_row, 0xff, cells * 8, st));
        return false;
    }
    __atomic_add_fetch(&g_first_tiled_chunks, 1ull, __ATOMIC_RELAXED);
    return true;
}

}  // namespace vh
