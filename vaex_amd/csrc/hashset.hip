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
#include <limits>
#include <memory>
#include <mutex>
#include <numeric>

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

template <typename T>
__global__ __launch_bounds__(256) void k_set_insert(const T *keys, const uint8_t *mask, const uint8_t *select, uint64_t n,
                                                    uint64_t row0, uint64_t *tab, uint64_t cap_mask, uint64_t limit,
                                                    uint64_t *ctr) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t row = row0 + i;
        if (select && !select[i]) continue;  // filtered out / not selected
        if (mask && mask[i]) {
            atomicMin((unsigned long long *)&ctr[C_NULL_FIRST], (unsigned long long)row);
            atomicAdd((unsigned long long *)&ctr[C_NULL_COUNT], 1ULL);
            continue;
        }
        const T v = keys[i];
        if (is_nan_v(v)) {
            atomicMin((unsigned long long *)&ctr[C_NAN_FIRST], (unsigned long long)row);
            atomicAdd((unsigned long long *)&ctr[C_NAN_COUNT], 1ULL);
            continue;
        }
        const uint64_t kb = key_bits(v);
        if (kb == SET_EMPTY) {
            atomicMin((unsigned long long *)&ctr[C_SPECIAL_FIRST], (unsigned long long)row);
            continue;
        }
        uint64_t pos = hash64(kb) & cap_mask;
        int p = 0;
        bool refused = false;
        for (; p <= SET_MAX_PROBE; p++) {
            uint64_t k = __hip_atomic_load(&tab[2 * pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (k == kb) break;
            if (k == SET_EMPTY) {
                // a new key: refuse it once the table holds `limit` keys (the host grows the
                // table and re-runs the chunk)
                if (__hip_atomic_load(&ctr[C_DISTINCT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= limit) {
                    refused = true;
                    break;
                }
                uint64_t old = atomicCAS((unsigned long long *)&tab[2 * pos], (unsigned long long)SET_EMPTY,
                                         (unsigned long long)kb);
                if (old == SET_EMPTY) {
                    atomicAdd((unsigned long long *)&ctr[C_DISTINCT], 1ULL);
                    break;
                }
                if (old == kb) break;
            }
            pos = (pos + 1) & cap_mask;
        }
        if (refused || p > SET_MAX_PROBE) {
            ctr[C_OVERFLOW] = 1;
            continue;
        }
        if (__hip_atomic_load(&tab[2 * pos + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > row)
            atomicMin((unsigned long long *)&tab[2 * pos + 1], (unsigned long long)row);
    }
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

__global__ void k_set_compact(const uint64_t *tab, uint64_t cap, uint64_t *slot, uint64_t *first, uint64_t *bits,
                              uint64_t *ctr) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t kb = tab[2 * i];
        if (kb == SET_EMPTY) continue;
        const uint64_t j = atomicAdd((unsigned long long *)&ctr[C_CURSOR], 1ULL);
        slot[j] = i;
        first[j] = tab[2 * i + 1];
        bits[j] = kb;
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
    hipLaunchKernelGGL(k_set_compact, dim3(blocks_for(cap, 256)), dim3(256), 0, stream(), s->tab.as<uint64_t>(), cap,
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

static void set_update(vh_set *s, const void *keys, const uint8_t *mask, const uint8_t *select, uint64_t n, int loc) {
    loc = resolve_loc(keys, loc);
    const int isz = dtype_itemsize(s->dtype);
    // Chunks start at cap/4 rows and double after every chunk that did not need the table
    // to grow, so a too-small table is found after a cheap chunk and a settled one is
    // streamed in a few large launches.  Inside a launch, new keys past `limit` (3/4 of the
    // capacity) are refused and flag overflow; the table then grows and the chunk re-runs.
    const uint64_t stage_max = loc == VH_LOC_HOST ? (uint64_t(1) << 24) : ~0ULL;
    uint64_t want = std::max<uint64_t>(s->cap / 4, 1 << 16);
    for (uint64_t row0 = 0, len = 0; row0 < n; row0 += len) {
        len = std::min({want, stage_max, n - row0});
        const void *dk = reinterpret_cast<const char *>(keys) + row0 * isz;
        const uint8_t *dm = mask ? mask + row0 : nullptr;
        const uint8_t *ds = select ? select + row0 : nullptr;
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
        bool grew = false;
        for (int attempt = 0;; attempt++) {
            {
                TimedScope ts("set_insert");
                const uint64_t limit = s->cap / 4 * 3;
                VH_DISPATCH_DTYPE(s->dtype, T,
                                  hipLaunchKernelGGL(k_set_insert<T>, dim3(std::min<uint64_t>(blocks_for(len, 256), 1 << 16)),
                                                     dim3(256), 0, stream(), reinterpret_cast<const T *>(dk), dm, ds, len,
                                                     s->rows_seen + row0, s->tab.as<uint64_t>(), s->cap - 1, limit,
                                                     s->ctr.as<uint64_t>()));
                VH_HIP(hipGetLastError());
            }
            auto c = read_ctr(s);
            const bool overflow = c[C_OVERFLOW] != 0;
            if (overflow || c[C_DISTINCT] * 2 > s->cap) {
                uint64_t nc = s->cap * 4;
                while (c[C_DISTINCT] * 2 > nc) nc *= 2;
                set_grow(s, nc);
                grew = true;
                uint64_t zero = 0;
                VH_HIP(hipMemcpyAsync(s->ctr.as<uint64_t>() + C_OVERFLOW, &zero, 8, hipMemcpyHostToDevice, stream()));
            }
            if (!overflow) break;
            if (attempt > 16) fail(VH_ERR_RUNTIME, "hash set could not grow enough");
        }
        want = grew ? std::max<uint64_t>(want, s->cap / 4) : want * 2;
    }
    s->rows_seen += n;
    {
        auto c = read_ctr(s);
        if (c[C_NAN_FIRST] != ~0ULL && s->nan_pos == ~0ULL) s->nan_pos = s->rows_seen;
        if (c[C_NULL_FIRST] != ~0ULL && s->null_pos == ~0ULL) s->null_pos = s->rows_seen;
    }
    s->sealed = false;
    VH_HIP(hipStreamSynchronize(stream()));
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
