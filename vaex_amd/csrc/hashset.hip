// ordered_set_<dtype> on the GPU: the groupby key set of vaex-core
// (packages/vaex-core/src/hash_primitives.hpp:417-621, hash.hpp:124-257),
// rebuilt as one open-address table in HBM instead of nmaps mutex-guarded
// hopscotch maps:
//   update      -- every row inserts its key with a CAS on an EMPTY slot
//                  (linear probing from _hash64(bits), hash.hpp:25-30) and
//                  lowers the slot's first-seen row with atomicMin;
//   seal        -- occupied slots are compacted and ordinals assigned in
//                  first-appearance order (the order a single-threaded
//                  reference update assigns `ordinal = map.size()`,
//                  hash_primitives.hpp:453-461, with nmaps = 1);
//   map_ordinal -- one probe per row (hash_primitives.hpp:556-583).
// NaN and null keys get their own ordinals (nan_value / null_value,
// hash_primitives.hpp:436-450).  The table grows x4 when half full or when a
// probe sequence exceeds SET_MAX_PROBE (the chunk is then re-run: inserts are
// idempotent).
#include <algorithm>
#include <limits>
#include <memory>
#include <numeric>

#include "common.hpp"
#include "hashset.hpp"

using namespace vh;

enum { C_DISTINCT = 0, C_OVERFLOW, C_NAN_FIRST, C_NULL_FIRST, C_SPECIAL_FIRST, C_NAN_COUNT, C_NULL_COUNT, C_CURSOR, C_N };

struct vh_set {
    int dtype = VH_I64;
    uint64_t cap = 0;
    DevBuf keys, first, ords, ctr;
    DevBuf stage_keys, stage_mask;
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
__global__ __launch_bounds__(256) void k_set_insert(const T *keys, const uint8_t *mask, uint64_t n, uint64_t row0,
                                                    uint64_t *tk, uint64_t *tf, uint64_t cap_mask, uint64_t *ctr) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t row = row0 + i;
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
        for (; p <= SET_MAX_PROBE; p++) {
            uint64_t k = __hip_atomic_load(&tk[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (k == kb) break;
            if (k == SET_EMPTY) {
                uint64_t old = atomicCAS((unsigned long long *)&tk[pos], (unsigned long long)SET_EMPTY,
                                         (unsigned long long)kb);
                if (old == SET_EMPTY) {
                    atomicAdd((unsigned long long *)&ctr[C_DISTINCT], 1ULL);
                    break;
                }
                if (old == kb) break;
            }
            pos = (pos + 1) & cap_mask;
        }
        if (p > SET_MAX_PROBE) {
            ctr[C_OVERFLOW] = 1;
            continue;
        }
        if (__hip_atomic_load(&tf[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > row)
            atomicMin((unsigned long long *)&tf[pos], (unsigned long long)row);
    }
}

__global__ void k_set_rehash(const uint64_t *ok, const uint64_t *of, uint64_t ocap, uint64_t *nk, uint64_t *nf,
                             uint64_t ncap_mask) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ocap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t kb = ok[i];
        if (kb == SET_EMPTY) continue;
        uint64_t pos = hash64(kb) & ncap_mask;
        for (;;) {
            uint64_t old = atomicCAS((unsigned long long *)&nk[pos], (unsigned long long)SET_EMPTY,
                                     (unsigned long long)kb);
            if (old == SET_EMPTY) break;
            pos = (pos + 1) & ncap_mask;
        }
        nf[pos] = of[i];
    }
}

__global__ void k_set_compact(const uint64_t *tk, const uint64_t *tf, uint64_t cap, uint64_t *slot, uint64_t *first,
                              uint64_t *bits, uint64_t *ctr) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t kb = tk[i];
        if (kb == SET_EMPTY) continue;
        const uint64_t j = atomicAdd((unsigned long long *)&ctr[C_CURSOR], 1ULL);
        slot[j] = i;
        first[j] = tf[i];
        bits[j] = kb;
    }
}

__global__ void k_set_scatter_ords(const uint64_t *slot, const int64_t *ord, uint64_t m, int64_t *ords) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < m;
         j += (uint64_t)gridDim.x * blockDim.x)
        ords[slot[j]] = ord[j];
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
    DevBuf nk, nf;
    nk.ensure(new_cap * 8);
    nf.ensure(new_cap * 8);
    VH_HIP(hipMemsetAsync(nk.ptr, 0xff, new_cap * 8, stream()));
    VH_HIP(hipMemsetAsync(nf.ptr, 0xff, new_cap * 8, stream()));
    if (s->cap) {
        hipLaunchKernelGGL(k_set_rehash, dim3(blocks_for(s->cap, 256)), dim3(256), 0, stream(), s->keys.as<uint64_t>(),
                           s->first.as<uint64_t>(), s->cap, nk.as<uint64_t>(), nf.as<uint64_t>(), new_cap - 1);
        VH_HIP(hipGetLastError());
    }
    VH_HIP(hipStreamSynchronize(stream()));
    std::swap(s->keys.ptr, nk.ptr);
    std::swap(s->keys.bytes, nk.bytes);
    std::swap(s->first.ptr, nf.ptr);
    std::swap(s->first.bytes, nf.bytes);
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
    hipLaunchKernelGGL(k_set_compact, dim3(blocks_for(cap, 256)), dim3(256), 0, stream(), s->keys.as<uint64_t>(),
                       s->first.as<uint64_t>(), cap, s->c_slot.as<uint64_t>(), s->c_first.as<uint64_t>(),
                       s->c_bits.as<uint64_t>(), s->ctr.as<uint64_t>());
    VH_HIP(hipGetLastError());
    c = read_ctr(s);
    const uint64_t m = c[C_CURSOR];
    std::vector<uint64_t> first(m), bits(m);
    VH_HIP(hipMemcpyAsync(first.data(), s->c_first.ptr, m * 8, hipMemcpyDeviceToHost, stream()));
    VH_HIP(hipMemcpyAsync(bits.data(), s->c_bits.ptr, m * 8, hipMemcpyDeviceToHost, stream()));
    VH_HIP(hipStreamSynchronize(stream()));
    // order: regular keys (index j < m), then the special, nan, null pseudo keys
    struct Ent {
        uint64_t first;
        int tie;
        int64_t j;
    };
    std::vector<Ent> ents(m);
    // sort keys: 2*row for keys, 2*end_of_call - 1 for NaN/null (after that call's keys,
    // before any key first seen by a later call)
    for (uint64_t j = 0; j < m; j++) ents[j] = {2 * first[j], 0, (int64_t)j};
    if (c[C_SPECIAL_FIRST] != ~0ULL) ents.push_back({2 * c[C_SPECIAL_FIRST], 0, -3});
    if (c[C_NAN_FIRST] != ~0ULL) ents.push_back({2 * s->nan_pos - 1, 1, -1});
    if (c[C_NULL_FIRST] != ~0ULL) ents.push_back({2 * s->null_pos - 1, 2, -2});
    std::sort(ents.begin(), ents.end(), [](const Ent &a, const Ent &b) {
        return a.first != b.first ? a.first < b.first : a.tie < b.tie;
    });
    std::vector<int64_t> ord_of(m);
    s->key_bits.assign(ents.size(), 0);
    s->key_kind.assign(ents.size(), 0);
    s->nan_ord = s->null_ord = s->special_ord = -1;
    for (size_t o = 0; o < ents.size(); o++) {
        const int64_t j = ents[o].j;
        if (j >= 0) {
            ord_of[j] = (int64_t)o;
            s->key_bits[o] = bits[j];
        } else if (j == -1) {
            s->nan_ord = (int64_t)o;
            s->key_kind[o] = 1;
        } else if (j == -2) {
            s->null_ord = (int64_t)o;
            s->key_kind[o] = 2;
        } else {
            s->special_ord = (int64_t)o;
            s->key_kind[o] = 3;
            s->key_bits[o] = SET_EMPTY;
        }
    }
    s->ords.ensure(cap * 8);
    if (m) {
        VH_HIP(hipMemcpyAsync(s->c_ord.ptr, ord_of.data(), m * 8, hipMemcpyHostToDevice, stream()));
        hipLaunchKernelGGL(k_set_scatter_ords, dim3(blocks_for(m, 256)), dim3(256), 0, stream(), s->c_slot.as<uint64_t>(),
                           s->c_ord.as<int64_t>(), m, s->ords.as<int64_t>());
        VH_HIP(hipGetLastError());
    }
    VH_HIP(hipStreamSynchronize(stream()));
    s->length = (int64_t)ents.size();
    s->nan_count = (int64_t)c[C_NAN_COUNT];
    s->null_count = (int64_t)c[C_NULL_COUNT];
    s->sealed = true;
}

SetDev set_device_view(vh_set *s) {
    set_seal(s);
    SetDev d{};
    d.keys = s->keys.as<uint64_t>();
    d.ords = s->ords.as<int64_t>();
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

int vh_set_update(vh_set *s, const void *keys, const uint8_t *mask, uint64_t n, int loc) {
    VH_API_BEGIN
    loc = resolve_loc(keys, loc);
    const int isz = dtype_itemsize(s->dtype);
    // Rows are inserted in chunks no longer than the table capacity while the table may
    // still need to grow (a chunk can add at most `len` keys), so a too-small table is
    // detected after one cheap chunk instead of after probing every row to the limit.
    const uint64_t stage_max = loc == VH_LOC_HOST ? (uint64_t(1) << 24) : ~0ULL;
    for (uint64_t row0 = 0, len = 0; row0 < n; row0 += len) {
        // at most cap/4 new keys per chunk on a table kept <= half full: load stays <= 3/4
        len = std::min({s->cap / 4, stage_max, n - row0});
        const void *dk = reinterpret_cast<const char *>(keys) + row0 * isz;
        const uint8_t *dm = mask ? mask + row0 : nullptr;
        if (loc == VH_LOC_HOST) {
            s->stage_keys.ensure(len * isz);
            VH_HIP(hipMemcpyAsync(s->stage_keys.ptr, dk, len * isz, hipMemcpyHostToDevice, stream()));
            dk = s->stage_keys.ptr;
            if (mask) {
                s->stage_mask.ensure(len);
                VH_HIP(hipMemcpyAsync(s->stage_mask.ptr, dm, len, hipMemcpyHostToDevice, stream()));
                dm = s->stage_mask.as<uint8_t>();
            }
        }
        for (int attempt = 0;; attempt++) {
            {
                TimedScope ts("set_insert");
                VH_DISPATCH_DTYPE(s->dtype, T,
                                  hipLaunchKernelGGL(k_set_insert<T>, dim3(blocks_for(len, 256)), dim3(256), 0, stream(),
                                                     reinterpret_cast<const T *>(dk), dm, len, s->rows_seen + row0,
                                                     s->keys.as<uint64_t>(), s->first.as<uint64_t>(), s->cap - 1,
                                                     s->ctr.as<uint64_t>()));
                VH_HIP(hipGetLastError());
            }
            auto c = read_ctr(s);
            const bool overflow = c[C_OVERFLOW] != 0;
            if (overflow || c[C_DISTINCT] * 2 > s->cap) {
                uint64_t nc = s->cap * 4;
                while (c[C_DISTINCT] * 2 > nc) nc *= 2;
                set_grow(s, nc);
                uint64_t zero = 0;
                VH_HIP(hipMemcpyAsync(s->ctr.as<uint64_t>() + C_OVERFLOW, &zero, 8, hipMemcpyHostToDevice, stream()));
            }
            if (!overflow) break;
            if (attempt > 8) fail(VH_ERR_RUNTIME, "hash set could not grow enough");
        }
    }
    s->rows_seen += n;
    {
        auto c = read_ctr(s);
        if (c[C_NAN_FIRST] != ~0ULL && s->nan_pos == ~0ULL) s->nan_pos = s->rows_seen;
        if (c[C_NULL_FIRST] != ~0ULL && s->null_pos == ~0ULL) s->null_pos = s->rows_seen;
    }
    s->sealed = false;
    VH_HIP(hipStreamSynchronize(stream()));
    VH_API_END
}

int vh_set_seal(vh_set *s) {
    VH_API_BEGIN
    set_seal(s);
    VH_API_END
}

int vh_set_info(vh_set *s, int64_t *length, int64_t *nan_count, int64_t *null_count, int64_t *nan_value,
                int64_t *null_value) {
    VH_API_BEGIN
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
    set_seal(s);
    VH_DISPATCH_DTYPE(s->dtype, T, write_keys<T>(s, reinterpret_cast<T *>(out)));
    VH_API_END
}

int vh_set_map_ordinal(vh_set *s, const void *keys, uint64_t n, int loc, void *out, int out_itemsize, int out_loc) {
    VH_API_BEGIN
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
