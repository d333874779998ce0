// Element-wise expression evaluation on HBM columns: the device side of vaex's expression
// evaluation for virtual columns, selections and filters (the reference evaluates them
// with numpy per chunk, cpu.py:542-581, execution.py:337-341, dataframe.py evaluate).
//
// An expression arrives as a small stack program compiled on the host
// (vaex_amd/expr.py): the host resolves numpy's type promotion for every node, so the
// device only runs typed operations on 64-bit slots (float64 or int64 bits) and applies
// the node's rounding (float32) or wrap-around (narrow ints) where numpy would.  The
// stack lives in registers: a push shifts the fixed slots up, a binary operation shifts
// them down, so no slot is ever indexed dynamically (no scratch memory).  Each thread
// evaluates EX_RPT rows per instruction fetch; the program is uniform, so every branch on
// the opcode is a scalar branch.
#include "common.hpp"

#include <algorithm>
#include <cmath>

namespace vh {

constexpr int EX_MAX_CODE = 128;
constexpr int EX_MAX_CONST = 32;
constexpr int EX_MAX_COLS = 16;
constexpr int EX_DEPTH = 8;
constexpr int EX_THREADS = 256;

// opcodes (vaex_amd/expr.py mirrors these numbers)
enum : uint32_t {
    OP_COL = 0, OP_CONST = 1, OP_I2F = 2, OP_F2I = 3, OP_ROUND_F32 = 4, OP_WRAP = 5, OP_U2F = 6,
    OP_ADD_F = 10, OP_SUB_F = 11, OP_MUL_F = 12, OP_DIV_F = 13, OP_FLOORDIV_F = 14, OP_MOD_F = 15,
    OP_POW_F = 16, OP_NEG_F = 17, OP_ABS_F = 18, OP_MIN_F = 19, OP_MAX_F = 20, OP_ARCTAN2 = 21,
    OP_ADD_I = 30, OP_SUB_I = 31, OP_MUL_I = 32, OP_FLOORDIV_I = 33, OP_MOD_I = 34, OP_NEG_I = 35,
    OP_ABS_I = 36, OP_AND_I = 37, OP_OR_I = 38, OP_XOR_I = 39, OP_INV_I = 40, OP_MIN_I = 41, OP_MAX_I = 42,
    OP_SHL_I = 43, OP_SHR_I = 44, OP_POW_I = 45,
    OP_LT_F = 50, OP_LE_F = 51, OP_GT_F = 52, OP_GE_F = 53, OP_EQ_F = 54, OP_NE_F = 55,
    OP_LT_I = 60, OP_LE_I = 61, OP_GT_I = 62, OP_GE_I = 63, OP_EQ_I = 64, OP_NE_I = 65,
    OP_LT_U = 66, OP_LE_U = 67, OP_GT_U = 68, OP_GE_U = 69,
    OP_NOT_B = 70,
    OP_SQRT = 80, OP_EXP = 81, OP_LOG = 82, OP_LOG10 = 83, OP_SIN = 84, OP_COS = 85, OP_TAN = 86,
    OP_ARCSIN = 87, OP_ARCCOS = 88, OP_ARCTAN = 89, OP_SINH = 90, OP_COSH = 91, OP_TANH = 92,
    OP_FLOOR = 93, OP_CEIL = 94, OP_ISNAN = 95, OP_ISFINITE = 96, OP_ISINF = 97, OP_LOG1P = 98,
    OP_EXPM1 = 99, OP_LOG2 = 100, OP_EXP2 = 101, OP_TRUNC = 102, OP_RINT = 103,
    OP_WHERE = 110,
};

struct ExprProg {
    uint32_t code[EX_MAX_CODE];  // op | arg << 8
    uint64_t consts[EX_MAX_CONST];
    const void *cols[EX_MAX_COLS];
    int32_t col_dtype[EX_MAX_COLS];
    int32_t ncode;
    int32_t out_dtype;
};

__device__ inline double as_f(uint64_t b) { return __builtin_bit_cast(double, b); }
__device__ inline uint64_t fb(double d) { return __builtin_bit_cast(uint64_t, d); }
__device__ inline int64_t as_i(uint64_t b) { return (int64_t)b; }

// a column value as its 64-bit slot: floats as float64 bits, integers sign/zero-extended
__device__ inline uint64_t load_slot(const void *p, int dtype, uint64_t i) {
    switch (dtype) {
    case VH_F64: return fb(static_cast<const double *>(p)[i]);
    case VH_F32: return fb((double)static_cast<const float *>(p)[i]);
    case VH_I64: return (uint64_t)static_cast<const int64_t *>(p)[i];
    case VH_I32: return (uint64_t)(int64_t)static_cast<const int32_t *>(p)[i];
    case VH_I16: return (uint64_t)(int64_t)static_cast<const int16_t *>(p)[i];
    case VH_I8: return (uint64_t)(int64_t)static_cast<const int8_t *>(p)[i];
    case VH_U64: return static_cast<const uint64_t *>(p)[i];
    case VH_U32: return static_cast<const uint32_t *>(p)[i];
    case VH_U16: return static_cast<const uint16_t *>(p)[i];
    default: return static_cast<const uint8_t *>(p)[i];  // uint8, bool (0 / 1)
    }
}

__device__ inline int64_t floordiv_i(int64_t a, int64_t b) {
    if (b == 0) return 0;  // numpy: 0 (with a warning)
    if (b == -1) return (int64_t)(0 - (uint64_t)a);
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) q -= 1;
    return q;
}

__device__ inline int64_t mod_i(int64_t a, int64_t b) {
    if (b == 0 || b == -1) return 0;
    int64_t r = a % b;
    if (r != 0 && ((r < 0) != (b < 0))) r += b;
    return r;
}

// numpy's float floor_divide / remainder (npy_divmod): the remainder takes the divisor's
// sign, the quotient is floored and corrected by one where fmod rounds
__device__ inline void divmod_f(double a, double b, double *q, double *r) {
    double mod = fmod(a, b);
    if (b == 0.0) {
        *r = mod;
        *q = a / b;
        return;
    }
    double div = (a - mod) / b;
    if (mod != 0.0) {
        if ((b < 0) != (mod < 0)) {
            mod += b;
            div -= 1.0;
        }
    } else {
        mod = copysign(0.0, b);
    }
    double fl;
    if (div != 0.0) {
        fl = floor(div);
        if (div - fl > 0.5) fl += 1.0;
    } else {
        fl = copysign(0.0, a / b);
    }
    *q = fl;
    *r = mod;
}

__device__ inline int64_t pow_i(int64_t base, int64_t e) {
    if (e < 0) return 0;  // numpy raises for integer ** negative; the host rejects constants
    int64_t r = 1;
    uint64_t ub = (uint64_t)base, ur = 1;
    while (e) {
        if (e & 1) ur *= ub;
        ub *= ub;
        e >>= 1;
    }
    r = (int64_t)ur;
    return r;
}

template <bool MATH> __device__ inline uint64_t unary(uint32_t op, uint32_t arg, uint64_t x) {
    const double f = as_f(x);
    const int64_t v = as_i(x);
    if constexpr (MATH) {
        switch (op) {
        case OP_SQRT: return fb(sqrt(f));
        case OP_EXP: return fb(exp(f));
        case OP_LOG: return fb(log(f));
        case OP_LOG10: return fb(log10(f));
        case OP_LOG2: return fb(log2(f));
        case OP_EXP2: return fb(exp2(f));
        case OP_LOG1P: return fb(log1p(f));
        case OP_EXPM1: return fb(expm1(f));
        case OP_SIN: return fb(sin(f));
        case OP_COS: return fb(cos(f));
        case OP_TAN: return fb(tan(f));
        case OP_ARCSIN: return fb(asin(f));
        case OP_ARCCOS: return fb(acos(f));
        case OP_ARCTAN: return fb(atan(f));
        case OP_SINH: return fb(sinh(f));
        case OP_COSH: return fb(cosh(f));
        case OP_TANH: return fb(tanh(f));
        }
    }
    switch (op) {
    case OP_I2F: return fb((double)v);
    case OP_U2F: return fb((double)x);
    case OP_F2I: return (uint64_t)(int64_t)f;
    case OP_ROUND_F32: return fb((double)(float)f);
    case OP_WRAP: {
        const uint32_t bits = arg & 0xff, sgn = arg >> 8;
        const uint64_t m = bits >= 64 ? ~0ull : ((1ull << bits) - 1);
        uint64_t u = x & m;
        if (sgn && bits < 64 && (u >> (bits - 1)) & 1) u |= ~m;
        return u;
    }
    case OP_NEG_F: return fb(-f);
    case OP_ABS_F: return fb(fabs(f));
    case OP_NEG_I: return (uint64_t)(0 - x);
    case OP_ABS_I: return v < 0 ? (uint64_t)(0 - x) : x;
    case OP_INV_I: return ~x;
    case OP_NOT_B: return x ? 0 : 1;
    case OP_FLOOR: return fb(floor(f));
    case OP_CEIL: return fb(ceil(f));
    case OP_TRUNC: return fb(trunc(f));
    case OP_RINT: return fb(rint(f));
    case OP_ISNAN: return f != f;
    case OP_ISFINITE: return isfinite(f) ? 1 : 0;
    case OP_ISINF: return isinf(f) ? 1 : 0;
    }
    return x;
}

template <bool MATH> __device__ inline uint64_t binary(uint32_t op, uint64_t a, uint64_t b) {
    const double fa = as_f(a), fbv = as_f(b);
    const int64_t ia = as_i(a), ib = as_i(b);
    switch (op) {
    case OP_ADD_F: return fb(fa + fbv);
    case OP_SUB_F: return fb(fa - fbv);
    case OP_MUL_F: return fb(fa * fbv);
    case OP_DIV_F: return fb(fa / fbv);
    case OP_FLOORDIV_F: {
        double q, r;
        divmod_f(fa, fbv, &q, &r);
        return fb(q);
    }
    case OP_MOD_F: {
        double q, r;
        divmod_f(fa, fbv, &q, &r);
        return fb(r);
    }
    case OP_POW_F: if constexpr (MATH) return fb(pow(fa, fbv)); else return a;
    case OP_MIN_F: return fb((fa != fa || fbv != fbv) ? (fa != fa ? fa : fbv) : (fa < fbv ? fa : fbv));
    case OP_MAX_F: return fb((fa != fa || fbv != fbv) ? (fa != fa ? fa : fbv) : (fa > fbv ? fa : fbv));
    case OP_ARCTAN2: if constexpr (MATH) return fb(atan2(fa, fbv)); else return a;
    case OP_ADD_I: return a + b;
    case OP_SUB_I: return a - b;
    case OP_MUL_I: return a * b;
    case OP_FLOORDIV_I: return (uint64_t)floordiv_i(ia, ib);
    case OP_MOD_I: return (uint64_t)mod_i(ia, ib);
    case OP_AND_I: return a & b;
    case OP_OR_I: return a | b;
    case OP_XOR_I: return a ^ b;
    case OP_MIN_I: return ia < ib ? a : b;
    case OP_MAX_I: return ia > ib ? a : b;
    case OP_SHL_I: return (ib < 0 || ib >= 64) ? 0 : a << ib;
    case OP_SHR_I: return (ib < 0 || ib >= 64) ? (uint64_t)(ia < 0 ? -1 : 0) : (uint64_t)(ia >> ib);
    case OP_POW_I: return (uint64_t)pow_i(ia, ib);
    case OP_LT_F: return fa < fbv;
    case OP_LE_F: return fa <= fbv;
    case OP_GT_F: return fa > fbv;
    case OP_GE_F: return fa >= fbv;
    case OP_EQ_F: return fa == fbv;
    case OP_NE_F: return fa != fbv;
    case OP_LT_I: return ia < ib;
    case OP_LE_I: return ia <= ib;
    case OP_GT_I: return ia > ib;
    case OP_GE_I: return ia >= ib;
    case OP_EQ_I: return a == b;
    case OP_NE_I: return a != b;
    case OP_LT_U: return a < b;
    case OP_LE_U: return a <= b;
    case OP_GT_U: return a > b;
    case OP_GE_U: return a >= b;
    }
    return a;
}

__host__ __device__ inline bool is_binary(uint32_t op) {
    return (op >= OP_ADD_F && op <= OP_ARCTAN2 && op != OP_NEG_F && op != OP_ABS_F) ||
           (op >= OP_ADD_I && op <= OP_POW_I && op != OP_NEG_I && op != OP_ABS_I && op != OP_INV_I) ||
           (op >= OP_LT_F && op <= OP_GE_U);
}

// MATH: the program calls transcendental functions (pow, exp, sin, ...), whose inlined
// libm bodies need many registers, so that variant evaluates one row per thread; the
// arithmetic / comparison / logic variant evaluates EX_RPT
__host__ __device__ inline bool is_math(uint32_t op) {
    return op == OP_POW_F || op == OP_ARCTAN2 || (op >= OP_SQRT && op <= OP_TANH) || op == OP_LOG2 ||
           op == OP_EXP2 || op == OP_LOG1P || op == OP_EXPM1;
}

template <bool MATH, int EX_RPT>
__global__ __launch_bounds__(EX_THREADS) void k_expr(ExprProg prog, uint64_t n, void *out) {
    const uint64_t stride = (uint64_t)gridDim.x * EX_THREADS * EX_RPT;
    for (uint64_t base = (uint64_t)blockIdx.x * EX_THREADS * EX_RPT + threadIdx.x; base < n; base += stride) {
        uint64_t s[EX_RPT][EX_DEPTH];
        uint64_t row[EX_RPT];
#pragma unroll
        for (int r = 0; r < EX_RPT; r++) {
            row[r] = base + (uint64_t)r * EX_THREADS;
#pragma unroll
            for (int d = 0; d < EX_DEPTH; d++) s[r][d] = 0;
        }
        for (int pc = 0; pc < prog.ncode; pc++) {
            const uint32_t ins = prog.code[pc];
            const uint32_t op = ins & 0xff, arg = ins >> 8;
            if (op == OP_COL || op == OP_CONST) {
                const void *col = op == OP_COL ? prog.cols[arg] : nullptr;
                const int dt = op == OP_COL ? prog.col_dtype[arg] : 0;
                const uint64_t c = op == OP_CONST ? prog.consts[arg] : 0;
#pragma unroll
                for (int r = 0; r < EX_RPT; r++) {
#pragma unroll
                    for (int d = EX_DEPTH - 1; d > 0; d--) s[r][d] = s[r][d - 1];
                    s[r][0] = op == OP_COL ? (row[r] < n ? load_slot(col, dt, row[r]) : 0) : c;
                }
            } else if (op == OP_WHERE) {
#pragma unroll
                for (int r = 0; r < EX_RPT; r++) {
                    s[r][0] = s[r][2] ? s[r][1] : s[r][0];
#pragma unroll
                    for (int d = 1; d < EX_DEPTH - 2; d++) s[r][d] = s[r][d + 2];
                }
            } else if (is_binary(op)) {
#pragma unroll
                for (int r = 0; r < EX_RPT; r++) {
                    s[r][0] = binary<MATH>(op, s[r][1], s[r][0]);
#pragma unroll
                    for (int d = 1; d < EX_DEPTH - 1; d++) s[r][d] = s[r][d + 1];
                }
            } else {
#pragma unroll
                for (int r = 0; r < EX_RPT; r++) s[r][0] = unary<MATH>(op, arg, s[r][0]);
            }
        }
#pragma unroll
        for (int r = 0; r < EX_RPT; r++) {
            if (row[r] >= n) continue;
            const uint64_t v = s[r][0];
            const uint64_t i = row[r];
            switch (prog.out_dtype) {
            case VH_F64: static_cast<double *>(out)[i] = as_f(v); break;
            case VH_F32: static_cast<float *>(out)[i] = (float)as_f(v); break;
            case VH_I64: case VH_U64: static_cast<uint64_t *>(out)[i] = v; break;
            case VH_I32: case VH_U32: static_cast<uint32_t *>(out)[i] = (uint32_t)v; break;
            case VH_I16: case VH_U16: static_cast<uint16_t *>(out)[i] = (uint16_t)v; break;
            default: static_cast<uint8_t *>(out)[i] = (uint8_t)v; break;
            }
        }
    }
}

// ---- conjunctions / disjunctions of column-vs-constant comparisons -----------------------
// The common filter and selection shape, (a > c1) & (b <= c2) & ...: the interpreter above
// issues each column's loads inside its program step and shifts the register stack per push
// (`w > 0.4` over 1e9 float64 rows: 7.4 ms, 1.2 TB/s, profiles/r06_filter_tl.txt).  Here each
// lane takes 8 consecutive rows: a term's column is read with 16-byte loads (8 rows of its
// dtype), compared with the term's constant by the interpreter's own `binary` / `unary`
// (identical results by construction), folded into the 8 keep bytes, stored as one 8-byte
// word.  vh_expr_eval recognises the program shape; anything else runs the interpreter.
constexpr int EX_MAX_TERMS = 8;
constexpr int EXT_RPT = 8;
struct ExprTerms {
    const void *col[EX_MAX_TERMS];
    uint64_t c[EX_MAX_TERMS];
    int32_t dt[EX_MAX_TERMS];
    uint32_t ucol[EX_MAX_TERMS], ucon[EX_MAX_TERMS], cmp[EX_MAX_TERMS];  // ucol / ucon: 0 or op | arg << 8
    int32_t nt, conj, neg;
};

// 8 consecutive rows' 64-bit slots (load_slot's widening) from 16-byte loads when the column
// block is aligned and whole, else element by element
__device__ inline void load_slots8(const void *p, int dt, uint64_t base, uint32_t cnt, uint64_t (&v)[EXT_RPT]) {
    const int isz = dt == VH_F64 || dt == VH_I64 || dt == VH_U64 ? 8 : dt == VH_F32 || dt == VH_I32 || dt == VH_U32 ? 4
                  : dt == VH_I16 || dt == VH_U16 ? 2 : 1;
    const char *b = static_cast<const char *>(p) + base * isz;
    if (cnt == EXT_RPT && (reinterpret_cast<uintptr_t>(b) & 15) == 0 && isz >= 2) {
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (q * 16 < EXT_RPT * isz) {
                const uint4 u = reinterpret_cast<const uint4 *>(b)[q];
                w[4 * q] = u.x;
                w[4 * q + 1] = u.y;
                w[4 * q + 2] = u.z;
                w[4 * q + 3] = u.w;
            }
        }
#pragma unroll
        for (int r = 0; r < EXT_RPT; r++) {
            uint64_t raw;
            if (isz == 8) raw = (uint64_t)w[2 * r] | ((uint64_t)w[2 * r + 1] << 32);
            else if (isz == 4) raw = w[r];
            else raw = (w[r >> 1] >> (16 * (r & 1))) & 0xffffu;
            switch (dt) {
            case VH_F32: v[r] = fb((double)__builtin_bit_cast(float, (uint32_t)raw)); break;
            case VH_I32: v[r] = (uint64_t)(int64_t)(int32_t)(uint32_t)raw; break;
            case VH_I16: v[r] = (uint64_t)(int64_t)(int16_t)(uint16_t)raw; break;
            default: v[r] = raw;  // float64 bits, int64, uint64 / 32 / 16
            }
        }
        return;
    }
#pragma unroll
    for (int r = 0; r < EXT_RPT; r++) v[r] = (uint32_t)r < cnt ? load_slot(p, dt, base + r) : 0;
}

__global__ __launch_bounds__(EX_THREADS) void k_expr_terms(ExprTerms t, uint64_t n, uint8_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * EX_THREADS * EXT_RPT;
    for (uint64_t base = ((uint64_t)blockIdx.x * EX_THREADS + threadIdx.x) * EXT_RPT; base < n; base += stride) {
        const uint32_t cnt = (uint32_t)min<uint64_t>(EXT_RPT, n - base);
        uint32_t acc[EXT_RPT];
#pragma unroll
        for (int r = 0; r < EXT_RPT; r++) acc[r] = t.conj ? 1u : 0u;
        for (int k = 0; k < t.nt; k++) {
            uint64_t v[EXT_RPT];
            load_slots8(t.col[k], t.dt[k], base, cnt, v);
            const uint32_t uc = t.ucol[k], cop = t.cmp[k];
            const uint64_t c = t.ucon[k] ? unary<false>(t.ucon[k] & 0xff, t.ucon[k] >> 8, t.c[k]) : t.c[k];
#pragma unroll
            for (int r = 0; r < EXT_RPT; r++) {
                const uint64_t x = uc ? unary<false>(uc & 0xff, uc >> 8, v[r]) : v[r];
                const uint32_t bit = (uint32_t)binary<false>(cop, x, c);
                acc[r] = t.conj ? (acc[r] & bit) : (acc[r] | bit);
            }
        }
        uint64_t word = 0;
#pragma unroll
        for (int r = 0; r < EXT_RPT; r++) word |= (uint64_t)((acc[r] ^ (uint32_t)t.neg) & 1u) << (8 * r);
        if (cnt == EXT_RPT && (reinterpret_cast<uintptr_t>(out + base) & 7) == 0) {
            *reinterpret_cast<uint64_t *>(out + base) = word;
        } else {
            for (uint32_t r = 0; r < cnt; r++) out[base + r] = (uint8_t)(word >> (8 * r));
        }
    }
}

// the program as T (T COMB)* [NOT_B] with T = COL [cvt] CONST [cvt] CMP, one COMB kind
// (AND_I or OR_I) and a 1-byte output; false: another shape
static bool match_terms(const uint32_t *code, int ncode, const uint64_t *consts, const void *const *cols,
                        const int *col_dtypes, int out_dtype, ExprTerms &t) {
    if (dtype_itemsize(out_dtype) != 1) return false;
    auto cvt = [](uint32_t op) { return op == OP_I2F || op == OP_U2F || op == OP_ROUND_F32 || op == OP_WRAP; };
    auto cmp = [](uint32_t op) { return op >= OP_LT_F && op <= OP_GE_U; };
    t = ExprTerms{};
    t.conj = -1;
    int i = 0;
    while (i < ncode) {
        if (t.nt == EX_MAX_TERMS) return false;
        uint32_t op = code[i] & 0xff;
        if (op != OP_COL) break;
        const int k = t.nt;
        t.col[k] = cols[code[i] >> 8];
        t.dt[k] = col_dtypes[code[i] >> 8];
        i++;
        if (i < ncode && cvt(code[i] & 0xff)) t.ucol[k] = code[i++];
        if (i >= ncode || (code[i] & 0xff) != OP_CONST) return false;
        t.c[k] = consts[code[i] >> 8];
        i++;
        if (i < ncode && cvt(code[i] & 0xff)) t.ucon[k] = code[i++];
        if (i >= ncode || !cmp(code[i] & 0xff)) return false;
        t.cmp[k] = code[i] & 0xff;
        i++;
        t.nt++;
        if (k > 0) {  // a combiner follows every term after the first
            if (i >= ncode) return false;
            op = code[i] & 0xff;
            const int cj = op == OP_AND_I ? 1 : op == OP_OR_I ? 0 : -1;
            if (cj < 0 || (t.conj >= 0 && cj != t.conj)) return false;
            t.conj = cj;
            i++;
        }
    }
    if (t.nt == 0) return false;
    if (t.conj < 0) t.conj = 1;
    if (i < ncode && (code[i] & 0xff) == OP_NOT_B) {
        t.neg = 1;
        i++;
    }
    return i == ncode;
}

}  // namespace vh

using namespace vh;

static bool getenv_off_expr(const char *name) {  // NAME=0: the interpreter for every program (A/Bs)
    const char *e = getenv(name);
    return e && e[0] == '0' && e[1] == 0;
}

extern "C" int vh_expr_eval(const uint32_t *code, int ncode, const uint64_t *consts, int nconsts,
                            const void *const *cols, const int *col_dtypes, int ncols, uint64_t n, int out_dtype,
                            void *out) {
    VH_API_BEGIN
    if (ncode <= 0 || ncode > EX_MAX_CODE) fail(VH_ERR_ARG, "expression program too long");
    if (nconsts < 0 || nconsts > EX_MAX_CONST) fail(VH_ERR_ARG, "too many expression constants");
    if (ncols < 0 || ncols > EX_MAX_COLS) fail(VH_ERR_ARG, "too many expression columns");
    ExprProg p{};
    // host-side check of the program: operands in range, stack depth within the slots
    int depth = 0, maxd = 0;
    bool math = false;
    for (int i = 0; i < ncode; i++) {
        const uint32_t op = code[i] & 0xff, arg = code[i] >> 8;
        math = math || is_math(op);
        if (op == OP_COL) {
            if ((int)arg >= ncols) fail(VH_ERR_ARG, "expression column index out of range");
            depth++;
        } else if (op == OP_CONST) {
            if ((int)arg >= nconsts) fail(VH_ERR_ARG, "expression constant index out of range");
            depth++;
        } else if (op == OP_WHERE) {
            depth -= 2;
        } else if (is_binary(op)) {
            depth -= 1;
        }
        if (depth < 1) fail(VH_ERR_ARG, "malformed expression program (stack underflow)");
        maxd = std::max(maxd, depth);
        p.code[i] = code[i];
    }
    if (depth != 1) fail(VH_ERR_ARG, "malformed expression program (stack not 1 at the end)");
    if (maxd > EX_DEPTH) fail(VH_ERR_ARG, "expression too deeply nested for the device stack");
    for (int i = 0; i < nconsts; i++) p.consts[i] = consts[i];
    for (int i = 0; i < ncols; i++) {
        p.cols[i] = cols[i];
        p.col_dtype[i] = col_dtypes[i];
        dtype_itemsize(col_dtypes[i]);
    }
    dtype_itemsize(out_dtype);
    p.ncode = ncode;
    p.out_dtype = out_dtype;
    ExprTerms terms;
    if (n && !getenv_off_expr("VH_EXPR_TERMS") &&
        match_terms(code, ncode, consts, cols, col_dtypes, out_dtype, terms)) {
        TimedScope ts("expr");
        const uint64_t per_block = (uint64_t)EX_THREADS * EXT_RPT;
        const unsigned grid = (unsigned)std::min<uint64_t>((n + per_block - 1) / per_block, (uint64_t)cu_count() * 8);
        hipLaunchKernelGGL(k_expr_terms, dim3(grid), dim3(EX_THREADS), 0, stream(), terms, n, static_cast<uint8_t *>(out));
        VH_HIP(hipGetLastError());
    } else if (n) {
        TimedScope ts("expr");
        const uint64_t per_block = (uint64_t)EX_THREADS * (math ? 1 : 4);
        const uint64_t want = (n + per_block - 1) / per_block;
        const unsigned grid = (unsigned)std::min<uint64_t>(want, (uint64_t)cu_count() * 8);
        if (math) hipLaunchKernelGGL((k_expr<true, 1>), dim3(grid), dim3(EX_THREADS), 0, stream(), p, n, out);
        else hipLaunchKernelGGL((k_expr<false, 4>), dim3(grid), dim3(EX_THREADS), 0, stream(), p, n, out);
        VH_HIP(hipGetLastError());
    }
    VH_API_END
}
